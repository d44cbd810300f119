"""Fallback process image: answers 200 on every declared container port (KFAMD_CONTAINER_PORTS).

Used for images that have no dedicated recipe so that Services, probes and the gateway see a
live endpoint; the container log records the image it stands in for.
"""
from __future__ import annotations

import os
import sys
import time

from ._http import JsonHandler, run_forever, serve


class H(JsonHandler):
    def do_GET(self):
        self.send_json(200, {"ok": True, "container": os.environ.get("KFAMD_CONTAINER_NAME"), "path": self.path})

    do_POST = do_GET
    do_PUT = do_GET
    do_DELETE = do_GET


def main(argv=None) -> int:
    ports = [int(p) for p in (os.environ.get("KFAMD_CONTAINER_PORTS") or "").split(",") if p]
    print(f"[kflite-generic] container={os.environ.get('KFAMD_CONTAINER_NAME')} argv={argv} ports={ports}", flush=True)
    if not ports:
        while True:
            time.sleep(3600)
    run_forever([serve(H, p) for p in ports])
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
