"""TensorBoard event files without TensorFlow: TFRecord framing (masked CRC32C) + the few protobuf
fields of ``Event`` / ``Summary`` that scalar dashboards need, encoded/decoded by hand.

Writer: ``SummaryWriter(logdir).add_scalar(tag, value, step)`` (used by notebooks and the
training examples to log loss / TFLOPS). Reader: ``read_scalars(path)`` (used by the
tensorboard image). Format: tensorflow/core/util/event.proto, summary.proto, tensor.proto.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Iterator

# ---- CRC32C (Castagnoli), table driven -------------------------------------------------------
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---- protobuf wire helpers -------------------------------------------------------------------
def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _read_varint(buf: bytes, i: int) -> tuple[int, int]:
    shift = n = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7


def _fields(buf: bytes) -> Iterator[tuple[int, int, object]]:
    i = 0
    while i < len(buf):
        k, i = _read_varint(buf, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(buf, i)
        elif w == 1:
            v = buf[i:i + 8]
            i += 8
        elif w == 2:
            n, i = _read_varint(buf, i)
            v = buf[i:i + n]
            i += n
        elif w == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def encode_scalar_event(tag: str, value: float, step: int, wall_time: float | None = None) -> bytes:
    val = _ld(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))
    summary = _ld(1, val)
    return (_key(1, 1) + struct.pack("<d", wall_time if wall_time is not None else time.time())
            + _key(2, 0) + _varint(int(step)) + _ld(5, summary))


def _file_version_event() -> bytes:
    return _key(1, 1) + struct.pack("<d", time.time()) + _ld(3, b"brain.Event:2")


def frame(record: bytes) -> bytes:
    hdr = struct.pack("<Q", len(record))
    return hdr + struct.pack("<I", masked_crc(hdr)) + record + struct.pack("<I", masked_crc(record))


class SummaryWriter:
    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}{filename_suffix}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._f.write(frame(_file_version_event()))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, step: int, wall_time: float | None = None) -> None:
        self._f.write(frame(encode_scalar_event(tag, value, step, wall_time)))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if len(hdr) < 12:
                return
            (n,) = struct.unpack("<Q", hdr[:8])
            if verify and struct.unpack("<I", hdr[8:])[0] != masked_crc(hdr[:8]):
                raise ValueError(f"{path}: corrupt record header")
            data = f.read(n)
            crc = f.read(4)
            if len(data) < n or len(crc) < 4:
                return  # partially written tail
            if verify and struct.unpack("<I", crc)[0] != masked_crc(data):
                raise ValueError(f"{path}: corrupt record")
            yield data


def _tensor_scalar(buf: bytes) -> float | None:
    dtype = None
    for f, w, v in _fields(buf):
        if f == 1 and w == 0:
            dtype = v
        elif f == 4 and w == 2:  # tensor_content
            if dtype == 2 and len(v) >= 8:
                return struct.unpack("<d", v[:8])[0]
            if len(v) >= 4:
                return struct.unpack("<f", v[:4])[0]
        elif f == 5:  # float_val (packed or not)
            if w == 2 and len(v) >= 4:
                return struct.unpack("<f", v[:4])[0]
            if w == 5:
                return struct.unpack("<f", v)[0]
        elif f == 6:  # double_val
            if w == 2 and len(v) >= 8:
                return struct.unpack("<d", v[:8])[0]
            if w == 1:
                return struct.unpack("<d", v)[0]
    return None


def decode_event(buf: bytes) -> dict:
    ev: dict = {"wall_time": 0.0, "step": 0, "scalars": []}
    for f, w, v in _fields(buf):
        if f == 1 and w == 1:
            ev["wall_time"] = struct.unpack("<d", v)[0]
        elif f == 2 and w == 0:
            ev["step"] = v
        elif f == 3 and w == 2:
            ev["file_version"] = v.decode(errors="replace")
        elif f == 5 and w == 2:
            for sf, sw, sv in _fields(v):
                if sf != 1 or sw != 2:
                    continue
                tag, val = None, None
                for vf, vw, vv in _fields(sv):
                    if vf == 1 and vw == 2:
                        tag = vv.decode(errors="replace")
                    elif vf == 2 and vw == 5:
                        val = struct.unpack("<f", vv)[0]
                    elif vf == 8 and vw == 2:
                        val = _tensor_scalar(vv)
                if tag is not None and val is not None:
                    ev["scalars"].append((tag, val))
    return ev


def read_scalars(path: str) -> dict[str, list[tuple[float, int, float]]]:
    """tag -> [(wall_time, step, value)] for one event file."""
    out: dict[str, list] = {}
    for rec in read_records(path):
        ev = decode_event(rec)
        for tag, val in ev["scalars"]:
            out.setdefault(tag, []).append((ev["wall_time"], ev["step"], val))
    return out


def find_runs(logdir: str) -> dict[str, list[str]]:
    """run name (dir relative to logdir, "." for the root) -> event files."""
    runs: dict[str, list[str]] = {}
    for root, _dirs, files in os.walk(logdir):
        ev = sorted(os.path.join(root, f) for f in files if "tfevents" in f)
        if ev:
            rel = os.path.relpath(root, logdir)
            runs[rel] = ev
    return runs
