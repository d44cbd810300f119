"""Status phases the frontends understand (crud_backend/status.py contract)."""


class STATUS_PHASE:
    READY = "ready"
    WAITING = "waiting"
    WARNING = "warning"
    ERROR = "error"
    UNINITIALIZED = "uninitialized"
    UNAVAILABLE = "unavailable"
    TERMINATING = "terminating"
    STOPPED = "stopped"


def create_status(phase: str = "", message: str = "", state: str = "") -> dict:
    return {"phase": phase, "message": message, "state": state}
