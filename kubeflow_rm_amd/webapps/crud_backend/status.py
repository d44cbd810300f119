"""Status vocabulary shared by the backends and the frontends' status icons.

Every list row carries ``status = {phase, message, state}``; ``phase`` is one of the names below
(the frontends map them to icons: kf.js ``statusCell``).
"""
import enum


class Phase(str, enum.Enum):
    READY = "ready"
    WAITING = "waiting"
    WARNING = "warning"
    ERROR = "error"
    UNINITIALIZED = "uninitialized"
    UNAVAILABLE = "unavailable"
    TERMINATING = "terminating"
    STOPPED = "stopped"


# attribute-style access used by the app modules (STATUS_PHASE.READY == "ready")
STATUS_PHASE = type("STATUS_PHASE", (), {p.name: p.value for p in Phase})


def create_status(phase: str = "", message: str = "", state: str = "") -> dict:
    return dict(phase=str(phase), message=message, state=state)
