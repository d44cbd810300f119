"""Environment settings of the CRUD backends (reference crud_backend/settings.py semantics)."""
import os


def _bool(name: str, default: str) -> bool:
    return os.getenv(name, default).lower() == "true"


SECURE_COOKIES = _bool("APP_SECURE_COOKIES", "true")
DISABLE_AUTH = _bool("APP_DISABLE_AUTH", "false")
USER_HEADER = os.getenv("USERID_HEADER", "kubeflow-userid")
USER_PREFIX = os.getenv("USERID_PREFIX", ":")
CSRF_SAMESITE = os.getenv("CSRF_SAMESITE", "Strict")


def reload() -> None:
    """Re-read the environment (tests change it between apps)."""
    global SECURE_COOKIES, DISABLE_AUTH, USER_HEADER, USER_PREFIX, CSRF_SAMESITE
    SECURE_COOKIES = _bool("APP_SECURE_COOKIES", "true")
    DISABLE_AUTH = _bool("APP_DISABLE_AUTH", "false")
    USER_HEADER = os.getenv("USERID_HEADER", "kubeflow-userid")
    USER_PREFIX = os.getenv("USERID_PREFIX", ":")
    CSRF_SAMESITE = os.getenv("CSRF_SAMESITE", "Strict")
