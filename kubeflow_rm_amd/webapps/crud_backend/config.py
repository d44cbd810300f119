"""Backend modes: dev / development (auth checks skipped) and prod / production."""
import logging
import os

from flask import current_app

DEV_MODES = ("dev", "development")
PROD_MODES = ("prod", "production")


class Config:
    ENV = "production"
    DEBUG = False
    LOG_LEVEL = logging.INFO
    PREFIX = "/"
    STATIC_DIR = ""
    JSON_SORT_KEYS = False

    def __init__(self, mode: str | None = None, prefix: str | None = None):
        mode = (mode or os.getenv("BACKEND_MODE", "prod")).lower()
        if mode not in DEV_MODES + PROD_MODES:
            raise RuntimeError(f"Backend mode '{mode}' is not implemented. Choose one of {list(DEV_MODES + PROD_MODES)}")
        self.ENV = "development" if mode in DEV_MODES else "production"
        self.DEBUG = self.ENV == "development"
        if self.DEBUG or os.getenv("LOG_LEVEL_DEBUG", "false") == "true":
            self.LOG_LEVEL = logging.DEBUG
        self.PREFIX = prefix or os.getenv("APP_PREFIX", "/")


def dev_mode_enabled() -> bool:
    return current_app.config.get("ENV") == "development"
