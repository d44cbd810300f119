"""CSRF protection for the AJAX frontends: double-submit cookie (XSRF-TOKEN refreshed whenever
index.html is served, readable by JS) checked against the X-XSRF-TOKEN header on every
non-safe method; SameSite from CSRF_SAMESITE, Secure from APP_SECURE_COOKIES."""
import secrets

from flask import current_app, request
from werkzeug.exceptions import Forbidden

from . import settings

CSRF_COOKIE = "XSRF-TOKEN"
CSRF_HEADER = "X-" + CSRF_COOKIE
SAMESITE_VALUES = ("Strict", "Lax", "None")
SAFE_METHODS = ("GET", "HEAD", "OPTIONS", "TRACE")
NO_CACHE = "no-cache, no-store, must-revalidate, max-age=0"


def set_cookie(resp):
    samesite = settings.CSRF_SAMESITE if settings.CSRF_SAMESITE in SAMESITE_VALUES else "Strict"
    resp.set_cookie(key=CSRF_COOKIE, value=secrets.token_urlsafe(32), samesite=samesite, httponly=False,
                    secure=settings.SECURE_COOKIES, path=current_app.config["PREFIX"])
    resp.headers["Cache-Control"] = NO_CACHE


def check_endpoint():
    if request.method in SAFE_METHODS:
        return None
    if CSRF_COOKIE not in request.cookies:
        raise Forbidden(f"Could not find CSRF cookie {CSRF_COOKIE} in the request.")
    if CSRF_HEADER not in request.headers:
        raise Forbidden(f"Could not detect CSRF protection header {CSRF_HEADER}.")
    if request.headers[CSRF_HEADER] != request.cookies[CSRF_COOKIE]:
        raise Forbidden(f"CSRF check failed. Token in cookie {CSRF_COOKIE} doesn't match token in header {CSRF_HEADER}.")
    return None
