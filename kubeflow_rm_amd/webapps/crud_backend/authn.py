"""Authentication: the user comes from a trusted header set by the ingress (USERID_HEADER minus
USERID_PREFIX); every route requires it unless dev mode, APP_DISABLE_AUTH or @no_authentication."""
import logging

from flask import current_app, request
from werkzeug.exceptions import Unauthorized

from . import config, settings

log = logging.getLogger(__name__)


def get_username():
    if settings.USER_HEADER not in request.headers:
        return None
    return request.headers[settings.USER_HEADER].replace(settings.USER_PREFIX, "")


def no_authentication(func):
    func.no_authentication = True
    return func


def check_authentication():
    if config.dev_mode_enabled() or settings.DISABLE_AUTH:
        return None
    if request.endpoint and getattr(current_app.view_functions.get(request.endpoint), "no_authentication", False):
        return None
    if get_username() is None:
        raise Unauthorized("No user detected.")
    return None
