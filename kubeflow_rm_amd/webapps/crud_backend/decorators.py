"""Body validation for the mutating routes: a JSON content type, an object body, named fields.

A failed check is a 400 with the reference's messages, so the frontends' error snack-bars read the
same text.
"""
import functools

from flask import request
from werkzeug import exceptions


def _check_json_type():
    if request.content_type != "application/json":
        raise exceptions.BadRequest("Request is not in JSON format.")


def _json_object():
    body = request.get_json(silent=True)
    if not isinstance(body, dict):
        raise exceptions.BadRequest("Request doesn't have a JSON object body.")
    return body


def request_is_json_type(view):
    @functools.wraps(view)
    def checked(*args, **kwargs):
        _check_json_type()
        return view(*args, **kwargs)
    return checked


def required_body_params(*names):
    def wrap(view):
        @functools.wraps(view)
        def checked(*args, **kwargs):
            missing = [n for n in names if n not in _json_object()]
            if missing:
                raise exceptions.BadRequest(f"Parameter '{missing[0]}' is missing from the request's body.")
            return view(*args, **kwargs)
        return checked
    return wrap
