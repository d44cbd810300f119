"""Route decorators: JSON content type and required body fields (400 otherwise)."""
import functools

from flask import request
from werkzeug import exceptions


def request_is_json_type(func):
    @functools.wraps(func)
    def wrapper(*a, **kw):
        if request.content_type != "application/json":
            raise exceptions.BadRequest("Request is not in JSON format.")
        return func(*a, **kw)
    return wrapper


def required_body_params(*params):
    def deco(func):
        @functools.wraps(func)
        def runner(*a, **kw):
            body = request.get_json(silent=True)
            if not isinstance(body, dict):
                raise exceptions.BadRequest("Request doesn't have a JSON object body.")
            for p in params:
                if p not in body:
                    raise exceptions.BadRequest(f"Parameter '{p}' is missing from the request's body.")
            return func(*a, **kw)
        return runner
    return deco
