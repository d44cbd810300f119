"""Authorization: one SubjectAccessReview per Kubernetes call made on the user's behalf."""
import functools
import logging

from werkzeug.exceptions import Forbidden, Unauthorized

from . import authn, config, k8s, settings

log = logging.getLogger(__name__)


def is_authorized(user, verb, group, version, resource, namespace=None, subresource=None) -> bool:
    if config.dev_mode_enabled() or settings.DISABLE_AUTH:
        return True
    if user is None:
        raise Unauthorized(description="No user credentials were found!")
    sar = k8s.client().subject_access_review(user, verb, group, resource, namespace=namespace, subresource=subresource)
    status = sar.get("status")
    return bool(status and status.get("allowed"))


def unauthorized_message(user, verb, group, version, resource, subresource=None, namespace=None) -> str:
    msg = f"User '{user}' is not authorized to {verb}"
    msg += f" {version}/{resource}" if group == "" else f" {group}/{version}/{resource}"
    if subresource is not None:
        msg += f"/{subresource}"
    if namespace is not None:
        msg += f" in namespace '{namespace}'"
    return msg


def ensure_authorized(verb, group, version, resource, namespace=None, subresource=None) -> None:
    user = authn.get_username()
    if not is_authorized(user, verb, group, version, resource, namespace=namespace, subresource=subresource):
        raise Forbidden(description=unauthorized_message(user, verb, group, version, resource, subresource, namespace))


def needs_authorization(verb, group, version, resource, namespace=None, subresource=None):
    def wrapper(func):
        @functools.wraps(func)
        def runner(*a, **kw):
            ensure_authorized(verb, group, version, resource, namespace=namespace, subresource=subresource)
            return func(*a, **kw)
        return runner
    return wrapper
