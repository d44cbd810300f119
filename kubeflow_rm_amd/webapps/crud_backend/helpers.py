"""Helpers: prefixed index.html, parameterised YAML templates, human uptime."""
from __future__ import annotations

import datetime as dt
import logging
import os
import re

import yaml
from flask import current_app

log = logging.getLogger(__name__)


def get_prefixed_index_html() -> str:
    prefix = os.path.join("/", current_app.config["PREFIX"].strip("/"), "")
    with open(os.path.join(current_app.config["STATIC_DIR"], "index.html")) as f:
        html = f.read()
    return re.sub(r"<base href=\".*\".*>", f'<base href="{prefix}">', html)


def load_yaml(path):
    try:
        with open(path) as f:
            text = f.read()
    except OSError:
        log.error("Error opening: %s", path)
        return None
    try:
        data = yaml.safe_load(text)
    except yaml.YAMLError:
        return None
    return {} if data is None else data


def load_param_yaml(path, **kwargs):
    """YAML with `{var}` placeholders substituted before parsing."""
    try:
        with open(path) as f:
            text = f.read().format(**kwargs)
    except OSError:
        log.error("Error opening: %s", path)
        return None
    try:
        data = yaml.safe_load(text)
    except yaml.YAMLError:
        return None
    return {} if data is None else data


def get_uptime(then) -> str:
    if isinstance(then, str):
        then = dt.datetime.strptime(then, "%Y-%m-%dT%H:%M:%SZ")
    diff = dt.datetime.utcnow() - then.replace(tzinfo=None)
    days, hours, mins = diff.days, diff.seconds // 3600, (diff.seconds % 3600) // 60
    if days > 0:
        return f"{days} day{'s' if days != 1 else ''} ago"
    if hours > 0:
        return f"{hours} hour{'s' if hours != 1 else ''} ago"
    if mins == 0:
        return "just now"
    return f"{mins} min{'s' if mins != 1 else ''} ago"
