"""Native YAML reader (core/yaml.cc) against PyYAML's safe loader.

Corpus: every YAML file of the reference tree (manifests, CRDs, kustomizations, swagger) when it
is present, plus hand-written edge cases. Loaded with yaml.safe_load_all only.
"""
import glob
import json
import os

import pytest
import yaml

REF = "/root/reference"


def _safe(text):
    return json.loads(json.dumps([d for d in yaml.safe_load_all(text) if d is not None], default=str))


CASES = [
    "a: 1\nb: [1, 2, {c: d}]\n",
    "- a\n- b: 1\n  c: 2\n- - x\n  - y\n",
    "k: |\n  line1\n  line2\n\nj: >-\n  folded\n  text\n",
    'q: "esc \\" \\n \\u00e9"\nr: \'it\'\'s\'\n',
    "key:\n- a\n- b\nother: ~\nt: true\nf: 1.5e+3\nh: 0x1F\n",
    "---\na: 1\n---\nb: 2\n...\n",
    "long: this is a\n  plain multi line\n  - scalar\n",
    "m: {a: 1, b: [x, y], 'c d': \"e\"}\n",
    "desc: \"first\\\n  \\ second\"\n",
]


@pytest.mark.parametrize("text", CASES)
def test_edge_cases(native, text):
    assert [d for d in native.call("parse_yaml_all", text=text) if d is not None] == _safe(text)


def test_dump_roundtrip(native):
    v = {"a": [1, {"b": "x: y", "c": []}], "d": {"e": None, "f": "true"}, "g": "-lead"}
    text = native.call("dump_yaml", value=v)
    assert yaml.safe_load(text) == v


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_reference_corpus(native):
    files = [f for f in glob.glob(REF + "/**/*.y*ml", recursive=True) if f.endswith((".yaml", ".yml"))]
    bad = []
    for f in files:
        text = open(f, errors="replace").read()
        try:
            want = _safe(text)
        except yaml.YAMLError:
            continue
        got = [d for d in native.call("parse_yaml_all", text=text) if d is not None]
        if got != want:
            bad.append(f)
    assert not bad, bad[:10]
    assert len(files) > 100
