"""HyperPyYAML surface: the reference's doctest answers (ref:src/hyperpyyaml/core.py:144-151,
249-253, 284-291, 524-525, 580-584, 635-636, 696-699) plus the semantics the recipes use."""
import collections
import doctest
import io
import os

import pytest

import hyperpyyaml
from hyperpyyaml import core
from hyperpyyaml import load_hyperpyyaml, resolve_references, dump_hyperpyyaml
from hyperpyyaml.core import deref, parse_arithmetic, recursive_resolve, recursive_update


def test_doctest_answers():
    y = "\na: 3\nthing: !new:collections.Counter\n    b: !ref <a>\n"
    assert load_hyperpyyaml(y)["thing"] == collections.Counter({"b": 3})
    s = io.StringIO()
    dump_hyperpyyaml({"a": hyperpyyaml.Placeholder(), "b": hyperpyyaml.RefTag("<a>")}, s)
    assert s.getvalue() == "a: !PLACEHOLDER\nb: !ref <a>\n"
    y = "\nconstants:\n    a: 3\n    b: !ref <constants[a]>\n"
    assert resolve_references(y, {"constants": {"a": 4}}).getvalue() == "constants:\n  a: 4\n  b: 4\n"
    assert deref("constants[a][b]", {"constants": {"a": {"b": "c"}}}) == "c"
    tree = {"a": 3, "b": "x", "c": "<a>", "d": "<c>/<c>", "e": "<b>/<b>"}
    assert recursive_resolve("<d>", [], tree) == 1.0
    assert recursive_resolve("<e>", [], tree) == "x/x"
    assert parse_arithmetic("2 * 6") == 12
    d = {"a": 1, "b": {"c": 2}}
    recursive_update(d, {"b": {"d": 3}})
    assert d == {"a": 1, "b": {"c": 2, "d": 3}}


def test_module_doctests_pass():
    res = doctest.testmod(core)
    assert res.failed == 0 and res.attempted >= 9


def test_ref_identity_copy_tuple_arith_and_private_keys():
    y = """
__seed: !apply:operator.add [1, 2]
base: 8
dims: !ref <base> * 3
obj: !new:hyperpyyaml.TestThing
    x: 1
same: !ref <obj>
other: !copy <obj>
pair: (3, 4)
path: !ref runs/<base>/x
attr: !ref <obj.kwargs>
"""
    hp = load_hyperpyyaml(y)
    assert "__seed" not in hp
    assert hp["dims"] == 24
    assert hp["same"] is hp["obj"] and hp["other"] is not hp["obj"]
    assert hp["pair"] == (3, 4)
    assert hp["path"] == "runs/8/x"
    assert hp["attr"] == {"x": 1}


def test_placeholder_and_override_errors():
    with pytest.raises(ValueError, match="PLACEHOLDER"):
        load_hyperpyyaml("a: !PLACEHOLDER\nb: 1\n")
    with pytest.raises(KeyError):
        load_hyperpyyaml("a: 1\n", {"zzz": 2})
    assert load_hyperpyyaml("a: !PLACEHOLDER\n", {"a": 5})["a"] == 5
    with pytest.raises(ValueError):
        load_hyperpyyaml("a: !ref <missing>\n")


def test_include_with_child_overrides(tmp_path):
    child = tmp_path / "child.yaml"
    child.write_text("n: 50\nsize: !ref <input_size> * 2\nname: !ref <tag>-x\n")
    parent = tmp_path / "parent.yaml"
    parent.write_text("tag: run\nmodel: !PLACEHOLDER\n    input_size: 40\n    tag: !ref <tag>\n")
    with open(parent) as f:
        hp = load_hyperpyyaml(f, [{"model": {"n": 1}}, "model: !include:child.yaml\n"])
    assert hp["model"] == {"n": 1, "size": 80, "name": "run-x", "input_size": 40, "tag": "run"}


def test_name_module_apply():
    hp = load_hyperpyyaml("f: !name:collections.Counter\n    a: 1\nm: !module:collections\n"
                          "v: !apply:max [3, 9]\n")
    assert hp["f"]() == collections.Counter({"a": 1})
    assert hp["m"] is collections
    assert hp["v"] == 9
