"""HyperPyYAML surface on PyYAML alone (the reference vendors a ruamel.yaml-based copy:
ref:src/hyperpyyaml/core.py:25-717; ruamel is not available on the GPU hosts).

Supported, with the reference's semantics:
  !new:<class>      construct (mapping -> kwargs, sequence -> args)
  !name:<callable>  the callable, or functools.partial(callable, *args, **kwargs)
  !module:<mod>     the module object
  !apply:<callable> call it at load time (e.g. !apply:torch.manual_seed [123456])
  !ref <key[sub]>   reference (same object), string interpolation, simple arithmetic,
                    <key.attr> -> getattr; chains followed, cycles rejected
  !copy <key>       deep copy of the referenced node
  !include:<file>   load another file; a mapping under the tag overrides its keys
  !PLACEHOLDER      must be overridden, else ValueError
  (a, b)            implicit !tuple
  overrides         dict / yaml string / list of them, applied before resolution
                    (TaggedScalar override -> the tag is moved onto the node, as
                    ref:src/hyperpyyaml/core.py:703-717 does)
  keys "__*"        dropped after construction (side-effect-only entries)
"""
import ast
import collections.abc
import copy
import functools
import inspect
import io
import operator as op
import os
import pydoc
import re

import yaml

_REF_RE = re.compile(r"<[^>]*>")
_TUPLE_RE = re.compile(r"^\(.*\)$")


class Tagged:
    """A YAML node carrying an explicit tag (scalar, mapping or sequence value)."""

    __slots__ = ("tag", "value")

    def __init__(self, tag, value):
        self.tag, self.value = tag, value

    def is_scalar(self):
        return not isinstance(self.value, (dict, list))

    def __repr__(self):
        return f"Tagged({self.tag!r}, {self.value!r})"

    def __deepcopy__(self, memo):
        return Tagged(self.tag, copy.deepcopy(self.value, memo))


class RefTag:
    """Dump helper: a ``!ref`` scalar (ref:src/hyperpyyaml/core.py:197-219)."""

    yaml_tag = "!ref"

    def __init__(self, ref_str):
        self.ref_str = ref_str


class Placeholder:
    """Dump helper: a ``!PLACEHOLDER`` scalar."""

    yaml_tag = "!PLACEHOLDER"


# --------------------------------------------------------------------------- parsing
class _ScalarResolver(yaml.SafeLoader):
    pass


def _plain_scalar(node):
    """Resolve an untagged scalar node the way PyYAML would (int/float/bool/null/str)."""
    if node.tag == "tag:yaml.org,2002:str" and node.style is None and _TUPLE_RE.match(node.value):
        return Tagged("!tuple", node.value)
    loader = _ScalarResolver("")
    return loader.construct_object(node, deep=True)


def _from_node(node):
    tag = node.tag or ""
    explicit = tag.startswith("!")
    if isinstance(node, yaml.MappingNode):
        val = {}
        for k_node, v_node in node.value:
            key = _plain_scalar(k_node) if isinstance(k_node, yaml.ScalarNode) else _from_node(k_node)
            if isinstance(key, Tagged):
                key = key.value
            val[key] = _from_node(v_node)
        return Tagged(tag, val) if explicit else val
    if isinstance(node, yaml.SequenceNode):
        val = [_from_node(n) for n in node.value]
        return Tagged(tag, val) if explicit else val
    if explicit:
        return Tagged(tag, node.value)
    return _plain_scalar(node)


def _parse(stream):
    if hasattr(stream, "read"):
        text = stream.read()
    else:
        text = stream
    node = yaml.compose(text, Loader=yaml.SafeLoader) if text and text.strip() else None
    if node is None:
        return {}
    return _from_node(node)


# --------------------------------------------------------------------------- overrides
def recursive_update(d, u, must_match=False):
    """Nested dict.update (ref:src/hyperpyyaml/core.py:654-717).

    >>> d = {'a': 1, 'b': {'c': 2}}
    >>> recursive_update(d, {'b': {'d': 3}})
    >>> d
    {'a': 1, 'b': {'c': 2, 'd': 3}}
    """
    for k, v in u.items():
        cur = d.get(k) if isinstance(d, dict) else None
        if isinstance(v, collections.abc.Mapping) and not isinstance(v, Tagged) and k in d:
            if isinstance(cur, Tagged) and cur.is_scalar():
                d[k] = Tagged(cur.tag, {})  # tagged scalar becomes a tagged mapping
            target = d[k].value if isinstance(d[k], Tagged) else d[k]
            recursive_update(target, v)
        elif must_match and k not in d:
            raise KeyError(f"Override '{k}' not found in: {[key for key in d.keys()]}")
        elif isinstance(v, Tagged) and v.is_scalar() and k in d and isinstance(cur, (Tagged, dict, list)):
            # move the override's tag onto the existing node (e.g. --model !include:x.yaml)
            d[k] = Tagged(v.tag, cur.value if isinstance(cur, Tagged) else cur)
        else:
            d[k] = v


def _as_tree(overrides):
    if isinstance(overrides, str):
        return _parse(overrides) or {}
    return overrides


# --------------------------------------------------------------------------- references
def _ast_eval(node):
    ops = {ast.Add: op.add, ast.Sub: op.sub, ast.Mult: op.mul, ast.Div: op.truediv,
           ast.FloorDiv: op.floordiv, ast.Pow: op.pow, ast.Mod: op.mod, ast.USub: op.neg,
           ast.UAdd: op.pos}
    if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)):
        return node.value
    if isinstance(node, ast.BinOp):
        return ops[type(node.op)](_ast_eval(node.left), _ast_eval(node.right))
    if isinstance(node, ast.UnaryOp):
        return ops[type(node.op)](_ast_eval(node.operand))
    raise TypeError(node)


def parse_arithmetic(reference_string):
    """Evaluate +-*/ // ** % on numbers; anything else comes back unchanged.

    >>> parse_arithmetic('2 * 6')
    12
    """
    try:
        return _ast_eval(ast.parse(reference_string, mode="eval").body)
    except (TypeError, SyntaxError, KeyError, ValueError):
        return reference_string


def deref(ref, full_tree, copy_mode=False):
    """Follow ``key[sub][sub2]`` (plus an optional ``.attr``) into the tree.

    >>> deref('constants[a][b]', {'constants': {'a': {'b': 'c'}}})
    'c'
    """
    attr = None
    if "." in ref:
        ref, attr = ref.split(".", maxsplit=1)
    branch = full_tree
    for part in ref.split("["):
        part = part.strip("]")
        container = branch.value if isinstance(branch, Tagged) and not branch.is_scalar() else branch
        if not isinstance(container, (dict, list)):
            raise ValueError(f'The reference "{ref}" is not valid')
        if isinstance(container, list):
            try:
                branch = container[int(part)]
            except (ValueError, IndexError):
                raise ValueError(f'The reference "{ref}" is not valid')
        else:
            if part not in container:
                raise ValueError(f'The reference "{ref}" is not valid')
            branch = container[part]
    if copy_mode:
        return copy.deepcopy(branch)
    if attr is not None:
        return Tagged("!apply:getattr", [branch, attr])
    return branch


def _deref_resolved(ref, reference_list, full_tree, copy_mode):
    # a referent that is itself a not-yet-walked !ref/!copy is resolved on the spot
    v = deref(ref, full_tree, copy_mode)
    if isinstance(v, Tagged) and v.tag in ("!ref", "!copy") and v.is_scalar():
        v = recursive_resolve(v.value, list(reference_list), full_tree, copy_mode or v.tag == "!copy")
    return v


def recursive_resolve(reference, reference_list, full_tree, copy_mode=False):
    """Resolve ``<key>`` references in a string, following chains.

    >>> tree = {'a': 3, 'b': 'x', 'c': '<a>', 'd': '<c>/<c>', 'e': '<b>/<b>'}
    >>> recursive_resolve('<d>', [], tree)
    1.0
    >>> recursive_resolve('<e>', [], tree)
    'x/x'
    """
    if not isinstance(reference, str) or not _REF_RE.search(reference):
        return reference
    if len(reference_list) > 1 and reference in reference_list[1:]:
        raise ValueError("Circular reference detected: ", reference_list)
    if _REF_RE.fullmatch(reference):  # whole-value reference keeps the type/object
        value = _deref_resolved(reference.strip("<>"), reference_list, full_tree, copy_mode)
        reference_list += [reference]
        return recursive_resolve(value, reference_list, full_tree, copy_mode)
    reference_list += _REF_RE.findall(reference)

    def sub(m):
        v = _deref_resolved(m.group(0).strip("<>"), reference_list, full_tree, copy_mode)
        v = recursive_resolve(v, list(reference_list), full_tree, copy_mode)
        return str(v.value if isinstance(v, Tagged) and v.is_scalar() else v)

    out = recursive_resolve(_REF_RE.sub(sub, reference), reference_list, full_tree, copy_mode)
    return parse_arithmetic(out) if isinstance(out, str) else out


def _walk(key, node, tree, file_path):
    if isinstance(node, list):
        for i, sub in enumerate(node):
            node[i] = _walk(i if key == "root" else f"{key}[{i}]", sub, tree, file_path)
    elif isinstance(node, dict):
        for k in list(node.keys()):
            node[k] = _walk(k if key == "root" else f"{key}[{k}]", node[k], tree, file_path)
    elif isinstance(node, Tagged) and not node.is_scalar():
        _walk(key, node.value, tree, file_path)
    if isinstance(node, Tagged):
        tag = node.tag
        if tag == "!PLACEHOLDER":
            raise ValueError(f"'{key}' is a !PLACEHOLDER and must be replaced.")
        if tag in ("!ref", "!copy"):
            return recursive_resolve(node.value, [], tree, copy_mode=(tag == "!copy"))
        if tag.startswith("!include:"):
            filename = tag[len("!include:"):]
            if file_path is not None:
                filename = os.path.join(file_path, filename)
            child_overrides = dict(node.value) if isinstance(node.value, dict) else None
            with open(filename) as f:
                return _resolve(f, child_overrides, False)
    return node


def _resolve(stream, overrides=None, overrides_must_match=False):
    file_path = None
    if hasattr(stream, "name"):
        file_path = os.path.dirname(os.path.realpath(stream.name))
    tree = _parse(stream)
    if overrides:
        for o in (overrides if isinstance(overrides, list) else [overrides]):
            o = _as_tree(o)
            if o:
                recursive_update(tree, o, must_match=overrides_must_match)
    _walk("root", tree, tree, file_path)
    return tree


# --------------------------------------------------------------------------- construction
def _locate(name, what):
    obj = pydoc.locate(name)
    if obj is None:
        raise ImportError(f"There is no such {what} as {name}")
    return obj


def _build(node, memo):
    if id(node) in memo:
        return memo[id(node)]
    if isinstance(node, dict):
        out = {}
        memo[id(node)] = out
        for k, v in node.items():
            out[k] = _build(v, memo)
        return out
    if isinstance(node, list):
        out = []
        memo[id(node)] = out
        out.extend(_build(v, memo) for v in node)
        return out
    if not isinstance(node, Tagged):
        return node
    tag, val = node.tag, node.value
    if tag == "!tuple":
        return tuple(yaml.safe_load("[" + str(val)[1:-1] + "]"))
    if isinstance(val, dict):
        args, kwargs = [], {k: _build(v, memo) for k, v in val.items()}
    elif isinstance(val, list):
        args, kwargs = [_build(v, memo) for v in val], {}
    else:
        args, kwargs = [], {}
    if tag.startswith("!new:"):
        cls = _locate(tag[5:], "class")
        if not inspect.isclass(cls):
            raise ValueError(f"!new:{tag[5:]} should be a class, but is {cls}")
        try:
            out = cls(*args, **kwargs)
        except TypeError as e:
            e.args = (f"Invalid argument to class {tag[5:]}", *e.args)
            raise
    elif tag.startswith("!name:"):
        fn = _locate(tag[6:], "entity")
        if not (inspect.isclass(fn) or inspect.isroutine(fn)):
            if args or kwargs:
                raise ValueError(f"!name:{tag[6:]} should be class or function, if you specify "
                                 f"args or kwargs. Instead it is {fn}")
            out = fn
        else:
            out = functools.partial(fn, *args, **kwargs)
    elif tag.startswith("!module:"):
        mod = _locate(tag[8:], "module")
        if args or kwargs:
            raise ValueError("Cannot pass args to module")
        if not inspect.ismodule(mod):
            raise ValueError(f"!module:{tag[8:]} should be module, but is {mod}")
        out = mod
    elif tag.startswith("!apply:"):
        fn = _locate(tag[7:], "callable")
        if not inspect.isroutine(fn):
            raise ValueError(f"!apply:{tag[7:]} should be a callable, but is {fn}")
        try:
            out = fn(*args, **kwargs)
        except TypeError as e:
            e.args = (f"Invalid argument to callable {tag[7:]}", *e.args)
            raise
    else:
        raise ValueError(f"unknown tag {tag}")
    memo[id(node)] = out
    return out


def resolve_references(yaml_stream, overrides=None, overrides_must_match=False):
    """Apply overrides and resolve !ref/!copy/!include:, returning a yaml stream.

    >>> yaml_string = '''
    ... constants:
    ...     a: 3
    ...     b: !ref <constants[a]>
    ... '''
    >>> overrides = {'constants': {'a': 4}}
    >>> resolve_references(yaml_string, overrides).getvalue()
    'constants:\\n  a: 4\\n  b: 4\\n'
    """
    tree = _resolve(yaml_stream, overrides, overrides_must_match)
    out = io.StringIO()
    dump_hyperpyyaml(tree, out)
    out.seek(0)
    return out


def load_hyperpyyaml(yaml_stream, overrides=None, overrides_must_match=True):
    """Load HyperPyYAML into python objects (ref:src/hyperpyyaml/core.py:25-194).

    >>> yaml_string = '''
    ... a: 3
    ... thing: !new:collections.Counter
    ...     b: !ref <a>
    ... '''
    >>> params = load_hyperpyyaml(yaml_string)
    >>> params["thing"]
    Counter({'b': 3})
    """
    tree = _resolve(yaml_stream, overrides, overrides_must_match)
    hparams = _build(tree, {})
    if isinstance(hparams, dict):
        for k in [k for k in hparams if isinstance(k, str) and k.startswith("__")]:
            del hparams[k]
    return hparams


# --------------------------------------------------------------------------- dumping
class _Dumper(yaml.SafeDumper):
    pass


def _repr_tagged(dumper, t):
    if isinstance(t.value, dict):
        return dumper.represent_mapping(t.tag, t.value)
    if isinstance(t.value, list):
        return dumper.represent_sequence(t.tag, t.value)
    return dumper.represent_scalar(t.tag, str(t.value))


_Dumper.add_representer(Tagged, _repr_tagged)
_Dumper.add_representer(RefTag, lambda d, r: d.represent_scalar("!ref", r.ref_str))
_Dumper.add_representer(Placeholder, lambda d, p: d.represent_scalar("!PLACEHOLDER", "", style=""))
_Dumper.add_representer(tuple, lambda d, t: d.represent_sequence("tag:yaml.org,2002:seq", list(t)))


def dump_hyperpyyaml(yaml_tree, output_stream, *args, **kwargs):
    """Dump a tree keeping !ref / !PLACEHOLDER tags.

    >>> to_yaml = {'a': Placeholder(), 'b': RefTag('<a>')}
    >>> stringio = io.StringIO()
    >>> dump_hyperpyyaml(to_yaml, stringio)
    >>> stringio.getvalue()
    'a: !PLACEHOLDER\\nb: !ref <a>\\n'
    """
    kwargs.setdefault("default_flow_style", False)
    kwargs.setdefault("sort_keys", False)
    text = yaml.dump(yaml_tree, Dumper=_Dumper, *args, **kwargs)
    # PyYAML single-quotes every scalar carrying an explicit local tag; emit such scalars
    # plain when that is unambiguous, as HyperPyYAML files are written.
    text = _TAGGED_QUOTED.sub(_unquote, text)
    output_stream.write(text)


_TAGGED_QUOTED = re.compile(r"(![^\s']+) '((?:[^'\n]|'')*)'")


def _unquote(m):
    body = m.group(2).replace("''", "'")
    if body == "":
        return m.group(1)
    if ": " in body or " #" in body or body[0] in "!&*[]{}|>'\"%@`,?-#" or body != body.strip():
        return m.group(0)
    return f"{m.group(1)} {body}"
