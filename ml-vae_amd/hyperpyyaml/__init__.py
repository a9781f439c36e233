"""HyperPyYAML surface (ref:src/hyperpyyaml/__init__.py), PyYAML-only implementation."""
from .core import (  # noqa: F401
    Placeholder,
    RefTag,
    dump_hyperpyyaml,
    load_hyperpyyaml,
    recursive_update,
    resolve_references,
)


class TestThing:
    """Test helper kept for the surface (constructed by the doctest-style tests)."""

    def __init__(self, *args, **kwargs):
        self.args = args
        self.kwargs = kwargs

    @classmethod
    def from_keys(cls, args, kwargs):
        obj = cls()
        obj.specific_key = kwargs["thing1"]
        obj.args = args
        obj.kwargs = kwargs
        return obj
