"""The drop-in boundary, pinned mechanically.

`tests/golden/ref_signatures.json` holds every public class method and module-level function of
the reference's src/model.py and src/retrieval.py as `ast` saw them (gen_signatures.py; the
reference read as text in the build container). Each must exist in triad_amd's mirror with the
same parameter names in the same order, the same kinds and the same defaults. The mirror may add
parameters only after the reference's, and only optional ones (a caller written against the
reference then binds identically).
"""
import ast
import importlib
import inspect
import json
import os

import pytest

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "ref_signatures.json")
SIGS = json.load(open(FIXTURE))


def _cases():
    for mod, spec in sorted(SIGS.items()):
        for cls, c in sorted(spec["classes"].items()):
            for meth, m in sorted(c["methods"].items()):
                yield pytest.param(mod, cls, meth, m, id=f"{mod.split('.')[-1]}.{cls}.{meth}")
        for fn, f in sorted(spec["functions"].items()):
            yield pytest.param(mod, None, fn, f, id=f"{mod.split('.')[-1]}.{fn}")


def check_signature(obj, ref_params, where):
    """Assert `obj`'s signature binds like the reference's `ref_params` (list of name / kind /
    default-source dicts). Returns nothing; raises AssertionError naming the first drift."""
    params = list(inspect.signature(obj).parameters.values())
    assert len(params) >= len(ref_params), f"{where}: {len(params)} parameters, reference has {len(ref_params)}"
    for i, rp in enumerate(ref_params):
        p = params[i]
        assert p.name == rp["name"], f"{where}: parameter {i} is {p.name!r}, reference {rp['name']!r}"
        assert p.kind.name == rp["kind"], f"{where}: {p.name} is {p.kind.name}, reference {rp['kind']}"
        if rp["default"] is None:
            assert p.default is inspect.Parameter.empty, f"{where}: {p.name} has a default, reference has none"
        else:
            want = ast.literal_eval(rp["default"])
            assert p.default is not inspect.Parameter.empty, f"{where}: {p.name} lacks the default {want!r}"
            assert type(p.default) is type(want) and p.default == want, \
                f"{where}: default of {p.name} is {p.default!r}, reference {want!r}"
    for p in params[len(ref_params):]:
        assert p.default is not inspect.Parameter.empty or p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD), \
            f"{where}: added parameter {p.name} must be optional"


@pytest.mark.parametrize("mod,cls,name,spec", list(_cases()))
def test_public_signature_matches_reference(mod, cls, name, spec):
    m = importlib.import_module(mod)
    owner = m if cls is None else getattr(m, cls, None)
    assert owner is not None, f"{mod} has no class {cls}"
    obj = getattr(owner, name, None)
    assert obj is not None, f"{mod}.{cls + '.' if cls else ''}{name} is missing (reference line {spec['line']})"
    check_signature(obj, spec["params"], f"{mod}.{cls + '.' if cls else ''}{name}")


def test_fixture_covers_the_boundary_classes():
    """The fixture is the reference's whole public surface of the two modules, not a hand pick."""
    model = SIGS["triad_amd.model"]["classes"]
    assert set(model) == {"AudioEmbedder", "TextEmbedder", "ViTEmbedder", "ViTLoRAEmbedder", "MultiModalModel"}
    assert len(model["MultiModalModel"]["methods"]) == 12
    assert model["TextEmbedder"]["methods"]["__init__"]["params"][2]["default"] == "'answerdotai/ModernBERT-base'"


def test_checker_catches_a_drifted_default():
    """The comparison itself fails on a changed default, a renamed or reordered parameter, and an
    added required one."""
    ref = SIGS["triad_amd.model"]["classes"]["TextEmbedder"]["methods"]["__init__"]["params"]

    def drifted(self, embedding_dim=512, model_name="distilbert/distilbert-base-uncased"):
        pass

    def renamed(self, embedding_dim=512, name="answerdotai/ModernBERT-base"):
        pass

    def required_extra(self, embedding_dim=512, model_name="answerdotai/ModernBERT-base", x=None, y=...):
        pass

    def required(self, embedding_dim=512, model_name="answerdotai/ModernBERT-base", z=None, *, w):
        pass

    def ok(self, embedding_dim=512, model_name="answerdotai/ModernBERT-base", extra=None):
        pass

    for bad in (drifted, renamed, required):
        with pytest.raises(AssertionError):
            check_signature(bad, ref, bad.__name__)
    check_signature(required_extra, ref, "required_extra")   # `...` is a default, still optional
    check_signature(ok, ref, "ok")
