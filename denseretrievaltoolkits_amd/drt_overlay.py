"""Drop-in overlay: serve the hot-path modules of the user's DRT package from this build.

    import denseretrievaltoolkits_amd.drt_overlay as o; o.install()
    # or, with the reference scripts unchanged:
    python -m denseretrievaltoolkits_amd.run run_random_sampling.py --model_name_or_path ... (same args)

Only the modules on the north-star path are replaced; everything
else (DRT.arguments, DRT.dataset, DRT.dataloader, DRT.trainer.sampler,
DRT.evaluator.nq_eval, ...) keeps resolving to the user's own DRT package.
"""
from __future__ import annotations

import importlib
import sys
import types

HOT_PATH_MODULES = {
    "DRT.model.biencoder": "denseretrievaltoolkits_amd.model.biencoder",
    "DRT.model.linear": "denseretrievaltoolkits_amd.model.linear",
    "DRT.model.reranker": "denseretrievaltoolkits_amd.model.reranker",
    "DRT.evaluator.index": "denseretrievaltoolkits_amd.evaluator.index",
    "DRT.evaluator.metrics": "denseretrievaltoolkits_amd.evaluator.metrics",
    "DRT.trainer.trainer": "denseretrievaltoolkits_amd.trainer.trainer",
    "DRT.trainer.losses": "denseretrievaltoolkits_amd.trainer.losses",
}


def _ensure_package(name: str):
    if name in sys.modules:
        return sys.modules[name]
    try:
        return importlib.import_module(name)
    except ImportError:
        mod = types.ModuleType(name)
        mod.__path__ = []  # namespace-like placeholder when the user's DRT is absent
        sys.modules[name] = mod
        parent, _, child = name.rpartition(".")
        if parent:
            setattr(_ensure_package(parent), child, mod)
        return mod


def install(modules=None):
    """Register the MI355X implementations under the reference's module names."""
    from . import _native
    _native.load()  # fail loudly up front if the HIP extension is missing
    for ref_name, ours in (modules or HOT_PATH_MODULES).items():
        mod = importlib.import_module(ours)
        parent, _, child = ref_name.rpartition(".")
        pkg = _ensure_package(parent)
        sys.modules[ref_name] = mod
        setattr(pkg, child, mod)
    return sorted(HOT_PATH_MODULES)
