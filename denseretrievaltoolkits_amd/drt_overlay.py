"""Drop-in overlay: serve the hot-path modules of the user's DRT package from this build.

    import denseretrievaltoolkits_amd.drt_overlay as o; o.install()
    # or, with the reference scripts unchanged:
    python -m denseretrievaltoolkits_amd.run run_random_sampling.py --model_name_or_path ... (same args)

Only the modules on the north-star path are replaced; everything
else (DRT.arguments, DRT.dataset, DRT.dataloader, DRT.trainer.sampler,
DRT.evaluator.nq_eval, ...) keeps resolving to the user's own DRT package.
"""
from __future__ import annotations

import builtins
import importlib
import importlib.util
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


# Names the overlay module re-exports from the user's own module when it exists: they are off the
# hot path but other reference modules import them from there (DRT/trainer/sampler.py:5 imports
# BM25Retriever from DRT.evaluator.index; BM25Negatives builds one, sampler.py:55).
USER_REEXPORTS = {"DRT.evaluator.index": ("BM25Retriever", "FaissRetriever")}


class _MissingModule(types.ModuleType):
    """Stands in for an optional dependency of the user's module that is not installed; any use
    raises (e.g. faiss for FaissRetriever, which the overlay does not serve)."""

    def __getattr__(self, attr):
        raise ImportError(f"{self.__name__} is not installed (needed for {self.__name__}.{attr})")


def _user_module(name: str, optional=("faiss",)):
    """The user's own module `name` before the overlay replaces it, or None.  If it only fails
    to import because an optional third-party dependency is absent (the reference's index.py
    imports faiss at module level, index.py:2), it is executed with that import bound to a
    placeholder that raises on use, so its other classes (BM25Retriever) stay reachable."""
    cur = sys.modules.get(name)
    if cur is not None and not getattr(cur, "__drt_overlay__", False):
        return cur
    try:
        spec = importlib.util.find_spec(name)
    except (ImportError, ValueError):
        return None
    if spec is None or spec.origin is None or spec.loader is None:
        return None
    mod = importlib.util.module_from_spec(spec)
    real_import = builtins.__import__

    def _import(nm, globals=None, locals=None, fromlist=(), level=0):
        if level == 0 and nm.split(".")[0] in optional:
            try:
                return real_import(nm, globals, locals, fromlist, level)
            except ImportError:
                return _MissingModule(nm)
        return real_import(nm, globals, locals, fromlist, level)

    mod.__dict__["__builtins__"] = dict(builtins.__dict__, __import__=_import)
    try:
        spec.loader.exec_module(mod)
    except Exception:
        return None
    return mod


def install(modules=None):
    """Register the MI355X implementations under the reference's module names."""
    from . import _native
    _native.load()  # fail loudly up front if the HIP extension is missing
    for ref_name, ours in (modules or HOT_PATH_MODULES).items():
        mod = importlib.import_module(ours)
        parent, _, child = ref_name.rpartition(".")
        pkg = _ensure_package(parent)
        names = USER_REEXPORTS.get(ref_name, ())
        user = _user_module(ref_name) if names else None
        if user is not None:
            for n in names:
                if hasattr(user, n):
                    setattr(mod, n, getattr(user, n))
        mod.__drt_overlay__ = True
        sys.modules[ref_name] = mod
        setattr(pkg, child, mod)
    return sorted(HOT_PATH_MODULES)
