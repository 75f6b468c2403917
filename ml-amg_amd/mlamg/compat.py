"""Install this package under the reference's module names, so the reference's callers
(utils/common.py, utils/evaluate_dataset.py, utils/evaluate_model.py, utils/train_dataset.py,
demos/lloyd_seeds_hist.py) run unchanged on the MI355X path.

    import mlamg.compat; mlamg.compat.install()

registers ns.lib.multigrid / graph / sparse / sparse_tensor -> mlamg.multigrid / graph / sparse /
sparse_tensor, and — when pyamg is not importable (or pyamg=True) — pyamg, pyamg.aggregation,
pyamg.graph, pyamg.strength, pyamg.relaxation(.relaxation) -> mlamg.pyamg_compat. Returns the
{name: module} map it installed. uninstall(installed) removes exactly those entries.
"""
from __future__ import annotations

import importlib
import importlib.util
import sys
import types

NS = {
    "ns.lib.multigrid": "mlamg.multigrid",
    "ns.lib.graph": "mlamg.graph",
    "ns.lib.sparse": "mlamg.sparse",
    "ns.lib.sparse_tensor": "mlamg.sparse_tensor",
}
PYAMG = {
    "pyamg": "mlamg.pyamg_compat",
    "pyamg.aggregation": "mlamg.pyamg_compat.aggregation",
    "pyamg.graph": "mlamg.pyamg_compat.graph",
    "pyamg.strength": "mlamg.pyamg_compat.strength",
    "pyamg.relaxation": "mlamg.pyamg_compat.relaxation",
    "pyamg.relaxation.relaxation": "mlamg.pyamg_compat.relaxation.relaxation",
}


def _pyamg_present():
    m = sys.modules.get("pyamg")
    if m is not None:
        return not getattr(m, "__name__", "").startswith("mlamg")
    try:
        return importlib.util.find_spec("pyamg") is not None
    except (ImportError, ValueError):
        return False


def install(ns=True, pyamg=None):
    """pyamg=None: alias pyamg only when the real package is absent; True / False: always /
    never."""
    table = dict(NS) if ns else {}
    if pyamg or (pyamg is None and not _pyamg_present()):
        table.update(PYAMG)
    installed = {}
    for name, target in table.items():
        mod = importlib.import_module(target)
        parent, _, leaf = name.rpartition(".")
        if parent:
            setattr(_package(parent, installed), leaf, mod)
        sys.modules[name] = mod
        installed[name] = mod
    return installed


def _package(name, installed):
    """The parent package of an alias, imported (the reference's own empty ns/__init__.py,
    ns/lib/__init__.py when it is on sys.path) or else created empty, so that `import
    ns.lib.graph` binds ns.lib.graph — the import system sets that attribute only when it loads
    the child itself."""
    if name in sys.modules:
        return sys.modules[name]
    parent, _, leaf = name.rpartition(".")
    try:
        mod = importlib.import_module(name)
    except ImportError:
        mod = types.ModuleType(name)
        mod.__path__ = []
        sys.modules[name] = mod
        installed[name] = mod
    if parent:
        setattr(_package(parent, installed), leaf, mod)
    return mod


def uninstall(installed):
    for name, mod in installed.items():
        if sys.modules.get(name) is mod:
            del sys.modules[name]
