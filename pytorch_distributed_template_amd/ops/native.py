"""Loader for the in-tree native extension (``pytorch_distributed_template_amd/_C.so``).

``native.C`` is the extension module.  It is imported on first use; if the shared object is missing
it is built in-tree (set PDT_AUTOBUILD=1 to also rebuild a stale one) with ``ops._build`` (hipcc for gfx950).  There is no silent fallback:
a GPU code path that needs a kernel raises if the extension cannot be loaded.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import threading

_lock = threading.Lock()
_mod = None


def _so_path() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")


def load(build: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        import torch  # noqa: F401  (loads libtorch / the HIP runtime the extension links against)

        alt = os.environ.get("PDT_NATIVE_SO")  # A/B runs: load another build of the extension
        if alt:
            spec = importlib.util.spec_from_file_location("pytorch_distributed_template_amd._C", alt)
            _mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_mod)
            return _mod
        if build and (not os.path.exists(_so_path()) or os.environ.get("PDT_AUTOBUILD", "0") == "1"):
            from . import _build
            _build.build()
        if not os.path.exists(_so_path()):
            raise ImportError(f"native extension not found at {_so_path()}; run `python -m "
                              "pytorch_distributed_template_amd.ops._build`")
        _mod = importlib.import_module("pytorch_distributed_template_amd._C")
        return _mod


def available() -> bool:
    try:
        load()
        return True
    except Exception:  # pragma: no cover - diagnostic helper
        return False


class _Proxy:
    """``native.C``: attribute access on the extension.  With ``PDT_VALIDATE`` >= 1 (read once, at the first
    access) extension functions come back wrapped by :mod:`.validate` (launch-checked / non-finite tracking)."""

    def __init__(self):
        self._wrapped = None  # None: not decided yet; False: validation off; dict: name -> checked wrapper

    def __getattr__(self, name):
        obj = getattr(load(), name)
        if name.startswith("_"):
            return obj
        w = self._wrapped
        if w is None:
            from . import validate
            w = self._wrapped = {} if validate.level_from_env() > 0 else False
        if w is False:
            return obj
        f = w.get(name)
        if f is None:
            from . import validate
            f = w[name] = validate.maybe_wrap(name, obj)
        return f


C = _Proxy()
