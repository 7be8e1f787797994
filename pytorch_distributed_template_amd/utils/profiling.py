"""Tracing / profiling helpers (SURVEY §5 "Tracing / profiling": the reference only has wall clocks).

* :func:`roctx_range` -- ROCm ``roctx`` ranges (``libroctx64``, loaded with ctypes) around training
  phases; they show up in ``rocprofv3 --marker-trace`` timelines.  No-ops when the library is absent.
* :class:`PhaseTimer` -- HIP-event timing of named phases (forward/backward/optimizer/comm) without
  host synchronisation inside the step; ``summary()`` synchronises once and returns milliseconds.
* :class:`ThroughputMeter` -- images/s over a window of steps (synchronised at the window edges only).
"""
from __future__ import annotations

import contextlib
import ctypes
import glob
import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch

_ROCTX = None
_ROCTX_TRIED = False


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if _ROCTX_TRIED:
        return _ROCTX
    _ROCTX_TRIED = True
    cands = glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so*"))
    cands += ["/opt/rocm/lib/libroctx64.so"]
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePop.argtypes = []
            _ROCTX = lib
            break
        except OSError:
            continue
    return _ROCTX


@contextlib.contextmanager
def roctx_range(name: str, enabled: bool = True):
    lib = _roctx() if enabled else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


class PhaseTimer:
    """Accumulate GPU time per named phase with events (one event pair per phase instance)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._events: Dict[str, List] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        with roctx_range(name):
            yield
        b.record()
        self._events[name].append((a, b))

    def summary(self, reset: bool = True) -> Dict[str, float]:
        if not self.enabled:
            return {}
        torch.cuda.synchronize()
        out = {k: sum(a.elapsed_time(b) for a, b in v) for k, v in self._events.items()}
        if reset:
            self._events.clear()
        return out


class ThroughputMeter:
    def __init__(self, device: Optional[torch.device] = None):
        self.device = device
        self.reset()

    def reset(self) -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        self.samples = 0

    def update(self, n: int) -> None:
        self.samples += n

    def rate(self) -> float:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dt = time.perf_counter() - self.t0
        return self.samples / dt if dt > 0 else 0.0
