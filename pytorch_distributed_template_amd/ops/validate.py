"""Validation mode for the native ops (the debug / sanitizer counterpart of ``CUDA_LAUNCH_BLOCKING=1`` +
``torch.autograd.detect_anomaly`` for our own kernels; SURVEY §5 "race detection / sanitizers").

Enabled with ``PDT_VALIDATE=<level>`` before the extension is first used (``native.C`` then hands out
checked wrappers of every extension *function*; classes such as the communicator pass through):

* level 1 -- launch-checked: every native op is followed by a device synchronisation, so an asynchronous
  HIP error (illegal address, invalid launch, a kernel trap) is raised AT the op that caused it, with the
  op's name, its tensor arguments and the last ``PDT_VALIDATE_HISTORY`` (default 32) ops in the message.
  ``PDT_VALIDATE_LOG=<file>`` also appends each op name to a file (flushed) BEFORE it launches: a fault the
  HIP runtime turns into a process abort (GPU memory access fault) leaves the faulting op as the last line.
* level 2 -- level 1 plus non-finite tracking: every floating-point tensor argument is scanned before and
  after the op, and an op that turns a finite tensor into one holding NaN/Inf raises
  :class:`NonFiniteError` naming the op and the argument.  (An fp16 AMP step that overflows on purpose --
  the GradScaler then skips it -- trips this too, exactly like torch's anomaly mode.)
* level 3 -- level 1 plus replay determinism (an intra-kernel race detector): before each op every tensor
  argument is snapshotted; after it ran, the op is re-run ``PDT_VALIDATE_REPLAYS`` (default 3) times from the
  snapshot and every argument must come out BIT-identical to the first run.  A kernel whose result depends on
  wave timing (a missing barrier / ``s_waitcnt``, an LDS read racing an LDS-DMA, an order-dependent reduction)
  raises :class:`NondeterminismError` naming the op, the argument, and how many elements differed
  (``PDT_VALIDATE_COLLECT=1``: record in ``Validator.findings`` and continue instead).

Guard bands (any level, ``PDT_VALIDATE_GUARD=<elements>``): :class:`~..optim.flat.FlatParams` leaves that many
extra elements after every parameter slot and fills them in the GRADIENT buffer with a finite canary; after every
op the canaries are checked, and an op that wrote past the end of a gradient slice (e.g. a side-stream weight
gradient spilling into the BN-gradient slot a main-stream kernel writes concurrently) raises
:class:`GuardBandError` naming the op and the parameter whose guard it hit.

Steps being captured into a HIP graph are not checked (nothing may synchronise inside a capture).
Everything here costs a device round trip per op: it is a debugging mode, never on in a benchmark.
"""
from __future__ import annotations

import collections
import os
import threading
from typing import Any, Callable, Deque, List, Optional, Tuple

import torch


class ValidationError(RuntimeError):
    """A native op failed (synchronous TORCH_CHECK or an asynchronous HIP error surfaced at its sync)."""


class NonFiniteError(ValidationError):
    """A native op produced NaN/Inf in a tensor argument that was finite before the op."""


class NondeterminismError(ValidationError):
    """Re-running a native op from identical inputs produced different bits (level 3)."""


class GuardBandError(ValidationError):
    """A native op wrote into a canary guard band after a flat-buffer slot."""


CANARY_BITS = 0x0BADC0DE  # a finite fp32 (~7e-32): harmless if a whole-buffer op reads it, unmistakable if overwritten


def canary_bits(t: torch.Tensor) -> torch.Tensor:
    """Integer view of a guard tail for canary comparisons."""
    return _bits(t)


def canary_value(t: torch.Tensor) -> int:
    return {8: 0x0BADC0DE0BADC0DE, 4: CANARY_BITS, 2: 0x0BAD, 1: 0xA5}[t.element_size()] if t.element_size() != 1 \
        else (0xA5 if t.dtype == torch.uint8 else -91)


def fill_canary(t: torch.Tensor) -> None:
    canary_bits(t).fill_(canary_value(t))


def _bits(t: torch.Tensor) -> torch.Tensor:
    """Bitwise view for comparisons (NaN payloads compare equal to themselves)."""
    t = t.detach().contiguous().reshape(-1)
    if t.dtype in (torch.float64, torch.int64):
        return t.view(torch.int64)
    if t.dtype in (torch.float32, torch.int32):
        return t.view(torch.int32)
    if t.dtype in (torch.float16, torch.bfloat16, torch.int16):
        return t.view(torch.int16)
    return t.view(torch.uint8)


def _describe(args) -> str:
    parts = []
    for i, a in enumerate(args):
        if isinstance(a, torch.Tensor):
            parts.append(f"#{i}:{str(a.dtype).replace('torch.', '')}{list(a.shape)}")
    return " ".join(parts) if parts else "(no tensors)"


class Validator:
    """Wraps extension functions; one instance per process (see :func:`validator`)."""

    def __init__(self, level: int = 1, history: int = 32, log_path: Optional[str] = None,
                 sync: Optional[Callable[[], None]] = None, capturing: Optional[Callable[[], bool]] = None):
        self.level = int(level)
        self.history: Deque[str] = collections.deque(maxlen=max(1, int(history)))
        self.calls = 0
        self._lock = threading.Lock()
        self._log = open(log_path, "a", buffering=1) if log_path else None
        self._sync = sync or (lambda: torch.cuda.synchronize() if torch.cuda.is_available() else None)
        self._capturing = capturing or (lambda: torch.cuda.is_available() and torch.cuda.is_current_stream_capturing())
        self.replays = int(os.environ.get("PDT_VALIDATE_REPLAYS", "3"))
        self.collect = os.environ.get("PDT_VALIDATE_COLLECT", "0") == "1"
        self.findings: List[str] = []
        self.replayed = 0
        self.replay_host = False  # replay host-tensor ops too (CPU tests of the mechanism)
        self._guards: List[Tuple[torch.Tensor, torch.Tensor, List[Tuple[int, str]]]] = []
        self._tails = {}

    def register_guard(self, buf: torch.Tensor, idx: torch.Tensor, owners: List[Tuple[int, str]]) -> None:
        """``buf[idx]`` holds canaries; ``owners`` = (first position in idx, parameter name) per slot guard."""
        self._guards.append((buf, idx, owners))

    def register_tail_guard(self, name: str, tail: torch.Tensor) -> None:
        """``tail`` (the guard elements allocated behind a work buffer, any dtype) was canary-filled by
        :func:`fill_canary`; an op writing past the end of the buffer in front of it overwrites them."""
        self._tails[name] = tail

    def _check_tails(self, name: str, args) -> None:
        for owner, tail in self._tails.items():
            b = canary_bits(tail)
            if not bool((b == canary_value(tail)).all()):
                n = int((b != canary_value(tail)).sum())
                raise GuardBandError(f"native op `{name}` wrote past the end of work buffer `{owner}` ({n} guard "
                                     f"element(s) overwritten)\n  args: {_describe(args)}\n  last native ops "
                                     f"(oldest first):\n  {self._recent()}")

    def _check_guards(self, name: str, args) -> None:
        for buf, idx, owners in self._guards:
            v = buf.view(torch.int32)[idx]
            bad = (v != CANARY_BITS).nonzero()
            if bad.numel():
                pos = int(bad[0])
                who = [n for start, n in owners if start <= pos][-1]
                raise GuardBandError(f"native op `{name}` wrote into the guard band after parameter `{who}` "
                                     f"({int(bad.numel())} canary element(s) overwritten)\n  args: {_describe(args)}"
                                     f"\n  last native ops (oldest first):\n  {self._recent()}")

    def _replay(self, name: str, fn, args, kwargs):
        """Run ``fn`` once, then ``self.replays`` more times from the same inputs; returns the first result."""
        ts = [(i, a) for i, a in enumerate(args) if isinstance(a, torch.Tensor) and a.numel() > 0]
        if not ts or not (self.replay_host or any(a.is_cuda for _, a in ts)):
            res = fn(*args, **kwargs)
            self._sync()
            return res
        pre = [a.clone() for _, a in ts]
        res = fn(*args, **kwargs)
        self._sync()
        post = [_bits(a).clone() for _, a in ts]
        self.replayed += 1
        for r in range(self.replays):
            for (_, a), p in zip(ts, pre):
                a.copy_(p)
            fn(*args, **kwargs)
            self._sync()
            for (i, a), want in zip(ts, post):
                got = _bits(a)
                if torch.equal(got, want):
                    continue
                nd = int((got != want).sum())
                msg = (f"native op `{name}` is not deterministic: replay {r + 1} changed {nd} of {a.numel()} "
                       f"element(s) of argument #{i} ({str(a.dtype).replace('torch.', '')}{list(a.shape)})")
                for (_, a2), w2 in zip(ts, post):  # keep the first run's result so the step can go on
                    a2.copy_(w2.view(a2.dtype).view(a2.shape))
                if self.collect:
                    self.findings.append(msg)
                    return res
                raise NondeterminismError(msg + f"\n  args: {_describe(args)}\n  last native ops (oldest first):"
                                          f"\n  {self._recent()}")
        return res

    def _recent(self) -> str:
        return "\n  ".join(self.history)

    @staticmethod
    def _finite_args(args) -> List[Tuple[int, torch.Tensor, bool]]:
        out = []
        for i, a in enumerate(args):
            if isinstance(a, torch.Tensor) and a.is_floating_point() and a.numel() > 0:
                out.append((i, a, bool(torch.isfinite(a).all())))
        return out

    def wrap(self, name: str, fn: Callable[..., Any]) -> Callable[..., Any]:
        def checked(*args, **kwargs):
            if self._capturing():
                return fn(*args, **kwargs)
            entry = f"{name} {_describe(args)}"
            with self._lock:
                self.calls += 1
                self.history.append(entry)
                if self._log is not None:
                    self._log.write(entry + "\n")
            pre = self._finite_args(args) if self.level == 2 else []
            try:
                if self.level >= 3:
                    res = self._replay(name, fn, args, kwargs)
                else:
                    res = fn(*args, **kwargs)
                    self._sync()
            except ValidationError:
                raise
            except Exception as e:  # TORCH_CHECK in the binding, or an async HIP error at the sync
                raise ValidationError(f"native op `{name}` failed: {e}\n  args: {_describe(args)}\n"
                                      f"  last native ops (oldest first):\n  {self._recent()}") from e
            if self._guards:
                self._check_guards(name, args)
            if self._tails:
                self._check_tails(name, args)
            for i, t, was_finite in pre:
                if was_finite and not bool(torch.isfinite(t).all()):
                    bad = int((~torch.isfinite(t)).sum())
                    raise NonFiniteError(f"native op `{name}` wrote {bad} non-finite value(s) into argument #{i} "
                                         f"({str(t.dtype).replace('torch.', '')}{list(t.shape)}), finite before "
                                         f"the op\n  last native ops (oldest first):\n  {self._recent()}")
            return res
        checked.__name__ = name
        checked.__wrapped__ = fn
        return checked


_validator: Optional[Validator] = None
_vlock = threading.Lock()


def level_from_env() -> int:
    try:
        return int(os.environ.get("PDT_VALIDATE", "0") or 0)
    except ValueError:
        return 1


def validator() -> Optional[Validator]:
    """The process-wide validator, created on first use when ``PDT_VALIDATE`` >= 1, else None."""
    global _validator
    lvl = level_from_env()
    if lvl <= 0:
        return None
    with _vlock:
        if _validator is None or _validator.level != lvl:
            _validator = Validator(lvl, int(os.environ.get("PDT_VALIDATE_HISTORY", "32")),
                                   os.environ.get("PDT_VALIDATE_LOG") or None)
        return _validator


def maybe_wrap(name: str, obj: Any) -> Any:
    """``obj`` unchanged unless validation is on and it is an extension function (not a class/constant)."""
    v = validator()
    if v is None or isinstance(obj, type) or not callable(obj):
        return obj
    return v.wrap(name, obj)
