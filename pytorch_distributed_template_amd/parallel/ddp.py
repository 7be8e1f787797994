"""Data-parallel gradient bucketer (our replacement for the C++ DDP Reducer).

Reference behaviour being reproduced (SURVEY §2.3 "DDP", X2-X4): one process per GPU; at
construction parameters and buffers are broadcast from rank 0 (`T/nn/parallel/distributed.py:862-864`);
before every grad-enabled forward the BatchNorm buffers are re-broadcast from rank 0 (X3); during
backward, gradients are averaged across ranks in buckets (reverse registration order, first bucket
small) with the all-reduces overlapping the rest of backward (X4).

MI355X-native design:
* gradients live in ONE flat fp32 buffer (:class:`~..optim.flat.FlatParams`), so a bucket is a
  contiguous slice -- no copy-in/copy-out, no per-bucket division (the 1/world factor is folded into
  the fused SGD kernel);
* a bucket's all-reduce is launched (``async_op=True`` on the RCCL communicator, which orders itself
  after the compute stream's work already enqueued) the moment its last gradient is produced --
  either by the native executor's explicit backward (``grad_ready(pid)``) or by autograd
  post-accumulate hooks on the generic path;
* bucket sizes: DDP's policy (1 MiB first-produced bucket, 25 MiB after) or -- the native trainer's
  default -- a small LAST-produced bucket (1 MiB, stem side) and 25 MiB caps elsewhere: each ring
  all-reduce stays large enough to use all seven xGMI links of an MI355X node, and the one all-reduce
  that cannot overlap backward (the last bucket's) is small;
* ``finish()`` makes the compute stream wait for every bucket (no host synchronisation).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..optim.flat import FlatBuffers, FlatParams


class GradBucketer:
    def __init__(self, flat: FlatParams, process_group=None, bucket_cap_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, enabled: Optional[bool] = None, last_bucket_mb: Optional[float] = None,
                 rebuild: bool = False):
        """Buckets over parameters in the order their gradients are produced (reverse registration).

        ``last_bucket_mb=None``: DDP's policy -- the FIRST-produced bucket closes at ``first_bucket_mb``, the rest
        at ``bucket_cap_mb``.  ``last_bucket_mb=x``: built from the other end -- the LAST-produced bucket (stem /
        layer1 side, ready only when backward ends, so its all-reduce is exposed) closes at ``x`` and the rest at
        the cap; every other bucket is launched while backward still has whole stages to run.  With DDP's policy
        on ResNet-18 the last bucket holds 15 MiB (part of layer4, layer3, layer2, layer1, stem) and its ring
        all-reduce trails backward on every step.

        ``rebuild=True`` (the autograd / torch-engine path): like upstream DDP after its first iteration
        (`distributed.py:144`; `T/nn/parallel/distributed.py:1195-1247`, Reducer::rebuild_buckets), the buckets are
        rebuilt ONCE from the order in which gradients actually became ready in step 1 (rank 0's order, broadcast,
        so every rank builds the same buckets), and the flat buffers are re-laid so each new bucket is again a
        contiguous slice.  The native executor's production order is fixed by construction and needs no rebuild."""
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.enabled = (self.world > 1) if enabled is None else enabled
        self._policy = (bucket_cap_mb, first_bucket_mb, last_bucket_mb)
        self._assign(list(range(len(flat.slots) - 1, -1, -1)))
        self._works = []
        self._next = 0  # next bucket index to launch
        self.launch_log: List[int] = []  # bucket ids in launch order, this step
        self.last_launch_order: List[int] = []  # ... of the last finished step (tests)
        self._observed: Optional[List[int]] = [] if (rebuild and self.enabled) else None
        self.rebuilt = False

    def _assign(self, production: List[int]) -> None:
        """Buckets over ``production`` (parameter ids in gradient-production order); the flat buffer's memory order
        must be its reverse (so every bucket is a contiguous slice)."""
        bucket_cap_mb, first_bucket_mb, last_bucket_mb = self._policy
        cap = int(bucket_cap_mb * 1024 * 1024)
        slots = self.flat.slots
        self.buckets: List[dict] = []
        self.bucket_of = {}
        groups: List[List[int]] = []
        cur: List[int] = []
        cur_bytes = 0
        if last_bucket_mb is None:
            order, limit = list(production), int(first_bucket_mb * 1024 * 1024)
        else:
            order, limit = list(reversed(production)), int(last_bucket_mb * 1024 * 1024)
        for i in order:
            cur.append(i)
            cur_bytes += slots[i].numel * 4
            if cur_bytes >= limit:
                groups.append(cur)
                cur, cur_bytes, limit = [], 0, cap
        if cur:
            groups.append(cur)
        if last_bucket_mb is not None:  # built from the last-produced end: put them in production order
            groups = [list(reversed(g)) for g in reversed(groups)]
        for g in groups:
            self._close(g)
        self._pending = [len(b["params"]) for b in self.buckets]

    def production_order(self) -> List[int]:
        return [i for b in self.buckets for i in b["params"]]

    def _rebuild_from_observed(self) -> bool:
        """End of step 1: rank 0's observed gradient-ready order -> new buckets + flat re-layout (every rank).
        Returns True when the layout changed."""
        obs, self._observed = self._observed, None
        seen = set(obs)
        obs = obs + [i for i in self.production_order() if i not in seen]  # never-ready params last (unused)
        if dist.is_initialized() and self.world > 1:
            on_dev = dist.get_backend(self.pg) == "nccl"
            t = torch.tensor(obs, dtype=torch.int64, device=self.flat.device if on_dev else "cpu")
            dist.broadcast(t, src=0, group=self.pg)
            obs = [int(v) for v in t.tolist()]
        if obs == self.production_order():
            return False
        self.flat.reorder(list(reversed(obs)))
        self._assign(obs)
        self.rebuilt = True
        return True

    def _close(self, idxs: List[int]) -> None:
        slots = [self.flat.slots[i] for i in idxs]
        lo = min(s.offset for s in slots)
        hi = max(s.offset + s.numel for s in slots)
        b = {"params": list(idxs), "lo": lo, "hi": hi, "id": len(self.buckets)}
        for i in idxs:
            self.bucket_of[i] = b["id"]
        self.buckets.append(b)

    def bucket_sizes_mb(self) -> List[float]:
        return [(b["hi"] - b["lo"]) * 4 / 2 ** 20 for b in self.buckets]

    # -- per-step protocol ---------------------------------------------------------------------
    def grad_ready(self, pid: int) -> None:
        if not self.enabled:
            return
        if self._observed is not None:
            self._observed.append(pid)
        bid = self.bucket_of[pid]
        self._pending[bid] -= 1
        # launch strictly in bucket-index order (upstream Reducer::mark_bucket_ready / next_bucket_): a rank whose
        # local ready order differs from rank 0's still issues the same collective sequence as every other rank
        while self._next < len(self.buckets) and self._pending[self._next] == 0:
            self._launch(self._next)
            self._next += 1

    def _launch(self, bid: int) -> None:
        b = self.buckets[bid]
        view = self.flat.grad[b["lo"]:b["hi"]]
        self._works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
        self.launch_log.append(bid)

    def finish(self) -> bool:
        """Wait (stream-wise) for every bucket; launch any bucket whose params produced no grad.  After the first
        step of a ``rebuild`` bucketer, rebuild the buckets from the observed order; returns True when it did."""
        if not self.enabled:
            return False
        # buckets not launched yet (unused parameters, or held behind one): reduce whatever is in the buffer (zeros for
        # unused parameters) in index order, to stay in lock-step
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        for w in self._works:
            w.wait()
        self._works.clear()
        self._pending = [len(b["params"]) for b in self.buckets]
        self._next = 0
        self.last_launch_order, self.launch_log = self.launch_log, []
        if self._observed is not None:
            return self._rebuild_from_observed()
        return False

    def grad_scale(self) -> float:
        """Factor the optimizer applies to the summed gradients (mean over ranks)."""
        return 1.0 / self.world if self.enabled else 1.0

    # -- autograd path -------------------------------------------------------------------------
    def register_autograd_hooks(self) -> None:
        """Generic (autograd) path: notify readiness from post-accumulate-grad hooks."""
        for s, p in zip(self.flat.slots, self.flat.params):
            p.register_post_accumulate_grad_hook(lambda _p, i=s.index: self.grad_ready(i))


def broadcast_parameters(flat: FlatParams, buffers: Optional[FlatBuffers], process_group=None, src: int = 0) -> None:
    """DDP constructor semantics: every rank starts from rank 0's parameters and buffers (X2)."""
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1:
        return
    dist.broadcast(flat.data, src=src, group=process_group)
    if buffers is not None:
        sync_buffers(buffers, process_group, src)
    flat.refresh_shadow()


def sync_buffers(buffers: FlatBuffers, process_group=None, src: int = 0) -> None:
    """DDP ``broadcast_buffers=True``: BN running statistics from rank 0 before a forward (X3)."""
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1:
        return
    if buffers.n_float:
        dist.broadcast(buffers.fdata, src=src, group=process_group)
    if buffers.n_int:
        dist.broadcast(buffers.idata, src=src, group=process_group)
