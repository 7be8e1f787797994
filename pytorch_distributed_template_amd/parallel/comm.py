"""Native collectives: our RCCL communicator and C++ gradient bucketer (csrc/comm.cpp).

The default data-parallel path drives RCCL through ``torch.distributed`` (backend ``nccl`` IS RCCL on
ROCm).  ``--comm native`` instead uses this module: one ``ncclComm_t`` per process whose unique id is
exchanged through the launcher's TCP store, collectives on our own HIP stream ordered by events against
the compute stream (no host synchronisation), and the bucketed gradient all-reduce run from C++
(``Bucketer.ready`` launches a bucket's in-place SUM all-reduce the moment its last gradient is written).
Reference counterparts: c10d ``ProcessGroupNCCL`` + ``TCPStore`` and the DDP ``Reducer`` (SURVEY §2.7,
X1-X9; `distributed.py:124,144`).
"""
from __future__ import annotations

import itertools
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import native
from .store import NativeStore

_COUNTER = itertools.count()


class NativeComm:
    """A process-group-like wrapper over :class:`_C.Communicator`."""

    def __init__(self, device: torch.device, process_group=None, store=None, timeout_s: float = 0.0):
        """The RCCL unique id travels through ``store``: c10d's store when torch.distributed is up,
        otherwise (or when given) our native TCP store (:class:`~.store.NativeStore`, env://).

        ``timeout_s > 0`` starts the C++ watchdog (csrc/comm.cpp): a collective pending longer than that, or
        an asynchronous RCCL error, aborts the communicator and exits the process non-zero (the launcher
        then tears the group down) -- the counterpart of ProcessGroupNCCL's watchdog + ``timeout``."""
        self.device = torch.device(device)
        key = f"pdt_rccl_uid_{next(_COUNTER)}"
        if store is None and dist.is_initialized():
            store = dist.distributed_c10d._get_default_store()
        elif store is None and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            store = NativeStore.from_env()
        if store is not None:
            if isinstance(store, NativeStore):
                self.rank, self.world = store.rank, store.world
            else:
                self.rank = dist.get_rank(process_group)
                self.world = dist.get_world_size(process_group)
            if self.rank == 0:
                uid = native.C.rccl_unique_id()
                store.set(key, uid)
            else:
                uid = store.get(key)
        else:
            self.rank, self.world = 0, 1
            uid = native.C.rccl_unique_id()
        self.store = store
        self.comm = native.C.Communicator(bytes(uid), self.world, self.rank, self.device.index or 0,
                                          float(timeout_s))

    def count(self) -> int:
        """Ranks in the RCCL communicator (``ncclCommCount``)."""
        return self.comm.count()

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False) -> None:
        self.comm.all_reduce(t, op, async_op)

    def all_reduce_inline(self, t: torch.Tensor, op: str = "sum") -> None:
        """All-reduce on the caller's stream (no comm-stream round trip); the caller guarantees that no
        comm-stream collective can be reordered against it (see csrc/comm.cpp)."""
        self.comm.all_reduce_inline(t, op)

    def broadcast_inline(self, t: torch.Tensor, src: int = 0) -> None:
        """Broadcast on the caller's stream (same ordering contract as :meth:`all_reduce_inline`)."""
        self.comm.broadcast_inline(t, src)

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False) -> None:
        self.comm.broadcast(t, src, async_op)

    def all_gather(self, inp: torch.Tensor, out: torch.Tensor, async_op: bool = False) -> None:
        self.comm.all_gather(inp, out, async_op)

    def wait(self) -> None:
        self.comm.wait()

    def barrier(self) -> None:
        self.comm.barrier()

    def check(self) -> None:
        """Raise if RCCL reported an asynchronous error (failure detection hook)."""
        err = self.comm.async_error()
        if err:
            self.comm.abort()
            raise RuntimeError(f"RCCL communicator failed: {err}")

    def abort(self) -> None:
        self.comm.abort()

    def destroy(self) -> None:
        """Collective teardown (every rank, same point): stop the watchdog, ncclCommDestroy."""
        self.comm.destroy()


class NativeBucketer:
    """Drop-in for :class:`~.ddp.GradBucketer` backed by the C++ bucketer (same bucket layout)."""

    def __init__(self, layout, comm: NativeComm, compress: str = "none"):
        """``compress="bf16"``: buckets are all-reduced in bf16 (cast on the comm stream, half the bytes on
        xGMI, widened back into the fp32 gradient) -- upstream DDP's ``bf16_compress_hook``; off by default, as
        the reference all-reduces fp32 gradients."""
        if compress not in ("none", "bf16"):
            raise ValueError(f"gradient compression must be 'none' or 'bf16', got {compress!r}")
        self.world = comm.world
        self.comm = comm
        self.compress = compress
        self.buckets = layout.buckets
        pb: List[int] = [0] * len(layout.flat.slots)
        for pid, bid in layout.bucket_of.items():
            pb[pid] = bid
        self._impl = native.C.Bucketer(comm.comm, layout.flat.grad, [b["lo"] for b in self.buckets],
                                       [b["hi"] for b in self.buckets], pb, 1 if compress == "bf16" else 0)

    def grad_ready(self, pid: int) -> None:
        self._impl.ready(pid)

    def finish(self) -> None:
        self._impl.finish()

    def grad_scale(self) -> float:
        return 1.0 / self.world

    def bucket_sizes_mb(self) -> List[float]:
        return [(b["hi"] - b["lo"]) * 4 / 2 ** 20 for b in self.buckets]
