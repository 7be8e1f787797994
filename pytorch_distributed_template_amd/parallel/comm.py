"""Native collectives: our RCCL communicator and C++ gradient bucketer (csrc/comm.cpp).

The default data-parallel path drives RCCL through ``torch.distributed`` (backend ``nccl`` IS RCCL on
ROCm).  ``--comm native`` instead uses this module: one ``ncclComm_t`` per process whose unique id is
exchanged through the launcher's TCP store, collectives on our own HIP stream ordered by events against
the compute stream (no host synchronisation), and the bucketed gradient all-reduce run from C++
(``Bucketer.ready`` launches a bucket's in-place SUM all-reduce the moment its last gradient is written).
Reference counterparts: c10d ``ProcessGroupNCCL`` + ``TCPStore`` and the DDP ``Reducer`` (SURVEY §2.7,
X1-X9; `distributed.py:124,144`).

Transports (csrc/comm.cpp): ``rccl`` (the production path: one rank per GPU over xGMI) or ``host`` (a POSIX
shared-memory group, csrc/shm_group.h) for ranks that share a GPU -- RCCL refuses duplicate devices -- or run on
the CPU.  The host transport runs the same C++ Communicator / Bucketer code, synchronously, so the multi-rank
bucketer logic is exercised by the CPU test suite (world 2 / 4, host tensors) and by 1-GPU DDP rehearsals
(``bench.py --gpus 2 --dist-backend gloo``).  ``auto`` = host on the CPU or when ranks share a GPU, else rccl.
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


def _gpus_shared(world: int) -> bool:
    """More ranks on this node than visible GPUs (a rehearsal with ranks sharing devices)."""
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return torch.cuda.is_available() and local > torch.cuda.device_count()


def single_node(world: int) -> bool:
    """Every rank on this node (the host shared-memory transport maps ONE segment: it cannot span nodes)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", world)) >= world


class NativeComm:
    """A process-group-like wrapper over :class:`_C.Communicator`."""

    def __init__(self, device: torch.device, process_group=None, store=None, timeout_s: float = 0.0,
                 transport: str = "auto"):
        """The RCCL unique id (or the host group's segment name) travels through ``store``: c10d's store when
        torch.distributed is up, otherwise (or when given) our native TCP store (:class:`~.store.NativeStore`).

        ``timeout_s > 0`` starts the C++ watchdog (csrc/comm.cpp): a collective pending longer than that, or
        an asynchronous RCCL error, aborts the communicator and exits the process non-zero (the launcher
        then tears the group down) -- the counterpart of ProcessGroupNCCL's watchdog + ``timeout``.  On the host
        transport a barrier waiting longer than ``timeout_s`` raises (and aborts the group for every rank)."""
        self.device = torch.device(device)
        seq = next(_COUNTER)
        key = f"pdt_rccl_uid_{seq}"
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
        else:
            self.rank, self.world = 0, 1
        self.store = store
        if transport == "auto":
            transport = "host" if self.device.type != "cuda" or _gpus_shared(self.world) else "rccl"
        if transport not in ("rccl", "host"):
            raise ValueError(f"comm transport must be auto, rccl or host, got {transport!r}")
        if transport == "host" and self.world > 1 and not single_node(self.world):
            # fail fast: the other nodes would retry shm_open on a segment that exists only on node 0 until the timeout
            raise ValueError(f"the host shared-memory comm transport needs every rank on one node (WORLD_SIZE="
                             f"{self.world}, LOCAL_WORLD_SIZE={os.environ.get('LOCAL_WORLD_SIZE')}); use --comm torch "
                             "(c10d / gloo) or one rank per GPU (rccl) across nodes")
        if transport == "rccl" and self.device.type != "cuda":
            raise ValueError("the rccl transport needs GPU tensors; use transport='host' on the CPU")
        self.transport = transport
        dev_index = (self.device.index or 0) if self.device.type == "cuda" else -1
        if transport == "host":
            # rank 0 publishes a fresh segment name and creates it; the others open it (retrying until it exists);
            # the constructor's barrier returns once every rank mapped it, and rank 0 then unlinks the name
            if self.rank == 0:
                name = f"/pdt_comm_{os.getpid()}_{seq}_{os.urandom(4).hex()}"
                if store is not None:
                    store.set(key, name.encode())
            else:
                name = bytes(store.get(key)).decode()
            slot = int(os.environ.get("PDT_HOST_COMM_SLOT_MB", "8")) << 20
            self.comm = native.C.host_communicator(name, self.world, self.rank, dev_index, self.rank == 0, slot,
                                                   float(timeout_s) if timeout_s and timeout_s > 0 else 600.0)
            return
        if store is not None:
            if self.rank == 0:
                uid = native.C.rccl_unique_id()
                store.set(key, uid)
            else:
                uid = store.get(key)
        else:
            uid = native.C.rccl_unique_id()
        self.comm = native.C.Communicator(bytes(uid), self.world, self.rank, dev_index, float(timeout_s))

    def count(self) -> int:
        """Ranks in the communicator (``ncclCommCount`` on RCCL)."""
        return self.comm.count()

    def track_compute(self, what: str = "graph replay") -> None:
        """Watchdog: one tracked event on the compute stream (after a HIP-graph replay, whose captured
        collectives are otherwise invisible to the timeout)."""
        self.comm.track_compute(what)

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
        _trace(f"rank {self.rank}/{self.world}: {self.transport} communicator aborted")

    def destroy(self) -> None:
        """Collective teardown (every rank, same point): stop the watchdog, ncclCommDestroy."""
        self.comm.destroy()
        _trace(f"rank {self.rank}/{self.world}: {self.transport} communicator destroyed")


def live_watchdogs() -> int:
    """Native communicator watchdog threads still running in this process (0 after a clean teardown)."""
    return int(native.C.Communicator.live_watchdogs())


def _trace(msg: str) -> None:
    """PDT_COMM_TRACE=1: communicator lifecycle events on stderr (teardown tests)."""
    if os.environ.get("PDT_COMM_TRACE") == "1":
        import sys
        sys.stderr.write(f"[pdt comm] {msg}\n")
        sys.stderr.flush()


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
        self.layout = layout
        self._make_impl()

    def _make_impl(self) -> None:
        layout = self.layout
        self.buckets = layout.buckets
        self.bucket_of = layout.bucket_of
        pb: List[int] = [0] * len(layout.flat.slots)
        for pid, bid in layout.bucket_of.items():
            pb[pid] = bid
        self._impl = native.C.Bucketer(self.comm.comm, layout.flat.grad, [b["lo"] for b in self.buckets],
                                       [b["hi"] for b in self.buckets], pb, 1 if self.compress == "bf16" else 0)

    def grad_ready(self, pid: int) -> None:
        if self.layout._observed is not None:  # step 1 of a rebuilding layout (GradBucketer rebuild=True)
            self.layout._observed.append(pid)
        self._impl.ready(pid)

    def finish(self) -> bool:
        self._impl.finish()
        if self.layout._observed is not None and self.layout._rebuild_from_observed():
            self._make_impl()
            return True
        return False

    def grad_scale(self) -> float:
        return 1.0 / self.world

    def bucket_sizes_mb(self) -> List[float]:
        return [(b["hi"] - b["lo"]) * 4 / 2 ** 20 for b in self.buckets]
