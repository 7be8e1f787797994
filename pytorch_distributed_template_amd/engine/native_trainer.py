"""One data-parallel training step on the native (HIP kernel) path.

Mirrors the reference step (`distributed.py:237-263`, `distributed_syncBN_amp.py:250-278`):

    [DDP buffer broadcast] -> forward -> CE loss -> top-1 accuracy -> [metric all-reduce]
    -> (scaled) backward with bucketed gradient all-reduce -> (unscale, overflow check) SGD step
    -> (scaler update)

with every piece on device and no host synchronisation inside the step: the loss/accuracy pair is
returned as a device tensor (reduced across ranks with ONE 2-float all-reduce instead of a barrier and
two scalar all-reduces) and read by the caller only when it logs.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from ..amp.scaler import DeviceGradScaler
from ..models.executor_vgg import make_executor
from ..optim.flat import FlatBuffers, FlatParams
from ..optim.sgd import FusedSGD
from ..parallel.ddp import GradBucketer, broadcast_parameters, sync_buffers
from ..parallel.syncbn import native_syncbn_wiring


class NativeTrainer:
    def __init__(self, model, device, dtype: torch.dtype = torch.bfloat16, lr: float = 0.1, momentum: float = 0.9,
                 weight_decay: float = 1e-4, use_amp: bool = False, sync_bn: bool = False,
                 bucket_cap_mb: float = 25.0, first_bucket_mb: float = 1.0, broadcast_buffers: bool = True,
                 process_group=None, reduce_metrics: bool = True, autotune: bool = False, comm: str = "torch",
                 force_comm: bool = False, graph: bool = False, last_bucket_mb: Optional[float] = 1.0,
                 comm_timeout_s: float = 0.0, time_comm: bool = False, eval_fp32: bool = False,
                 grad_compress: str = "none", comm_transport: str = "auto"):
        self.device = torch.device(device)
        self.dtype = dtype
        self.buffer_syncs = 0  # buffer broadcasts issued (tests: one per train step after the first + one per eval epoch)
        self.model = model
        self.pg = process_group
        self.distributed = dist.is_initialized() and dist.get_world_size(process_group) > 1
        self.world = dist.get_world_size(process_group) if self.distributed else 1
        # fp32 (the reference's distributed.py precision): kernels read the fp32 master directly, no shadow
        self.flat = FlatParams(model, self.device, dtype if dtype != torch.float32 else None)
        self.buffers = FlatBuffers(model, self.device)
        # collectives: torch.distributed (RCCL via c10d) or our own RCCL communicator + C++ bucketer
        # (--comm native; force_comm exercises it on a single rank).  With the native communicator EVERY
        # GPU collective of the step (constructor broadcast, buffer broadcast, gradient buckets, SyncBN
        # statistics, metrics) goes through it; torch.distributed only provides the rendezvous store.
        self.ncomm = None
        if comm == "native" and (self.distributed or force_comm):
            from ..parallel.comm import NativeComm
            self.ncomm = NativeComm(self.device, process_group, timeout_s=comm_timeout_s, transport=comm_transport)
        self._broadcast_initial()
        layout = GradBucketer(self.flat, process_group, bucket_cap_mb, first_bucket_mb, enabled=self.distributed,
                              last_bucket_mb=last_bucket_mb)
        if self.ncomm is not None:
            from ..parallel.comm import NativeBucketer
            self.bucketer = NativeBucketer(layout, self.ncomm, compress=grad_compress)
        elif grad_compress != "none":
            raise ValueError("--grad-compress needs the native communicator (--comm native)")
        else:
            self.bucketer = layout
        # HIP events around bucketer.finish(): the time the compute stream waits for gradient all-reduces
        # that backward did not hide (exposed communication)
        self._comm_events = [] if time_comm else None
        # SyncBN collectives: which communicator / stream every statistic all-reduce uses (parallel/syncbn.py)
        self.ncomm_bn, sync_kw = native_syncbn_wiring(sync_bn, self.ncomm, process_group, self.distributed, dtype,
                                                      comm_timeout_s, comm_transport)
        if dtype == torch.float32:
            from ..models.executor32 import ResNetExecutor32
            self.executor = ResNetExecutor32(model, self.flat, self.device, grad_ready=self.bucketer.grad_ready,
                                             **sync_kw)
        else:
            self.executor = make_executor(model, self.flat, self.device, dtype, grad_ready=self.bucketer.grad_ready,
                                          autotune=autotune, **sync_kw)
        # --eval-precision fp32: validation on the fp32 executor over the fp32 master weights (the reference
        # validates without autocast, `distributed_syncBN_amp.py:311-317`), whatever the training dtype
        self._eval32 = None
        self._eval32_at = -1  # optimizer step count its derived layouts were gathered at
        from ..models.executor32 import fp32_supported
        if eval_fp32 and dtype != torch.float32 and not fp32_supported(model):
            import warnings
            warnings.warn("--eval-precision fp32: no native fp32 kernels for this model; validating in the compute dtype")
            eval_fp32 = False
        if eval_fp32 and dtype != torch.float32:
            from ..models.executor32 import ResNetExecutor32
            self._eval32 = ResNetExecutor32(model, self.flat, self.device)
        self.optimizer = FusedSGD(self.flat, lr, momentum, weight_decay)
        self.optimizer.post_step_hooks.append(self.executor.update_derived)
        # fp16 needs dynamic loss scaling; bf16 has fp32's exponent range and does not
        self.scaler = DeviceGradScaler(self.device, enabled=use_amp and dtype == torch.float16)
        self.broadcast_buffers = broadcast_buffers and (self.distributed or self.ncomm is not None)
        self.reduce_metrics = reduce_metrics and (self.distributed or self.ncomm is not None)
        self._steps = 0
        self._eval_sync_pending = False  # a train step ran since the last eval-forward buffer broadcast
        # whole-step HIP graph (launch-bound small batches, e.g. the reference's -b 1200 split over 8 GPUs = 150
        # per GPU): single process, or any world on the native communicator, whose collectives (buffer
        # broadcast, gradient buckets, SyncBN statistics, metrics) are captured into the graph with the kernels
        # (RCCL supports stream capture; every rank captures and replays the same sequence).  c10d's
        # ProcessGroupNCCL collectives stay eager, so world > 1 on --comm torch runs without a graph.
        # (the host shared-memory transport synchronises the host inside every collective: not capturable)
        self.use_graph = graph and (self.ncomm is None or self.ncomm.transport == "rccl") and (
            not self.distributed or self.ncomm is not None)
        self._graphs = {}
        self._graph_warm = 0

    def _broadcast_initial(self) -> None:
        """DDP constructor semantics (X2): every rank starts from rank 0's parameters and buffers."""
        if self.ncomm is None:
            broadcast_parameters(self.flat, self.buffers, self.pg)
            return
        if self.ncomm.world > 1:
            self.ncomm.broadcast(self.flat.data, 0)
            self._sync_buffers()
            self.flat.refresh_shadow()

    def close(self) -> None:
        """Collective teardown of the native communicators (every rank, same point: runner._finish after its barrier,
        bench.py after the timed steps): ncclCommDestroy, watchdog threads joined.  Idempotent.

        Captured step graphs hold collectives on these communicators, and RCCL's destroy waits until every graph
        referencing a communicator is freed: release the graphs (after the device drained) BEFORE destroying."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if self._graphs:
            self._graphs.clear()
            import gc
            gc.collect()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
        for c in (self.ncomm_bn, self.ncomm):
            if c is not None:
                c.destroy()
        self.ncomm_bn = None
        self.ncomm = None

    def abort(self) -> None:
        """Failure path (an exception left the epoch loop): abort the communicators -- pending RCCL work is cancelled
        and the watchdog stops -- so this rank can exit instead of hanging in a collective; not collective."""
        for c in (self.ncomm_bn, self.ncomm):
            if c is not None:
                c.abort()
        self.ncomm_bn = None
        self.ncomm = None

    def on_state_loaded(self) -> None:
        """After ``model.load_state_dict`` (resume): re-derive the 16-bit shadow and the kernel weight layouts."""
        self.flat.refresh_shadow()
        self.executor.update_derived()
        self._eval32_at = -1

    def exposed_comm_ms(self) -> Optional[float]:
        """Mean per-step exposed gradient-communication time since the last call (needs ``time_comm``)."""
        if not self._comm_events:
            return None
        torch.cuda.synchronize(self.device)
        ms = sum(a.elapsed_time(b) for a, b in self._comm_events) / len(self._comm_events)
        self._comm_events.clear()
        return ms

    def param_checksum(self) -> torch.Tensor:
        """[sum, sum of squares, position-weighted sum] of the fp32 master parameters (fp64): equal on every
        rank iff the data-parallel replicas stayed in lock-step."""
        d = self.flat.data.double()
        w = torch.linspace(0.5, 1.5, d.numel(), dtype=torch.float64, device=d.device)
        return torch.stack([d.sum(), (d * d).sum(), (d * w).sum()])

    def _reduce(self, met: torch.Tensor) -> torch.Tensor:
        if self.reduce_metrics:
            if self.ncomm is not None:
                self.ncomm.all_reduce(met)
            else:
                dist.all_reduce(met, group=self.pg)
            met.div_(self.world)
        return met

    def _sync_buffers(self) -> None:
        self.buffer_syncs += 1
        if self.ncomm is not None:
            # start of a step: every earlier collective was joined into the compute stream, so the broadcasts
            # go straight onto it (no comm-stream round trip; same RCCL order on every rank)
            if self.buffers.n_float:
                self.ncomm.broadcast_inline(self.buffers.fdata, 0)
            if self.buffers.n_int:
                self.ncomm.broadcast_inline(self.buffers.idata, 0)
        else:
            sync_buffers(self.buffers, self.pg)

    def train_step(self, images: torch.Tensor, target: torch.Tensor):
        if self.use_graph:
            return self._graphed_step(images, target)
        # Single-GPU runs at large batch issue the step on a HIGH-priority stream, so the weight gradients of the
        # (normal-priority) side stream fill CUs the critical path leaves idle instead of delaying it.  Same-box A/Bs
        # (profiles/r6_ab_summary.md): ResNet-18 B=1200 -0.15 / -0.21 ms, ResNet-50 fp16 -0.13 ms; but B=400 +0.06 ms
        # and B=150 +0.08 ms (the starved weight-gradient tail then ends the step), hence the batch threshold, and
        # ResNeXt-50 +0.41 ms (its grouped weight gradients are the heavier tail), hence no grouped convs; VGG-16 at
        # B=150 -0.10 ms (a long step at a small batch), hence VGG's lower threshold.  Not with a
        # communicator: bucket all-reduces queue behind the side stream and would be delayed the same way (unmeasured
        # on a multi-GPU node).  PDT_MAIN_PRIO=-1 / 0 forces it on / off.
        env = os.environ.get("PDT_MAIN_PRIO")
        if env is not None:
            prio = int(env)
        else:
            if getattr(self, "_grouped", None) is None:
                from ..models.classic import VGG
                self._grouped = any(getattr(m, "groups", 1) > 1 for m in self.model.modules()
                                    if isinstance(m, torch.nn.Conv2d))
                # VGG's step is long at any batch it trains at: on from 128 images (VGG-16 B=150 -0.10 ms)
                self._prio_batch = 128 if isinstance(self.model, VGG) else 800
            prio = -1 if (self.world == 1 and images.shape[0] >= self._prio_batch and not self._grouped) else 0
        if prio == 0 or self.device.type != "cuda":
            return self._train_step_eager(images, target)
        if getattr(self, "_main_stream", None) is None:
            self._main_stream = torch.cuda.Stream(device=self.device, priority=prio)
        cur = torch.cuda.current_stream(self.device)
        self._main_stream.wait_stream(cur)
        with torch.cuda.stream(self._main_stream):
            out = self._train_step_eager(images, target)
        cur.wait_stream(self._main_stream)
        return out

    def _graphed_step(self, images: torch.Tensor, target: torch.Tensor):
        """Replay one captured training step (forward, loss, backward, SGD, scaler update) as a HIP graph.

        Two eager warm-up steps settle every lazily created buffer and per-shape kernel choice (and the
        momentum initialisation of the first SGD step); the graph is keyed by input shape / dtype and the
        learning rate (a kernel argument), so an LR-schedule change captures a new graph."""
        key = (tuple(images.shape), images.dtype, float(self.optimizer.lr))
        ent = self._graphs.get(key)
        if ent is None:
            if self._graph_warm < 2:
                self._graph_warm += 1
                return self._train_step_eager(images, target)
            sx, st = images.clone(), target.clone()
            g = torch.cuda.CUDAGraph()
            steps, sc = self._steps, self.optimizer.step_count
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                out = self._train_step_eager(sx, st)
            self._steps, self.optimizer.step_count = steps, sc  # capture does not run the step
            ent = self._graphs[key] = (g, sx, st, out)
        g, sx, st, out = ent
        sx.copy_(images)
        st.copy_(target)
        g.replay()
        if self.ncomm is not None:
            self.ncomm.track_compute("graph replay of a training step")
        self._steps += 1
        self._eval_sync_pending = True
        self.optimizer.step_count += 1
        return out

    def _train_step_eager(self, images: torch.Tensor, target: torch.Tensor):
        if self.broadcast_buffers and self._steps > 0:
            self._sync_buffers()
        if self.buffers.n_int:
            # BatchNorm num_batches_tracked: issued ahead of the step so it is not a launch in the tail between the
            # last weight gradient and SGD (rocprof: ~20 us there)
            self.buffers.idata.add_(1)
        logits, met = self.executor.train_step(images, target, loss_scale=self.scaler.scale_tensor,
                                               grad_div=float(images.shape[0]))
        met = self._reduce(met)
        if self._comm_events is not None and not torch.cuda.is_current_stream_capturing():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.bucketer.finish()
            e1.record()
            self._comm_events.append((e0, e1))
        else:
            self.bucketer.finish()
        self.scaler.unscale_check(self.flat.grad)
        self.optimizer.step(grad_scale=self.bucketer.grad_scale(), loss_scale=self.scaler.scale_tensor,
                            found_inf=self.scaler.found_inf)
        self.scaler.update()
        self._steps += 1
        self._eval_sync_pending = True
        return logits, met

    @torch.no_grad()
    def eval_step(self, images: torch.Tensor, target: torch.Tensor):
        if self.broadcast_buffers and self._eval_sync_pending:
            # DDP: only the FIRST eval forward after training re-broadcasts the buffers; the following
            # no-grad forwards see require_forward_param_sync = False (`T/nn/parallel/distributed.py:1557-1558`)
            self._sync_buffers()
            self._eval_sync_pending = False
        if self._eval32 is not None:
            if self._eval32_at != self.optimizer.step_count:  # once per weight version, not per batch
                self._eval32.update_derived()  # fp32 layouts of the current master weights
                self._eval32_at = self.optimizer.step_count
            logits, met = self._eval32.eval_step(images, target)
        else:
            logits, met = self.executor.eval_step(images, target)
        return logits, self._reduce(met)
