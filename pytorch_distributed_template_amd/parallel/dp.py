"""Single-process multi-GPU DataParallel on the native executor (reference C09, `dataparallel.py:119`).

Reference semantics (``nn.DataParallel``) kept here:
* ONE process drives all visible GPUs; the node-total batch ``-b`` is scattered along dim 0;
* every forward replicates the parameters (and BN buffers) from GPU 0 to the other GPUs;
* the loss is the mean over the FULL batch, i.e. each replica's backward seed is divided by the
  node-total batch size;
* gradients are reduce-added onto GPU 0 and the optimizer runs on GPU 0 only;
* BatchNorm running statistics come from GPU 0's replica only (other replicas' updates are discarded).

MI355X-native mechanics: replicas are :class:`ResNetExecutor` instances (one per device, each with
its own 16-bit weight shadow).  Collectives go through our single-process RCCL device group
(csrc/dp_group.cpp: ``ncclCommInitAll`` over the visible GPUs, one grouped call per collective on each
device's current stream): the per-forward weight broadcast moves the 16-bit shadow (half the bytes of
the fp32 parameters) and the BN buffers from GPU 0 over xGMI, and gradients are reduce-added in place
into GPU 0's flat gradient buffer.  All devices run concurrently because every launch is asynchronous on
its device's stream; no host synchronisation is needed anywhere in the step.

One host thread drives every device, so eager launching would serialise: a replica's step is ~300 kernel
launches (a few ms of host time) while its GPU work at the reference's per-GPU batch is only a few ms, and
N replicas would wait on one launching thread.  With ``graph=True`` (the default on > 1 device) each
replica's forward + backward (plus its derived weight layouts) is captured once per input shape as a HIP
graph on its own device and replayed: per step the host issues the broadcast, N graph launches, the
gradient reduce and the SGD -- the devices' work overlaps instead of queueing behind the host.

What a replica receives each forward (``_replicate``): the 16-bit shadow (conv / fc weights as the kernels read
them), the fp32 values of the 1-D parameters that the executor reads from the MASTER copy (BatchNorm gamma / beta
in every finalize / eval / backward coefficient, the fc bias in the loss kernel; ``FlatParams.master_read_index``,
~10 K floats for ResNet-18) packed into one buffer, and the BN running statistics.  On the fp32 path the master
itself is the compute copy and is broadcast whole.

Replicas may share a device (``device_ids=[0, 0]``): their collectives are then plain device copies / adds in a
fixed order (:class:`_LocalGroup`), which rehearses the whole multi-replica step -- scatter, replication, per-
replica BN statistics, gradient reduce -- on one GPU, bit-comparable with a single-executor oracle.

Host batches: when the loader yields :class:`ShardedBatch` objects (``data/loader.py`` builds them for native DP
on > 1 device), each shard was copied host -> its own GPU already and ``_scatter`` only hands them out; a plain
tensor batch is split and copied from wherever it lives (``nn.DataParallel``'s scatter).
"""
from __future__ import annotations

import copy
from typing import List, Optional

import torch

from ..amp.scaler import DeviceGradScaler
from ..data.loader import ShardedBatch
from ..models.executor_vgg import make_executor
from ..optim.flat import FlatBuffers, FlatParams
from ..optim.sgd import FusedSGD


def _fp32_supported(model) -> bool:
    """Whether the native fp32 executor (models/executor32.py) can run ``model`` -- the same predicate
    NativeTrainer applies before building its fp32 validation executor."""
    from ..models.executor32 import fp32_supported
    return fp32_supported(model)


class _LocalGroup:
    """DataParallel collectives when replicas share a device (RCCL refuses duplicate GPUs): device copies and
    adds on the current streams, reduced in replica order (deterministic)."""

    def broadcast(self, ts, root: int) -> None:
        for i, t in enumerate(ts):
            if i != root:
                t.copy_(ts[root], non_blocking=True)

    def reduce(self, ts, root: int) -> None:
        acc = ts[root]
        for i, t in enumerate(ts):
            if i != root:
                acc.add_(t.to(acc.device, non_blocking=True))


class NativeDataParallelTrainer:
    def __init__(self, model, device_ids: List[int], dtype: torch.dtype = torch.bfloat16, lr: float = 0.1,
                 momentum: float = 0.9, weight_decay: float = 1e-4, use_amp: bool = False,
                 graph: Optional[bool] = None, eval_fp32: bool = False):
        self.device_ids = list(device_ids)
        distinct = len(set(self.device_ids))
        # per-replica HIP graphs (see module doc); two eager warm-up steps settle buffers and tile choices
        self.use_graph = (distinct > 1) if graph is None else bool(graph)
        self._graphs = {}
        self._graph_warm = 0
        self.devices = [torch.device("cuda", i) for i in self.device_ids]
        self.dtype = dtype
        replicas = [model] + [copy.deepcopy(model) for _ in self.devices[1:]]
        self.flats = []
        self.buffers = []
        self.executors = []
        for m, d in zip(replicas, self.devices):
            with torch.cuda.device(d):
                f = FlatParams(m, d, dtype if dtype != torch.float32 else None, guards=len(self.devices) == 1)
                b = FlatBuffers(m, d)
                self.flats.append(f)
                self.buffers.append(b)
                if dtype == torch.float32:  # the reference's dataparallel.py precision
                    from ..models.executor32 import ResNetExecutor32
                    self.executors.append(ResNetExecutor32(m, f, d))
                else:
                    self.executors.append(make_executor(m, f, d, dtype))
        self.model = model
        self.flat = self.flats[0]
        # eval_fp32: validation of the fp32 model like the reference's DataParallel (`dataparallel.py:243-262`, no
        # autocast anywhere): each replica evaluates its shard on the fp32 kernels over the fp32 master weights, which
        # are broadcast from GPU 0 to the replicas once per weight version (16-bit training replicates only the 16-bit
        # shadow and the master-read parameters)
        self._eval32 = None
        self._eval32_at = -1
        if eval_fp32 and dtype != torch.float32 and not _fp32_supported(model):
            import warnings
            warnings.warn("--eval-precision fp32: no native fp32 kernels for this model; validating in the compute dtype")
            eval_fp32 = False
        if eval_fp32 and dtype != torch.float32:
            from ..models.executor32 import ResNetExecutor32
            self._eval32 = []
            for m, f, d in zip(replicas, self.flats, self.devices):
                with torch.cuda.device(d):
                    self._eval32.append(ResNetExecutor32(m, f, d))
        self.optimizer = FusedSGD(self.flat, lr, momentum, weight_decay)
        self.optimizer.post_step_hooks.append(self.executors[0].update_derived)
        self.scaler = DeviceGradScaler(self.devices[0], enabled=use_amp and dtype == torch.float16)
        # fp32 values the 16-bit executors read from the master (BN affine, fc bias): packed on GPU 0, broadcast,
        # unpacked into each replica's master (see module doc)
        self._aux_idx, self._aux = [], []
        if dtype != torch.float32 and len(self.devices) > 1:
            idx = self.flat.master_read_index()
            for d in self.devices:
                self._aux_idx.append(idx.to(d))
                self._aux.append(torch.zeros(idx.numel(), dtype=torch.float32, device=d))
        self.group = None
        # the runner hands batches over as they come from the loader: ShardedBatch (already on every GPU) or a
        # tensor that _scatter splits; no copy to the runner's device first
        self.host_batches = len(self.devices) > 1
        if len(self.devices) > 1:
            if distinct == len(self.devices):
                from ..ops import native
                self.group = native.C.DeviceGroup(self.device_ids)
            else:
                self.group = _LocalGroup()

    def on_state_loaded(self) -> None:
        """After ``model.load_state_dict`` (resume): GPU 0's shadow and derived layouts, then every replica's full
        compute state (shadow, master-read parameters, BN buffers, derived layouts)."""
        self._eval32_at = -1
        with torch.cuda.device(self.devices[0]):
            self.flat.refresh_shadow()
            self.executors[0].update_derived()
        self._replicate(derived=True)

    def _replicate(self, derived: bool = True) -> None:
        if len(self.devices) == 1:
            return
        # the compute copy: the 16-bit shadow, or the fp32 master itself on the fp32 path
        self.group.broadcast([f.shadow if f.shadow is not None else f.data for f in self.flats], 0)
        if self._aux:
            from ..ops import native
            with torch.cuda.device(self.devices[0]):
                native.C.gather32(self.flat.data, self._aux_idx[0], self._aux[0])
            self.group.broadcast(self._aux, 0)
            for i in range(1, len(self.devices)):
                with torch.cuda.device(self.devices[i]):
                    native.C.scatter32(self._aux[i], self._aux_idx[i], self.flats[i].data)
        if self.buffers[0].n_float:
            self.group.broadcast([b.fdata for b in self.buffers], 0)
        if derived:
            for i in range(1, len(self.devices)):
                with torch.cuda.device(self.devices[i]):
                    self.executors[i].update_derived()

    def _replica_step(self, i: int, x, t, ls, B: int, derived: bool):
        """Replica i's forward + backward on its device (gradients into its flat buffer)."""
        if derived and i > 0:
            self.executors[i].update_derived()
        return self.executors[i].train_step(x, t, loss_scale=ls, grad_div=float(B))

    def _run_replicas(self, xs, ts, B: int):
        """Every replica's step: eager, or -- once warm -- one captured HIP graph replay per device."""
        scale = self.scaler.scale_tensor
        res = []
        warm = self.use_graph and self._graph_warm >= 2
        for i, (x, t) in enumerate(zip(xs, ts)):
            if x.shape[0] == 0:
                res.append(None)
                continue
            with torch.cuda.device(self.devices[i]):
                ls = scale if i == 0 or scale is None else scale.to(self.devices[i])
                if not warm:
                    res.append(self._replica_step(i, x, t, ls, B, derived=False))
                    continue
                key = (i, tuple(x.shape), x.dtype, B)
                # executor 0's derived layouts are gathered eagerly by the post-step hook (on its side stream when
                # split): order them before the capture / replay here, never through an event waited on inside
                # the capture (a capture-time wait on an outside event does not order a later replay)
                self.executors[i]._wait_derived()
                ent = self._graphs.get(key)
                if ent is None:
                    sx, st = x.clone(), t.clone()
                    sls = ls.clone() if ls is not None else None
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, capture_error_mode="thread_local"):
                        out = self._replica_step(i, sx, st, sls, B, derived=True)
                    ent = self._graphs[key] = (g, sx, st, sls, out)
                g, sx, st, sls, out = ent
                sx.copy_(x, non_blocking=True)
                st.copy_(t, non_blocking=True)
                if sls is not None:
                    sls.copy_(ls, non_blocking=True)
                g.replay()
                res.append(tuple(o.clone() for o in out))
        if self.use_graph and not warm:
            self._graph_warm += 1
        return res, warm

    def _scatter(self, images, target):
        if isinstance(images, ShardedBatch):  # the loader already put shard i on device i
            assert len(images.parts) == len(self.devices), "ShardedBatch built for another device list"
            return list(images.parts), list(target.parts)
        n = len(self.devices)
        chunks = torch.tensor_split(torch.arange(images.shape[0]), n)
        xs, ts = [], []
        for d, c in zip(self.devices, chunks):
            lo, hi = int(c[0]) if len(c) else 0, int(c[-1]) + 1 if len(c) else 0
            xs.append(images[lo:hi].to(d, non_blocking=True))
            ts.append(target[lo:hi].to(d, non_blocking=True))
        return xs, ts

    def train_step(self, images, target):
        B = images.size(0)
        warm = self.use_graph and self._graph_warm >= 2
        self._replicate(derived=not warm)  # graphed replicas gather their derived layouts inside the graph
        xs, ts = self._scatter(images, target)
        scale = self.scaler.scale_tensor
        outs, mets = [], []
        res, _ = self._run_replicas(xs, ts, B)
        for x, r in zip(xs, res):
            if r is None:
                continue
            logits, met = r
            outs.append(logits)
            mets.append(met.to(self.devices[0]) * (x.shape[0] / B))
        if self.buffers[0].n_int:
            self.buffers[0].idata.add_(1)  # num_batches_tracked of GPU 0's BatchNorms, as nn.DataParallel
        if self.group is not None:
            self.group.reduce([f.grad for f in self.flats], 0)  # in place into GPU 0's flat gradient
        self.scaler.unscale_check(self.flat.grad)
        self.optimizer.step(grad_scale=1.0, loss_scale=scale, found_inf=self.scaler.found_inf)
        self.scaler.update()
        logits = torch.cat([o.to(self.devices[0]) for o in outs])
        return logits, torch.stack(mets).sum(0)

    def _replicate_fp32(self) -> None:
        """fp32 validation: the fp32 master on every replica + each replica's fp32 derived layouts, once per weight
        version (optimizer step or state load)."""
        if self._eval32_at == self.optimizer.step_count:
            return
        if len(self.devices) > 1:
            self.group.broadcast([f.data for f in self.flats], 0)
        for i, ex in enumerate(self._eval32):
            with torch.cuda.device(self.devices[i]):
                ex.update_derived()
        self._eval32_at = self.optimizer.step_count

    @torch.no_grad()
    def eval_step(self, images, target):
        B = images.size(0)
        self._replicate()
        executors = self.executors
        if self._eval32 is not None:
            self._replicate_fp32()
            executors = self._eval32
        xs, ts = self._scatter(images, target)
        outs, mets = [], []
        for i, (ex, x, t) in enumerate(zip(executors, xs, ts)):
            if x.shape[0] == 0:
                continue
            with torch.cuda.device(self.devices[i]):
                logits, met = ex.eval_step(x, t)
            outs.append(logits)
            mets.append(met.to(self.devices[0]) * (x.shape[0] / B))
        return torch.cat([o.to(self.devices[0]) for o in outs]), torch.stack(mets).sum(0)
