"""Multi-GPU tests (>= 2 visible MI355X): the native RCCL communicator and C++ bucketer at world = 2 over
xGMI, native DataParallel over two devices, and the single-process device group.  Skipped on 1-GPU boxes
(the gloo rehearsals in test_ddp_numerics_gpu.py / test_comm_gpu.py cover the logic there)."""
import os
import sys

import pytest
import torch

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")]
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _ddp_common import make_batch, make_model  # noqa: E402
from test_ddp_numerics_gpu import B, HW, _run_ranks  # noqa: E402


def test_native_comm_ddp_bit_equals_c10d_ddp(tmp_path):
    """Same buckets, same RCCL, same order: our communicator + C++ bucketer and c10d give identical weights."""
    a = _run_ranks(tmp_path, PDT_TEST_BACKEND="gloo", PDT_TEST_COMM="native", PDT_TEST_STEPS=2)
    b = _run_ranks(tmp_path, PDT_TEST_BACKEND="nccl", PDT_TEST_COMM="torch", PDT_TEST_STEPS=2)
    assert torch.equal(a["data"], b["data"])
    assert torch.equal(a["fbuf"], b["fbuf"])


def test_native_comm_syncbn_two_gpus(tmp_path):
    """SyncBN statistics through the native communicator on two real devices == the gloo rehearsal."""
    a = _run_ranks(tmp_path, PDT_TEST_BACKEND="gloo", PDT_TEST_COMM="native", PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=2)
    b = _run_ranks(tmp_path, PDT_TEST_BACKEND="gloo", PDT_TEST_COMM="torch", PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=2)
    rel = ((a["data"] - b["data"]).norm() / b["data"].norm()).item()
    assert rel < 1e-6, rel


def test_native_dataparallel_two_devices_equals_averaged_halves():
    """DP over 2 devices == per-shard gradients (BN per shard) summed onto GPU 0 with the full-batch mean."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    X, T = make_batch(2 * B, HW)
    dp = NativeDataParallelTrainer(make_model(seed=0), [0, 1], dtype=torch.bfloat16)
    before = dp.flat.data.clone()
    dp.train_step(X.cuda(0), T.cuda(0))
    torch.cuda.synchronize()
    tr = NativeTrainer(make_model(seed=0), "cuda:0", dtype=torch.bfloat16)
    tr.executor.train_step(X[:B].cuda(), T[:B].cuda(), grad_div=float(2 * B))
    ga = tr.flat.grad.clone()
    tr.executor.train_step(X[B:].cuda(), T[B:].cuda(), grad_div=float(2 * B))
    tr.flat.grad.add_(ga)
    tr.optimizer.step()
    torch.cuda.synchronize()
    d1, d2 = dp.flat.data - before, tr.flat.data - before
    assert ((d1 - d2).norm() / d2.norm()).item() < 1e-3


def test_device_group_broadcast_and_reduce():
    from pytorch_distributed_template_amd.ops import native
    n = torch.cuda.device_count()
    g = native.C.DeviceGroup(list(range(n)))
    ts = [torch.full((1 << 20,), float(i + 1), device=f"cuda:{i}") for i in range(n)]
    g.reduce(ts, 0)
    torch.cuda.synchronize()
    assert torch.all(ts[0] == n * (n + 1) / 2)
    g.broadcast(ts, 0)
    torch.cuda.synchronize()
    for t in ts:
        assert torch.all(t == n * (n + 1) / 2)
