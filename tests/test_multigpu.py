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


@pytest.mark.parametrize("ndev", [2, 4])
def test_native_dataparallel_multi_device_equals_oracle(ndev):
    """Native DP over ``ndev`` real devices (RCCL device group), 3 steps + an eval, against the single-executor
    oracle (per-shard BN statistics, gradients summed onto GPU 0, GPU 0's running statistics): bit-identical at 2
    devices (a 2-term sum is exact in any order); at 4 devices RCCL's reduce order is its own and the chaotic 16-bit
    backward amplifies last-bit differences, so one step is compared by its update (relative 1e-3)."""
    if torch.cuda.device_count() < ndev:
        pytest.skip(f"needs {ndev} GPUs")
    from _ddp_common import dp_oracle
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    X, T = make_batch(ndev * B, HW)
    x, t = X.cuda(0), T.cuda(0)
    dp = NativeDataParallelTrainer(make_model(seed=0), list(range(ndev)), dtype=torch.bfloat16)
    steps = 3 if ndev == 2 else 1
    before = dp.flat.data.clone()
    mets = torch.stack([dp.train_step(x, t)[1] for _ in range(steps)])
    logits, _ = dp.eval_step(x, t)
    torch.cuda.synchronize()
    tr, omets, ologits = dp_oracle(x, t, ndev, steps)
    if ndev == 2:
        assert torch.equal(dp.flat.data, tr.flat.data)
        assert torch.equal(dp.buffers[0].fdata, tr.buffers.fdata)
        assert torch.equal(logits, ologits)
    else:
        d1, d2 = dp.flat.data - before, tr.flat.data - before
        assert ((d1 - d2).norm() / d2.norm()).item() < 1e-3
    assert torch.allclose(mets, omets, rtol=1e-4, atol=1e-5)
    assert torch.equal(dp.buffers[0].idata, tr.buffers.idata)


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
