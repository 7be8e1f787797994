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
from test_ddp_numerics_gpu import B, HW, _run_ranks, check_syncbn_fp32_full_batch  # noqa: E402


def test_native_comm_ddp_bit_equals_c10d_ddp(tmp_path):
    """Same buckets, same RCCL, same order: our communicator + C++ bucketer and c10d give identical weights."""
    a = _run_ranks(tmp_path, PDT_TEST_BACKEND="gloo", PDT_TEST_COMM="native", PDT_TEST_STEPS=2)
    b = _run_ranks(tmp_path, PDT_TEST_BACKEND="nccl", PDT_TEST_COMM="torch", PDT_TEST_STEPS=2)
    assert torch.equal(a["data"], b["data"])
    assert torch.equal(a["fbuf"], b["fbuf"])


@pytest.mark.parametrize("syncbn_comm", ["shared", "own"])
def test_native_comm_syncbn_two_gpus(tmp_path, syncbn_comm):
    """SyncBN through the native RCCL communicator on two real devices against the full-batch oracle: in fp32, one
    step, every parameter update within 1e-4 and running statistics within 1e-5 of ONE process running both ranks'
    batches with plain BN (test_ddp_numerics_gpu.check_syncbn_fp32_full_batch) -- with the statistics on the gradient
    buckets' communicator (PDT_SYNCBN_COMM=shared) and on a communicator of their own running concurrently with the
    bucket all-reduces (own, the default since round 6); then the bf16 path against c10d's SyncBN within 1e-6."""
    a = _run_ranks(tmp_path, PDT_TEST_BACKEND="gloo", PDT_TEST_COMM="native", PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=1,
                   PDT_TEST_DTYPE="fp32", PDT_SYNCBN_COMM=syncbn_comm)
    assert a["transport"] == "rccl"
    check_syncbn_fp32_full_batch(a, 2)
    a = _run_ranks(tmp_path, PDT_TEST_BACKEND="gloo", PDT_TEST_COMM="native", PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=2,
                   PDT_SYNCBN_COMM=syncbn_comm)
    b = _run_ranks(tmp_path, PDT_TEST_BACKEND="gloo", PDT_TEST_COMM="torch", PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=2)
    rel = ((a["data"] - b["data"]).norm() / b["data"].norm()).item()
    assert rel < 1e-6, rel


@pytest.mark.parametrize("ndev", [2, 4, 8])
def test_native_dataparallel_fp32_multi_device_equals_oracle(ndev):
    """Native DP in fp32 (the reference's `dataparallel.py:119` precision) over ``ndev`` real devices, 3 steps,
    against the single-executor oracle: without 16-bit chaos the only difference is RCCL's reduce order, so every
    parameter update stays within 1e-5 relative and the running statistics / num_batches_tracked match."""
    if torch.cuda.device_count() < ndev:
        pytest.skip(f"needs {ndev} GPUs")
    from _ddp_common import dp_oracle
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    X, T = make_batch(ndev * B, HW)
    x, t = X.cuda(0), T.cuda(0)
    dp = NativeDataParallelTrainer(make_model(seed=0), list(range(ndev)), dtype=torch.float32)
    before = dp.flat.data.clone()
    mets = torch.stack([dp.train_step(x, t)[1] for _ in range(3)])
    torch.cuda.synchronize()
    tr, omets, _ = dp_oracle(x, t, ndev, 3, dtype=torch.float32)
    bad = []
    for s in tr.flat.slots:
        d1 = (dp.flat.data - before)[s.offset:s.offset + s.numel]
        d2 = (tr.flat.data - before)[s.offset:s.offset + s.numel]
        rel = ((d1 - d2).norm() / d2.norm().clamp_min(1e-12)).item()
        if rel > 1e-5:
            bad.append((s.name, rel))
    assert not bad, bad[:8]
    fb, ofb = dp.buffers[0].fdata, tr.buffers.fdata
    assert ((fb - ofb).norm() / ofb.norm()).item() < 1e-5
    assert torch.equal(dp.buffers[0].idata, tr.buffers.idata)
    assert torch.allclose(mets, omets, rtol=1e-5, atol=1e-6)


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
    """The single-process device group (ncclCommInitAll, grouped calls) with rank-dependent random data: reduce onto
    device 0 equals the host-side sum (fp64 reference, fp32 summation-order tolerance; small integers exactly), and
    broadcast copies device 0's tensor bit for bit -- several tensors per call, sizes not a multiple of anything."""
    from pytorch_distributed_template_amd.ops import native
    n = torch.cuda.device_count()
    g = native.C.DeviceGroup(list(range(n)))
    gen = torch.Generator().manual_seed(5)
    sizes = [(1 << 20) + 3, 4097, 1]
    host = [[torch.randn(sz, generator=gen) * (i + 1) for sz in sizes] for i in range(n)]
    ints = [torch.randint(-1000, 1000, ((1 << 16) + 5,), generator=gen).float() for _ in range(n)]
    for k, sz in enumerate(sizes):
        ts = [host[i][k].to(f"cuda:{i}") for i in range(n)]
        g.reduce(ts, 0)
        torch.cuda.synchronize()
        terms = torch.stack([host[i][k].double() for i in range(n)])
        want, absum = terms.sum(0), terms.abs().sum(0)
        got = ts[0].cpu().double()
        assert ((got - want).abs() <= 1e-6 * absum).all()  # fp32 summation in any order: <= (n - 1) eps sum|x|
        bc = [torch.randn(sz, generator=gen).to(f"cuda:{i}") for i in range(n)]
        src = bc[0].cpu()
        g.broadcast(bc, 0)
        torch.cuda.synchronize()
        for t in bc:
            assert torch.equal(t.cpu(), src)
    ti = [ints[i].to(f"cuda:{i}") for i in range(n)]
    g.reduce(ti, 0)
    torch.cuda.synchronize()
    assert torch.equal(ti[0].cpu(), torch.stack(ints).sum(0))  # integers in fp32: exact in any order


def test_entry_script_rccl_graph_teardown(tmp_path):
    """Communicator lifecycle on two real GPUs (reference teardown `distributed_syncBN_amp.py:236-237`): distributed.py
    at world 2 on the native RCCL communicator with the whole step captured as a HIP graph (its collectives live in
    the graph).  At the end every rank releases its graphs BEFORE ncclCommDestroy (RCCL's destroy waits for every
    graph that references the communicator), the watchdog thread that was running stops, and the job exits 0 well
    inside the time bound instead of hanging at exit."""
    import re
    import subprocess
    root = os.path.dirname(HERE)
    out = str(tmp_path / "output_rccl_teardown")
    env = dict(os.environ, PYTHONUNBUFFERED="1", PDT_COMM_TRACE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc_per_node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29641", "distributed.py", "--outpath", out, "-b", "16", "--comm", "native", "--graph",
           "--dist-timeout", "120", "--synthetic", "--synthetic-train-size", "96", "--synthetic-val-size", "16",
           "--image-size", "64", "--num-classes", "10", "-j", "0", "--epochs", "1", "--exist-policy", "delete",
           "-p", "1"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    for rk in (0, 1):
        assert f"[pdt comm] rank {rk}/2: rccl communicator destroyed" in log, log[-3000:]
        m = re.search(rf"\[pdt comm\] rank {rk}: trainer closed, live watchdogs (\d+) -> (\d+)", log)
        assert m is not None, log[-3000:]
        assert int(m.group(1)) > 0 and int(m.group(2)) == 0, m.group(0)
    assert "communicator aborted" not in log
