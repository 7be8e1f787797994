"""Native DataParallel (reference C09, `dataparallel.py:119,211,221`) over several steps, against the single-
executor oracle of ``_ddp_common.dp_oracle``: parameters, running statistics, metrics and evaluation logits must be
BIT-identical.  On one GPU the replicas share cuda:0 (``device_ids=[0, 0]``, fixed-order local collectives), which
exercises every replica-state path (shadow + master-read parameters + BN buffers + derived layouts); the >= 2-GPU
variants run the RCCL device group (tests/test_multigpu.py)."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _ddp_common import dp_oracle, make_batch, make_model  # noqa: E402

B = 32  # node batch: two 16-image shards
HW = 224
STEPS = 3


def _dp_run(device_ids, x, t, steps, graph=None, sharded=False):
    from pytorch_distributed_template_amd.data.loader import ShardedBatch, shard_bounds
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    dp = NativeDataParallelTrainer(make_model(seed=0), device_ids, dtype=torch.bfloat16, graph=graph)
    if sharded:  # the loader's form: shard i already on device i
        bs = shard_bounds(x.shape[0], len(device_ids))
        x = ShardedBatch([x[lo:hi].to(f"cuda:{d}") for (lo, hi), d in zip(bs, device_ids)])
        t = ShardedBatch([t[lo:hi].to(f"cuda:{d}") for (lo, hi), d in zip(bs, device_ids)])
    mets = [dp.train_step(x, t)[1] for _ in range(steps)]
    logits, _ = dp.eval_step(x, t)
    torch.cuda.synchronize()
    return dp, torch.stack(mets), logits


@pytest.mark.parametrize("graph,sharded", [(False, False), (True, False), (False, True)])
def test_dp_shared_device_equals_oracle(graph, sharded):
    X, T = make_batch(B, HW)
    x, t = X.cuda(), T.cuda()
    dp, mets, logits = _dp_run([0, 0], x, t, STEPS, graph=graph, sharded=sharded)
    tr, omets, ologits = dp_oracle(x, t, 2, STEPS)
    assert torch.equal(dp.flat.data, tr.flat.data)
    assert torch.equal(dp.buffers[0].fdata, tr.buffers.fdata)
    assert torch.equal(dp.buffers[0].idata, tr.buffers.idata)
    assert torch.allclose(mets, omets, rtol=1e-6, atol=1e-6)
    assert torch.equal(logits, ologits)
    # every replica ends holding GPU 0's compute state (the round-2 bug: stale BN affine / fc bias on replica 1)
    dp._replicate()
    torch.cuda.synchronize()
    idx = dp.flat.master_read_index().long().cuda()
    assert torch.equal(dp.flats[1].data[idx], dp.flat.data[idx])
    assert torch.equal(dp.flats[1].shadow, dp.flat.shadow)


def test_dp_replica_eval_matches_replica0_after_training():
    """After 3 SGD steps a replica evaluates exactly like replica 0 (same images on both)."""
    X, T = make_batch(16, HW)
    x, t = X.cuda(), T.cuda()
    dp, _, _ = _dp_run([0, 0], torch.cat([x, x]), torch.cat([t, t]), STEPS)
    dp._replicate()
    l0, _ = dp.executors[0].eval_step(x, t)
    l1, _ = dp.executors[1].eval_step(x, t)
    torch.cuda.synchronize()
    assert torch.equal(l0, l1)


def test_dp_resume_refreshes_every_replica():
    """--resume into native DP on shared devices: every replica evaluates with the loaded weights at once."""
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    X, T = make_batch(B, 64)
    x, t = X.cuda(), T.cuda()
    a = NativeDataParallelTrainer(make_model(seed=0), [0, 0], dtype=torch.bfloat16)
    for _ in range(2):
        a.train_step(x, t)
    la, _ = a.eval_step(x, t)
    sd = {k: v.detach().cpu().clone() for k, v in a.model.state_dict().items()}
    b = NativeDataParallelTrainer(make_model(seed=5), [0, 0], dtype=torch.bfloat16)
    b.model.load_state_dict(sd)
    b.on_state_loaded()
    l1, _ = b.executors[1].eval_step(x[16:], t[16:])  # replica 1 directly, before any forward replicated state
    lb, _ = b.eval_step(x, t)
    torch.cuda.synchronize()
    assert torch.equal(la, lb)
    assert torch.equal(l1, la[16:])


def test_dp_runner_sharded_synthetic(tmp_path, monkeypatch):
    """dataparallel.py end to end with two replicas on cuda:0: the loader yields ShardedBatch pairs."""
    from pytorch_distributed_template_amd.engine import runner
    monkeypatch.setenv("PDT_DP_DEVICES", "0,0")
    out = tmp_path / "o"
    rc = runner.main("dp", ["--synthetic", "--synthetic-train-size", "64", "--synthetic-val-size", "32",
                            "--iters-per-epoch", "2", "--epochs", "1", "-b", "32", "--image-size", "64",
                            "--outpath", str(out), "--exist-policy", "delete", "-j", "0"])
    assert rc == 0
    log = (tmp_path / "o_resnet18" / "experiment.log").read_text()
    assert "||==> Val epoch" in log


@pytest.mark.parametrize("device_ids", [[0], [0, 0]])
def test_dp_fp32_eval_equals_executor32(device_ids):
    """dataparallel.py validates the fp32 model (reference `dataparallel.py:243-262`: no autocast anywhere), so native
    DataParallel with eval_fp32 (--eval-precision auto) evaluates each shard on the fp32 kernels over the fp32 master
    after bf16 training steps: its logits equal ResNetExecutor32.eval_step on the same master weights and running
    statistics, shard by shard, bit for bit (one replica, and two replicas sharing cuda:0)."""
    from pytorch_distributed_template_amd.data.loader import shard_bounds
    from pytorch_distributed_template_amd.models.executor32 import ResNetExecutor32
    from pytorch_distributed_template_amd.optim.flat import FlatBuffers, FlatParams
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    X, T = make_batch(B, HW)
    x, t = X.cuda(), T.cuda()
    dp = NativeDataParallelTrainer(make_model(seed=0), device_ids, dtype=torch.bfloat16, eval_fp32=True)
    for _ in range(2):
        dp.train_step(x, t)
    logits, met = dp.eval_step(x, t)
    logits2, _ = dp.eval_step(x, t)  # same weight version: no re-replication, same result
    ref_model = make_model(seed=1)
    ref_model.load_state_dict({k: v.detach().clone() for k, v in dp.model.state_dict().items()})
    flat = FlatParams(ref_model, "cuda:0", None)
    FlatBuffers(ref_model, "cuda:0")
    ex = ResNetExecutor32(ref_model, flat, "cuda:0")
    ref = torch.cat([ex.eval_step(x[lo:hi], t[lo:hi])[0] for lo, hi in shard_bounds(B, len(device_ids))])
    torch.cuda.synchronize()
    assert torch.equal(logits, ref)
    assert torch.equal(logits2, ref)
    # the bf16 evaluation differs (it is not what the reference validates)
    dp16 = NativeDataParallelTrainer(make_model(seed=0), device_ids, dtype=torch.bfloat16)
    for _ in range(2):
        dp16.train_step(x, t)
    assert not torch.equal(dp16.eval_step(x, t)[0], ref)


def test_dp_resnext_default_eval_precision_builds_and_runs():
    """native DataParallel of a grouped-conv model with the default eval precision (fp32 validation
    requested) must build and validate (round 6: the fp32 executor runs grouped convs too, so the fp32 evaluation
    executor is built; a model it cannot run falls back to the compute dtype instead of raising)."""
    import warnings
    from pytorch_distributed_template_amd.models import registry
    from pytorch_distributed_template_amd.models.executor32 import fp32_supported
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    torch.manual_seed(0)
    model = registry.create("resnext50_32x4d")
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        dp = NativeDataParallelTrainer(model, [0, 0], dtype=torch.bfloat16, eval_fp32=True)
    assert (dp._eval32 is not None) == fp32_supported(model)
    x = torch.randn(8, 3, 64, 64, device="cuda")
    t = torch.randint(0, 1000, (8,), device="cuda")
    _, met = dp.train_step(x, t)
    logits, _ = dp.eval_step(x, t)
    torch.cuda.synchronize()
    assert torch.isfinite(met).all() and torch.isfinite(logits.float()).all()
