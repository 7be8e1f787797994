"""Native-executor DDP and SyncBN numerics at world = 2, at the real 224x224 geometry (so the specialised
layer1 / stem / ping-pong kernels run), rehearsed on ONE GPU: two ranks share cuda:0 over gloo (RCCL refuses
duplicate GPUs).  Each 2-rank result is compared with a single-process oracle on the same kernels:

* DDP (2 x B/2, per-rank BN)  ==  one process computing each half's gradient and averaging them
  (the upstream DDP contract, `distributed.py:144`);
* SyncBN DDP (2 x B/2)        ==  one process running the full batch B with plain BN
  (SyncBN's contract, `distributed_syncBN_amp.py:142-147`; upstream semantics SURVEY §3.5).

Parameter UPDATES (after - before) are compared per parameter, so a wrong gradient scale on any tensor
(e.g. BN gamma/beta gradients world x too large) fails the test rather than hiding in a sum.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _ddp_common import make_batch, make_model  # noqa: E402

B = 16  # per rank
HW = 224


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(tmp_path, nproc=2, **env):
    out = str(tmp_path / "rank0.pt")
    e = dict(os.environ, PYTHONUNBUFFERED="1", PDT_TEST_OUT=out, PDT_TEST_B=str(B), PDT_TEST_HW=str(HW))
    e.update({k: str(v) for k, v in env.items()})
    r = subprocess.run([sys.executable, "-m", "pytorch_distributed_template_amd.launch", f"--nproc_per_node={nproc}",
                        f"--master_port={_free_port()}", "--no_local_rank", os.path.join(HERE, "_native_ddp_worker.py")],
                       cwd=ROOT, env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return torch.load(out, weights_only=True)


def _single(steps_fn, dtype=torch.bfloat16):
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    model = make_model(seed=0)
    tr = NativeTrainer(model, "cuda:0", dtype=dtype)
    before = tr.flat.data.clone()
    steps_fn(tr)
    torch.cuda.synchronize()
    return tr, before


def _compare_updates(tr, before, data, per_tensor_tol, total_tol):
    before = before.cpu()
    ours = data - before
    want = tr.flat.data.cpu() - before
    bad = []
    for s in tr.flat.slots:
        a = ours[s.offset:s.offset + s.numel]
        b = want[s.offset:s.offset + s.numel]
        rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        if rel > per_tensor_tol:
            bad.append((s.name, round(rel, 4), round(b.norm().item(), 6), round(a.norm().item(), 6)))
    total = ((ours - want).norm() / want.norm()).item()
    assert not bad, bad[:8]
    assert total < total_tol, total


@pytest.mark.parametrize("comm,nproc", [("torch", 2), ("native", 2), ("native", 4)])
def test_native_ddp_equals_averaged_half_batches(tmp_path, comm, nproc):
    """DDP at world ``nproc`` == one process averaging the ranks' gradients, bit for bit.  ``native`` runs this
    framework's C++ communicator + bucketer (ranks share cuda:0, so it selects the host shared-memory transport,
    which sums in rank order -- the order the oracle accumulates in)."""
    res = _run_ranks(tmp_path, nproc=nproc, PDT_TEST_SYNCBN=0, PDT_TEST_STEPS=1, PDT_TEST_COMM=comm)
    if comm == "native":
        assert res["transport"] == "host" and res["bucketer"] == "NativeBucketer"
    X, T = make_batch(nproc * B, HW)
    box = {}

    def steps(tr):
        acc = None
        for r in range(nproc):
            _, m = tr.executor.train_step(X[r * B:(r + 1) * B].cuda(), T[r * B:(r + 1) * B].cuda(), grad_div=float(B))
            if r == 0:
                box["fbuf"] = tr.buffers.fdata.clone()  # rank 0's running stats come from its own batch only
                acc = tr.flat.grad.clone()
                box["met"] = m.clone()
            else:
                acc.add_(tr.flat.grad)
                box["met"] = box["met"] + m
        tr.flat.grad.copy_(acc)
        tr.optimizer.step(grad_scale=1.0 / nproc)
        box["met"] = box["met"] / nproc

    tr, before = _single(steps)
    # the statistics path is deterministic (per-block partial rows + fixed-order reduction, conv_fwd.h) and the
    # all-reduce sums in the oracle's order (two addends: any order): gradients and the update are BIT-identical
    grad = tr.flat.grad.cpu()
    bad = [s.name for s in tr.flat.slots
           if not torch.equal(res["grad"][s.offset:s.offset + s.numel], grad[s.offset:s.offset + s.numel])]
    assert not bad, bad[:8]
    assert torch.equal(res["data"], tr.flat.data.cpu())
    _compare_updates(tr, before, res["data"], per_tensor_tol=2e-3, total_tol=5e-4)
    assert torch.equal(res["fbuf"], box["fbuf"].cpu())
    assert torch.allclose(res["met"][0], box["met"].cpu(), rtol=1e-4, atol=1e-5)


def _update_errors(tr, before, a, b):
    """Per-parameter relative error of update (a - before) against update (b - before)."""
    out = {}
    for s in tr.flat.slots:
        da = (a - before)[s.offset:s.offset + s.numel]
        db = (b - before)[s.offset:s.offset + s.numel]
        out[s.name] = ((da - db).norm() / db.norm().clamp_min(1e-12)).item()
    return out


@pytest.mark.parametrize("nproc", [2, 4])
def test_native_syncbn_fp32_equals_full_batch(tmp_path, nproc):
    """SyncBN correctness without 16-bit chaos: in fp32 (the reference's `distributed.py` precision, exact-fp32
    MFMA kernels) SyncBN DDP over ``nproc`` ranks x B (the native communicator: ranks share cuda:0, host transport)
    must equal ONE process running the full batch nproc x B with plain BN after one step -- every parameter's
    update within max(1e-4, 3 x ITS OWN reorder floor: the same full-batch step with the ranks' slices rotated, or
    every image permuted),
    running mean / var within 1e-5, num_batches_tracked exact, loss / accuracy within 1e-5.  A count, eps,
    variance-bias or gradient-scale error in the native SyncBN path is orders of magnitude larger
    (`distributed_syncBN_amp.py:142-147`; upstream semantics SURVEY §3.5)."""
    res = _run_ranks(tmp_path, nproc=nproc, PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=1, PDT_TEST_COMM="native",
                     PDT_TEST_DTYPE="fp32")
    assert res["transport"] == "host"
    check_syncbn_fp32_full_batch(res, nproc)


def check_syncbn_fp32_full_batch(res, nproc):
    """The fp32 SyncBN contract (see test_native_syncbn_fp32_equals_full_batch) for rank 0's saved state ``res``
    after one step at world ``nproc``; also used by the >= 2-GPU tests (tests/test_multigpu.py)."""
    X, T = make_batch(nproc * B, HW)
    box = {}

    def run_on(x, t, key):
        def run(tr):
            _, m = tr.train_step(x.cuda(), t.cuda())
            box[key] = m.clone()
        return run

    tr, before = _single(run_on(X, T, "met"), dtype=torch.float32)
    before, full = before.cpu(), tr.flat.data.cpu()
    # reorder floor: the same full batch with the ranks' slices rotated -- mathematically the identical step, so its
    # difference is pure fp32 summation order, amplified through the random-init network's backward chain (a ReLU
    # flip of a near-zero pre-activation moves whole blocks' gradients, test_fp32_gpu.py); a SyncBN count, eps,
    # variance-bias or gradient-scale error is far above it
    tr2, _ = _single(run_on(torch.roll(X, B, 0), torch.roll(T, B, 0), "met2"), dtype=torch.float32)
    floor = _update_errors(tr, before, tr2.flat.data.cpu(), full)
    # a second reorder sample (every image permuted) so each parameter's own floor is not one lucky draw
    perm = torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(11))
    tr3, _ = _single(run_on(X[perm], T[perm], "met3"), dtype=torch.float32)
    floor3 = _update_errors(tr, before, tr3.flat.data.cpu(), full)
    floor = {k: max(v, floor3[k]) for k, v in floor.items()}
    e = _update_errors(tr, before, res["data"], full)
    # the classifier's update depends on the forward (SyncBN statistics, counts, eps, variance bias) and the loss
    # gradient only -- no backward ReLU decision that reordering could flip -- so it is held to the plain 1e-4 bound.
    # (Already the last block's conv2 / bn2 see ~1e-3 at W = 4: one flipped block-output ReLU mask among the 32 x 49
    # positions per channel of layer4 moves those sums by ~1/1568 -- measured; hence the reorder floor below.)
    strict = [k for k in e if k.startswith("fc.")]
    assert len(strict) == 2, strict
    bad = [(k, e[k]) for k in strict if e[k] > 1e-4]
    assert not bad, bad
    # each parameter against its OWN reorder floor (one noisy layer must not widen every other layer's bound)
    bad = [(k, v, floor[k]) for k, v in e.items() if v > max(1e-4, 3 * floor[k])]
    assert not bad, sorted(bad, key=lambda kv: -kv[1])[:8]
    assert torch.allclose(box["met2"], box["met"], rtol=1e-5, atol=1e-6)
    fb = tr.buffers.fdata.cpu()
    # every running mean / var element within 1e-5 relative (plus 1e-7 absolute for means that are ~0)
    rs_err = ((res["fbuf"] - fb).abs() - 1e-5 * fb.abs()).max().item()
    assert ((res["fbuf"] - fb).norm() / fb.norm()).item() < 1e-5 and rs_err < 1e-7, rs_err
    assert torch.equal(res["ibuf"], tr.buffers.idata.cpu())  # num_batches_tracked
    assert torch.allclose(res["met"][0], box["met"].cpu(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("steps,comm", [(1, "torch"), (1, "native"), (2, "torch"), (2, "native")])
def test_native_syncbn_equals_full_batch(tmp_path, steps, comm):
    """A random-init ResNet's gradient is chaotic in 16-bit arithmetic: nudging the INPUT by one part in 1e6
    already moves the parameter updates by 10-60 % (the "floor", measured here).  SyncBN(2 x B/2) must
    agree with the full batch within that floor, and far better than plain DDP(2 x B/2), whose per-rank
    BN statistics genuinely differ; a scale error on any tensor (e.g. gamma/beta gradients world x) is
    >= 100 % and fails.  Running statistics, num_batches_tracked and the loss must match closely.
    One step: the original strict bounds (better than DDP everywhere, fc within 2e-2 / 1e-3, running statistics
    within 1e-3); two steps: bounds relative to the measured floor (the second step sees the chaotic first update).
    The chaos-free check of the same path is test_native_syncbn_fp32_equals_full_batch."""
    res = _run_ranks(tmp_path, PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=steps, PDT_TEST_COMM=comm)
    nosync = _run_ranks(tmp_path, PDT_TEST_SYNCBN=0, PDT_TEST_STEPS=steps, PDT_TEST_COMM=comm)["data"]
    X, T = make_batch(2 * B, HW)
    x, t = X.cuda(), T.cuda()
    mets = []

    def run(tr, xx, keep):
        for _ in range(steps):
            _, m = tr.train_step(xx, t)
            if keep:
                mets.append(m.clone())

    tr, before = _single(lambda tr: run(tr, x, True))
    floor_tr, _ = _single(lambda tr: run(tr, x * (1 + 1e-6), False))
    before, full = before.cpu(), tr.flat.data.cpu()
    e_sync = _update_errors(tr, before, res["data"], full)
    e_nosync = _update_errors(tr, before, nosync, full)
    e_floor = _update_errors(tr, before, floor_tr.flat.data.cpu(), full)
    # "better than plain DDP" is only testable where the input-noise floor is well below the DDP error: a parameter
    # whose floor is itself ~ the DDP error (e.g. 0.54 vs 0.58) is noise-dominated, and only the floor bound applies
    strict = steps == 1
    bad = [(k, round(e_sync[k], 4), round(e_floor[k], 4), round(e_nosync[k], 4)) for k in e_sync
           if e_sync[k] > max(1.5 * e_floor[k], 0.02) or
           (e_nosync[k] > 0.05 and (strict or e_floor[k] < 0.5 * e_nosync[k]) and e_sync[k] > 0.75 * e_nosync[k])]
    assert not bad, bad[:8]
    fb = tr.buffers.fdata.cpu()
    fb_err = ((res["fbuf"] - fb).norm() / fb.norm()).item()
    if strict:
        assert e_sync["fc.weight"] < 0.02 and e_sync["fc.bias"] < 1e-3, (e_sync["fc.weight"], e_sync["fc.bias"])
        assert fb_err < 1e-3, fb_err  # running mean / var (unbiased, global count)
    else:
        # the fc layer sees the chaos only through its input features: its own measured floor widens the bound
        assert e_sync["fc.weight"] < max(0.02, 2 * e_floor["fc.weight"]), (e_sync["fc.weight"], e_floor["fc.weight"])
        assert e_sync["fc.bias"] < max(1e-3, 2 * e_floor["fc.bias"]), (e_sync["fc.bias"], e_floor["fc.bias"])
        # running statistics after step 1 see the chaotic update: bounded by the floor too
        fb_floor = ((floor_tr.buffers.fdata.cpu() - fb).norm() / fb.norm()).item()
        assert fb_err < max(1e-3, 2 * fb_floor), (fb_err, fb_floor)
    assert torch.equal(res["ibuf"], tr.buffers.idata.cpu())  # num_batches_tracked
    assert torch.allclose(res["met"], torch.stack(mets).cpu(), rtol=2e-3, atol=2e-3)


def test_native_dp_state_reload_refreshes_derived_layouts():
    """--resume into the native DataParallel trainer: the kernels' derived weight layouts follow the loaded
    weights (evaluation logits equal the saving trainer's)."""
    from pytorch_distributed_template_amd.models import registry
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    torch.manual_seed(0)
    a = NativeDataParallelTrainer(registry.create("resnet18"), [0], dtype=torch.bfloat16)
    X, T = make_batch(16, 64)
    x, t = X.cuda(), T.cuda()
    a.train_step(x, t)
    assert int(a.buffers[0].idata[0].item()) == 1  # num_batches_tracked advances like nn.DataParallel
    la, _ = a.eval_step(x, t)
    sd = {k: v.detach().cpu().clone() for k, v in a.model.state_dict().items()}
    torch.manual_seed(1)
    b = NativeDataParallelTrainer(registry.create("resnet18"), [0], dtype=torch.bfloat16)
    b.model.load_state_dict(sd)
    b.on_state_loaded()
    lb, _ = b.eval_step(x, t)
    torch.cuda.synchronize()
    assert torch.equal(la, lb)


def test_seeded_training_is_bitwise_repeatable():
    """Two identically seeded trainers on identical data end bit-identical after three steps (224 px)."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    X, T = make_batch(B, HW)
    x, t = X.cuda(), T.cuda()
    outs = []
    for _ in range(2):
        tr = NativeTrainer(make_model(seed=0), "cuda:0", dtype=torch.bfloat16)
        for _ in range(3):
            tr.train_step(x, t)
        torch.cuda.synchronize()
        outs.append((tr.flat.data.clone(), tr.buffers.fdata.clone()))
        del tr
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
