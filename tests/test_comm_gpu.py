"""Native RCCL communicator and C++ gradient bucketer (csrc/comm.cpp) on one GPU.

RCCL refuses two ranks on one device, so multi-rank numerics are covered by the torch.distributed path
(test_distributed_cpu.py, test_training_gpu.py); here the native layer runs as a 1-rank communicator:
collectives must be identities, stream ordering must hold (results read on the compute stream without
host synchronisation), and a training step through the C++ bucketer must equal the default path.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_rccl_single_rank_collectives():
    from pytorch_distributed_template_amd.parallel.comm import NativeComm
    c = NativeComm(torch.device(DEV, 0))
    assert c.world == 1 and c.rank == 0
    x = torch.randn(1 << 20, device=DEV)
    ref = x.clone()
    x.mul_(2.0)  # enqueued on the compute stream; the collective must run after it
    c.all_reduce(x)
    assert torch.equal(x, ref * 2.0)
    y = torch.arange(1000, device=DEV, dtype=torch.int64)
    c.broadcast(y, 0)
    assert torch.equal(y, torch.arange(1000, device=DEV, dtype=torch.int64))
    out = torch.empty(4096, device=DEV, dtype=torch.bfloat16)
    inp = torch.randn(4096, device=DEV).to(torch.bfloat16)
    c.all_gather(inp, out)
    assert torch.equal(out, inp)
    m = torch.tensor([3.0, -1.0], device=DEV)
    c.all_reduce(m, "max")
    assert m.tolist() == [3.0, -1.0]
    c.barrier()
    c.check()


def test_native_bucketer_step_matches_default():
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry

    def one(comm):
        torch.manual_seed(0)
        model = registry.create("resnet18", num_classes=100)
        tr = NativeTrainer(model, DEV, dtype=torch.bfloat16, comm=comm, force_comm=True, bucket_cap_mb=4.0)
        g = torch.Generator(device=DEV).manual_seed(5)
        x = torch.randn(16, 3, 64, 64, device=DEV, generator=g)
        t = torch.randint(0, 100, (16,), device=DEV, generator=g)
        for _ in range(2):
            _, met = tr.train_step(x, t)
        return tr, met

    tn, mn = one("native")
    assert tn.ncomm is not None and len(tn.bucketer.buckets) > 1
    tt, mt = one("torch")
    assert tt.ncomm is None
    assert torch.equal(tn.flat.data, tt.flat.data)
    assert torch.allclose(mn, mt)


def test_bucketer_bf16_gradient_compression():
    """--grad-compress bf16: each bucket is cast to bf16 on the comm stream, all-reduced in bf16 and widened back,
    so at a world of one the fp32 gradient comes back exactly bf16-rounded; a training step runs on it."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    torch.manual_seed(0)
    tr = NativeTrainer(registry.create("resnet18", num_classes=100), DEV, dtype=torch.bfloat16, comm="native",
                       force_comm=True, bucket_cap_mb=4.0, grad_compress="bf16")
    assert tr.bucketer.compress == "bf16" and len(tr.bucketer.buckets) > 1
    g = tr.flat.grad
    g.copy_(torch.randn_like(g) * 1e-2)
    ref = g.clone()
    covered = torch.zeros(g.numel(), dtype=torch.bool, device=DEV)  # buckets skip the flat buffer's alignment pads
    for b in tr.bucketer.buckets:
        covered[b["lo"]:b["hi"]] = True
    ref[covered] = ref[covered].to(torch.bfloat16).float()
    assert not torch.equal(g, ref)
    for pid in range(len(tr.flat.slots)):
        tr.bucketer.grad_ready(pid)
    tr.bucketer.finish()
    torch.cuda.synchronize()
    assert torch.equal(g, ref)
    x = torch.randn(8, 3, 64, 64, device=DEV)
    t = torch.randint(0, 100, (8,), device=DEV)
    _, met = tr.train_step(x, t)
    assert torch.isfinite(met).all() and torch.isfinite(tr.flat.data).all()
    with pytest.raises(ValueError, match="native communicator"):
        NativeTrainer(registry.create("resnet18", num_classes=100), DEV, dtype=torch.bfloat16, comm="torch",
                      grad_compress="bf16")


@pytest.mark.parametrize("comm,sync_bn", [("torch", False), ("native", False), ("native", True)])
def test_graphed_training_step_matches_eager(comm, sync_bn):
    """Whole-step HIP graph replay == eager steps (same data, same updates), including an LR change.  With the
    native communicator (a real RCCL communicator of one rank, watchdog on) the buffer broadcast, gradient
    bucket all-reduces, metric all-reduce and SyncBN statistic all-reduces are captured into the graph too."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry

    def run(graph):
        torch.manual_seed(0)
        kw = dict(comm="native", force_comm=True, comm_timeout_s=120.0, sync_bn=sync_bn) if comm == "native" else {}
        tr = NativeTrainer(registry.create("resnet18", num_classes=100), DEV, dtype=torch.bfloat16, graph=graph,
                           **kw)
        assert tr.use_graph == graph and (tr.ncomm is not None) == (comm == "native")
        g = torch.Generator(device=DEV).manual_seed(3)
        batches = [(torch.randn(8, 3, 64, 64, device=DEV, generator=g),
                    torch.randint(0, 100, (8,), device=DEV, generator=g)) for _ in range(3)]
        mets = []
        for i in range(6):
            if i == 4:
                tr.optimizer.param_groups[0]["lr"] = 0.01
            _, met = tr.train_step(*batches[i % 3])
            mets.append(met.clone())
        torch.cuda.synchronize()
        return tr, torch.stack(mets)

    tg, mg = run(True)
    te, me = run(False)
    assert len(tg._graphs) == 2 and tg.optimizer.step_count == te.optimizer.step_count == 6
    if comm == "native":
        # the watchdog drains every tracked collective (one recorded inside the capture would never complete
        # as an event and would end the process with a false timeout)
        import time
        time.sleep(0.3)
        assert tg.ncomm.comm.pending() == 0
    assert torch.allclose(mg, me, rtol=1e-3, atol=1e-3)
    assert ((tg.flat.data - te.flat.data).norm() / te.flat.data.norm()).item() < 1e-4


def test_device_group_single_process_collectives():
    """Single-process DP collectives (csrc/dp_group.cpp, ncclCommInitAll) on the visible device(s):
    broadcast from the root, in-place reduce-add into the root, all-reduce; ordered on the current
    stream behind earlier compute without host synchronisation."""
    from pytorch_distributed_template_amd.ops import native
    n = torch.cuda.device_count()
    g = native.C.DeviceGroup(list(range(n)))
    assert g.size == n
    xs = []
    for d in range(n):
        with torch.cuda.device(d):
            xs.append(torch.full((1 << 16,), float(d + 1), device=f"cuda:{d}"))
    with torch.cuda.device(0):
        xs[0].mul_(3.0)  # compute-stream work the collective must follow
    g.reduce(xs, 0)
    assert torch.allclose(xs[0], torch.full_like(xs[0], 3.0 + sum(range(2, n + 1))))
    g.broadcast(xs, 0)
    for x in xs:
        assert torch.equal(x.cpu(), xs[0].cpu())
    g.all_reduce(xs)
    assert torch.allclose(xs[0], torch.full_like(xs[0], n * (3.0 + sum(range(2, n + 1)))))


def test_native_comm_over_native_tcp_store():
    """The native communicator rendezvousing through our C++ TCP store instead of c10d's."""
    from pytorch_distributed_template_amd.parallel.comm import NativeComm
    from pytorch_distributed_template_amd.parallel.store import NativeStore
    st = NativeStore("127.0.0.1", 0, 0, 1)
    c = NativeComm(torch.device(DEV, 0), store=st)
    assert c.world == 1 and c.rank == 0
    x = torch.randn(4096, device=DEV)
    ref = x.clone()
    c.all_reduce(x)
    assert torch.equal(x, ref)
    c.barrier()


def test_watchdog_quiet_on_completed_collectives():
    """With a short timeout, collectives that complete never trip the watchdog and its queue drains."""
    import time
    from pytorch_distributed_template_amd.parallel.comm import NativeComm
    c = NativeComm(torch.device(DEV, 0), timeout_s=2.0)
    x = torch.randn(1 << 16, device=DEV)
    for _ in range(20):
        c.all_reduce(x)
    torch.cuda.synchronize()
    assert c.count() == 1
    deadline = time.time() + 5
    while c.comm.pending() and time.time() < deadline:
        time.sleep(0.05)
    assert c.comm.pending() == 0
    time.sleep(2.5)  # past the timeout: nothing pending, nothing fires
    c.destroy()


def test_watchdog_aborts_a_stalled_collective(tmp_path):
    """A collective pending past the timeout aborts the communicator and exits the process non-zero
    (simulated with the test hook: a pending entry that never completes -- no GPU hang involved)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, time, torch; sys.path.insert(0, %r)\n"
            "from pytorch_distributed_template_amd.parallel.comm import NativeComm\n"
            "c = NativeComm(torch.device('cuda', 0), timeout_s=1.0)\n"
            "x = torch.ones(16, device='cuda'); c.all_reduce(x); torch.cuda.synchronize()\n"
            "c.comm.inject_stall(0.0)\n"
            "time.sleep(30)\n"
            "print('NOT ABORTED')\n" % root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 75, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "[pdt comm watchdog]" in r.stderr and "injected stall" in r.stderr
    assert "NOT ABORTED" not in r.stdout


def test_bench_native_comm_single_rank_json():
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "bench.py", "--force-comm", "--batch-per-gpu", "32", "--steps", "2",
                        "--warmup", "1"], cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 1 and rec["config"]["rccl_world"] == 1 and rec["config"]["comm"] == "native"
    assert rec["config"]["params_equal_across_ranks"] and rec["config"]["comm_selftest"]


def test_bench_two_ranks_gloo_rehearsal_json():
    """bench.py --gpus 2 spawns two ranks itself; on a 1-GPU box only as a gloo rehearsal."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [sys.executable, "bench.py", "--gpus", "2", "--batch-per-gpu", "16", "--steps", "2", "--warmup", "1"]
    if torch.cuda.device_count() < 2:
        r = subprocess.run(args, cwd=root, capture_output=True, text=True, timeout=120)
        assert r.returncode != 0 and "needs 2 visible GPUs" in r.stderr
        args += ["--dist-backend", "gloo"]
    r = subprocess.run(args, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 32
    assert rec["config"]["params_equal_across_ranks"] and len(rec["config"]["bucket_sizes_mb"]) > 1
