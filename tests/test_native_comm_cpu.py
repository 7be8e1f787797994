"""The native collective layer's multi-rank C++ logic on the CPU (csrc/comm.cpp over the host shared-memory
transport, csrc/shm_group.h): the same Communicator and Bucketer classes the GPU path runs over RCCL, here at
world 2 and 4 with host tensors (SURVEY §4 layer 2; reference `start.sh:3-4`, `distributed.py:124,144`).

* raw collectives (all_reduce sum/max over f32 / f64 / bf16 / i64 with payloads larger than a slot, broadcast,
  all_gather, barrier) against closed forms;
* the C++ Bucketer: every bucket all-reduced once per step, in production order, launched the moment its last
  parameter is ready, leftovers launched by finish(), results the rank-order sum;
* DDP through the runner's CPU path with ``--comm native`` (the C++ bucketer behind autograd hooks) bit-equal to
  c10d/gloo at world 2 and replicas bit-identical at world 4;
* failure handling: a rank that dies makes its peers' next collective raise within the timeout; an abort reaches
  every rank;
* the shared-memory group itself under AddressSanitizer + UBSan and ThreadSanitizer (csrc/tests/shm_stress.cpp).
"""
import os
import shutil
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


def _spawn(fn, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, v = q.get(timeout=240)
        res[r] = v
    for p in ps:
        p.join(timeout=60)
    return res, [p.exitcode for p in ps]


def _collectives_worker(rank, world, port, q):
    _init(rank, world, port)
    os.environ["PDT_HOST_COMM_SLOT_MB"] = "1"
    from pytorch_distributed_template_amd.parallel.comm import NativeComm
    c = NativeComm(torch.device("cpu"), timeout_s=60.0)
    out = {"transport": c.transport, "world": c.world, "count": c.count()}
    x = torch.full((700_000,), float(rank + 1))  # 2.8 MB > 1 MB slot: chunked
    c.all_reduce(x)
    out["sum_ok"] = bool(torch.all(x == world * (world + 1) / 2))
    d = torch.arange(1000, dtype=torch.float64) + 1000 * rank
    c.all_reduce(d, "max")
    out["max_ok"] = bool(torch.equal(d, torch.arange(1000, dtype=torch.float64) + 1000 * (world - 1)))
    h = torch.full((4096,), 0.5 * (rank + 1), dtype=torch.bfloat16)
    c.all_reduce(h)
    out["bf16_ok"] = bool(torch.all(h.float() == 0.5 * world * (world + 1) / 2))
    i = torch.full((3,), 10 ** 12 + rank, dtype=torch.int64)
    c.all_reduce(i, "min")
    out["i64_ok"] = bool(torch.all(i == 10 ** 12))
    b = torch.full((5000,), -1.0) if rank != 1 else torch.arange(5000.0)
    c.broadcast(b, 1)
    out["bcast_ok"] = bool(torch.equal(b, torch.arange(5000.0)))
    g_in = torch.full((300,), float(rank))
    g_out = torch.empty(300 * world)
    c.all_gather(g_in, g_out)
    out["gather_ok"] = bool(torch.equal(g_out, torch.arange(world, dtype=torch.float32).repeat_interleave(300)))
    c.barrier()
    c.check()
    c.destroy()
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_host_transport_collectives(world):
    res, codes = _spawn(_collectives_worker, world)
    assert codes == [0] * world
    for r in range(world):
        o = res[r]
        assert o["transport"] == "host" and o["world"] == world and o["count"] == world
        assert all(o[k] for k in ("sum_ok", "max_ok", "bf16_ok", "i64_ok", "bcast_ok", "gather_ok")), o


def _bucketer_worker(rank, world, port, q):
    _init(rank, world, port)
    from pytorch_distributed_template_amd.ops import native
    from pytorch_distributed_template_amd.parallel.comm import NativeComm
    c = NativeComm(torch.device("cpu"), timeout_s=60.0)
    # 6 parameters in 3 buckets over a flat buffer of 64 elements (slots 0..5 at offsets 0, 8, 16, 24, 40, 48)
    offs, sizes = [0, 8, 16, 24, 40, 48], [8, 8, 8, 16, 8, 16]
    param_bucket = [2, 2, 1, 1, 0, 0]  # buckets in production order: params 5, 4 -> bucket 0, ...
    lo, hi = [40, 16, 0], [64, 40, 16]
    grad = torch.zeros(64)
    bk = native.C.Bucketer(c.comm, grad, lo, hi, param_bucket, 0)
    out = {"launched": [], "orders": [], "grads": []}
    for step in range(3):
        for p, (o, n) in enumerate(zip(offs, sizes)):
            grad[o:o + n] = (rank + 1) * (p + 1) + step
        # backward produces parameters 5, 4, 3, 2 (bucket 0 then 1); parameters 1, 0 "unused" -> finish()
        for p in (5, 4, 3, 2):
            bk.ready(p)
            out["launched"].append(bk.launched())
        bk.finish()
        out["orders"].append(list(bk.last_launch_order()))
        out["grads"].append(grad.numpy().copy())  # numpy: tensors would travel as shared memory of a dying process
    # rank-dependent ready order: odd ranks finish bucket 1 before bucket 0.  Launches stay in bucket-index order
    # (bucket 1 is held until bucket 0 completes), so every rank issues the same collective sequence
    out["skew_launched"] = []
    for p, (o, n) in enumerate(zip(offs, sizes)):
        grad[o:o + n] = (rank + 1) * (p + 1) + 3
    for p in ((3, 2, 5, 4) if rank % 2 else (5, 4, 3, 2)):
        bk.ready(p)
        out["skew_launched"].append(bk.launched())
    bk.finish()
    out["skew_order"] = list(bk.last_launch_order())
    out["skew_grad"] = grad.numpy().copy()
    try:
        bk.ready(5)
        bk.ready(4)  # bucket 0 complete (launched on every rank)
        bk.ready(5)
        out["double_ready"] = "accepted"
    except RuntimeError as e:
        out["double_ready"] = str(e)
    c.destroy()
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_cpp_bucketer_multi_rank(world):
    res, codes = _spawn(_bucketer_worker, world)
    assert codes == [0] * world
    tri = world * (world + 1) / 2
    offs, sizes = [0, 8, 16, 24, 40, 48], [8, 8, 8, 16, 8, 16]
    for r in range(world):
        o = res[r]
        # bucket 0 launches when param 4 (its last) is ready, bucket 1 when param 2 is; bucket 2 only in finish()
        assert o["launched"] == [0, 1, 1, 2] * 3
        assert o["orders"] == [[0, 1, 2]] * 3
        for step, g in enumerate(o["grads"]):
            want = torch.zeros(64)
            for p, (off, n) in enumerate(zip(offs, sizes)):
                want[off:off + n] = sum((q + 1) * (p + 1) + step for q in range(world))
            assert torch.equal(torch.from_numpy(g), want), (r, step)
        assert "reported ready twice" in o["double_ready"]
        assert o["skew_order"] == [0, 1, 2]
        assert o["skew_launched"] == ([0, 0, 0, 2] if r % 2 else [0, 1, 1, 2])
        want = torch.zeros(64)
        for p, (off, n) in enumerate(zip(offs, sizes)):
            want[off:off + n] = sum((q + 1) * (p + 1) + 3 for q in range(world))
        assert torch.equal(torch.from_numpy(o["skew_grad"]), want), r
    assert all((res[0]["grads"][-1] == res[r]["grads"][-1]).all() for r in range(world))
    assert tri > 0


def _ddp_worker(rank, world, port, q, comm):
    _init(rank, world, port)
    from pytorch_distributed_template_amd.engine.torch_trainer import TorchTrainer
    from pytorch_distributed_template_amd.models import registry
    torch.manual_seed(100 + rank)  # different init per rank: the constructor broadcast must equalise them
    model = registry.create("resnet18", num_classes=10)
    tr = TorchTrainer(model, "cpu", lr=0.1, momentum=0.9, weight_decay=1e-4, bucket_cap_mb=2.0,
                      first_bucket_mb=0.5, comm=comm, comm_timeout_s=120.0)
    g = torch.Generator().manual_seed(42)
    x = torch.randn(4 * world, 3, 32, 32, generator=g)
    t = torch.randint(0, 10, (4 * world,), generator=g)
    mets = []
    for _ in range(2):
        _, met = tr.train_step(x[rank * 4:(rank + 1) * 4], t[rank * 4:(rank + 1) * 4])
        mets.append(met.clone())
    kind = type(tr.bucketer).__name__
    q.put((rank, (tr.flat.data.numpy().copy(), tr.buffers.fdata.numpy().copy(), torch.stack(mets).numpy().copy(),
                  kind, len(tr.bucketer.buckets))))
    if tr.ncomm is not None:
        tr.ncomm.destroy()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ddp_native_comm_cpu(world):
    nat, codes = _spawn(_ddp_worker, world, "native")
    nat = {r: [torch.from_numpy(v) if hasattr(v, "dtype") else v for v in o] for r, o in nat.items()}
    assert codes == [0] * world
    assert nat[0][3] == "NativeBucketer" and nat[0][4] > 1
    for r in range(1, world):  # DDP invariant: parameters bit-identical (buffers are synced at forward START, so
        assert torch.equal(nat[r][0], nat[0][0])  # after the last step each rank holds its own running-stat update)
    ref, codes = _spawn(_ddp_worker, world, "torch")
    ref = {r: [torch.from_numpy(v) if hasattr(v, "dtype") else v for v in o] for r, o in ref.items()}
    assert codes == [0] * world and ref[0][3] == "GradBucketer"
    if world == 2:  # two fp32 addends: the sum is exact in any order -> bit-identical to gloo
        assert torch.equal(nat[0][0], ref[0][0])
        assert torch.equal(nat[0][1], ref[0][1])
    else:
        rel = ((nat[0][0] - ref[0][0]).norm() / ref[0][0].norm()).item()
        assert rel < 1e-3, rel  # rank-order vs gloo-order fp32 sums, amplified by BN backward at batch 4
    assert torch.allclose(nat[0][2], ref[0][2], rtol=1e-5, atol=1e-6)


def _dead_peer_worker(rank, world, port, q):
    _init(rank, world, port)
    from pytorch_distributed_template_amd.parallel.comm import NativeComm
    c = NativeComm(torch.device("cpu"), timeout_s=3.0)
    x = torch.ones(10)
    c.all_reduce(x)
    if rank == 1:
        q.put((rank, "exiting"))
        q.close()
        q.join_thread()  # flush the queue's feeder thread before dying
        os._exit(0)  # a crashed rank: no teardown
    try:
        c.all_reduce(x)
        msg = "returned"
    except RuntimeError as e:
        msg = str(e)
    q.put((rank, msg))
    q.close()
    q.join_thread()
    os._exit(0)


def test_host_transport_dead_peer_times_out():
    res, codes = _spawn(_dead_peer_worker, 2)
    assert "peer dead or hung" in res[0], res[0]


def _abort_worker(rank, world, port, q):
    _init(rank, world, port)
    from pytorch_distributed_template_amd.parallel.comm import NativeComm
    c = NativeComm(torch.device("cpu"), timeout_s=60.0)
    c.barrier()
    if rank == 0:
        c.abort()
        q.put((rank, "aborted"))
        q.close()
        q.join_thread()
        os._exit(0)
    try:
        c.barrier()
        msg = "returned"
    except RuntimeError as e:
        msg = str(e)
    q.put((rank, msg))
    q.close()
    q.join_thread()
    os._exit(0)


def test_host_transport_abort_reaches_every_rank():
    res, _ = _spawn(_abort_worker, 3)
    assert all("aborted the group" in res[r] for r in (1, 2)), res


SRC = os.path.join(ROOT, "csrc", "tests", "shm_stress.cpp")
GXX = shutil.which("g++")


def _stress(tmp_path, flags, env):
    exe = str(tmp_path / "shm_stress")
    b = subprocess.run([GXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", *flags,
                        f"-I{os.path.join(ROOT, 'csrc')}", SRC, "-o", exe], capture_output=True, text=True)
    if b.returncode != 0 and "cannot find" in b.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {b.stderr[-300:]}")
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([exe, "4", "15"], capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "0 errors" in out
    return out


@pytest.mark.skipif(GXX is None, reason="needs g++")
def test_shm_group_under_asan_ubsan(tmp_path):
    out = _stress(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                  {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "AddressSanitizer" not in out and "runtime error" not in out


@pytest.mark.skipif(GXX is None, reason="needs g++")
def test_shm_group_under_tsan(tmp_path):
    out = _stress(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
    assert "ThreadSanitizer" not in out
