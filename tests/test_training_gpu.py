"""GPU end-to-end: entry scripts on the native engine, native DataParallel, AMP fp16 loss scaling, and
the native DDP/SyncBN path with two ranks sharing one GPU over gloo (RCCL refuses duplicate GPUs)."""
import os
import re
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--synthetic", "--synthetic-train-size", "1024", "--synthetic-val-size", "256", "--image-size", "64",
          "-j", "0", "--epochs", "2", "--step", "1", "--exist-policy", "delete", "-p", "2", "-b", "128"]


def _run(args, timeout=600, env_extra=None):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.update(env_extra or {})
    r = subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


@pytest.mark.parametrize("script,extra", [("distributed.py", []), ("dataparallel.py", []),
                                          ("distributed_syncBN_amp.py", []),
                                          ("distributed.py", ["--autotune", "--profile"])])
def test_entry_scripts_native_gpu(tmp_path, script, extra):
    out = str(tmp_path / "out")
    _run([script, "--outpath", out] + COMMON + extra)
    log = open(os.path.join(out + "_resnet18", "experiment.log")).read()
    assert "=> engine: native" in log
    losses = [float(x) for x in re.findall(r"\|\|==> Train epoch: \[\d/2\]\tlr=[\d.]+\tce_loss=([\d.]+)", log)]
    assert len(losses) == 2 and all(l == l and l < 20 for l in losses)
    if script == "distributed_syncBN_amp.py":
        assert "compute dtype: float16" in log
    peaks = [float(x) for x in re.findall(r"Peak GPU memory: ([\d.]+) GiB allocated", log)]
    assert len(peaks) == 2 and all(0 < p < 300 for p in peaks)  # per-epoch peak memory (README memory column)
    ck = torch.load(os.path.join(out + "_resnet18", "checkpoint.pth.tar"), map_location="cpu", weights_only=True)
    assert ck["epoch"] == 2 and torch.isfinite(ck["state_dict"]["conv1.weight"]).all()


def test_amp_scaler_backoff_on_overflow():
    """A huge loss scale overflows fp16 gradients: the step is skipped and the scale backs off."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    torch.manual_seed(0)
    tr = NativeTrainer(registry.create("resnet18"), "cuda", dtype=torch.float16, use_amp=True)
    tr.scaler._scale.fill_(2.0 ** 40)
    before = tr.flat.data.clone()
    x = torch.randn(8, 3, 64, 64, device="cuda")
    t = torch.randint(0, 1000, (8,), device="cuda")
    tr.train_step(x, t)
    torch.cuda.synchronize()
    assert torch.equal(before, tr.flat.data)  # skipped
    assert tr.scaler.get_scale() == 2.0 ** 39
    tr.scaler._scale.fill_(1024.0)
    tr.train_step(x, t)
    torch.cuda.synchronize()
    assert not torch.equal(before, tr.flat.data)
    assert torch.isfinite(tr.flat.data).all()


def test_native_dataparallel_single_device_matches_ddp_world1():
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    torch.manual_seed(0)
    m1 = registry.create("resnet18")
    m2 = registry.create("resnet18")
    m2.load_state_dict(m1.state_dict())
    a = NativeTrainer(m1, "cuda", dtype=torch.bfloat16)
    b = NativeDataParallelTrainer(m2, [0], dtype=torch.bfloat16)
    x = torch.randn(16, 3, 64, 64, device="cuda")
    t = torch.randint(0, 1000, (16,), device="cuda")
    for _ in range(2):
        _, ma = a.train_step(x, t)
        _, mb = b.train_step(x, t)
    torch.cuda.synchronize()
    assert torch.allclose(ma, mb, atol=1e-4)
    assert torch.allclose(a.flat.data, b.flat.data, atol=1e-5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_native_ddp_two_ranks_one_gpu_gloo(tmp_path):
    """Bucketed all-reduce + SyncBN + buffer broadcast of the NATIVE executor, 2 ranks on cuda:0 over gloo."""
    script = tmp_path / "ddp2.py"
    script.write_text(r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, %r)
dist.init_process_group("gloo")
rank = dist.get_rank()
from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
from pytorch_distributed_template_amd.models import registry
torch.manual_seed(rank)  # different init: the constructor broadcast must equalise it
tr = NativeTrainer(registry.create("resnet18"), "cuda:0", dtype=torch.bfloat16, sync_bn=True,
                   bucket_cap_mb=4, first_bucket_mb=1)
g = torch.Generator(device="cuda").manual_seed(10 + rank)
x = torch.randn(8, 3, 64, 64, device="cuda", generator=g)
t = torch.randint(0, 1000, (8,), device="cuda", generator=g)
for _ in range(2):
    _, met = tr.train_step(x, t)
torch.cuda.synchronize()
s = torch.stack([tr.flat.data.double().sum(), tr.buffers.fdata.double().sum(), met[0].double()]).cpu()
out = [torch.zeros(3, dtype=torch.float64) for _ in range(2)]
dist.all_gather(out, s)
if rank == 0:
    print("SUMS", out[0].tolist(), out[1].tolist(), len(tr.bucketer.buckets), flush=True)
    assert torch.allclose(out[0], out[1], rtol=1e-9, atol=1e-6), out
dist.destroy_process_group()
''' % ROOT)
    r = _run(["-m", "pytorch_distributed_template_amd.launch", "--nproc_per_node=2", f"--master_port={_free_port()}",
              "--no_local_rank", str(script)], timeout=600)
    assert "SUMS" in r.stdout


@pytest.mark.parametrize("arch", ["regnet_y_400mf", "convnext_tiny", "swin_t", "swin_v2_t", "efficientnet_v2_s",
                                  "vit_b_32", "maxvit_t"])
def test_modern_families_torch_engine_gpu(arch):
    """RegNet / ConvNeXt / Swin / EfficientNetV2 / ViT train (bf16 autocast, SGD) and evaluate on cuda:0."""
    from pytorch_distributed_template_amd.engine.torch_trainer import TorchTrainer
    from pytorch_distributed_template_amd.models import registry
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    kw = {"vit_b_32": {"image_size": 64}, "maxvit_t": {"input_size": (64, 64), "partition_size": 2}}.get(arch, {})
    tr = TorchTrainer(registry.create(arch, num_classes=10, **kw), dev, dtype=torch.bfloat16, lr=0.01)
    x = torch.randn(8, 3, 64, 64, device=dev)
    t = torch.randint(0, 10, (8,), device=dev)
    for _ in range(2):
        _, met = tr.train_step(x, t)
    assert torch.isfinite(torch.as_tensor(met[0])).all()
    out = tr.eval_step(x, t)
    torch.cuda.synchronize()
    assert out is not None


def test_native_dataparallel_graph_replay_matches_eager():
    """Per-replica HIP-graph replay (the multi-device default) == eager replicas, bit for bit (one device
    forced into graph mode; 2 eager warm-up steps, then capture + replays)."""
    from pytorch_distributed_template_amd.models import registry
    from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(32, 3, 64, 64, generator=g) for _ in range(5)]
    ts = [torch.randint(0, 1000, (32,), generator=g) for _ in range(5)]
    out = []
    for graph in (False, True):
        torch.manual_seed(0)
        tr = NativeDataParallelTrainer(registry.create("resnet18"), [0], dtype=torch.bfloat16, graph=graph)
        mets = []
        for x, t in zip(xs, ts):
            _, m = tr.train_step(x.cuda(), t.cuda())
            mets.append(m.clone())
        torch.cuda.synchronize()
        out.append((tr.flat.data.clone(), tr.buffers[0].fdata.clone(), torch.stack(mets)))
        if graph:
            assert len(tr._graphs) == 1
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][2], out[1][2])
