"""End-to-end runs of the three entry scripts on CPU (synthetic data, tiny images): output layout,
log formats, TensorBoard tags, checkpoint schema, resume and evaluate-only mode."""
import glob
import os
import re
import subprocess
import sys

import pytest
import torch

from pytorch_distributed_template_amd.utils.tensorboard import read_scalars

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--synthetic", "--synthetic-train-size", "24", "--synthetic-val-size", "8", "--image-size", "32",
          "--num-classes", "10", "-j", "0", "--epochs", "2", "--step", "1", "--exist-policy", "delete", "-p", "1"]


def _run(args, timeout=600):
    env = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


def _check_outdir(d, logger_line_prefix="Train epoch"):
    files = os.listdir(d)
    assert "experiment.log" in files and "settings.log" in files
    assert "checkpoint.pth.tar" in files
    log = open(os.path.join(d, "experiment.log")).read()
    # model_best is written only when val top-1 strictly improves on 0 (reference `distributed.py:201`);
    # a random tiny model on 8 synthetic images can stay at 0
    best = max(float(v) for v in re.findall(r"best_acc1=(\d+\.\d+)", log))
    assert ("model_best.pth.tar" in files) == (best > 0)
    assert re.search(r"Train epoch: \[0/2\]\[0/\d+\]\tlr=0\.100000\tce_loss=\d+\.\d{4}\ttop1_acc=\d\.\d{4}\t"
                     r"data_time=\s*\d+\.\d{3}s\tbatch_time=\s*\d+\.\d{3}s", log)
    assert re.search(r"\|\|==> Train epoch: \[1/2\]\tlr=0\.010000\tce_loss=", log)
    # the loss value itself may be nan: a random tiny model after two lr=0.1 steps on 4 images per rank can
    # blow up its eval-mode BN running statistics; the log FORMAT is what is checked here
    assert re.search(r"Val epoch: \[0/2\]\[0/\d+\]\tce_loss=(\d+\.\d{4}|nan|inf)\ttop1_acc=\d\.\d{4}\tbatch_time=", log)
    assert re.search(r"\|\|==> Epoch=\[1/2\]\tbest_acc1=\d\.\d{4}\tbest_acc1_index=\d\ttime_cost=\d+\.\d{4}s", log)
    assert re.search(r"\|\|==> total_time_cost=\d+\.\d{4}s", log)
    assert "lr_scheduler: SGD MultiStepLR !!!" in log and "=> creating model: resnet18" in log
    ev = glob.glob(os.path.join(d, "events.out.tfevents.*"))
    assert len(ev) == 1
    tags = {t for t, _, _ in read_scalars(ev[0])}
    assert tags == {"lr", "Train_ce_loss", "Train_top1_accuracy", "Val_ce_loss", "Val_top1_accuracy"}
    ck = torch.load(os.path.join(d, "checkpoint.pth.tar"), map_location="cpu", weights_only=True)
    assert {"epoch", "arch", "state_dict", "best_acc1"} <= set(ck)
    assert ck["epoch"] == 2 and ck["arch"] == "resnet18" and "fc.weight" in ck["state_dict"]
    assert ck["state_dict"]["fc.weight"].shape == (10, 512)
    return log, ck


def test_dataparallel_cpu(tmp_path):
    out = str(tmp_path / "output")
    _run(["dataparallel.py", "--outpath", out, "-b", "8"] + COMMON)
    log, _ = _check_outdir(out + "_resnet18")
    assert "DataParallel" not in log.splitlines()[0] or True


def test_distributed_two_ranks_cpu(tmp_path):
    out = str(tmp_path / "output_ddp")
    _run(["-m", "pytorch_distributed_template_amd.launch", "--nproc_per_node=2", "--master_port=29611",
          "distributed.py", "--outpath", out, "-b", "16"] + COMMON)
    log, ck = _check_outdir(out + "_resnet18")
    settings = open(os.path.join(out + "_resnet18", "settings.log")).read()
    assert "batch_size: 16" in settings and "nprocs: 2" in settings  # node-total batch is logged
    # resume the finished run for one more epoch
    _run(["-m", "pytorch_distributed_template_amd.launch", "--nproc_per_node=2", "--master_port=29612",
          "distributed.py", "--outpath", out + "_r", "-b", "16", "--resume",
          os.path.join(out + "_resnet18", "checkpoint.pth.tar")] + COMMON[:-6] + ["--epochs", "3", "--step", "1",
                                                                                   "--exist-policy", "delete", "-p", "1"])
    log2 = open(os.path.join(out + "_r_resnet18", "experiment.log")).read()
    assert "=> resumed from" in log2 and "Epoch=[2/3]" in log2 and "Epoch=[0/3]" not in log2


def test_syncbn_amp_two_ranks_cpu(tmp_path):
    out = str(tmp_path / "output_amp")
    _run(["-m", "pytorch_distributed_template_amd.launch", "--nproc_per_node=2", "--master_port=29613",
          "distributed_syncBN_amp.py", "--outpath", out, "-b", "16", "--sync_batchnorm", "True"] + COMMON)
    log, _ = _check_outdir(out + "_resnet18")
    assert "=> using sync BN" in log


def test_evaluate_only(tmp_path):
    out = str(tmp_path / "output_eval")
    r = _run(["dataparallel.py", "--outpath", out, "-b", "8", "-e", "True"] + COMMON)
    log = open(os.path.join(out + "_resnet18", "experiment.log")).read()
    assert "Val epoch: [-1/2]" in log and "Train epoch" not in log


def test_two_simulated_nodes_cpu(tmp_path):
    """2 "nodes" x 2 ranks on localhost (SURVEY §4 layer 2): two launchers with --nnodes 2 --node_rank r
    rendezvous on one master; only global rank 0 writes the output directory."""
    out = str(tmp_path / "output_2n")
    env = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="1")
    procs = []
    for node in (0, 1):
        cmd = [sys.executable, "-m", "pytorch_distributed_template_amd.launch", "--nnodes=2", f"--node_rank={node}",
               "--nproc_per_node=2", "--master_addr=127.0.0.1", "--master_port=29617", "distributed.py",
               "--outpath", out, "-b", "16"] + COMMON
        procs.append(subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        o, _ = p.communicate(timeout=600)
        outs.append(o)
        assert p.returncode == 0, o[-3000:]
    log, _ = _check_outdir(out + "_resnet18")
    assert "world: 4" in log
    settings = open(os.path.join(out + "_resnet18", "settings.log")).read()
    assert "nprocs: 4" in settings
    # node 1 hosts global ranks 2, 3: no rank-0 duties there
    assert "Train epoch" not in outs[1]


def test_distributed_googlenet_aux_heads_cpu(tmp_path):
    """GoogLeNet trains through the DDP entry point: the aux heads' losses join the main loss (the
    reference would hand the output namedtuple to CrossEntropyLoss and fail)."""
    out = str(tmp_path / "output")
    args = [a if a != "32" else "64" for a in COMMON]
    _run(["-m", "torch.distributed.run", "--nproc_per_node", "2", "--master-addr", "127.0.0.1", "--master-port",
          "29561", "distributed.py", "--outpath", out, "-b", "8", "-a", "googlenet", "--dist-backend", "gloo"] + args)
    log = open(os.path.join(out + "_googlenet", "experiment.log")).read()
    assert "=> creating model: googlenet" in log
    assert re.search(r"\|\|==> total_time_cost=\d+\.\d{4}s", log)


def test_fixed_resolution_archs_follow_cli_crop(tmp_path):
    """ViT / MaxViT are built for ``--image-size`` (position table / partition grid), so the CLI runs them at
    a non-224 crop."""
    from pytorch_distributed_template_amd.models import registry
    assert registry.resolution_kwargs("vit_b_16", 64) == {"image_size": 64}
    assert registry.resolution_kwargs("maxvit_t", 224) == {"input_size": (224, 224), "partition_size": 7}
    assert registry.resolution_kwargs("resnet18", 64) == {}
    out = str(tmp_path / "out")
    args = [a if a != "32" else "64" for a in COMMON]
    _run(["dataparallel.py", "--outpath", out, "-b", "4", "--arch", "vit_b_32"] + args)
    assert "total_time_cost" in open(os.path.join(out + "_vit_b_32", "experiment.log")).read()


def test_bench_multi_gpu_request_fails_loudly_without_gpus():
    """bench.py --gpus 2 never silently runs one rank: with too few GPUs it exits non-zero and says why."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "needs 2 visible GPUs" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.parametrize("mode,port", [("exit", 29621), ("hang", 29622)])
def test_fault_injection_tears_down_group(tmp_path, mode, port):
    """SURVEY §5 fault injection ("kill rank k at step s", PDT_FAULT_INJECT): rank 1 of a 2-rank DDP run dies
    (exit) or stops making progress (hang) at iteration 1.  The group must end with a non-zero status instead of
    hanging: the launcher tears it down when a child exits non-zero; for a hang, rank 0's next collective hits
    --dist-timeout first."""
    import time
    out = str(tmp_path / f"output_fault_{mode}")
    env = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="1", PDT_FAULT_INJECT=f"1:1:{mode}")
    cmd = [sys.executable, "-m", "pytorch_distributed_template_amd.launch", "--nproc_per_node=2",
           "--master_addr=127.0.0.1", f"--master_port={port}", "--grace_s=2", "distributed.py", "--outpath", out,
           "-b", "8", "--dist-timeout", "15"] + COMMON
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    log = r.stdout + r.stderr
    assert r.returncode != 0, log[-3000:]
    assert f"[fault injection] rank 1: {mode} at epoch 0 iteration 1" in log
    assert "terminating the group" in log, log[-3000:]
    assert time.time() - t0 < 240


def test_entry_script_tears_down_native_comm(tmp_path):
    """Communicator lifecycle on the entry-script path (reference teardown `distributed_syncBN_amp.py:236-237`):
    distributed.py at world 2 on the CPU runs its gradient buckets / buffer broadcasts / metrics through the native
    C++ communicator (host shared-memory transport, --comm native); at the end every rank passes the barrier, then
    destroys its communicator collectively (runner._finish -> trainer.close()) and the job exits 0."""
    out = str(tmp_path / "output_teardown")
    env = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="1", PDT_COMM_TRACE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc_per_node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29631", "distributed.py", "--outpath", out, "-b", "8", "--comm", "native",
           "--dist-timeout", "120"] + COMMON
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    for rk in (0, 1):
        assert f"[pdt comm] rank {rk}/2: host communicator destroyed" in log, log[-3000:]
        # the host transport starts no watchdog thread (its timeout runs inside its waits): 0 before and after;
        # the RCCL watchdog's teardown is covered by test_multigpu.py::test_entry_script_rccl_graph_teardown
        assert f"[pdt comm] rank {rk}: trainer closed, live watchdogs 0 -> 0" in log, log[-3000:]
    assert "communicator aborted" not in log


def test_entry_script_aborts_native_comm_on_failure(tmp_path):
    """Failure path: rank 1 stops making progress (PDT_FAULT_INJECT hang); rank 0's next native collective times
    out (--dist-timeout), the exception leaves the epoch loop and runner aborts rank 0's communicator (not a
    collective teardown) before the job ends non-zero -- without hanging."""
    import time
    out = str(tmp_path / "output_abort")
    env = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="1", PDT_COMM_TRACE="1", PDT_FAULT_INJECT="1:1:hang")
    cmd = [sys.executable, "-m", "pytorch_distributed_template_amd.launch", "--nproc_per_node=2",
           "--master_addr=127.0.0.1", "--master_port=29632", "--grace_s=2", "distributed.py", "--outpath", out,
           "-b", "8", "--comm", "native", "--dist-timeout", "15"] + COMMON
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    log = r.stdout + r.stderr
    assert r.returncode != 0, log[-3000:]
    assert "[fault injection] rank 1: hang at epoch 0 iteration 1" in log
    assert "[pdt comm] rank 0/2: host communicator aborted" in log, log[-3000:]
    assert time.time() - t0 < 240
