"""Logger, meters, accuracy, settings, output dir policy, checkpoint schema, TensorBoard, LR schedule."""
import logging
import os

import pytest
import torch

from pytorch_distributed_template_amd import cli
from pytorch_distributed_template_amd.optim.lr import MultiStepLR, build_scheduler
from pytorch_distributed_template_amd.utils import io, meters, tensorboard
from pytorch_distributed_template_amd.utils.logging import close_logger, ddp_print, get_logger


def test_average_meter():
    m = meters.AverageMeter("Loss", ":.4f")
    m.update(2.0, 4)
    m.update(4.0, 12)
    assert m.count == 16 and m.sum == 56.0 and m.avg == 3.5 and m.val == 4.0
    assert str(m) == "Loss 4.0000 (3.5000)"
    m.update(torch.tensor(1.0), 16)
    assert abs(float(m.avg) - 2.25) < 1e-6


def test_accuracy_fraction():
    scores = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1], [0.2, 0.3, 0.5], [0.5, 0.4, 0.1]])
    tgt = torch.tensor([1, 0, 0, 1])
    acc = meters.accuracy(scores, tgt, 1)
    assert acc.dim() == 0 and abs(acc.item() - 0.5) < 1e-6
    assert abs(meters.accuracy(scores, tgt, 2).item() - 0.75) < 1e-6


def test_get_learning_rate():
    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=0.3)
    assert meters.get_learning_rate(opt) == 0.3


def test_logger_formats(tmp_path, capsys):
    lg = get_logger(str(tmp_path), "DistributedDataParallel_test")
    ddp_print("hello world", lg, 0)
    ddp_print("not printed", lg, 1)
    close_logger(lg)
    text = open(tmp_path / "experiment.log").read().strip().splitlines()
    assert len(text) == 1 and text[0].endswith(" INFO: hello world")
    assert "hello world" in capsys.readouterr().out


def test_settings_log(tmp_path):
    a = cli.parse_args("ddp", ["--outpath", str(tmp_path)])
    io.write_settings(a)
    lines = open(tmp_path / "settings.log").read().splitlines()
    assert "arch: resnet18" in lines and "batch_size: 1200" in lines and "step: [3, 4]" in lines


def test_output_process_policies(tmp_path):
    d = tmp_path / "out_resnet18"
    io.output_process(str(d), "prompt")
    assert d.is_dir()
    (d / "x").write_text("1")
    with pytest.raises(OSError):
        io.output_process(str(d), "quit")
    with pytest.raises(OSError):  # prompt policy without a TTY refuses instead of hanging
        io.output_process(str(d), "prompt")
    io.output_process(str(d), "reuse")
    assert (d / "x").exists()
    io.output_process(str(d), "delete")
    assert d.is_dir() and not (d / "x").exists()


def test_checkpoint_schema_roundtrip(tmp_path):
    from pytorch_distributed_template_amd.models import registry
    m = registry.create("resnet18")
    st = io.make_checkpoint_state(3, "resnet18", m, torch.tensor(0.25))
    io.save_checkpoint(st, True, str(tmp_path))
    assert (tmp_path / "checkpoint.pth.tar").exists() and (tmp_path / "model_best.pth.tar").exists()
    ck = io.load_checkpoint(str(tmp_path / "checkpoint.pth.tar"))
    assert set(ck) == {"epoch", "arch", "state_dict", "best_acc1"}
    assert ck["epoch"] == 3 and ck["arch"] == "resnet18"
    assert ck["best_acc1"].dim() == 0 and ck["best_acc1"].device.type == "cpu"
    assert not any(k.startswith("module.") for k in ck["state_dict"])
    m2 = registry.create("resnet18")
    m2.load_state_dict(ck["state_dict"])
    io.save_checkpoint(st, False, str(tmp_path / ".."))


def test_tensorboard_roundtrip(tmp_path):
    w = tensorboard.SummaryWriter(str(tmp_path))
    for e in range(3):
        w.add_scalar("lr", 0.1 * (e + 1), e)
        w.add_scalar("Train_ce_loss", torch.tensor(6.9 - e), e)
    w.close()
    files = [f for f in os.listdir(tmp_path) if f.startswith("events.out.tfevents.")]
    assert len(files) == 1
    rec = tensorboard.read_scalars(str(tmp_path / files[0]))
    assert [(t, s) for t, s, _ in rec] == [("lr", 0), ("Train_ce_loss", 0), ("lr", 1), ("Train_ce_loss", 1),
                                          ("lr", 2), ("Train_ce_loss", 2)]
    assert abs(rec[-1][2] - 4.9) < 1e-5


def test_crc32c_known_vector():
    assert tensorboard.crc32c(b"123456789") == 0xE3069283


def test_multistep_closed_form():
    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=0.1)
    s = build_scheduler("steplr", opt, [3, 4], 0.1)
    lrs = []
    for e in range(5):
        s.step(e)
        lrs.append(opt.param_groups[0]["lr"])
    assert lrs == pytest.approx([0.1, 0.1, 0.1, 0.01, 0.001])
    with pytest.raises(ValueError):
        build_scheduler("cosine", opt, [3], 0.1)
    # matches upstream MultiStepLR with the deprecated step(epoch) closed form
    opt2 = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=0.1)
    up = torch.optim.lr_scheduler.MultiStepLR(opt2, milestones=[3, 4], gamma=0.1)
    for e in range(1, 6):
        up.step()
        s.step(e)
        assert opt2.param_groups[0]["lr"] == pytest.approx(opt.param_groups[0]["lr"])
