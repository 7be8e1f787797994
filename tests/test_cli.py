"""CLI parity with the reference parsers and quirk resolutions (§2.9)."""
import pytest

from pytorch_distributed_template_amd import cli


@pytest.mark.parametrize("mode,gpus,outpath", [("dp", "5,6,7", "./output"), ("ddp", "0,1,2", "./output_ddp_test"),
                                               ("ddp_amp", "0,1,2", "./output_ddp_amp")])
def test_defaults(mode, gpus, outpath):
    a = cli.parse_args(mode, [])
    assert a.data == "/mnt/cephfs/mixed/dataset/imagenet/"
    assert a.arch == "resnet18" and a.workers == 8 and a.epochs == 5 and a.step == [3, 4]
    assert a.start_epoch == 0 and a.batch_size == 1200 and a.lr == 0.1 and a.momentum == 0.9
    assert a.weight_decay == 1e-4 and a.print_freq == 10 and a.evaluate is False and a.pretrained is False
    assert a.seed is None and a.gpus == gpus and a.outpath == outpath
    assert a.lr_scheduler == "steplr" and a.gamma == 0.1
    if mode == "ddp_amp":
        assert a.use_amp is True and a.sync_batchnorm is False
    else:
        assert not hasattr(a, "use_amp")
    assert hasattr(a, "local_rank") == (mode != "dp")


def test_reference_spellings():
    a = cli.parse_args("ddp_amp", ["-a", "resnet50", "-j", "4", "-b", "256", "--learning-rate", "0.2", "--wd", "5e-5",
                                   "-p", "3", "--start-epoch", "2", "--lr-scheduler", "steplr", "--local_rank=1"])
    assert (a.arch, a.workers, a.batch_size, a.lr, a.weight_decay, a.print_freq, a.start_epoch, a.local_rank) == \
        ("resnet50", 4, 256, 0.2, 5e-5, 3, 2, 1)
    b = cli.parse_args("ddp", ["--local-rank", "3", "--weight-decay", "0.001"])
    assert b.local_rank == 3 and b.weight_decay == 0.001


@pytest.mark.parametrize("val,expect", [("True", True), ("False", False), ("false", False), ("0", False), ("1", True),
                                        ("", False), ("yes", True), ("no", False)])
def test_bool_flags(val, expect):
    a = cli.parse_args("ddp_amp", ["--use_amp", val, "--sync_batchnorm", val, "-e", val, "--pretrained", val])
    assert a.use_amp is expect and a.sync_batchnorm is expect and a.evaluate is expect and a.pretrained is expect


def test_bare_bool_flag():
    assert cli.parse_args("ddp_amp", ["--sync_batchnorm"]).sync_batchnorm is True


@pytest.mark.parametrize("argv", [["--step", "3", "4"], ["--step", "3,4"], ["--step", "[3,4]"], ["--step", "[3,", "4]"]])
def test_step_forms(argv):
    assert cli.parse_args("dp", argv).step == [3, 4]


def test_seed_and_arch_choices():
    assert cli.parse_args("dp", ["--seed", "7"]).seed == 7
    with pytest.raises(SystemExit):
        cli.parse_args("dp", ["-a", "not_a_model"])
    assert {"resnet18", "resnet34", "resnet50", "resnet101", "resnet152"} <= set(cli.build_parser("dp")._option_string_actions["--arch"].choices)


def test_local_rank_env(monkeypatch):
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert cli.parse_args("ddp", []).local_rank == 5


def test_native_engine_covers_resnets_resnexts_vgg_and_alexnet():
    """--engine auto picks the native HIP engine for the ResNet / Wide-ResNet / ResNeXt registry entries on a GPU in
    every precision (grouped convs: channel slices in the 16-bit and the fp32 executor), for VGG and AlexNet in 16-bit
    (their fp32 runs stay on the torch engine), and the torch engine elsewhere."""
    import argparse

    import torch
    from pytorch_distributed_template_amd.engine.runner import resolve_engine
    gpu, cpu = torch.device("cuda"), torch.device("cpu")
    for arch in ("resnet18", "resnet50", "wide_resnet101_2", "resnext50_32x4d", "resnext101_32x8d", "resnext101_64x4d"):
        a = argparse.Namespace(engine="auto", arch=arch)
        assert resolve_engine(a, gpu, torch.bfloat16) == "native", arch
        assert resolve_engine(a, gpu, torch.float16) == "native", arch
        assert resolve_engine(a, gpu, torch.float32) == "native", arch
        assert resolve_engine(a, cpu, torch.float32) == "torch", arch
    for arch in ("vgg11", "vgg16", "vgg19_bn", "alexnet"):  # the VGG / AlexNet executor: 16-bit only
        assert resolve_engine(argparse.Namespace(engine="auto", arch=arch), gpu, torch.bfloat16) == "native", arch
        assert resolve_engine(argparse.Namespace(engine="auto", arch=arch), gpu, torch.float32) == "torch", arch
