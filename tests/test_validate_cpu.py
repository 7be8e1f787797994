"""Validation mode (ops/validate.py): launch-checked native ops with an op history, non-finite tracking,
and the pre-launch op log -- exercised on CPU with stand-in extension functions (the GPU test in
tests/test_executor_gpu.py runs it over the real kernels)."""
import pytest
import torch

from pytorch_distributed_template_amd.ops import validate


def _v(level, **kw):
    return validate.Validator(level, history=4, sync=lambda: None, capturing=lambda: False, **kw)


def test_level1_names_the_failing_op_and_history():
    v = _v(1)
    ok = v.wrap("ok_op", lambda t: t.add_(1))
    def boom(t):
        raise RuntimeError("invalid device function")
    bad = v.wrap("bad_op", boom)
    t = torch.zeros(3)
    for _ in range(5):
        ok(t)
    assert torch.equal(t, torch.full((3,), 5.0))
    with pytest.raises(validate.ValidationError) as e:
        bad(torch.ones(2, 2))
    msg = str(e.value)
    assert "`bad_op` failed: invalid device function" in msg and "float32[2, 2]" in msg
    assert msg.count("ok_op") == 3  # history holds the last 4 ops: 3 x ok_op + bad_op
    assert v.calls == 6


def test_level2_flags_the_op_that_creates_nonfinite():
    v = _v(2)
    src = torch.tensor([1.0, float("nan"), 2.0])  # already non-finite: not this op's fault
    out = torch.zeros(3)
    copy = v.wrap("copy_op", lambda s, o: o.copy_(torch.nan_to_num(s)))
    poison = v.wrap("poison_op", lambda s, o: o.copy_(s))
    copy(src, out)
    with pytest.raises(validate.NonFiniteError) as e:
        poison(src, out)
    assert "`poison_op` wrote 1 non-finite value(s) into argument #1" in str(e.value)
    # level 1 does not scan
    _v(1).wrap("poison_op", lambda s, o: o.copy_(s))(src, torch.zeros(3))


def test_capture_and_log(tmp_path):
    log = tmp_path / "ops.log"
    v = validate.Validator(1, sync=lambda: (_ for _ in ()).throw(RuntimeError("sync inside capture")),
                           capturing=lambda: True, log_path=str(log))
    v.wrap("captured", lambda: 7)()  # no sync, no record while capturing
    assert v.calls == 0
    v2 = validate.Validator(1, sync=lambda: None, capturing=lambda: False, log_path=str(log))
    v2.wrap("first", lambda: None)()
    v2.wrap("second", lambda x: None)(torch.ones(1, dtype=torch.float16))
    assert log.read_text().splitlines() == ["first (no tensors)", "second #0:float16[1]"]


def test_env_wrapping(monkeypatch):
    monkeypatch.setenv("PDT_VALIDATE", "0")
    f = lambda: 1  # noqa: E731
    assert validate.maybe_wrap("f", f) is f
    monkeypatch.setenv("PDT_VALIDATE", "2")
    w = validate.maybe_wrap("f", f)
    assert w is not f and w.__wrapped__ is f and w() == 1
    assert validate.maybe_wrap("T", torch.nn.Module) is torch.nn.Module  # classes pass through


def test_level3_replay_flags_a_timing_dependent_op():
    """Replay determinism: an op whose output depends on something other than its inputs (here a call counter,
    standing in for wave timing) is named; a pure op passes and keeps its first result."""
    v = _v(3)
    v.replay_host = True
    pure = v.wrap("pure_op", lambda a, o: o.copy_(a * 2 + 1))
    a, o = torch.arange(6.0), torch.zeros(6)
    pure(a, o)
    assert torch.equal(o, torch.arange(6.0) * 2 + 1) and v.replayed == 1
    calls = [0]

    def racy(a, o):
        calls[0] += 1
        o.copy_(a)
        if calls[0] == 3:  # the second replay differs in one element
            o[4] += 1e-3
    with pytest.raises(validate.NondeterminismError) as e:
        v.wrap("racy_op", racy)(torch.arange(6.0), torch.zeros(6))
    assert "`racy_op` is not deterministic: replay 2 changed 1 of 6 element(s) of argument #1" in str(e.value)
    # accumulate-style ops are replayed from the snapshot, so they are not falsely flagged
    acc = v.wrap("acc_op", lambda a, o: o.add_(a))
    o2 = torch.ones(3)
    acc(torch.ones(3), o2)
    assert torch.equal(o2, torch.full((3,), 2.0))
    # collect mode: recorded, the first run's result kept
    v.collect = True
    calls[0] = 0
    o3 = torch.zeros(6)
    v.wrap("racy_op", racy)(torch.arange(6.0), o3)
    assert len(v.findings) == 1 and torch.equal(o3, torch.arange(6.0))


def test_guard_band_names_the_overrunning_op():
    v = _v(1)
    buf = torch.zeros(16)
    gi = torch.tensor([4, 5, 6, 7, 12, 13, 14, 15])  # guards after slot "a" [0,4) and slot "b" [8,12)
    buf.view(torch.int32)[gi] = validate.CANARY_BITS
    v.register_guard(buf, gi, [(0, "a"), (4, "b")])
    v.wrap("in_bounds", lambda t: t[8:12].fill_(3.0))(buf)
    with pytest.raises(validate.GuardBandError) as e:
        v.wrap("overrun", lambda t: t[8:13].fill_(3.0))(buf)
    assert "`overrun` wrote into the guard band after parameter `b`" in str(e.value)


def test_flat_params_guard_layout(monkeypatch):
    """PDT_VALIDATE_GUARD leaves a canary gap after every slot (CPU: layout only)."""
    from pytorch_distributed_template_amd.optim.flat import FlatParams
    monkeypatch.setenv("PDT_VALIDATE", "1")
    monkeypatch.setenv("PDT_VALIDATE_GUARD", "16")
    m = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.BatchNorm1d(8))
    f = FlatParams(m, "cpu")
    for a, b in zip(f.slots, f.slots[1:]):
        assert b.offset - (a.offset + a.numel) >= 16
    idx = f.master_read_index()
    assert idx.numel() == 8 + 8 + 8  # linear bias, bn weight, bn bias
