"""Profiling tools on synthetic rocprofv3 kernel-trace CSVs (CPU only)."""
import csv
import re
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, kernels):
    cols = ["Kind", "Queue_Id", "Stream_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for name, s, e, q in kernels:
            w.writerow({"Kind": "KERNEL_DISPATCH", "Queue_Id": q, "Stream_Id": q, "Kernel_Name": name,
                        "Start_Timestamp": s, "End_Timestamp": e})


def test_timeline_gaps_busy_union_and_gaps(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    # step 0: conv 0-100 us on stream 0 overlapping wgrad 50-150 us on stream 1, 20 us idle, sgd 170-180
    # step 1: conv 200-300, 40 us idle, sgd 340-350
    ns = 1000
    _trace(p, [("void pdt::conv_fwd_kernel<0>(A)", 0, 100 * ns, 0), ("pdt::wgrad(B)", 50 * ns, 150 * ns, 1),
               ("void pdt::sgd_kernel<0>(C)", 170 * ns, 180 * ns, 0),
               ("void pdt::conv_fwd_kernel<0>(A)", 200 * ns, 300 * ns, 0),
               ("void pdt::sgd_kernel<0>(C)", 340 * ns, 350 * ns, 0)])
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "timeline_gaps.py"), str(p), "--step", "1"],
                       capture_output=True, text=True, check=True)
    out = r.stdout.splitlines()
    assert out[0] == "2 steps in trace"
    assert out[1].startswith("step 0: wall 0.180 ms  busy 0.160 ms  idle 0.020 ms  kernel-sum 0.210 ms  kernels 3")
    assert out[2].startswith("step 1: wall 0.170 ms  busy 0.110 ms  idle 0.060 ms")
    gaps = [ln for ln in out if "gap" in ln]
    assert "40.0 us" in gaps[0] and "after conv_fwd_kernel<0>" in gaps[0] and "before sgd_kernel<0>" in gaps[0]
    assert "20.0 us" in gaps[1] and "after sgd_kernel<0>" in gaps[1]  # previous step's last kernel


def test_counted_waits_in_layer1_pingpong_kernel():
    """The 8-wave layer1 kernel counts its asm DMA / operand loads itself (s_waitcnt vmcnt(11) / vmcnt(7)); a spill
    or a store scheduled into those windows would be a silent race.  Compile it (hipcc -S, gfx950) and check every
    instantiation's ISA: no scratch instructions, each counted window holds at least its count of younger ops."""
    import shutil
    import subprocess
    import sys
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "check_counted_waits.py")
    r = subprocess.run([sys.executable, tool], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok ") >= 8, r.stdout


def test_isa_hazard_checker_detects_planted_hazards():
    """The ISA checker itself (tools/check_isa_hazards.py) on synthetic instruction streams: an asm load whose
    destination is read before a covering wait is reported, one read after its wait is not; a counted DMA window
    with too few younger operations is reported; a packed-FP32 op is reported."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import check_isa_hazards as c
    bad = ["global_load_dwordx4 v[4:7], v[0:1], off", "buffer_load_dwordx4 v2, s[0:3], 0 offen lds",
           "v_mov_b32 v9, v5", "s_waitcnt vmcnt(0)", "s_endpgm"]
    good = ["global_load_dwordx4 v[4:7], v[0:1], off", "buffer_load_dwordx4 v2, s[0:3], 0 offen lds",
            "s_waitcnt vmcnt(1)", "v_mov_b32 v9, v5", "s_endpgm"]
    early = ["global_load_dwordx4 v[4:7], v[0:1], off", "buffer_load_dwordx4 v2, s[0:3], 0 offen lds",
             "s_waitcnt vmcnt(2)", "v_mov_b32 v9, v5", "s_endpgm"]  # vmcnt(2) leaves the load in flight
    assert c.check_register_hazards(*c.parse(bad))
    assert not c.check_register_hazards(*c.parse(good))
    assert c.check_register_hazards(*c.parse(early))
    # a hazard behind an unconditional branch (followed)
    br = ["global_load_dwordx2 v[4:5], v[0:1], off", "s_branch .L1", "s_waitcnt vmcnt(0)", "s_endpgm",
          ".L1:", "v_add_u32_e32 v6, v4, v6", "s_endpgm"]
    assert c.check_register_hazards(*c.parse(br))
    # a younger load into the same register is not a hazard (loads return in issue order)
    waw = ["global_load_dwordx2 v[4:5], v[0:1], off", "global_load_dword v5, v[2:3], off", "s_waitcnt vmcnt(0)",
           "v_mov_b32 v9, v5", "s_endpgm"]
    assert not c.check_register_hazards(*c.parse(waw))
    win = ["buffer_load_dwordx4 v2, s[0:3], 0 offen lds"] + ["global_store_dwordx2 v[0:1], v[2:3], off"] * 3 + \
          ["s_waitcnt vmcnt(4)", "s_endpgm"]
    probs, _ = c.check_windows(*c.parse(win), {4: "dma"})
    assert probs
    win3 = [t.replace("vmcnt(4)", "vmcnt(3)") for t in win]
    probs, found = c.check_windows(*c.parse(win3), {3: "dma"})
    assert not probs and found == ["vmcnt(3):3"]
    probs, _ = c.check_kernel("_Zk", ["v_pk_fma_f32 v[0:1], v[2:3], v[4:5], v[6:7]", "s_endpgm"])
    assert probs
    # a loop whose counted wait is covered in the steady state (latch path: 3 stores behind the DMA) but not on the
    # path from the prologue (the DMA right before the loop): the SHORTEST path fails unless the kernel annotates
    # that wait as flag-guarded (GUARDED), and the annotation then applies the steady-state count
    loop = ["buffer_load_dwordx4 v2, s[0:3], 0 offen lds", ".Lloop:", "s_waitcnt vmcnt(3)",
            "buffer_load_dwordx4 v2, s[0:3], 0 offen lds"] + ["global_store_dwordx2 v[0:1], v[2:3], off"] * 3 + \
           ["s_cbranch_scc1 .Lloop", "s_endpgm"]
    probs, found = c.check_windows(*c.parse(loop), {3: "dma"}, "_Zloopk")
    assert probs and found == ["vmcnt(3):0"]
    c.GUARDED["_Zloopk"] = {3: "test: the first iteration waits vmcnt(0)"}
    try:
        used = set()
        probs, found = c.check_windows(*c.parse(loop), {3: "dma"}, "_Zloopk", used)
        assert not probs and found == ["vmcnt(3):3"] and used == {("_Zloopk", 3)}
    finally:
        del c.GUARDED["_Zloopk"]


def test_isa_hazards_every_kernel():
    """Every kernel's compiled ISA (hipcc -S, gfx950): no asm-load register hazard, every designated counted wait
    covers its window, no packed-FP32 op, no spill in a kernel that counts its own waits (tools/check_isa_hazards.py).
    Skipped only without hipcc."""
    import shutil
    import subprocess
    import sys
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "check_isa_hazards.py")
    r = subprocess.run([sys.executable, tool], capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    m = re.search(r"(\d+) kernels checked, 0 with violations", r.stdout)
    assert m and int(m.group(1)) > 300, r.stdout[-2000:]
    for k in ("conv_l1pp_kernel", "conv_l1_kernel", "stem_fwd_kernel", "wgrad_stem_quad_kernel",
              "wgrad_stem_rows_kernel"):
        assert k in r.stdout  # the designated windows were found and checked
