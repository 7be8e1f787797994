"""Profiling tools on synthetic rocprofv3 kernel-trace CSVs (CPU only)."""
import csv
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
    """The 8-wave layer1 kernel counts its asm DMA / operand loads itself (s_waitcnt vmcnt(11) / vmcnt(14)); a spill
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
