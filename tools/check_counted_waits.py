"""Static check of the counted ``s_waitcnt vmcnt(N)`` waits in kernels that issue asm LDS-DMA.

The 8-wave layer1 kernel (``conv_l1pp_kernel``, csrc/kernels/conv_l1.hip) issues its halo DMA and its epilogue
operand loads through inline asm, invisible to the compiler's waitcnt pass, and waits for them itself:

* ``vmcnt(11)`` after the operand loads + the 11 DMA pieces: the loads are done once at most 11 younger
  vector-memory operations remain -- safe iff at least 11 vm operations follow the last operand load;
* ``vmcnt(7)`` after the DMA + the epilogue's 7 (16-byte) stores: the DMA is done once at most 7 younger remain --
  safe iff at least 7 vm operations follow the last DMA piece;
* ``vmcnt(4)`` (EPI 3, the block-output BN-backward epilogue in two halves) after the second half's operand loads
  + the first half's 4 held stores: safe iff at least 4 vm operations follow the last operand load.
(Round 5: 16-byte epilogue stores and operand loads -- the counts were 14 and 8 with 8-byte ones.)

A compiler-inserted spill (``scratch_*``) or a reordered store inside those windows would break the count
silently (a race, not a crash), so this walks every instantiation's ISA backwards from each such wait and
checks the window, and checks that no instantiation spills at all.

    python tools/check_counted_waits.py [--asm /tmp/conv_l1.s]     # exit 1 on a violation
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VM = ("global_", "buffer_", "scratch_", "flat_")


def compile_asm(src: str, out: str) -> None:
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast", "-munsafe-fp-atomics",
           "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", f"-I{os.path.join(REPO, 'csrc')}",
           "--cuda-device-only", "-S", src, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)


def kernels(asm: str, prefix: str):
    for m in re.finditer(r"^(" + re.escape(prefix) + r"\w*):[ \t]*(;.*)?$", asm, re.M):
        name = m.group(1)
        end = asm.index(".Lfunc_end", m.end())
        yield name, asm[m.end():end].split("\n")


def check(lines):
    """Returns a list of problems of one kernel body."""
    ins = [l.strip() for l in lines]
    ins = [l for l in ins if l and not l.startswith((";", "."))]
    probs, windows = [], []
    nspill = sum(1 for l in ins if l.startswith("scratch_"))
    if nspill:
        probs.append(f"{nspill} scratch (spill) instructions")
    for i, l in enumerate(ins):
        m = re.match(r"s_waitcnt vmcnt\((\d+)\)$", l)
        if not m or m.group(1) not in ("4", "11", "7"):
            continue
        need = int(m.group(1))
        n = 0
        for k in range(i - 1, -1, -1):
            t = ins[k]
            if need == 7 and t.startswith("buffer_load_dwordx4") and t.endswith(" lds"):
                break
            if need in (4, 11) and t.startswith("buffer_load_dwordx") and not t.endswith(" lds"):
                break
            if t.startswith(VM):
                n += 1
            if t.startswith("s_barrier") or t.startswith("s_endpgm"):
                n = -1  # a barrier in between: not one of ours (the walk follows the linear layout, so the
                break   # other arm of an if / else -- e.g. the vmcnt(0) of the no-epilogue case -- is crossed)
        if n < 0:
            probs.append(f"vmcnt({need}) at instruction {i}: no asm load / DMA found before it (unrecognised window)")
        elif n < need:
            probs.append(f"vmcnt({need}) at instruction {i} has only {n} vm operations after the operations it waits for")
        windows.append(f"vmcnt({need}):{n}")
    return probs, windows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=None, help="existing hipcc -S listing of csrc/kernels/conv_l1.hip")
    ap.add_argument("--prefix", default="_ZN3pdt16conv_l1pp_kernel")
    a = ap.parse_args()
    path = a.asm
    if path is None:
        path = os.path.join(tempfile.mkdtemp(), "conv_l1.s")
        compile_asm(os.path.join(REPO, "csrc", "kernels", "conv_l1.hip"), path)
    asm = open(path).read()
    bad = 0
    seen = 0
    for name, body in kernels(asm, a.prefix):
        seen += 1
        probs, windows = check(body)
        print(f"{'FAIL' if probs else 'ok  '} {name}: windows {' '.join(windows)}" + ("; " + "; ".join(probs) if probs else ""))
        bad += bool(probs)
    if not seen:
        print("no kernel matched", a.prefix)
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
