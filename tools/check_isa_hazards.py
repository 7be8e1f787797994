"""Static hazard checks over the compiled gfx950 ISA of EVERY kernel in csrc/kernels/*.hip (a CPU test runs it).

Kernels that issue their own vector-memory operations through inline asm (LDS-DMA ``buffer_load ... lds`` pieces,
``gload16_asm`` / ``gload8_asm`` / ``buffer_load_dwordx2`` operand loads) and wait for them with COUNTED
``s_waitcnt vmcnt(N)`` are invisible to the compiler's waitcnt pass.  Three ways that silently races (a wrong
result under GPU contention, not a crash):

1. **register hazard** -- an asm load returns its destination as an ``"=v"`` output, so the compiler believes the
   value is present right after the asm statement.  Any instruction that reads or overwrites those VGPRs (a copy,
   a spill, an early use) before a wait that provably retired the load reads stale data.  Checked for every
   vector-memory load with a register destination in every kernel: a forward walk along the fall-through path from
   the load counts the vector-memory operations issued after it; the load is retired at the first
   ``s_waitcnt vmcnt(M)`` with at least M younger operations.  No instruction before that may touch the
   destination registers (the compiler's own loads pass by construction: its waits are exact).
2. **counted DMA windows** -- a designated wait ``vmcnt(N)`` must have at least N vector-memory operations between
   the youngest LDS-DMA piece (or asm operand load) it is meant to cover and the wait, on the kernel's loop path
   (walking back in layout order; entering a loop header continues from its latch: "the previous iteration").
   A spill or a reordered store inside the window breaks the count.  Windows: WINDOWS below.
4. **store data** -- a ``..._store_dwordx3/x4`` reads its data VGPRs after issue: no VALU instruction in the next two
   wait states may write them (hipcc pads the stores it emits; an asm store must end with ``s_nop 1`` itself -- found in
   round 5, where the missing pad corrupted stored rows of conv1x1x_bnb).
3. **packed FP32** -- no ``v_pk_{fma,mul,add}_f32`` anywhere: an LDS load into the source VGPRs of a packed FP32
   op issued right behind it raced on the last quarter-wave (profiles/r3_nondeterminism_root_cause.md); the build
   disables the feature (ops/_build.py), this checks it stays disabled.
Also: no ``scratch_`` (spill) instruction in a kernel that counts its own waits.

    python tools/check_isa_hazards.py [--keep DIR]      # exit 1 on a violation; prints one line per kernel
"""
import argparse
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VM_PREFIX = ("global_", "buffer_", "scratch_", "flat_")
# kernel-name substring -> {N: what the window must cover} (mangled names contain the plain kernel name)
WINDOWS = {
    "conv_l1pp_kernel": {7: "dma", 11: "load", 4: "load"},
    "conv_l1_kernel": {16: "dma", 12: "dma"},
    "stem_fwd_kernel": {14: "dma"},
    "wgrad_stem_quad_kernel": {12: "dma", 8: "load"},
    "wgrad_stem_rows_kernel": {12: "dma", 2: "load"},
    "conv_wgrad_wide_kernel": {6: ("dma", 6), 3: ("dma", 3)},
    "conv1x1_c64_kernel": {16: "dma"},  # the previous tile's 16 stores stay in flight
    "conv1x1_c64_bnb_kernel": {32: "dma", 40: "dma"},  # the previous tile's 24 (32) operand loads + 8 stores
    # conv1x1x.hip: the previous tile's stores (forward: (BM/16)*(NF/2) per wave) / operand loads + stores
    "conv1x1x_kernel": {8: "dma", 4: "dma", 2: "dma"},
}


def _x1_bnb_windows():
    """conv1x1x_bnb_kernel<DT, BR, KH, NF, BM, PJ> (conv1x1x.hip): per configuration, the loop-top wait covers the
    tile's DMA (SUB * NL younger loads; stores are not counted on), and the sub-tile waits cover that sub-tile's
    operand loads with the NL-load prefetch of the next sub-tile left in flight (skip NL), behind the next tile's DMA
    (XI, sub-tile 0).  (The walk counts stores too, so a window is >= the loads-only count.)"""
    out = {}
    for kh, nf, bm, pj, brs in ((1, 4, 64, 1, (1,)), (1, 2, 64, 2, (2,)), (2, 4, 64, 1, (1,)), (2, 2, 64, 2, (2,)),
                                (4, 2, 64, 2, (1, 2)),
                                (8, 2, 32, 1, (1, 2))):
        for br in brs:
            np_, sub = nf // 2, bm // (16 * pj)
            nl, ns, xi = pj * np_ * (4 if br == 2 else 3), pj * np_, bm * kh * 128 // 4096
            wins = {sub * nl: "dma", xi + nl: ("load", nl), nl: ("load", nl)}
            for dt in (0, 1):
                out[f"conv1x1x_bnb_kernelILi{dt}ELi{br}ELi{kh}ELi{nf}ELi{bm}ELi{pj}EE"] = wins
    return out


WINDOWS.update(_x1_bnb_windows())
COUNTING = ("conv_l1pp_kernel", "conv_l1_kernel", "stem_fwd_kernel", "wgrad_stem_kernel", "wgrad_stem_quad_kernel",
            "wgrad_stem_rows_kernel", "conv_pp_kernel",
            "conv_wgrad_pp_kernel", "wgrad3x3_c64_kernel", "conv_fwd_kernel", "conv_wgrad_wide_kernel",
            "conv1x1_c64_kernel", "conv1x1_c64_bnb_kernel", "conv1x1x_kernel", "conv1x1x_bnb_kernel")


def hip_flags():
    return ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast", "-munsafe-fp-atomics",
            "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", f"-I{os.path.join(REPO, 'csrc')}",
            "--cuda-device-only", "-S"]


def compile_all(out_dir):
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    srcs = sorted(glob.glob(os.path.join(REPO, "csrc", "kernels", "*.hip")))

    def one(src):
        out = os.path.join(out_dir, os.path.basename(src) + ".s")
        subprocess.run([hipcc] + hip_flags() + [src, "-o", out], check=True, capture_output=True)
        return out
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        return list(ex.map(one, srcs))


def kernels(asm):
    for m in re.finditer(r"^(_Z\w+):[ \t]*(;.*)?$", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        if end < 0:
            continue
        yield m.group(1), asm[m.end():end].split("\n")


def parse(lines):
    """-> instructions [(text)], label -> index of the next instruction."""
    ins, labels = [], {}
    for raw in lines:
        t = raw.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            labels[t[:-1]] = len(ins)
            continue
        if t.startswith("."):
            continue
        ins.append(t)
    return ins, labels


REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(4) is not None:
            out.add((k, int(m.group(4))))
        else:
            out.update((k, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def is_vm(t):
    return t.startswith(VM_PREFIX) and not t.startswith(("buffer_wbl2", "buffer_inv", "buffer_wbinvl1"))


def is_dma(t):
    return is_vm(t) and t.endswith(" lds")


def vm_wait(t):
    m = re.match(r"s_waitcnt\b.*\bvmcnt\((\d+)\)", t)
    return int(m.group(1)) if m else None


def branch(t):
    m = re.match(r"(s_branch|s_cbranch_\w+)\s+(\S+)", t)
    return (m.group(1), m.group(2)) if m else None


def touched(u):
    """Registers an instruction reads or writes -- except the destination of another vector-memory load: loads
    return in issue order, so a younger load into the same register lands after the older one (no hazard)."""
    if is_vm(u) and "load" in u.split()[0] and not u.endswith(" lds"):
        ops = u.split(None, 1)[1].split(",", 1) if len(u.split(None, 1)) > 1 else [""]
        return regs(ops[1]) if len(ops) > 1 else set()
    return regs(u.split(None, 1)[1]) if len(u.split(None, 1)) > 1 else set()


def check_register_hazards(ins, labels):
    """Forward walk from every register-destination VMEM load (module docstring, check 1) along the layout's
    fall-through path (unconditional branches followed): the region where the compiler would place a copy or spill of
    the loaded registers between an asm load and its asm wait.  (Conditional branches are not followed: the compiler
    threads block-uniform conditions through scalar flag registers, so most other paths are infeasible.)"""
    probs = []
    for i, t in enumerate(ins):
        if not is_vm(t) or "load" not in t.split()[0] or t.endswith(" lds"):
            continue
        ops = t.split(None, 1)
        if len(ops) < 2:
            continue
        dest = regs(ops[1].split(",")[0])
        if not dest:
            continue
        stack, seen = [(i + 1, 0)], set()
        while stack:
            j, k = stack.pop()
            while j < len(ins):
                key = (j, min(k, 64))
                if key in seen:
                    break
                seen.add(key)
                u = ins[j]
                w = vm_wait(u)
                if w is not None and k >= w:
                    break  # retired on this path
                if u.startswith("s_endpgm"):
                    break
                if not u.startswith("s_waitcnt") and touched(u) & dest:
                    probs.append(f"register hazard: '{u}' (instruction {j}) touches the destination of '{t}' "
                                 f"(instruction {i}) before a wait retires it ({k} younger vm ops)")
                    break
                if is_vm(u):
                    k += 1
                b = branch(u)
                if b is not None and b[0] == "s_branch":  # the only successor
                    tgt = labels.get(b[1])
                    if tgt is None:
                        break
                    j = tgt
                    continue
                j += 1  # conditional branches: the fall-through path (see check_register_hazards)
    return probs


def check_store_data(ins):
    """Module docstring, check 4: a >8-byte vector-memory store followed, within two wait states, by an instruction
    whose destination overlaps the store's data registers."""
    probs = []
    for i, t in enumerate(ins):
        op = t.split()[0]
        if not (is_vm(t) and "store" in op and op.endswith(("dwordx3", "dwordx4"))):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        data = regs(ops[0] if op.startswith("buffer_") else ops[1])  # global_/flat_: vaddr first, then vdata
        states, j = 0, i + 1
        while states < 2 and j < len(ins):
            u = ins[j]
            m = re.match(r"s_nop\s+(\d+)", u)
            if m:
                states += int(m.group(1)) + 1
            else:
                parts = u.split(None, 1)
                dest = regs(parts[1].split(",")[0]) if len(parts) > 1 and u.startswith("v_") else set()  # VALU
                if dest & data:
                    probs.append(f"store data hazard: '{u}' (instruction {j}) overwrites the data of '{t}' "
                                 f"(instruction {i}) {states} wait state(s) after it")
                    break
                states += 1
            j += 1
    return probs


def check_windows(ins, labels, wins):
    """Designated counted waits (module docstring, check 2).  Walking back from the wait in layout order, a label that
    is the target of backward branches (a loop header / latch block) may continue from any of those branches ("the
    previous iteration"); the window is the LARGEST count over these walks -- the kernel's steady-state path.  Paths
    through a latch that skips the epilogue (e.g. a tile with no rows to store) are guarded at run time by the
    kernel's own flag and are not reported; a spill or a store scheduled out of the steady-state window is.

    Why the LARGEST and not the smallest count (round-5 review): a path-insensitive minimum over the real control-flow
    graph was built and run over all 615 kernels -- it flags 20 of them, every one on a path the kernel's own
    loop-carried flag makes infeasible (``stores_behind`` / ``n_st`` / ``first`` select ``vmcnt(0)`` exactly when the
    previous tile issued no stores, and exec-mask store skips occur only on a partial last tile).  A checker that fails
    on correct code gets disabled; the flag-guarded first / last tiles are covered by the GPU numerics tests of each
    counted-wait kernel (bit-identity against the generic kernels, PDT_BUF_POISON on)."""
    latches = {}
    for j, t in enumerate(ins):
        b = branch(t)
        if b is not None and b[1] in labels and labels[b[1]] <= j:
            latches.setdefault(labels[b[1]], set()).add(j)

    def walk(j, cnt, what, depth, skip=0):
        """``skip``: the youngest ``skip`` matching operations are the group the wait leaves in flight (ring
        pipelines); the window is measured from the one before them."""
        best = None
        while j >= 0:
            u = ins[j]
            if (what == "dma" and is_dma(u)) or (what == "load" and is_vm(u) and "load" in u.split()[0]
                                                 and not u.endswith(" lds")):
                if skip == 0:
                    return cnt if best is None else max(best, cnt)
                skip -= 1
            if is_vm(u):
                cnt += 1
            if j in latches and depth < 4:
                for l in latches[j]:
                    r = walk(l, cnt, what, depth + 1, skip)
                    if r is not None:
                        best = r if best is None else max(best, r)
            j -= 1
        return best

    probs, found = [], []
    for i, t in enumerate(ins):
        n = vm_wait(t)
        if n is None or n == 0 or n not in wins:
            continue
        what, skip = wins[n] if isinstance(wins[n], tuple) else (wins[n], 0)
        cnt = walk(i, 0, what, 0, skip)  # from the wait itself: its block may be a loop header (latch walks)
        if cnt is None:
            probs.append(f"vmcnt({n}) at instruction {i}: no {what} found before it")
            continue
        if cnt < n:
            probs.append(f"vmcnt({n}) at instruction {i}: only {cnt} vm ops after the {what} it covers")
        found.append(f"vmcnt({n}):{cnt}")
    return probs, found


def check_kernel(name, body):
    ins, labels = parse(body)
    probs = []
    pk = [t for t in ins if re.match(r"v_pk_(fma|mul|add)_f32\b", t)]
    if pk:
        probs.append(f"{len(pk)} packed-FP32 instructions ({pk[0]})")
    if any(c in name for c in COUNTING):
        nsp = sum(1 for t in ins if t.startswith("scratch_"))
        if nsp:
            probs.append(f"{nsp} scratch (spill) instructions in a kernel that counts its own waits")
    probs += check_register_hazards(ins, labels)
    probs += check_store_data(ins)
    windows = []
    for key, wins in WINDOWS.items():
        if key in name:
            p, windows = check_windows(ins, labels, wins)
            probs += p
    return probs, windows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keep", default=None, help="directory for the .s listings (default: a temp dir)")
    a = ap.parse_args()
    out = a.keep or tempfile.mkdtemp()
    os.makedirs(out, exist_ok=True)
    listings = compile_all(out)
    bad = n = 0
    for path in listings:
        asm = open(path).read()
        for name, body in kernels(asm):
            n += 1
            probs, windows = check_kernel(name, body)
            tag = "FAIL" if probs else "ok  "
            if probs or windows:
                print(f"{tag} {os.path.basename(path)} {name[:90]}: {' '.join(windows)}" +
                      ("; " + "; ".join(probs[:4]) if probs else ""))
            bad += bool(probs)
    print(f"{n} kernels checked, {bad} with violations")
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
