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


# Counted waits whose SHORTEST layout path is known to be short by design, per kernel-name substring and wait count,
# with the run-time guard that makes that path infeasible (round-6 review: explicit annotations instead of taking the
# longest path everywhere).  Every other designated wait must hold on EVERY path (the shortest).  An annotation that
# no compiled kernel needs any more is itself reported (stale), so the list cannot silently cover a new short path.
_FIRST = "the first tile skips this wait (flag `first`); the walk's short path enters it from the kernel prologue"
_TAIL = ("only a walker's LAST tile can be the partial M tail, whose stores are exec-masked, so no wait follows the "
         "short store sequence")
GUARDED = {
    # conv_l1.hip: n_st (4 stores per pixel group of the PREVIOUS tile) selects vmcnt(12 | 16); the first tile of a
    # block and a tile behind no stores take vmcnt(0)
    "conv_l1_kernel": {12: "n_st == 12: " + _FIRST, 16: "n_st == 16: " + _FIRST},
    # stem.hip: stores_behind is false (vmcnt(0)) for the first tile and after an epilogue with fewer stores
    "stem_fwd_kernel": {14: "stores_behind: " + _FIRST},
    # conv1x1.hip / conv1x1x.hip persistent walkers: the loop-top / sub-tile waits count the previous tile's stores
    "conv1x1_c64_kernel": {16: _FIRST + "; " + _TAIL},
    "conv1x1_c64_bnb_kernel": {32: _FIRST + "; " + _TAIL, 40: _FIRST + "; " + _TAIL},
    "conv1x1x_kernel": {2: _FIRST + "; " + _TAIL, 4: _FIRST + "; " + _TAIL, 8: _FIRST + "; " + _TAIL},
    "conv1x1x_bnb_kernel": {n: _FIRST + "; sub-tile s == 0 after the prologue's operand loads; " + _TAIL
                            for n in (8, 12, 16, 24)},
}


def check_windows(ins, labels, wins, name="", used=None):
    """Designated counted waits (module docstring, check 2).  Walking back from the wait in layout order, a label that
    is the target of backward branches (a loop header / latch block) may continue from any of those branches ("the
    previous iteration") or fall through (the first iteration).  The window of a wait is the SMALLEST count over these
    walks, so a short path into a counted wait fails the check -- unless the kernel annotates that wait in GUARDED
    (a first / last tile whose run-time flag selects ``vmcnt(0)`` or skips the stores the count relies on), in which
    case the largest count (the steady-state path) must still cover it.  ``used`` collects the annotations applied."""
    latches = {}
    for j, t in enumerate(ins):
        b = branch(t)
        if b is not None and b[1] in labels and labels[b[1]] <= j:
            latches.setdefault(labels[b[1]], set()).add(j)

    def walk(j, cnt, what, depth, skip=0):
        """-> (min, max) count over the walks from ``j`` back to the covered operation, or None.  ``skip``: the
        youngest ``skip`` matching operations are the group the wait leaves in flight (ring pipelines); the window is
        measured from the one before them."""
        lo = hi = None

        def add(r):
            nonlocal lo, hi
            if r is None:
                return
            lo = r[0] if lo is None else min(lo, r[0])
            hi = r[1] if hi is None else max(hi, r[1])
        while j >= 0:
            u = ins[j]
            if (what == "dma" and is_dma(u)) or (what == "load" and is_vm(u) and "load" in u.split()[0]
                                                 and not u.endswith(" lds")):
                if skip == 0:
                    add((cnt, cnt))
                    return (lo, hi)
                skip -= 1
            if is_vm(u):
                cnt += 1
            if j in latches and depth < 4:
                for l in latches[j]:
                    add(walk(l, cnt, what, depth + 1, skip))
            j -= 1
        return None if lo is None else (lo, hi)

    guarded = {}
    for key, g in GUARDED.items():
        if key in name:
            guarded.update({n: (key, why) for n, why in g.items()})
    probs, found = [], []
    for i, t in enumerate(ins):
        n = vm_wait(t)
        if n is None or n == 0 or n not in wins:
            continue
        what, skip = wins[n] if isinstance(wins[n], tuple) else (wins[n], 0)
        r = walk(i, 0, what, 0, skip)  # from the wait itself: its block may be a loop header (latch walks)
        if r is None:
            probs.append(f"vmcnt({n}) at instruction {i}: no {what} found before it")
            continue
        lo, hi = r
        if lo < n and n in guarded:
            if used is not None:
                used.add((guarded[n][0], n))
            lo = hi  # annotated: the short path is guarded at run time (GUARDED)
        if lo < n:
            probs.append(f"vmcnt({n}) at instruction {i}: only {lo} vm ops after the {what} it covers on the shortest "
                         f"path (longest {hi})")
        found.append(f"vmcnt({n}):{lo}")
    return probs, found


def check_kernel(name, body, used=None):
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
            p, windows = check_windows(ins, labels, wins, name, used)
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
    used = set()
    for path in listings:
        asm = open(path).read()
        for name, body in kernels(asm):
            n += 1
            probs, windows = check_kernel(name, body, used)
            tag = "FAIL" if probs else "ok  "
            if probs or windows:
                print(f"{tag} {os.path.basename(path)} {name[:90]}: {' '.join(windows)}" +
                      ("; " + "; ".join(probs[:4]) if probs else ""))
            bad += bool(probs)
    stale = sorted((k, w) for k, g in GUARDED.items() for w in g if (k, w) not in used)
    for k, w in stale:
        print(f"FAIL stale GUARDED annotation {k} vmcnt({w}): no compiled kernel has a short path into it any more")
    print(f"{n} kernels checked, {bad} with violations, {len(stale)} stale annotations")
    return 1 if bad or stale or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
