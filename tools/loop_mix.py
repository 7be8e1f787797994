"""Static instruction mix of each kernel's MFMA loops in compiled gfx950 assembly.

    python tools/loop_mix.py <file.s> [--kernel SUBSTR] [--top N]

A kernel whose loop issues more than ~2 VALU per 16x16x32 MFMA per wave is VALU-issue bound: an MFMA blocks its
SIMD's vector issue for 8 of its 16 cycles and a VALU op takes 4, so with two waves per SIMD the MFMA pipe is fed
only while VALU <= ~2 x MFMA (MI355X_MICROARCH.md, cycle constants).  For every loop (the basic blocks LLVM's
comments assign to one loop header) that contains MFMAs, prints the per-iteration
counts of MFMA, VALU, SALU, LDS reads / writes and vector-memory instructions.  Round 6 used it to find the
VALU-bound wide weight-gradient and stem weight-gradient kernels (profiles/r6_ab_summary.md).
"""
import argparse
import collections
import re


def loops(body):
    """{header label: [line ranges]}: LLVM labels every basic block of a loop with "; in Loop: Header=BBx_y" (the
    header itself with "=>This Loop Header"); a rotated loop's blocks can sit before or after its header."""
    blocks = collections.defaultdict(list)
    starts = [k for k, l in enumerate(body) if re.match(r"^(\.LBB\w+:|; %bb\.\d+:)", l)] + [len(body)]
    for k, nxt in zip(starts, starts[1:]):
        line = body[k]
        lab = line.split(":")[0].replace("; %", ".%")
        m = re.search(r"Header=(BB\w+)", line)
        if "Loop Header" in line:
            blocks["." + lab[1:] if lab.startswith(".") else lab].append((k, nxt))
        elif m:
            blocks[".L" + m.group(1)].append((k, nxt))
    for lab, rng in blocks.items():
        yield lab, rng


def kind(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("ds_read"):
        return "lds_r"
    if op.startswith("ds_write"):
        return "lds_w"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--top", type=int, default=0)
    a = ap.parse_args()
    s = open(a.asm).read()
    rows = []
    for m in re.finditer(r"^(_ZN3pdt\w+):", s, re.M):
        name = m.group(1)
        if a.kernel not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end].split("\n")
        for lab, rng in loops(body):
            c = collections.Counter()
            for k, e in rng:
                for line in body[k:e]:
                    line = line.strip()
                    if line and line[0] not in ";.":
                        c[kind(line.split()[0])] += 1
            if c["mfma"]:
                rows.append((name, lab, c))
    rows.sort(key=lambda r: -r[2]["valu"] / r[2]["mfma"])
    for name, lab, c in rows[:a.top or None]:
        print(f"{name[:88]:88s} {lab:10s} mfma {c['mfma']:4d} valu {c['valu']:5d} salu {c['salu']:4d} "
              f"lds_r {c['lds_r']:4d} lds_w {c['lds_w']:3d} vmem {c['vmem']:3d}  valu/mfma {c['valu'] / c['mfma']:.2f}")


if __name__ == "__main__":
    main()
