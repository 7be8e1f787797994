"""Outline a kernel's main structure from a hipcc ``-S`` listing: barriers, waits, branches and
setprio, with the MFMA / ds_read / LDS-DMA counts between them.

    python tools/isa_outline.py /tmp/cf.s <mangled-kernel-name-substring> [--max 200]
"""
import argparse


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--max", type=int, default=200)
    a = ap.parse_args()
    s = open(a.asm).read()
    start = next(i for i in range(len(s)) if s.startswith(a.kernel, i) and s[i + len(a.kernel):].startswith(":"))
    body = s[start:s.index(".Lfunc_end", start)].split("\n")
    cnt = {"mfma": 0, "ds_read": 0, "dma": 0, "valu": 0}
    out = []
    for line in body:
        t = line.strip()
        if t.startswith("v_mfma"):
            cnt["mfma"] += 1
        elif t.startswith("ds_read"):
            cnt["ds_read"] += 1
        elif t.startswith("buffer_load") and "lds" in t:
            cnt["dma"] += 1
        elif t.startswith("v_"):
            cnt["valu"] += 1
        elif t.startswith(("s_barrier", "s_waitcnt", "s_cbranch", ".LBB", "s_setprio", "s_branch", "s_endpgm")):
            if any(cnt.values()):
                out.append("    [" + " ".join(f"{k} {v}" for k, v in cnt.items() if v) + "]")
                cnt = {k: 0 for k in cnt}
            out.append(t)
    print("\n".join(out[:a.max]))


if __name__ == "__main__":
    main()
