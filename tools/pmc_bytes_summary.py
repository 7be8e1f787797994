"""Per-kernel HBM bytes (FETCH_SIZE / WRITE_SIZE, KiB per dispatch in rocprofv3's derived counters) from the two
passes of tools/pmc_bytes.sh, next to the kernel time of the same dispatches (GRBM_GUI_ACTIVE at 2.4 GHz) and the
implied bandwidth (GRBM_GUI_ACTIVE is summed over the 8 XCDs: divided by 8).  The bench run covers 3 training steps (1 warm-up + 2 timed); per-step numbers divide by 3.

    python tools/pmc_bytes_summary.py gpurun_out/pmc_bytes [--steps 3] [--top 30]
"""
import argparse
import collections
import csv
import glob
import os
import re


def load(path, counter):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    assert f, f"no counter CSV under {path}"
    per = collections.OrderedDict()
    for r in csv.DictReader(open(f[0])):
        per.setdefault((r["Dispatch_Id"], re.sub(r"\(.*", "", r["Kernel_Name"])), {})[r["Counter_Name"]] = \
            float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for (_, name), c in per.items():
        agg[name][counter] += c.get(counter, 0.0)
        agg[name]["cycles"] += c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        agg[name]["n"] += 1
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    a = ap.parse_args()
    fe = load(os.path.join(a.dir, "fetch"), "FETCH_SIZE")
    wr = load(os.path.join(a.dir, "write"), "WRITE_SIZE")
    names = sorted(fe, key=lambda n: -fe[n]["cycles"])
    tot_f = sum(c["FETCH_SIZE"] for c in fe.values()) * 1024 / a.steps
    tot_w = sum(c["WRITE_SIZE"] for c in wr.values()) * 1024 / a.steps
    tot_t = sum(c["cycles"] for c in fe.values()) / (a.clock_ghz * 1e9) / a.steps
    print(f"- HBM bytes per training step: read **{tot_f / 1e9:.2f} GB**, write **{tot_w / 1e9:.2f} GB** "
          f"(kernel time {tot_t * 1e3:.2f} ms/step under counter collection; "
          f"mean {(tot_f + tot_w) / tot_t / 1e12:.2f} TB/s)\n")
    print("| kernel | calls/step | ms/step | read GB/step | write GB/step | TB/s |")
    print("|---|---:|---:|---:|---:|---:|")
    for n in names[:a.top]:
        t = fe[n]["cycles"] / (a.clock_ghz * 1e9) / a.steps
        rb = fe[n]["FETCH_SIZE"] * 1024 / a.steps
        wb = wr.get(n, {}).get("WRITE_SIZE", 0.0) * 1024 / a.steps
        print(f"| `{n[:64]}` | {fe[n]['n'] / a.steps:.0f} | {t * 1e3:.3f} | {rb / 1e9:.3f} | {wb / 1e9:.3f} | "
              f"{(rb + wb) / max(t, 1e-9) / 1e12:.2f} |")


if __name__ == "__main__":
    main()
