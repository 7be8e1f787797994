"""Per-kernel table (markdown) from a rocprofv3 ``--kernel-trace --stats`` run of bench.py.

    python tools/kernel_table.py gpurun_out/prof/run_kernel_stats.csv --steps 7 --title "..." [--top 45] > profiles/x.md

``--steps`` = the number of training steps the profiled process dispatched (warm-up + timed), so the table is per step.
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_csv")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--title", default="kernel time per step")
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    own = sum(float(r["TotalDurationNs"]) for r in rows if "pdt::" in r["Name"])
    print(f"# {a.title}\n")
    if a.note:
        print(a.note + "\n")
    print(f"- total GPU kernel time: {tot / 1e6:.2f} ms over {a.steps} steps = **{tot / 1e6 / a.steps:.2f} ms/step**")
    print(f"- share of kernel time in this framework's own HIP kernels (`pdt::`): **{100 * own / tot:.1f}%**\n")
    print("| ms/step | calls/step | % | kernel |\n|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        t = float(r["TotalDurationNs"])
        name = re.sub(r"\(.*", "", r["Name"]).strip()
        print(f"| {t / 1e6 / a.steps:.3f} | {int(r['Calls']) / a.steps:g} | {100 * t / tot:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
