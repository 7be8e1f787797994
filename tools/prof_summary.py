"""Summarise a rocprofv3 ``--kernel-trace --stats --output-format csv`` run into markdown.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv --steps 7 --title "..." > profiles/x.md

``--steps`` = number of training steps inside the profiled region (warmup + timed steps of the bench
run) so per-step milliseconds can be reported.
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_csv")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    ours = sum(float(r["TotalDurationNs"]) for r in rows if "pdt::" in r["Name"])
    print(f"# {a.title}\n")
    print(f"- total GPU kernel time: {tot / 1e6:.2f} ms over {a.steps} steps = **{tot / 1e6 / a.steps:.2f} ms/step**")
    print(f"- share of kernel time in this framework's own HIP kernels (`pdt::`): **{100 * ours / tot:.1f}%**\n")
    print("| ms/step | calls | % | kernel |")
    print("|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        name = re.sub(r"\(.*", "", r["Name"]).replace("|", "\\|")
        print(f"| {float(r['TotalDurationNs']) / 1e6 / a.steps:.3f} | {int(r['Calls'])} | "
              f"{100 * float(r['TotalDurationNs']) / tot:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
