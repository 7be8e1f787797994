"""Per-kernel PMC summary of a rocprofv3 ``--pmc`` counter-collection CSV (tools/pmc_step.sh).

    python tools/pmc_summary.py gpurun_out/pmc_step/run/run_counter_collection.csv [--top 40]

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); wait / stall / active are the
SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY shares of SQ_WAVE_CYCLES.  Aggregated per kernel
name (dispatches summed), sorted by GPU time (GRBM_GUI_ACTIVE/8 cycles).
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    per = collections.OrderedDict()
    for r in csv.DictReader(open(a.csv)):
        per.setdefault((r["Dispatch_Id"], re.sub(r"\(.*", "", r["Kernel_Name"])), {})[r["Counter_Name"]] = \
            float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for (_, name), c in per.items():
        for k, v in c.items():
            agg[name][k] += v
        agg[name]["n"] += 1
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"])
    tot = sum(c["GRBM_GUI_ACTIVE"] for _, c in rows)
    print("| kernel | calls | % time | MFMA busy | wait | issue stall | active | LDS conflict |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for name, c in rows[:a.top]:
        g = c["GRBM_GUI_ACTIVE"]
        wc = max(c["SQ_WAVE_CYCLES"], 1.0)
        print(f"| `{name[:70]}` | {int(c['n'])} | {100 * g / tot:.1f} | "
              f"{100 * c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(g / 8 * 1024, 1):.1f}% | {c['SQ_WAIT_ANY'] / wc:.2f} | "
              f"{c['SQ_WAIT_INST_ANY'] / wc:.2f} | {c['SQ_ACTIVE_INST_ANY'] / wc:.2f} | "
              f"{c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f} |")


if __name__ == "__main__":
    main()
