"""Print the kernel sequence of one training step from a rocprofv3 kernel-trace CSV.

    python tools/prof_step.py gpurun_out/prof/run_kernel_trace.csv [--step -1]

Steps are delimited by the fused SGD kernel (one per step).  Shows duration, grid, VGPRs and LDS for
every dispatch so per-layer costs can be read off directly.
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_csv")
    ap.add_argument("--step", type=int, default=-2)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd_kernel" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    st = steps[a.step]
    tot = 0.0
    for r in st:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("pdt::", "")
        grid = f'{int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))}x{r["Grid_Size_Y"]}'
        print(f"{d:9.1f} us  {grid:>12}  v{r['VGPR_Count']:>3}/a{r['Accum_VGPR_Count']:>3} lds{r['LDS_Block_Size']:>6}  {name[:90]}")
    span = (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e6
    print(f"kernel sum {tot / 1e3:.2f} ms, wall span {span:.2f} ms, {len(st)} dispatches")


if __name__ == "__main__":
    main()
