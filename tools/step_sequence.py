"""One training step's dispatch sequence from a rocprofv3 ``--kernel-trace`` CSV (serial run, PDT_WGRAD_STREAM=0).

    python tools/step_sequence.py gpurun_out/profs/run_kernel_trace.csv [--step -2] > profiles/x.txt

A step is delimited by the fused SGD kernel (``sgd_kernel``); ``--step`` picks one (Python index, default the
second-to-last complete step).  Prints start offset, duration, grid and the shortened kernel name per dispatch, then
the per-step total, so each kernel can be mapped to its layer by position.
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("pdt::", "")
    return name[:90]


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
    t0 = int(st[0]["Start_Timestamp"])
    tot = 0
    for r in st:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        tot += e - s
        grid = f'{r.get("Grid_Size_X", "")}x{r.get("Grid_Size_Y", "")}'
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {grid:>14}  {short(r['Kernel_Name'])}")
    print(f"# {len(st)} dispatches, kernel time {tot / 1e6:.3f} ms, wall {(int(st[-1]['End_Timestamp']) - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
