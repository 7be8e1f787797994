"""Where is the GPU idle inside a training step?  Reads a rocprofv3 kernel-trace CSV of the OVERLAPPED
(two-stream) bench run and, per step, reports the wall time, the union of kernel-busy intervals and the
largest idle gaps with the kernels on either side.

    python tools/timeline_gaps.py gpurun_out/prof/run_kernel_trace.csv [--step -2] [--gaps 15]

Steps are delimited by the fused SGD kernel (one per step).  A gap is a time span covered by no kernel on
any stream: host launch latency, a cross-stream event wait that left both streams empty, or a blocking host
synchronisation.
"""
import argparse
import csv
import re


def _name(r):
    return re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("pdt::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_csv")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--gaps", type=int, default=15)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd_kernel" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    print(f"{len(steps)} steps in trace")
    for si in range(len(steps)):
        st = steps[si]
        iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in st]
        t0 = iv[0][0] if si == 0 else int(steps[si - 1][-1]["End_Timestamp"])
        t1 = max(e for _, e, _ in iv)
        busy, gaps, end, prev = 0, [], t0, (steps[si - 1][-1] if si else None)
        for s, e, r in iv:
            if s > end:
                gaps.append((s - end, prev, r))
            if e > end:
                busy += e - max(s, end)
                end = e
                prev = r
        ksum = sum(e - s for s, e, _ in iv)
        print(f"step {si}: wall {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(t1 - t0 - busy) / 1e6:.3f} ms"
              f"  kernel-sum {ksum / 1e6:.3f} ms  kernels {len(iv)}")
        if si == (a.step % len(steps)):
            gaps.sort(key=lambda g: -g[0])
            for d, p, r in gaps[:a.gaps]:
                print(f"    gap {d / 1e3:8.1f} us  after {_name(p) if p else '<trace start>':60s} before {_name(r)}")


if __name__ == "__main__":
    main()
