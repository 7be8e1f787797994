"""Cross-stream ordering probe (the suspected cause of the intermittent native-DDP / repeatability mismatches).

Pattern under test, exactly as the executor and the bucketer use it: stream A runs a slow kernel and then writes
a marker into X; an event recorded on A after the write is waited on by stream B; B then reads X.  If the wait is
ever not enforced, B sees the previous marker.  Variants:
  event   : torch Event.record(A) + B.wait_event (torch's wait_stream idiom)
  native  : the C++ communicator's join_compute (hipEventRecord of ONE reused event + hipStreamWaitEvent) followed
            by a host-transport all_reduce of X on the comm stream (world 1: identity; it stages X through the host)
  chain   : A waits on the main stream, main waits on A again later (the executor's _side_wgrad / _join_side)
Prints the number of violations per variant; exit 1 if any.
"""
import argparse
import sys

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--sleep", type=int, default=200000, help="spin cycles before the marker write")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    A = torch.cuda.Stream(device=dev)
    B = torch.cuda.Stream(device=dev)
    X = torch.zeros(1 << 20, device=dev)
    Y = torch.zeros_like(X)
    bad = {"event": 0, "chain": 0}
    for i in range(1, a.iters + 1):
        with torch.cuda.stream(A):
            torch.cuda._sleep(a.sleep)
            X.fill_(float(i))
            ev = torch.cuda.Event()
            ev.record(A)
        B.wait_event(ev)
        with torch.cuda.stream(B):
            Y.copy_(X)
        torch.cuda.synchronize()
        bad["event"] += int(Y[0].item() != i or Y[-1].item() != i)
    main_s = torch.cuda.current_stream(dev)
    for i in range(1, a.iters + 1):
        X.fill_(0.0)                      # main
        A.wait_stream(main_s)
        with torch.cuda.stream(A):
            torch.cuda._sleep(a.sleep)
            X.add_(float(i))              # A reads main's write, then writes
        main_s.wait_stream(A)             # join
        Y.copy_(X)                        # main reads A's write
        torch.cuda.synchronize()
        bad["chain"] += int(Y[0].item() != i)
    try:
        sys.path.insert(0, ".")
        from pytorch_distributed_template_amd.ops import native
        c = native.C.host_communicator(f"/pdt_soc_{torch.randint(0, 1 << 30, (1,)).item()}", 1, 0, 0, True, 8 << 20, 60.0)
        bad["native"] = 0
        for i in range(1, a.iters + 1):
            with torch.cuda.stream(A):
                torch.cuda._sleep(a.sleep)
                X.fill_(float(i))
                c.all_reduce(X, "sum", True)   # join_compute on A, staged through the host on the comm stream
            c.wait()
            torch.cuda.synchronize()
            bad["native"] += int(X[0].item() != i)
        # producer on the legacy default (null) stream -- the stream torch uses as "current" unless told otherwise
        bad["native_null"] = 0
        for i in range(1, a.iters + 1):
            torch.cuda._sleep(a.sleep)
            X.fill_(float(i))
            c.all_reduce(X, "sum", True)
            c.wait()
            torch.cuda.synchronize()
            bad["native_null"] += int(X[0].item() != i)
        bad["native_null_many"] = 0  # many small kernels queued on the null stream before the join
        for i in range(1, a.iters + 1):
            for _ in range(50):
                X.add_(0.0)
            X.fill_(float(i))
            c.all_reduce(X, "sum", True)
            c.wait()
            torch.cuda.synchronize()
            bad["native_null_many"] += int(X[0].item() != i)
    except Exception as e:  # pragma: no cover - diagnostic
        print("native variant skipped:", e)
    print({k: f"{v} violations / {a.iters}" for k, v in bad.items()}, flush=True)
    return 1 if any(bad.values()) else 0


if __name__ == "__main__":
    sys.exit(main())
