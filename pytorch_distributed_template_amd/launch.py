"""torchrun-style launcher (reference C01: ``python -m torch.distributed.launch --nproc_per_node=3
--master_port=23334 <script>``, `start.sh:3-4`).

    python -m pytorch_distributed_template_amd.launch [--nproc_per_node N] [--nnodes M --node_rank R]
        [--master_addr A] [--master_port P] [--no_local_rank] script.py [script args...]

Environment contract for every child (same as the upstream launchers): ``MASTER_ADDR``,
``MASTER_PORT``, ``WORLD_SIZE``, ``RANK``, ``LOCAL_RANK``, ``LOCAL_WORLD_SIZE``; the legacy
``--local_rank=<i>`` argument is appended unless ``--no_local_rank`` is given (SURVEY Q5 -- our
entry scripts accept both spellings and the env variable).

Failure handling (the reference has none): the launcher polls its children; if any exits
non-zero, the remaining ones are terminated (SIGTERM, then SIGKILL after a grace period) so a crashed
rank cannot leave the others hanging in a collective, and the launcher exits with that code.
``--max_restarts`` re-launches the whole group after a failure (simple elastic-style retry).
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time
from typing import List


def parse(argv=None):
    p = argparse.ArgumentParser(description="Launch one process per GPU (torch.distributed env contract)")
    p.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=1)
    p.add_argument("--nnodes", type=int, default=1)
    p.add_argument("--node_rank", "--node-rank", type=int, default=0)
    p.add_argument("--master_addr", "--master-addr", default="127.0.0.1")
    p.add_argument("--master_port", "--master-port", type=int, default=29500)
    p.add_argument("--no_local_rank", "--no-local-rank", "--use_env", "--use-env", action="store_true",
                   help="do not append --local_rank=<i> (children read LOCAL_RANK from the env)")
    p.add_argument("--max_restarts", type=int, default=0)
    p.add_argument("--grace_s", type=float, default=10.0)
    p.add_argument("--module", "-m", action="store_true", help="run the target as a python module")
    p.add_argument("script")
    p.add_argument("script_args", nargs=argparse.REMAINDER)
    return p.parse_args(argv)


def _spawn(a) -> List[subprocess.Popen]:
    world = a.nnodes * a.nproc_per_node
    procs = []
    for local in range(a.nproc_per_node):
        rank = a.node_rank * a.nproc_per_node + local
        env = dict(os.environ, MASTER_ADDR=a.master_addr, MASTER_PORT=str(a.master_port), WORLD_SIZE=str(world),
                   RANK=str(rank), LOCAL_RANK=str(local), LOCAL_WORLD_SIZE=str(a.nproc_per_node),
                   GROUP_RANK=str(a.node_rank))
        # ROCm IPC: hosts whose amdgpu driver only supports dmabuf-based IPC need the non-legacy mode, otherwise RCCL's
        # intra-node transport (and CUDA-tensor sharing between processes) fails with `hipIpcGetMemHandle: invalid
        # argument`.  setdefault: an explicit user setting wins.
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        cmd = [sys.executable, "-u"] + (["-m", a.script] if a.module else [a.script])
        if not a.no_local_rank:
            cmd.append(f"--local_rank={local}")
        cmd += a.script_args
        procs.append(subprocess.Popen(cmd, env=env))
    return procs


def _terminate(procs, grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t0 = time.time()
    while time.time() - t0 < grace and any(p.poll() is None for p in procs):
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.kill()
    for p in procs:
        p.wait()


def run(a) -> int:
    attempt = 0
    while True:
        procs = _spawn(a)
        rc = 0
        try:
            while True:
                done = [p for p in procs if p.poll() is not None]
                bad = [p for p in done if p.returncode != 0]
                if bad:
                    rc = bad[0].returncode
                    sys.stderr.write(f"[launch] rank process exited with code {rc}; terminating the group\n")
                    _terminate(procs, a.grace_s)
                    break
                if len(done) == len(procs):
                    break
                time.sleep(0.2)
        except KeyboardInterrupt:
            _terminate(procs, a.grace_s)
            return 130
        if rc == 0 or attempt >= a.max_restarts:
            return rc
        attempt += 1
        sys.stderr.write(f"[launch] restart {attempt}/{a.max_restarts}\n")


def main(argv=None) -> int:
    return run(parse(argv))


if __name__ == "__main__":
    sys.exit(main())
