"""Native TCP rendezvous store (csrc/store.cpp) across processes on CPU: env:// contract, set/get
(blocking), atomic add, barriers, timeouts -- the rendezvous that ``--comm native`` uses to exchange
the RCCL unique id (SURVEY §2.4 X1, §4 layer 2)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1), RANK=str(rank), WORLD_SIZE=str(world))
    from pytorch_distributed_template_amd.parallel.store import NativeStore
    st = NativeStore.from_env(timeout_s=30.0)
    assert st.port == port
    # rank 0 publishes a 128-byte "unique id", everybody blocks on it (published after a delay)
    if rank == 0:
        import time
        time.sleep(0.3)
        st.set("uid", bytes(range(128)))
    uid = st.get("uid")
    # every rank contributes to a counter; after the barrier all see the total
    st.add("count", rank + 1)
    st.barrier()
    total = st.add("count", 0)
    st.set(f"from_{rank}", str(rank * rank).encode())
    st.barrier()
    others = [int(st.get(f"from_{r}")) for r in range(world)]
    st.barrier()  # keep the server (rank 0) alive until everyone has read
    q.put((rank, uid == bytes(range(128)), total, others))


def test_native_store_rendezvous_four_ranks():
    from pytorch_distributed_template_amd.ops import native
    native.load(build=False)
    world, port = 4, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, uid_ok, total, others in res:
        assert uid_ok
        assert total == sum(range(1, world + 1))
        assert others == [r * r for r in range(world)]


def test_native_store_timeout_and_check():
    sys.path.insert(0, ROOT)
    from pytorch_distributed_template_amd.parallel.store import NativeStore
    st = NativeStore("127.0.0.1", 0, 0, 1, timeout_s=5.0)
    assert not st.check("k")
    st.set("k", b"v")
    assert st.check("k") and st.get("k") == b"v"
    st.delete_key("k")
    assert not st.check("k")
    with pytest.raises(RuntimeError, match="timed out"):
        st.get("never", timeout_s=0.2)
    assert st.add("c", 5) == 5 and st.add("c", -2) == 3
    st.barrier()  # world 1: returns immediately


def _barrier_worker(rank, world, port, rounds, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1), RANK=str(rank), WORLD_SIZE=str(world))
    from pytorch_distributed_template_amd.parallel.store import NativeStore
    st = NativeStore.from_env(timeout_s=30.0)
    for _ in range(rounds):
        st.barrier()
    q.put(rank)
    # rank 0 (the server) returns from the last barrier and tears its store down at once: its destructor must
    # linger until every client's last request -- possibly the SET that released it -- has been answered


def test_native_store_barrier_teardown():
    """Back-to-back barriers, the server exiting right after the last one (any rank may be the last arriver
    whose releasing SET races the server's teardown): every rank completes and exits 0."""
    from pytorch_distributed_template_amd.ops import native
    native.load(build=False)
    world, rounds, port = 6, 12, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_barrier_worker, args=(r, world, port, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    done = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert done == list(range(world))
