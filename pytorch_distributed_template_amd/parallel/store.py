"""Native TCP rendezvous store (csrc/store.cpp) -- counterpart of c10d ``TCPStore``.

``NativeStore.from_env()`` follows the launcher's env:// contract (``MASTER_ADDR``, ``MASTER_PORT``,
``RANK``, ``WORLD_SIZE``): rank 0 hosts the server, every rank connects as a client.  The native store
listens on ``MASTER_PORT + 1`` by default (``PDT_STORE_PORT`` overrides) so it can coexist with
torch.distributed's own store on ``MASTER_PORT``.  It is what ``--comm native`` uses to exchange the
RCCL unique id when torch.distributed is not initialised, and it works on CPU-only hosts (the store
is plain sockets + threads; only the communicator needs a GPU).
"""
from __future__ import annotations

import os
from typing import Optional

from ..ops import native


class NativeStore:
    def __init__(self, host: str, port: int, rank: int, world: int, timeout_s: float = 300.0):
        self.rank, self.world = rank, world
        self._impl = native.C.TCPStore(host, port, rank == 0, timeout_s)
        self._barriers = 0

    @classmethod
    def from_env(cls, timeout_s: float = 300.0, port: Optional[int] = None) -> "NativeStore":
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("PDT_STORE_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        return cls(host, port, int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), timeout_s)

    @property
    def port(self) -> int:
        return self._impl.port

    def set(self, key: str, value: bytes) -> None:
        self._impl.set(key, bytes(value))

    def get(self, key: str, timeout_s: float = -1.0) -> bytes:
        return bytes(self._impl.get(key, timeout_s))

    def add(self, key: str, delta: int) -> int:
        return self._impl.add(key, delta)

    def check(self, key: str) -> bool:
        return self._impl.check(key)

    def delete_key(self, key: str) -> None:
        self._impl.delete_key(key)

    def barrier(self) -> None:
        """All ``world`` ranks arrive; every call site must be reached by every rank in the same order."""
        self._barriers += 1
        self._impl.barrier(f"__barrier_{self._barriers}", self.world)
