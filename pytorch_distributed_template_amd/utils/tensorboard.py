"""Minimal TensorBoard event-file writer (tensorboardX is not installed).

Writes the standard ``events.out.tfevents.<time>.<host>`` TFRecord stream: each record is
``len(u64) | masked_crc32c(len)(u32) | data | masked_crc32c(data)(u32)`` and each payload a hand-encoded
``tensorflow.Event`` protobuf (wall_time=1: double, step=2: int64, file_version=3: string,
summary=5: Summary{value=1: Value{tag=1: string, simple_value=2: float}}).  The reference logs the
per-epoch scalars ``lr``, ``Train_ce_loss``, ``Train_top1_accuracy``, ``Val_ce_loss``,
``Val_top1_accuracy`` with ``global_step=epoch`` (`distributed.py:279-283, 329-332`).
A reader (:func:`read_scalars`) is included for tests.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, List, Tuple


def _make_table():
    poly = 0x82F63B78
    tab = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        tab.append(c)
    return tab


_CRC_TABLE = _make_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int = 0, file_version: str = None, scalars: List[Tuple[str, float]] = ()):
    ev = _key(1, 1) + struct.pack("<d", wall_time)
    if step:
        ev += _key(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _len_field(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, val in scalars:
            v = _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(val))
            summ += _len_field(1, v)
        ev += _len_field(5, summ)
    return ev


class SummaryWriter:
    """Subset of ``tensorboardX.SummaryWriter``: ``add_scalar``, ``flush``, ``close``."""

    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, "events.out.tfevents.{:010d}.{}{}".format(
            int(time.time()), socket.gethostname(), filename_suffix))
        self._f = open(self.path, "wb")
        self._write(encode_event(time.time(), file_version="brain.Event:2"))
        self.flush()

    def _write(self, data: bytes) -> None:
        hdr = struct.pack("<Q", len(data))
        self._f.write(hdr + struct.pack("<I", masked_crc32c(hdr)) + data + struct.pack("<I", masked_crc32c(data)))

    def add_scalar(self, tag: str, scalar_value, global_step: int = None, walltime: float = None) -> None:
        if hasattr(scalar_value, "item"):
            scalar_value = scalar_value.item()
        self._write(encode_event(walltime or time.time(), global_step or 0, scalars=[(tag, float(scalar_value))]))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        if not self._f.closed:
            self._f.flush()
            self._f.close()


# ------------------------------------------------------------------------------------------ reader
def _read_varint(b: bytes, i: int):
    shift = res = 0
    while True:
        c = b[i]
        i += 1
        res |= (c & 0x7F) << shift
        if not c & 0x80:
            return res, i
        shift += 7


def _parse(b: bytes) -> Dict[int, list]:
    out: Dict[int, list] = {}
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v = b[i:i + 8]
            i += 8
        elif w == 5:
            v = b[i:i + 4]
            i += 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError("unsupported wire type")
        out.setdefault(f, []).append(v)
    return out


def read_scalars(path: str, check_crc: bool = True) -> List[Tuple[str, int, float]]:
    """Return ``[(tag, step, value), ...]`` from an event file (verifies record CRCs)."""
    res = []
    with open(path, "rb") as fh:
        data = fh.read()
    i = 0
    while i < len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        payload = data[i + 12:i + 12 + n]
        (pc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if check_crc and (hc != masked_crc32c(hdr) or pc != masked_crc32c(payload)):
            raise ValueError("corrupt event record")
        i += 16 + n
        ev = _parse(payload)
        step = ev.get(2, [0])[0]
        for summ in ev.get(5, []):
            for val in _parse(summ).get(1, []):
                v = _parse(val)
                res.append((v[1][0].decode(), step, struct.unpack("<f", v[2][0])[0]))
    return res
