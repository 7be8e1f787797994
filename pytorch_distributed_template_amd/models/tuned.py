"""Shipped per-shape conv tile tables (the analogue of a ``cudnn.benchmark`` cache, `distributed.py:104`).

``load_table`` reads one JSON table ``{"note": ..., "tiles": [[key, tile], ...]}``.  A SHIPPED table that is
missing or malformed is a silent multi-millisecond regression (every shape falls back to the static rule), so it
warns -- once per path -- instead of passing quietly; extra tables (``PDT_TUNED_EXTRA``) are the user's own.
"""
from __future__ import annotations

import json
import os
import warnings
from typing import Dict, Optional, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
TABLE16 = os.path.join(HERE, "tuned_tiles_mi355x.json")
TABLE32 = os.path.join(HERE, "tuned_tiles32_mi355x.json")
# key arity per table and kind (ResNetExecutor._tile keys / ResNetExecutor32._tile32c keys)
ARITY16 = {"fwd": 10, "dgrad": 12}
ARITY32 = {"fwd": 7, "dgrad": 7}
_warned = set()


def load_table(path: str, arity: Optional[Dict[str, int]] = None, shipped: bool = True) -> Dict[Tuple, Tuple]:
    try:
        with open(path) as f:
            rows = json.load(f)["tiles"]
        out = {}
        for k, v in rows:
            k, v = tuple(k), tuple(v)
            if arity is not None and arity.get(k[0]) != len(k):
                raise ValueError(f"key {k} has {len(k)} fields, expected {arity.get(k[0])}")
            if len(v) != 2:
                raise ValueError(f"tile {v} for {k} is not (bm, bn)")
            out[k] = v
        return out
    except (OSError, ValueError, KeyError, TypeError) as e:
        if shipped and path not in _warned:
            _warned.add(path)
            warnings.warn(f"shipped conv tile table {path} could not be loaded ({e}); using the static tile rule "
                          "for every shape (slower)", RuntimeWarning, stacklevel=2)
        return {}
