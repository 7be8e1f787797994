import os
import sys

import pytest

# every executor work buffer starts as NaN / 0xFF (models/executor.py _buf): a kernel that silently does not run (e.g. a
# refused launch or a dtype branch that skips it) shows up as NaN instead of as a stale buffer's plausible values
os.environ.setdefault("PDT_BUF_POISON", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
