#!/usr/bin/env python
"""Entry point: nn.DataParallel single-process multi-GPU data parallel (reference dataparallel.py).

Argument-compatible with the reference script of the same name; see
pytorch_distributed_template_amd/cli.py for the flag table and pytorch_distributed_template_amd/engine/runner.py
for the training driver.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_distributed_template_amd.engine.runner import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main("dp"))
