#!/usr/bin/env python
"""Entry point: DDP + AMP (fp16 dynamic loss scaling) + optional SyncBN (reference distributed_syncBN_amp.py).

Argument-compatible with the reference script of the same name; see
pytorch_distributed_template_amd/cli.py for the flag table and pytorch_distributed_template_amd/engine/runner.py
for the training driver.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_distributed_template_amd.engine.runner import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main("ddp_amp"))
