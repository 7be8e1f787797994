"""Experiment logger and rank-0 printing (reference: `utils.py:17-37`, `utils.py:72-74`).

File handler ``<outpath>/experiment.log`` with ``'%(asctime)s %(levelname)s: %(message)s'`` and a
stdout handler with ``'%(message)s'``, level INFO -- identical to the reference so log files diff
cleanly.  Unlike the reference, calling :func:`get_logger` twice does not duplicate handlers.
"""
from __future__ import annotations

import logging
import os
import sys
from typing import Optional

FILE_FORMAT = "%(asctime)s %(levelname)s: %(message)s"
CONSOLE_FORMAT = "%(message)s"


def get_logger(save_path: str, logger_name: str) -> logging.Logger:
    logger = logging.getLogger(logger_name)
    for h in list(logger.handlers):
        logger.removeHandler(h)
        h.close()
    file_handler = logging.FileHandler(os.path.join(save_path, "experiment.log"))
    file_handler.setFormatter(logging.Formatter(FILE_FORMAT))
    console_handler = logging.StreamHandler(sys.stdout)
    console_handler.setFormatter(logging.Formatter(CONSOLE_FORMAT))
    logger.addHandler(file_handler)
    logger.addHandler(console_handler)
    logger.setLevel(logging.INFO)
    logger.propagate = False
    return logger


def ddp_print(output, logger: Optional[logging.Logger], rank: int) -> None:
    """Log only on rank 0 (the reference keys this on ``local_rank``; we key on the global rank,
    which is identical on one node -- SURVEY Q7)."""
    if rank == 0 and logger is not None:
        logger.info(output)


def close_logger(logger: Optional[logging.Logger]) -> None:
    if logger is None:
        return
    for h in list(logger.handlers):
        h.flush()
        h.close()
        logger.removeHandler(h)
