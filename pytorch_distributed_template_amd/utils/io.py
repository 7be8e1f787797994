"""Output directory, settings dump and checkpoints (reference: `utils.py:40-62`, `utils.py:114-118`).

Output-dir policy: when ``<outpath>`` exists the reference prompts
``Select Action: d (delete) / q (quit):`` on stdin.  We keep that prompt when stdin is a TTY and
add a non-interactive policy (``--exist-policy`` / ``$PDT_EXIST_POLICY``: ``prompt`` | ``delete`` |
``quit`` | ``reuse``) for automated runs, where an interactive prompt would hang the job.
"""
from __future__ import annotations

import os
import shutil
import sys
from typing import Optional

import torch


def output_process(output_path: str, policy: Optional[str] = None) -> None:
    policy = policy or os.environ.get("PDT_EXIST_POLICY", "prompt")
    if os.path.exists(output_path):
        print("{} file exist!".format(output_path))
        if policy == "prompt":
            if not sys.stdin or not sys.stdin.isatty():
                raise OSError("Directory {} exits! (non-interactive run: pass --exist-policy delete|reuse)"
                              .format(output_path))
            act = input("Select Action: d (delete) / q (quit):").lower().strip()
        else:
            act = {"delete": "d", "quit": "q", "reuse": "r"}.get(policy, "q")
        if act == "d":
            shutil.rmtree(output_path)
        elif act == "r":
            pass
        else:
            raise OSError("Directory {} exits!".format(output_path))
    if not os.path.exists(output_path):
        os.makedirs(output_path)


def write_settings(settings) -> None:
    """``<outpath>/settings.log`` with one ``key: value`` line per argument (`utils.py:54-62`)."""
    with open(os.path.join(settings.outpath, "settings.log"), "w") as f:
        for k, v in settings.__dict__.items():
            f.write(str(k) + ": " + str(v) + "\n")


def _cpu_state_dict(model) -> dict:
    """Contiguous CPU copies with the torchvision key names (no ``module.`` prefix)."""
    m = model.module if hasattr(model, "module") else model
    return {k: v.detach().cpu().contiguous().clone() for k, v in m.state_dict().items()}


def save_checkpoint(state: dict, is_best: bool, outpath: str) -> None:
    """``checkpoint.pth.tar`` every call, copied to ``model_best.pth.tar`` when best (`utils.py:114-118`)."""
    filename = os.path.join(outpath, "checkpoint.pth.tar")
    tmp = filename + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, filename)
    if is_best:
        shutil.copyfile(filename, os.path.join(outpath, "model_best.pth.tar"))


def make_checkpoint_state(epoch: int, arch: str, model, best_acc1, optimizer=None, scaler=None,
                          lr_scheduler=None, extra: Optional[dict] = None) -> dict:
    """Reference schema ``{'epoch', 'arch', 'state_dict', 'best_acc1'}`` (`distributed.py:212-218`);
    ``best_acc1`` is stored as a 0-d CPU tensor fraction.  Optimizer / scaler / scheduler
    state are added under extra keys for ``--resume`` (a superset the reference lacks)."""
    b = best_acc1.detach().float().cpu() if torch.is_tensor(best_acc1) else torch.tensor(float(best_acc1))
    state = {"epoch": int(epoch), "arch": arch, "state_dict": _cpu_state_dict(model), "best_acc1": b.reshape(())}
    if optimizer is not None:
        state["optimizer"] = optimizer.state_dict()
    if scaler is not None and hasattr(scaler, "state_dict"):
        state["scaler"] = scaler.state_dict()
    if lr_scheduler is not None:
        state["lr_scheduler"] = lr_scheduler.state_dict()
    if extra:
        state.update(extra)
    return state


def load_checkpoint(path: str) -> dict:
    """Load a checkpoint with the safe loader (tensors + plain containers only)."""
    return torch.load(path, map_location="cpu", weights_only=True)
