"""Diagnostic: native-communicator DDP (2 ranks sharing cuda:0, host shared-memory transport) vs c10d/gloo DDP on
the same inputs -- per-rank initial parameters after the constructor broadcast, each bucket's LOCAL gradient
just before its all-reduce, and the all-reduced gradient, compared slot by slot."""
import os
import sys
import tempfile

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
sys.path.insert(0, os.path.dirname(HERE))
import test_ddp_numerics_gpu as T  # noqa: E402
from pytorch_distributed_template_amd.models import registry  # noqa: E402
from pytorch_distributed_template_amd.optim.flat import FlatParams  # noqa: E402


class _P:
    def __init__(self, d):
        self.d = d

    def __truediv__(self, o):
        return os.path.join(self.d, o)


def main():
    flat = FlatParams(registry.create("resnet18"), "cpu")
    out = {}
    for comm in ("torch", "native"):
        d = tempfile.mkdtemp()
        T._run_ranks(_P(d), PDT_TEST_SYNCBN=0, PDT_TEST_STEPS=1, PDT_TEST_COMM=comm, PDT_TEST_SAVE_LOCAL=1)
        out[comm] = [torch.load(os.path.join(d, f"rank0.pt.r{r}"), weights_only=True) for r in range(2)]
    for r in range(2):
        for key in ("init", "local", "grad"):
            a, b = out["torch"][r][key], out["native"][r][key]
            bad = [s.name for s in flat.slots if not torch.equal(a[s.offset:s.offset + s.numel],
                                                                 b[s.offset:s.offset + s.numel])]
            print(f"rank {r} {key}: {len(bad)} slots differ {bad[:6]}", flush=True)
    i0, i1 = out["native"][0]["init"], out["native"][1]["init"]
    print("native init rank0 == rank1:", torch.equal(i0, i1), flush=True)


if __name__ == "__main__":
    main()
