"""Shared model / batch construction for the DDP numerics tests and their rank script."""
import torch


def make_model(seed: int = 0, arch: str = "resnet18"):
    from pytorch_distributed_template_amd.models import registry
    torch.manual_seed(seed)
    model = registry.create(arch)
    g = torch.Generator().manual_seed(seed + 7)
    for m in model.modules():  # non-trivial BN affine parameters, so their gradients matter
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
                m.bias.copy_(torch.rand(m.bias.shape, generator=g) * 0.4 - 0.2)
    return model


def make_batch(n: int, hw: int, seed: int = 1234):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 3, hw, hw, generator=g), torch.randint(0, 1000, (n,), generator=g)


def dp_oracle(x, t, n_shards: int, steps: int, dtype=torch.bfloat16, seed: int = 0):
    """Single-executor oracle of native DataParallel over ``n_shards`` replicas (nn.DataParallel semantics,
    `dataparallel.py:119`): per step each shard's gradient (its own BN batch statistics, loss divided by the NODE
    batch) is summed in replica order onto the master, the running statistics come from shard 0 only,
    num_batches_tracked advances by one, then one SGD step.  Returns the trainer (its flat / buffers hold the
    state after ``steps``), the per-step [loss, acc] and the eval logits of each shard concatenated."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    tr = NativeTrainer(make_model(seed=seed), x.device, dtype=dtype)
    B = x.shape[0]
    bounds = [(int(c[0]), int(c[-1]) + 1) for c in torch.tensor_split(torch.arange(B), n_shards)]
    mets = []
    for _ in range(steps):
        f_before = tr.buffers.fdata.clone()
        acc, f0, met = None, None, 0
        for k, (lo, hi) in enumerate(bounds):
            tr.buffers.fdata.copy_(f_before)
            _, m = tr.executor.train_step(x[lo:hi], t[lo:hi], grad_div=float(B))
            met = met + m * ((hi - lo) / B)
            if k == 0:
                f0 = tr.buffers.fdata.clone()
                acc = tr.flat.grad.clone()
            else:
                acc.add_(tr.flat.grad)
        tr.flat.grad.copy_(acc)
        tr.buffers.fdata.copy_(f0)
        tr.buffers.idata.add_(1)
        tr.optimizer.step()
        mets.append(met)
    logits = torch.cat([tr.executor.eval_step(x[lo:hi], t[lo:hi])[0] for lo, hi in bounds])
    return tr, torch.stack(mets), logits
