"""Sampler partition parity with torch.utils.data.DistributedSampler; transforms; ImageFolder; loaders."""
import numpy as np
import pytest
import torch
from PIL import Image
from torch.utils.data import DistributedSampler as TorchDS

from pytorch_distributed_template_amd.data import transforms as T
from pytorch_distributed_template_amd.data.datasets import ImageFolder, SyntheticImageNet
from pytorch_distributed_template_amd.data.sampler import DistributedSampler


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n", [1, 5, 17, 100, 1001])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [False, True])
def test_sampler_matches_torch(n, world, shuffle, drop_last):
    if drop_last and n < world:
        return
    for rank in range(world):
        ours = DistributedSampler(_Len(n), world, rank, shuffle=shuffle, drop_last=drop_last)
        ref = TorchDS(_Len(n), world, rank, shuffle=shuffle, drop_last=drop_last)
        for epoch in (0, 1, 7):
            ours.set_epoch(epoch)
            ref.set_epoch(epoch)
            assert list(ours) == list(ref)
            assert len(ours) == len(ref)


def _img(w=300, h=200, seed=0):
    rng = np.random.default_rng(seed)
    return Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8))


def test_train_val_transforms():
    torch.manual_seed(0)
    x = T.train_transform(224)(_img())
    assert x.shape == (3, 224, 224) and x.dtype == torch.float32
    v = T.val_transform(224)(_img())
    assert v.shape == (3, 224, 224)
    # Resize(256) keeps aspect ratio on the shorter side
    assert T.Resize(256)(_img(300, 200)).size == (384, 256)
    assert T.CenterCrop(224)(_img(384, 256)).size == (224, 224)


def test_normalize_and_totensor():
    img = Image.fromarray(np.full((4, 4, 3), 255, dtype=np.uint8))
    t = T.ToTensor()(img)
    assert torch.allclose(t, torch.ones(3, 4, 4))
    n = T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)(t)
    assert torch.allclose(n[0], torch.full((4, 4), (1 - 0.485) / 0.229))


def test_random_resized_crop_bounds():
    torch.manual_seed(1)
    img = _img(500, 375)
    for _ in range(50):
        i, j, h, w = T.RandomResizedCrop.get_params(img, (0.08, 1.0), (3 / 4, 4 / 3))
        assert 0 <= i and 0 <= j and i + h <= 375 and j + w <= 500 and h > 0 and w > 0


def test_image_folder(tmp_path):
    for ci, cls in enumerate(["b_cls", "a_cls"]):
        d = tmp_path / cls
        d.mkdir()
        for k in range(3):
            _img(40, 30, seed=ci * 10 + k).save(d / f"im{k}.png")
        (d / "notes.txt").write_text("skip me")
    ds = ImageFolder(str(tmp_path), T.val_transform(32, 36))
    assert ds.classes == ["a_cls", "b_cls"] and len(ds) == 6
    x, y = ds[0]
    assert x.shape == (3, 32, 32) and y == 0
    assert ds.targets == [0, 0, 0, 1, 1, 1]


def test_synthetic_deterministic():
    ds = SyntheticImageNet(10, 16, 5, seed=3)
    a, ya = ds[4]
    b, yb = ds[4]
    assert torch.equal(a, b) and ya == yb and a.shape == (3, 16, 16) and 0 <= ya < 5


def test_jpeg_draft_decode_matches_full_decode(tmp_path):
    """--jpeg-draft: a reduced-size DCT decode ahead of RandomResizedCrop / Resize gives the same output size and
    nearly the same pixels as the full decode (crop boxes drawn from the same RNG state)."""
    import numpy as np
    import torch
    from PIL import Image
    from pytorch_distributed_template_amd.data.datasets import lazy_pil_loader, pil_loader
    from pytorch_distributed_template_amd.data.transforms import (RandomResizedCrop, Resize, ToUint8Tensor,
                                                                  _draft)
    rng = np.random.default_rng(0)
    low = rng.integers(0, 256, size=(40, 60, 3)).astype(np.uint8)
    p = str(tmp_path / "big.jpg")
    Image.fromarray(low).resize((1800, 1200), Image.BICUBIC).save(p, quality=92)
    full = ToUint8Tensor()
    for seed in range(4):
        torch.manual_seed(seed)
        a = full(RandomResizedCrop(224)(pil_loader(p))).float()
        torch.manual_seed(seed)
        b = full(RandomResizedCrop(224, draft=True)(lazy_pil_loader(p))).float()
        assert a.shape == b.shape == (3, 224, 224)
        assert (a - b).abs().mean().item() < 6.0  # DCT-domain vs bilinear downscale of a smooth image
    img = lazy_pil_loader(p)
    assert _draft(img, 4.0) == (0.25, 0.25) and img.size == (450, 300)  # header-only until decoded
    r = Resize(256, draft=True)(lazy_pil_loader(p))
    assert min(r.size) == 256
