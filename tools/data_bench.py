"""Real-data input pipeline throughput (reference C16-C18: ImageFolder + RandomResizedCrop/flip/ToTensor/
Normalize through DataLoader workers, `distributed.py:157-179`).

Generates an ImageFolder of JPEGs with ImageNet-like sizes and content statistics (smooth low-frequency
structure + sensor-like noise, quality 90; no dataset download is possible here), then measures loader
images/s for several worker counts and pipeline variants:

  ref        reference pipeline: float32 ToTensor + Normalize on the CPU
  u8         --gpu-normalize: uint8 samples, normalisation fused into the native stem kernel on the GPU
  u8+draft   u8 plus --jpeg-draft (libjpeg DCT-scaled decode ahead of the crop)

    python tools/data_bench.py [--n 1536] [--workers 1,2,4,8] [--batch 128] [--md out.md]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_jpegs(root: str, n: int, classes: int = 8, seed: int = 0) -> None:
    from PIL import Image
    rng = np.random.default_rng(seed)
    done = os.path.join(root, f".done_{n}")
    if os.path.exists(done):
        return
    for c in range(classes):
        os.makedirs(os.path.join(root, "train", f"c{c:03d}"), exist_ok=True)
    sizes = [(500, 375), (500, 333), (375, 500), (500, 400), (640, 480), (333, 500), (500, 500), (400, 300)]
    for i in range(n):
        w, h = sizes[rng.integers(len(sizes))]
        low = rng.integers(0, 256, size=(max(2, h // 32), max(2, w // 32), 3)).astype(np.uint8)
        img = Image.fromarray(low).resize((w, h), Image.BICUBIC)
        arr = np.asarray(img).astype(np.int16) + rng.normal(0, 8, size=(h, w, 3)).astype(np.int16)
        img = Image.fromarray(np.clip(arr, 0, 255).astype(np.uint8))
        img.save(os.path.join(root, "train", f"c{i % classes:03d}", f"img{i:06d}.jpg"), quality=90)
    open(done, "w").close()


def measure(root: str, variant: str, workers: int, batch: int, batches: int) -> float:
    import torch
    from torch.utils.data import DataLoader
    from pytorch_distributed_template_amd.data.datasets import ImageFolder, lazy_pil_loader, pil_loader
    from pytorch_distributed_template_amd.data.transforms import train_transform
    u8 = variant != "ref"
    draft = variant == "u8+draft"
    ds = ImageFolder(os.path.join(root, "train"), train_transform(224, gpu_normalize=u8, draft=draft),
                     loader=lazy_pil_loader if draft else pil_loader)
    dl = DataLoader(ds, batch_size=batch, shuffle=True, num_workers=workers, persistent_workers=False,
                    prefetch_factor=4 if workers else None)
    it = iter(dl)
    next(it)  # worker start-up + first batch
    t0 = time.perf_counter()
    n = 0
    for _ in range(batches):
        x, _ = next(it)
        n += x.shape[0]
    dt = time.perf_counter() - t0
    del it, dl
    torch.set_num_threads(torch.get_num_threads())
    return n / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/pdt_jpegs")
    ap.add_argument("--n", type=int, default=1536)
    ap.add_argument("--workers", default="1,2,4,8")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--batches", type=int, default=0, help="timed batches (0: one pass over the files)")
    ap.add_argument("--variants", default="ref,u8,u8+draft")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    import torch
    torch.set_num_threads(1)
    make_jpegs(a.dir, a.n)
    rows = []
    for v in a.variants.split(","):
        for w in [int(x) for x in a.workers.split(",")]:
            nb = a.batches or max(2, a.n // a.batch - 2)
            ips = measure(a.dir, v, w, a.batch, nb)
            r = {"variant": v, "workers": w, "img_per_s": round(ips, 1), "img_per_s_per_worker": round(ips / max(w, 1), 1),
                 "cpus": os.cpu_count()}
            rows.append(r)
            print(json.dumps(r), flush=True)
    if a.md:
        with open(a.md, "w") as f:
            f.write("| variant | workers | img/s | img/s per worker |\n|---|---:|---:|---:|\n")
            for r in rows:
                f.write(f"| {r['variant']} | {r['workers']} | {r['img_per_s']} | {r['img_per_s_per_worker']} |\n")


if __name__ == "__main__":
    main()
