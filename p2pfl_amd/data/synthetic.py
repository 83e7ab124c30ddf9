"""Synthetic, learnable image-classification datasets.

There is no network on the build or GPU boxes, so the reference's torchvision
MNIST download (``mnistfederated_dm.py:85-101``) is replaced by deterministic
synthetic data of the same shapes.  Each class has a smooth random prototype
stroke-like image (zero background); a sample is its class prototype under a
weaker distractor prototype of another class, a random contrast,
multiplicative stroke noise, a faint background and a per-sample random
translation, stored as ``uint8`` like MNIST.  Models reach
high accuracy on it, so convergence tests are meaningful, and the same seed
gives bit-identical data on every peer.

If ``P2PFL_MNIST_DIR`` points at the four classic IDX files
(``train-images-idx3-ubyte[.gz]`` ...), real MNIST is read instead (plain
byte parsing, nothing executed).
"""

from __future__ import annotations

import gzip
import os
import threading
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch

SPECS: Dict[str, Tuple[Tuple[int, int, int], int, int, int]] = {
    # name: ((C, H, W), classes, n_train, n_test)
    "mnist": ((1, 28, 28), 10, 60000, 10000),
    "cifar10": ((3, 32, 32), 10, 50000, 10000),
    "imagenet": ((3, 224, 224), 1000, 12800, 1000),
}


@dataclass
class ImageSet:
    x: torch.Tensor  # uint8 [N, C, H, W]
    y: torch.Tensor  # int64 [N]

    def __len__(self) -> int:
        return int(self.y.shape[0])


def _prototypes(shape: Tuple[int, int, int], classes: int, g: torch.Generator) -> torch.Tensor:
    """Sparse, stroke-like class prototypes in [0, 1] (background exactly 0, like MNIST)."""
    c, h, w = shape
    low = torch.rand(classes, c, max(2, h // 4), max(2, w // 4), generator=g)
    protos = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=False)
    flat = protos.reshape(classes, -1)
    lo = torch.quantile(flat, 0.70, dim=1).view(classes, 1, 1, 1)
    hi = flat.amax(dim=1).view(classes, 1, 1, 1)
    return ((protos - lo) / (hi - lo + 1e-6)).clamp(min=0.0)


def make_split(
    shape: Tuple[int, int, int], classes: int, n: int, seed: int, protos: torch.Tensor, chunk: int = 8192
) -> ImageSet:
    """Samples = prototype x random contrast + stroke noise, translated by a per-sample random shift."""
    g = torch.Generator().manual_seed(seed)
    c, h, w = shape
    y = torch.randint(0, classes, (n,), generator=g)
    x = torch.empty((n, c, h, w), dtype=torch.uint8)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        yy = y[s:e]
        # the true class prototype plus a weaker distractor of another class
        other = (yy + torch.randint(1, classes, (e - s,), generator=g)) % classes
        mix = 0.75 * torch.rand(e - s, 1, 1, 1, generator=g)
        img = protos[yy] + mix * protos[other]
        contrast = 0.5 + 0.5 * torch.rand(e - s, 1, 1, 1, generator=g)
        img = img * contrast * (0.5 + torch.rand(img.shape, generator=g))
        img = img + 0.1 * torch.rand(img.shape, generator=g)
        shifts = torch.randint(-2, 3, (e - s, 2), generator=g)
        code = (shifts[:, 0] + 2) * 5 + (shifts[:, 1] + 2)
        for k in torch.unique(code).tolist():
            sel = code == k
            img[sel] = torch.roll(img[sel], shifts=(k // 5 - 2, k % 5 - 2), dims=(2, 3))
        x[s:e] = (img.clamp(0, 1) * 255).to(torch.uint8)
    return ImageSet(x, y)


_cache: Dict[Tuple[str, int, Optional[int]], Tuple[ImageSet, ImageSet]] = {}
_cache_lock = threading.Lock()


def _read_idx(path: str) -> np.ndarray:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    ndim = data[3]
    dims = [int.from_bytes(data[4 + 4 * i : 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def _real_mnist(root: str) -> Optional[Tuple[ImageSet, ImageSet]]:
    def find(stem: str) -> Optional[str]:
        for suffix in ("", ".gz"):
            p = os.path.join(root, stem + suffix)
            if os.path.exists(p):
                return p
        return None

    paths = [find(s) for s in ("train-images-idx3-ubyte", "train-labels-idx1-ubyte", "t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")]
    if any(p is None for p in paths):
        return None
    xtr, ytr, xte, yte = (_read_idx(p) for p in paths)  # type: ignore[arg-type]
    mk = lambda x, y: ImageSet(torch.from_numpy(x.copy()).unsqueeze(1), torch.from_numpy(y.astype(np.int64)))
    return mk(xtr, ytr), mk(xte, yte)


def get_dataset(name: str = "mnist", seed: int = 0, n_train: Optional[int] = None) -> Tuple[ImageSet, ImageSet]:
    """(train, test) for a dataset name; cached per process like the reference singletons."""
    key = (name, seed, n_train)
    with _cache_lock:
        if key in _cache:
            return _cache[key]
        if name == "mnist" and os.environ.get("P2PFL_MNIST_DIR"):
            real = _real_mnist(os.environ["P2PFL_MNIST_DIR"])
            if real is not None:
                _cache[key] = real
                return real
        shape, classes, ntr, nte = SPECS[name]
        if n_train is not None:
            ntr = n_train
        g = torch.Generator().manual_seed(1000 + seed)
        protos = _prototypes(shape, classes, g)
        train = make_split(shape, classes, ntr, seed * 2 + 1, protos)
        test = make_split(shape, classes, nte, seed * 2 + 2, protos)
        _cache[key] = (train, test)
        return train, test
