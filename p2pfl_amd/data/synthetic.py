"""Synthetic, learnable image-classification datasets.

There is no network on the build or GPU boxes, so the reference's torchvision
MNIST download (``mnistfederated_dm.py:85-101``) is replaced by deterministic
synthetic data of the same shapes.  Each class has a smooth random prototype
image; a sample is its class prototype under a random contrast, a small random
translation and additive noise, stored as ``uint8`` like MNIST.  Models reach
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
    c, h, w = shape
    low = torch.rand(classes, c, max(2, h // 4), max(2, w // 4), generator=g)
    protos = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=False)
    protos = (protos - protos.amin(dim=(1, 2, 3), keepdim=True)) / (
        protos.amax(dim=(1, 2, 3), keepdim=True) - protos.amin(dim=(1, 2, 3), keepdim=True) + 1e-6
    )
    return protos


def make_split(
    shape: Tuple[int, int, int], classes: int, n: int, seed: int, protos: torch.Tensor, chunk: int = 8192
) -> ImageSet:
    g = torch.Generator().manual_seed(seed)
    c, h, w = shape
    y = torch.randint(0, classes, (n,), generator=g)
    x = torch.empty((n, c, h, w), dtype=torch.uint8)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        yy = y[s:e]
        img = protos[yy]
        contrast = 0.6 + 0.4 * torch.rand(e - s, 1, 1, 1, generator=g)
        img = img * contrast + 0.25 * torch.rand(img.shape, generator=g)
        dx, dy = torch.randint(-2, 3, (2,), generator=g).tolist()
        img = torch.roll(img, shifts=(dy, dx), dims=(2, 3))
        x[s:e] = (img.clamp(0, 1.25) / 1.25 * 255).to(torch.uint8)
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
