"""Device-resident federated data modules.

:class:`FederatedDataModule` is the framework's counterpart of the reference's
Lightning ``MnistFederatedDM`` (``mnistfederated_dm.py:33-162``): it exposes
``train_dataloader()``, ``val_dataloader()`` and ``test_dataloader()``, whose
``.dataset`` supports ``len`` (used for the FedAvg sample weight,
``lightning_learner.py:95-107``).

The shard is kept as ``uint8`` tensors and moved to the learner's device once;
batches are produced by indexing on the device (no worker processes, no
per-batch host->device copies).  ``x`` is normalised to ``[0, 1]`` float per
batch, or handed raw to fused kernels that fold the ``/255`` into their first
layer.
"""

from __future__ import annotations

import math
from typing import Iterator, Optional, Tuple

import torch

from p2pfl_amd.data import partition
from p2pfl_amd.data.synthetic import ImageSet, get_dataset


class _Sized:
    def __init__(self, n: int) -> None:
        self._n = n

    def __len__(self) -> int:
        return self._n


class DeviceLoader:
    """Iterates ``(x, y)`` batches from tensors that already live on a device."""

    def __init__(
        self,
        x: torch.Tensor,
        y: torch.Tensor,
        batch_size: int,
        shuffle: bool,
        seed: int = 0,
        normalize: bool = True,
        drop_last: bool = False,
    ) -> None:
        self.x, self.y = x, y
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.normalize = normalize
        self.drop_last = drop_last
        self.dataset = _Sized(int(y.shape[0]))
        self._epoch = 0
        self._seed = seed

    def __len__(self) -> int:
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def to(self, device: torch.device) -> "DeviceLoader":
        self.x = self.x.to(device)
        self.y = self.y.to(device)
        return self

    def permutation(self, host: bool = False) -> torch.Tensor:
        """This epoch's sample order on the data's device, or (``host``) in pinned host
        memory for the caller to copy straight into its own device buffer."""
        n = len(self.dataset)
        if not self.shuffle:
            return torch.arange(n) if host else torch.arange(n, device=self.y.device)
        g = torch.Generator().manual_seed(self._seed * 100003 + self._epoch)
        self._epoch += 1
        perm = torch.randperm(n, generator=g)
        if host:
            return perm.pin_memory() if self.y.device.type == "cuda" else perm
        if self.y.device.type == "cuda":
            # pinned + non-blocking: the host never waits for the GPU's queue
            # to drain just to hand it the next epoch's batch order
            return perm.pin_memory().to(self.y.device, non_blocking=True)
        return perm.to(self.y.device)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        perm = self.permutation()
        n = len(self.dataset)
        stop = n - (n % self.batch_size) if self.drop_last else n
        for s in range(0, stop, self.batch_size):
            idx = perm[s : s + self.batch_size]
            xb = self.x.index_select(0, idx)
            if self.normalize:
                xb = xb.float().div_(255.0)
            yield xb, self.y.index_select(0, idx)


def wants_float(loader, model) -> bool:
    """Whether a batch of ``loader`` is normalised to [0, 1] float before ``model``:
    not for models that read the uint8 batch themselves (``takes_uint8``)."""
    return bool(loader.normalize) and not getattr(model, "takes_uint8", False)


class FederatedDataModule:
    def __init__(
        self,
        train: ImageSet,
        val: ImageSet,
        test: ImageSet,
        batch_size: int = 32,
        seed: int = 0,
        num_classes: int = 10,
    ) -> None:
        self.batch_size = batch_size
        self.num_classes = num_classes
        self.train_loader = DeviceLoader(train.x, train.y, batch_size, shuffle=True, seed=seed)
        self.val_loader = DeviceLoader(val.x, val.y, batch_size, shuffle=False)
        self.test_loader = DeviceLoader(test.x, test.y, batch_size, shuffle=False)
        self.device = torch.device("cpu")

    def to(self, device: torch.device) -> "FederatedDataModule":
        device = torch.device(device)
        if device != self.device:
            for ld in (self.train_loader, self.val_loader, self.test_loader):
                ld.to(device)
            self.device = device
        return self

    def train_dataloader(self) -> DeviceLoader:
        return self.train_loader

    def val_dataloader(self) -> DeviceLoader:
        return self.val_loader

    def test_dataloader(self) -> DeviceLoader:
        return self.test_loader

    # -- construction helpers ---------------------------------------------
    @classmethod
    def from_dataset(
        cls,
        name: str = "mnist",
        sub_id: int = 0,
        number_sub: int = 1,
        batch_size: int = 32,
        val_percent: float = 0.1,
        iid: bool = True,
        partitioner: Optional[str] = None,
        alpha: float = 0.5,
        seed: int = 0,
        n_train: Optional[int] = None,
    ) -> "FederatedDataModule":
        train, test = get_dataset(name, seed=0, n_train=n_train)
        kind = partitioner or ("iid" if iid else "label_sorted")
        if kind == "iid":
            tr_idx = partition.iid_shard(len(train), sub_id, number_sub)
            te_idx = partition.iid_shard(len(test), sub_id, number_sub)
        elif kind == "label_sorted":
            tr_idx = partition.label_sorted(train.y, sub_id, number_sub)
            te_idx = partition.label_sorted(test.y, sub_id, number_sub)
        elif kind == "dirichlet":
            tr_idx = partition.dirichlet(train.y, sub_id, number_sub, alpha=alpha, seed=seed)
            te_idx = partition.iid_shard(len(test), sub_id, number_sub)
        else:
            raise ValueError(f"unknown partitioner {kind!r}")
        if len(test) < number_sub:
            raise ValueError("Too much partitions")
        # 90/10 train/val split of the shard (reference random_split, seeded)
        g = torch.Generator().manual_seed(seed + 7919 * sub_id)
        perm = tr_idx[torch.randperm(len(tr_idx), generator=g)]
        n_val = round(len(perm) * val_percent)
        n_tr = len(perm) - n_val
        tr, va = perm[:n_tr], perm[n_tr:]
        mk = lambda s, idx: ImageSet(s.x.index_select(0, idx), s.y.index_select(0, idx))
        classes = {"mnist": 10, "cifar10": 10, "imagenet": 1000}.get(name, 10)
        return cls(mk(train, tr), mk(train, va), mk(test, te_idx), batch_size=batch_size, seed=seed + sub_id, num_classes=classes)


class MnistFederatedDM(FederatedDataModule):
    """Drop-in for the reference data module (same constructor arguments).

    ``num_workers`` is accepted for signature compatibility and ignored:
    batches are produced on the device.
    """

    def __init__(
        self,
        sub_id: int = 0,
        number_sub: int = 1,
        batch_size: int = 32,
        num_workers: int = 0,
        val_percent: float = 0.1,
        iid: bool = True,
        partitioner: Optional[str] = None,
        alpha: float = 0.5,
        seed: int = 0,
    ) -> None:
        dm = FederatedDataModule.from_dataset(
            "mnist", sub_id, number_sub, batch_size, val_percent, iid, partitioner, alpha, seed
        )
        self.__dict__.update(dm.__dict__)
        self.sub_id, self.number_sub = sub_id, number_sub


class Cifar10FederatedDM(FederatedDataModule):
    def __init__(self, sub_id: int = 0, number_sub: int = 1, batch_size: int = 32, partitioner: str = "iid", alpha: float = 0.5, seed: int = 0) -> None:
        dm = FederatedDataModule.from_dataset("cifar10", sub_id, number_sub, batch_size, 0.1, True, partitioner, alpha, seed)
        self.__dict__.update(dm.__dict__)


class ImageNetFederatedDM(FederatedDataModule):
    def __init__(self, sub_id: int = 0, number_sub: int = 1, batch_size: int = 32, n_train: int = 12800, partitioner: str = "iid", seed: int = 0) -> None:
        dm = FederatedDataModule.from_dataset("imagenet", sub_id, number_sub, batch_size, 0.1, True, partitioner, 0.5, seed, n_train=n_train)
        self.__dict__.update(dm.__dict__)
