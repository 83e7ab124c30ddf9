"""Synthetic datasets, partitioners and device-resident data modules."""

from p2pfl_amd.data.datamodule import (
    Cifar10FederatedDM,
    DeviceLoader,
    FederatedDataModule,
    ImageNetFederatedDM,
    MnistFederatedDM,
)
from p2pfl_amd.data.synthetic import ImageSet, get_dataset

__all__ = [
    "Cifar10FederatedDM",
    "DeviceLoader",
    "FederatedDataModule",
    "ImageNetFederatedDM",
    "MnistFederatedDM",
    "ImageSet",
    "get_dataset",
]
