"""Pre-tuned library GEMM selections for MI355X (gfx950).

The plain GEMMs of the PyTorch-path learners (ViT linear layers, ResNet/MLP
heads) go through hipBLASLt/rocBLAS.  Their default heuristic picks a poor
kernel for several of the ViT-B/16 shapes (the weight-gradient GEMMs with a
6304-long reduction ran at ~0.4 PFLOP/s).  PyTorch's TunableOp benchmarks
every hipBLASLt and rocBLAS solution for a shape and records the winner;
``tunableop_gfx950.csv`` holds those winners, measured on an MI355X with this
image's PyTorch / hipBLASLt / rocBLAS (its validator lines pin the versions,
so a mismatched stack ignores it).  :func:`enable_tuned_gemms` loads the
table without re-tuning; ``P2PFL_TUNABLEOP_TUNE=1`` tunes unseen shapes
(and writes them to ``P2PFL_TUNABLEOP_FILE``), ``P2PFL_TUNABLEOP=0``
disables the mechanism.
"""

from __future__ import annotations

import os

import torch

TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_gfx950.csv")
_done = False


def enable_tuned_gemms() -> bool:
    global _done
    if _done:
        return True
    if os.environ.get("P2PFL_TUNABLEOP", "1") == "0" or not torch.cuda.is_available():
        return False
    tun = getattr(torch.cuda, "tunable", None)
    if tun is None:
        return False
    tun.enable(True)
    tune = os.environ.get("P2PFL_TUNABLEOP_TUNE") == "1"
    tun.tuning_enable(tune)
    if tune:
        tun.set_filename(os.environ.get("P2PFL_TUNABLEOP_FILE", "tunableop_results%d.csv"))
    if os.path.exists(TABLE):
        tun.read_file(TABLE)
    _done = True
    return True
