"""Runnable examples (``python -m p2pfl_amd experiment list``).

Each module has a one-line docstring (shown by ``experiment list``) and runs
under ``python -m p2pfl_amd.examples.<name> [args]``.  Mirrors the
reference's ``p2pfl/examples`` (mnist.py, node1.py, node2.py) and adds the
BASELINE.json configurations (CIFAR ResNet, ViT, fault tolerance).
"""
