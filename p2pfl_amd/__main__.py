"""``python -m p2pfl_amd``: the command-line interface (see :mod:`p2pfl_amd.cli`)."""

from p2pfl_amd.cli import main

main()
