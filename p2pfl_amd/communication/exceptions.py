"""Communication errors (reference ``communication/exceptions.py:21-24``)."""


class NeighborNotConnectedError(Exception):
    """Send to an unknown neighbour, or to a non-direct one without ``create_connection``."""
