"""Learning errors (reference ``learning/exceptions.py:22-31``)."""


class DecodingParamsError(Exception):
    """A weights payload could not be decoded."""


class ModelNotMatchingError(Exception):
    """Decoded parameters do not match the local model (names, count or shapes)."""
