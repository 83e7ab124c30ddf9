"""Node lifecycle exceptions (reference ``p2pfl/exceptions.py:21-36``)."""


class NodeRunningException(Exception):
    """The node is (or is not) running when the opposite was required."""


class LearnerNotSetException(Exception):
    """Model/data changed after the learner was instantiated."""


class ZeroRoundsException(Exception):
    """``set_start_learning`` called with fewer than one round."""
