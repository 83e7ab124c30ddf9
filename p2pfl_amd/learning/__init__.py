"""Learning layer: learner contract, learners, aggregators, arenas, wire codec."""
