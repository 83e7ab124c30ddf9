"""The six stages of a federated-learning node."""
