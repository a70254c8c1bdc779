"""Regularizers for reward-model training (reference: src/imitation/regularization/)."""
