"""Imitation / reward-learning algorithms (API parity with ``imitation.algorithms``)."""
