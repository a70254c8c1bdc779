"""Helpers for tests: permutation-test reward improvement, expert trajectories,
mock reward nets, hypothesis strategies (reference: src/imitation/testing/)."""
