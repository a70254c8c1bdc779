"""Command-line experiments (reference: src/imitation/scripts/), on the in-tree config engine."""
