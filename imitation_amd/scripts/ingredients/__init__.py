"""Reusable config + capture functions shared by the scripts (reference: scripts/ingredients/)."""
