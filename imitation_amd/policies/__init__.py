"""Policies: custom actor-critics, non-trainable policies, wrappers and the policy registry."""
