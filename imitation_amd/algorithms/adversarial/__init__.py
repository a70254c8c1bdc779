"""Adversarial imitation: GAIL and AIRL on a shared :class:`~.common.AdversarialTrainer`."""
