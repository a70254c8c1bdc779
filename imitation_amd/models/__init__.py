"""Model recipes for the headline configurations (see :mod:`.recipes`)."""

from imitation_amd.models.recipes import RECIPES, Built, build, synthetic_demonstrations

__all__ = ["RECIPES", "Built", "build", "synthetic_demonstrations"]
