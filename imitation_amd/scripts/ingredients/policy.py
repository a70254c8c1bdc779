"""Policy ingredient (reference: scripts/ingredients/policy.py)."""

import logging
from typing import Any, Mapping, Type

from imitation_amd.policies import base
from imitation_amd.rl import policies
from imitation_amd.rl.policies import get_schedule_fn
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.util import networks

policy_ingredient = Ingredient("policy", ingredients=[logging_ingredient.logging_ingredient])
logger = logging.getLogger(__name__)


@policy_ingredient.config
def config():
    policy_cls = base.FeedForward32Policy
    policy_kwargs = {}
    locals()


@policy_ingredient.named_config
def sac():
    policy_cls = base.SAC1024Policy


NORMALIZE_RUNNING_POLICY_KWARGS = {
    "features_extractor_class": base.NormalizeFeaturesExtractor,
    "features_extractor_kwargs": {"normalize_class": networks.RunningNorm},
}


@policy_ingredient.named_config
def normalize_running():
    policy_kwargs = NORMALIZE_RUNNING_POLICY_KWARGS


@policy_ingredient.named_config
def cnn_policy():
    policy_cls = policies.ActorCriticCnnPolicy


@policy_ingredient.capture
def make_policy(venv, policy_cls: Type[policies.BasePolicy], policy_kwargs: Mapping[str, Any]) -> policies.BasePolicy:
    policy_kwargs = dict(policy_kwargs)
    if isinstance(policy_cls, type) and issubclass(policy_cls, policies.ActorCriticPolicy):
        policy_kwargs.update({"observation_space": venv.observation_space, "action_space": venv.action_space,
                              "lr_schedule": get_schedule_fn(1)})
    policy = policy_cls(**policy_kwargs)
    logger.info(f"Policy network summary:\n {policy}")
    return policy
