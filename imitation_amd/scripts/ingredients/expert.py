"""Expert policy ingredient (reference: scripts/ingredients/expert.py).

``policy_type``: ``ppo`` / ``sac`` / ``dqn`` (``loader_kwargs.path`` to a model.zip),
``<algo>-huggingface`` (local hub copy, see ``policies.serialize``), ``random``, ``zero``.
"""

from imitation_amd.policies import serialize
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.scripts.ingredients import environment

expert_ingredient = Ingredient("expert", ingredients=[environment.environment_ingredient])


@expert_ingredient.config
def config():
    policy_type = "ppo-huggingface"
    loader_kwargs = dict()
    locals()


@expert_ingredient.config_hook
def config_hook(config, command_name, logger):
    e_config = config["expert"]
    if "huggingface" in e_config["policy_type"]:
        e_config["loader_kwargs"].setdefault("organization", "HumanCompatibleAI")
        e_config["loader_kwargs"]["env_name"] = config["environment"]["gym_id"]
    if e_config["policy_type"] in ("ppo", "sac", "dqn") and "path" not in e_config["loader_kwargs"]:
        e_config["loader_kwargs"]["path"] = None
    return e_config


@expert_ingredient.capture
def get_expert_policy(venv, policy_type, loader_kwargs):
    return serialize.load_policy(policy_type, venv, **loader_kwargs)
