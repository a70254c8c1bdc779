"""SQIL ingredient (reference: scripts/ingredients/sqil.py)."""

from imitation_amd.policies import base
from imitation_amd.rl.dqn import DQN
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.scripts.ingredients import policy, rl

sqil_ingredient = Ingredient("sqil", ingredients=[rl.rl_ingredient, policy.policy_ingredient])


@sqil_ingredient.config
def config():
    total_timesteps = 3e5
    train_kwargs = dict(log_interval=4, progress_bar=False)
    locals()


@rl.rl_ingredient.config_hook
def override_rl_cls(config, command_name, logger):
    res = {}
    if command_name == "sqil" and config["rl"]["rl_cls"] is None:
        res["rl_cls"] = DQN
    return res


@policy.policy_ingredient.config_hook
def override_policy_cls(config, command_name, logger):
    res = {}
    if command_name == "sqil" and config["policy"]["policy_cls"] is base.FeedForward32Policy:
        res["policy_cls"] = "MlpPolicy"
    return res
