"""Weights & Biases ingredient (reference: scripts/ingredients/wb.py)."""

from typing import Any, Mapping, Optional

from imitation_amd.scripts.config_engine import Ingredient

wandb_ingredient = Ingredient("logging.wandb")


@wandb_ingredient.config
def wandb_config():
    wandb_tag = None
    wandb_name_prefix = ""
    wandb_kwargs = dict(project="imitation", monitor_gym=False, save_code=False)
    wandb_additional_info = dict()
    locals()


@wandb_ingredient.capture
def wandb_init(_run, wandb_name_prefix: str, wandb_tag: Optional[str], wandb_kwargs: Mapping[str, Any],
               wandb_additional_info: Mapping[str, Any], log_dir: str) -> None:
    env_name = _run.config["environment"]["gym_id"]
    root_seed = _run.config["seed"]
    kwargs = {**wandb_kwargs, "name": f"{wandb_name_prefix}-{env_name}-seed{root_seed}",
              "tags": [env_name, f"seed{root_seed}"] + ([wandb_tag] if wandb_tag else []), "dir": log_dir}
    try:
        import wandb
    except ModuleNotFoundError as e:
        raise ModuleNotFoundError("Trying to call `wandb.init()` but `wandb` not installed: try `pip install wandb`.") from e
    cfg = dict(**_run.config)
    cfg.update(wandb_additional_info)
    wandb.init(config=cfg, **kwargs)
