"""Logging ingredient: log dir, stdout/TensorBoard/W&B formats (reference: scripts/ingredients/logging.py)."""

import logging
import os
import pathlib
from typing import Sequence, Tuple, Union

from imitation_amd.policies.serialize import env_name_to_hub
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.scripts.ingredients import environment, wb
from imitation_amd.util import logger as imit_logger
from imitation_amd.util import sacred as sacred_util
from imitation_amd.util import util

logging_ingredient = Ingredient("logging", ingredients=[wb.wandb_ingredient, environment.environment_ingredient])
logger = logging.getLogger(__name__)


@logging_ingredient.config
def config():
    log_root = None  # Defaults to "output" (the log_dir then is <root>/<command>/<env>/<timestamp>)
    log_dir = None
    log_level = logging.INFO
    log_format_strs = ["tensorboard", "stdout"]
    log_format_strs_additional = {}
    locals()


@logging_ingredient.config
def update_log_format_strs(log_format_strs, log_format_strs_additional):
    log_format_strs = log_format_strs + list(log_format_strs_additional.keys())


@logging_ingredient.config_hook
def hook(config, command_name: str, logger):
    updates = {}
    if config["logging"]["log_dir"] is None:
        log_root = util.parse_path(config["logging"]["log_root"] or "output")
        env_sanitized = env_name_to_hub(config["environment"]["gym_id"])
        updates["log_dir"] = str(log_root / str(command_name) / env_sanitized / util.make_unique_timestamp())
    return updates


@logging_ingredient.named_config
def wandb_logging():
    log_format_strs_additional = {"wandb": None}


@logging_ingredient.capture
def make_log_dir(_run, log_dir: str, log_level: Union[int, str]) -> pathlib.Path:
    parsed = util.parse_path(log_dir)
    parsed.mkdir(parents=True, exist_ok=True)
    try:
        log_level = int(log_level)
    except ValueError:
        pass
    logging.basicConfig(level=log_level)
    logger.info("Logging to %s", parsed)
    sacred_util.build_sacred_symlink(parsed, _run)
    return parsed


@logging_ingredient.capture
def setup_logging(_run, log_format_strs: Sequence[str]) -> Tuple[imit_logger.HierarchicalLogger, pathlib.Path]:
    log_dir = make_log_dir()
    if "wandb" in log_format_strs:
        wb.wandb_init(log_dir=str(log_dir))
    # asynchronous format writes: the training loop only snapshots each dump; the tensorboard /
    # stdout writing runs on the writer thread while the host waits for the GPU (drained at exit;
    # IMITATION_AMD_LOG_ASYNC=0 writes synchronously)
    async_writes = os.environ.get("IMITATION_AMD_LOG_ASYNC", "1") != "0"
    custom_logger = imit_logger.configure(folder=log_dir / "log", format_strs=log_format_strs, async_writes=async_writes)
    return custom_logger, log_dir
