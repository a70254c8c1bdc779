"""Expert demonstrations ingredient (reference: scripts/ingredients/demonstrations.py).

``source``: ``local`` (HF dataset dir or legacy npz at ``path``), ``huggingface`` (a
dataset dir already present locally -- no network on the training nodes), or
``generated`` (roll out the expert ingredient's policy).
"""

import logging
import os
from typing import Any, Dict, Optional, Sequence

import numpy as np

from imitation_amd.data import huggingface_utils, rollout, serialize, types
from imitation_amd.policies.serialize import env_name_to_hub
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.scripts.ingredients import environment, expert
from imitation_amd.scripts.ingredients import logging as logging_ingredient

demonstrations_ingredient = Ingredient("demonstrations", ingredients=[expert.expert_ingredient,
                                                                      logging_ingredient.logging_ingredient,
                                                                      environment.environment_ingredient])
logger = logging.getLogger(__name__)


@demonstrations_ingredient.config
def config():
    source = "generated"  # local | huggingface | generated
    path = None
    loader_kwargs = dict(split="train")
    organization = "HumanCompatibleAI"
    algo_name = "ppo"
    n_expert_demos = None
    locals()


@demonstrations_ingredient.named_config
def fast():
    n_expert_demos = 10


@demonstrations_ingredient.capture
def get_expert_trajectories(source: str, path: str) -> Sequence[types.Trajectory]:
    if source == "local":
        if path is None:
            raise ValueError("When source is 'local', path must be set.")
        return _constrain_number_of_demos(serialize.load(path))
    if source == "huggingface":
        return _constrain_number_of_demos(_download_expert_rollouts())
    if source == "generated":
        if path is not None:
            logger.warning("Ignoring path when source is 'generated'")
        return _generate_expert_trajs()
    raise ValueError("`source` can either be `local` or `huggingface` or `generated`.")


@demonstrations_ingredient.capture
def _constrain_number_of_demos(demos: Sequence[types.Trajectory], n_expert_demos: Optional[int]):
    if n_expert_demos is None:
        return demos
    if len(demos) < n_expert_demos:
        raise ValueError(f"Want to use n_expert_demos={n_expert_demos} trajectories, but only {len(demos)} are available.")
    if len(demos) > n_expert_demos:
        logger.warning(f"Using only the first {n_expert_demos} trajectories out of {len(demos)} available.")
        return demos[:n_expert_demos]
    return demos


@demonstrations_ingredient.capture
def _generate_expert_trajs(n_expert_demos: Optional[int], _rnd: np.random.Generator):
    if n_expert_demos is None:
        raise ValueError("n_expert_demos must be specified when generating demos.")
    logger.info(f"Generating {n_expert_demos} expert trajectories")
    with environment.make_rollout_venv() as env:
        return rollout.rollout(expert.get_expert_policy(env), env, rollout.make_sample_until(min_episodes=n_expert_demos),
                               rng=_rnd)


@demonstrations_ingredient.capture
def _download_expert_rollouts(environment: Dict[str, Any], path: Optional[str], organization: Optional[str],
                              algo_name: Optional[str], loader_kwargs: Dict[str, Any]):
    """Resolve ``{organization}/{algo}-{env}`` against the local dataset hub
    (``$IMITATION_AMD_DATASETS``, default ``~/.cache/imitation_amd/datasets``)."""
    import datasets

    if path is not None:
        local = path
    else:
        root = os.environ.get("IMITATION_AMD_DATASETS", os.path.expanduser("~/.cache/imitation_amd/datasets"))
        local = os.path.join(root, organization, f"{algo_name}-{env_name_to_hub(environment['gym_id'])}")
    logger.info(f"Loading expert trajectories from {local}")
    if os.path.isdir(local):
        try:
            ds = datasets.load_from_disk(local)
        except Exception:
            ds = datasets.load_dataset(local, **loader_kwargs)
    else:
        raise FileNotFoundError(f"No local copy of dataset {local} (training nodes have no network access)")
    if isinstance(ds, datasets.DatasetDict):
        ds = ds[loader_kwargs.get("split", "train")]
    return huggingface_utils.TrajectoryDatasetSequence(ds)
