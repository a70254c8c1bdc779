"""Expert demonstrations for tests (reference: src/imitation/testing/expert_trajectories.py).

Experts come from ``policies.serialize.load_policy("ppo-huggingface", ...)`` which
resolves against a LOCAL hub directory (no network on the MI355X pool); the test
suite points it at ``tests/testdata/expert_models``. Generated rollouts are cached
on disk in the HF-dataset format under a file lock, so parallel pytest workers share
one generation.
"""

from __future__ import annotations

import os
import pathlib
import shutil
import warnings
from typing import Sequence

import numpy as np

from imitation_amd.algorithms import base as algo_base
from imitation_amd.data import rollout, serialize, types, wrappers
from imitation_amd.policies import serialize as policies_serialize
from imitation_amd.util import util


class _FileLock:
    """Minimal advisory lock (fcntl) so concurrent workers do not both generate."""

    def __init__(self, path: str):
        self.path = path
        self.fd = None

    def __enter__(self):
        import fcntl

        self.fd = open(self.path, "w")
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl

        fcntl.flock(self.fd, fcntl.LOCK_UN)
        self.fd.close()


def generate_expert_trajectories(env_id: str, num_trajectories: int, rng: np.random.Generator) -> Sequence[types.TrajectoryWithRew]:
    env = util.make_vec_env(env_id, post_wrappers=[lambda e, _: wrappers.RolloutInfoWrapper(e)], rng=rng)
    try:
        expert = policies_serialize.load_policy("ppo-huggingface", env, env_name=env_id)
        return rollout.rollout(expert, env, rollout.make_sample_until(min_episodes=num_trajectories), rng=rng)
    finally:
        env.close()


def lazy_generate_expert_trajectories(cache_path, env_id: str, num_trajectories: int,
                                      rng: np.random.Generator) -> Sequence[types.TrajectoryWithRew]:
    env_dir = pathlib.Path(cache_path) / policies_serialize.env_name_to_hub(env_id)
    env_dir.mkdir(parents=True, exist_ok=True)
    traj_path = env_dir / "rollout"
    with _FileLock(str(env_dir / "rollout.lock")):
        try:
            trajectories = serialize.load_with_rewards(traj_path)
        except FileNotFoundError:
            warnings.warn(f"Generating expert trajectories for {env_id} because the cache is cold.")
            trajectories = generate_expert_trajectories(env_id, num_trajectories, rng)
            serialize.save(traj_path, trajectories)
    if len(trajectories) >= num_trajectories:
        return trajectories[:num_trajectories]
    shutil.rmtree(traj_path) if traj_path.is_dir() else os.unlink(traj_path)
    return lazy_generate_expert_trajectories(cache_path, env_id, num_trajectories, rng)


def make_expert_transition_loader(cache_dir, batch_size: int, expert_data_type: str, env_name: str,
                                  rng: np.random.Generator, num_trajectories: int = 1, shuffle: bool = True):
    """Expert data as "trajectories", "data_loader", "ducktyped_data_loader" or "transitions"."""
    trajectories = lazy_generate_expert_trajectories(cache_dir, env_name, num_trajectories, rng)
    transitions = rollout.flatten_trajectories(trajectories)
    if len(transitions) < batch_size:  # pragma: no cover
        transitions = types.Transitions(
            obs=np.concatenate([transitions.obs] * (batch_size // len(transitions) + 1)),
            acts=np.concatenate([transitions.acts] * (batch_size // len(transitions) + 1)),
            infos=np.concatenate([transitions.infos] * (batch_size // len(transitions) + 1)),
            next_obs=np.concatenate([transitions.next_obs] * (batch_size // len(transitions) + 1)),
            dones=np.concatenate([transitions.dones] * (batch_size // len(transitions) + 1)),
        )
    if expert_data_type == "trajectories":
        return trajectories
    if expert_data_type == "data_loader":
        return algo_base.make_data_loader(transitions, batch_size=batch_size, data_loader_kwargs=dict(shuffle=shuffle, drop_last=True))
    if expert_data_type == "ducktyped_data_loader":
        class DucktypedDataset:
            def __init__(self, transitions, batch_size):
                self.transitions = transitions
                self.batch_size = batch_size

            def __iter__(self):
                for start in range(0, len(self.transitions) - self.batch_size + 1, self.batch_size):
                    yield types.transitions_collate_fn([self.transitions[i] for i in range(start, start + self.batch_size)])

        return DucktypedDataset(transitions, batch_size)
    if expert_data_type == "transitions":
        return transitions
    raise ValueError(f"Unexpected data type '{expert_data_type}'")
