"""Roll out a policy and report statistics (reference: src/imitation/scripts/eval_policy.py)."""

from __future__ import annotations

import logging
import pathlib
import time
from typing import Any, Mapping, Optional

import numpy as np

from imitation_amd.data import rollout, serialize
from imitation_amd.envs.vec_env import VecEnvWrapper
from imitation_amd.policies.exploration_wrapper import ExplorationWrapper
from imitation_amd.rewards import reward_wrapper
from imitation_amd.rewards.serialize import load_reward
from imitation_amd.scripts.config.eval_policy import eval_policy_ex
from imitation_amd.utils import watchdog
from imitation_amd.scripts.config_engine import FileStorageObserver
from imitation_amd.scripts.ingredients import environment, expert
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.util import video_wrapper


class InteractiveRender(VecEnvWrapper):
    """Render the wrapped environment(s) on every step."""

    def __init__(self, venv, fps):
        super().__init__(venv)
        self.render_fps = fps

    def reset(self):
        ob = self.venv.reset()
        self.venv.render()
        return ob

    def step_wait(self):
        out = self.venv.step_wait()
        if self.render_fps > 0:
            time.sleep(1 / self.render_fps)
        self.venv.render()
        return out


def video_wrapper_factory(log_dir: pathlib.Path, **kwargs):
    def f(env, i: int) -> video_wrapper.VideoWrapper:
        return video_wrapper.VideoWrapper(env, directory=log_dir / "videos" / str(i), **kwargs)

    return f


@eval_policy_ex.main
def eval_policy(eval_n_timesteps: Optional[int], eval_n_episodes: Optional[int], render: bool, render_fps: int,
                videos: bool, video_kwargs: Mapping[str, Any], _run, _rnd: np.random.Generator,
                reward_type: Optional[str] = None, reward_path: Optional[str] = None,
                rollout_save_path: Optional[str] = None, explore_kwargs: Optional[Mapping[str, Any]] = None):
    """Returns ``rollout_stats`` of the expert ingredient's policy (optionally reward-overridden / exploratory)."""
    log_dir = logging_ingredient.make_log_dir()
    sample_until = rollout.make_sample_until(eval_n_timesteps, eval_n_episodes)
    post_wrappers = [video_wrapper_factory(log_dir, **video_kwargs)] if videos else None
    with environment.make_venv(post_wrappers=post_wrappers) as venv:
        if render:
            venv = InteractiveRender(venv, render_fps)
        if reward_type is not None:
            venv = reward_wrapper.RewardVecEnvWrapper(venv, load_reward(reward_type, reward_path, venv))
            logging.info(f"Wrapped env in reward {reward_type} from {reward_path}.")
        policy = expert.get_expert_policy(venv)
        if explore_kwargs is not None:
            policy = ExplorationWrapper(policy, venv, rng=_rnd, **explore_kwargs)
            logging.info(f"Wrapped policy in ExplorationWrapper with kwargs {explore_kwargs}")
        with watchdog.cli_watchdog("eval_policy"):  # an evaluation that never ends aborts instead of hanging
            trajs = rollout.generate_trajectories(policy, venv, sample_until, rng=_rnd)
    if rollout_save_path:
        serialize.save(log_dir / rollout_save_path.replace("{log_dir}/", ""), trajs)
    return rollout.rollout_stats(trajs)


def main_console(argv=None):
    eval_policy_ex.observers.append(FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "eval_policy"))
    return eval_policy_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
