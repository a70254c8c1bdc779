"""Replay buffer whose sampled rewards are relabelled by a reward function
(reference: src/imitation/policies/replay_buffer_wrapper.py; used for SAC on a learned reward).

The inner buffer lives on the device. When ``reward_fn`` is a reward net's
``predict_processed`` (or the net itself), relabelling stays on the device through
``predict_processed_th``; otherwise the sampled batch goes through the numpy
``RewardFn`` protocol like the reference.
"""

from __future__ import annotations

from typing import Any, Dict, Type

import numpy as np
import torch as th

from imitation_amd.rewards.reward_function import RewardFn
from imitation_amd.rl.buffers import BaseBuffer, ReplayBuffer, ReplayBufferSamples
from imitation_amd.util import util


def _samples_to_reward_fn_input(samples: ReplayBufferSamples) -> Dict[str, np.ndarray]:
    return dict(state=samples.observations.cpu().numpy(), action=samples.actions.cpu().numpy(),
                next_state=samples.next_observations.cpu().numpy(), done=samples.dones.cpu().numpy())


def _device_reward_fn(reward_fn):
    from imitation_amd.rewards.reward_nets import RewardNet

    if isinstance(reward_fn, RewardNet):
        return reward_fn.predict_processed_th
    owner = getattr(reward_fn, "__self__", None)
    if isinstance(owner, RewardNet) and getattr(reward_fn, "__name__", "") == "predict_processed":
        return owner.predict_processed_th
    return None


class ReplayBufferRewardWrapper(BaseBuffer):
    def __init__(self, buffer_size: int, observation_space, action_space, *, replay_buffer_class: Type[ReplayBuffer],
                 reward_fn: RewardFn, **kwargs: Any):
        assert replay_buffer_class is ReplayBuffer, "only ReplayBuffer is supported"
        self.replay_buffer = replay_buffer_class(buffer_size, observation_space, action_space, **kwargs)
        self.reward_fn = reward_fn
        self._reward_th = _device_reward_fn(reward_fn)
        base_kwargs = {k: v for k, v in kwargs.items() if k in ("device", "n_envs")}
        super().__init__(buffer_size, observation_space, action_space, **base_kwargs)

    @property
    def pos(self) -> int:
        return self.replay_buffer.pos

    @pos.setter
    def pos(self, pos: int):
        if hasattr(self, "replay_buffer"):
            self.replay_buffer.pos = pos

    @property
    def full(self) -> bool:
        return self.replay_buffer.full

    @full.setter
    def full(self, full: bool):
        if hasattr(self, "replay_buffer"):
            self.replay_buffer.full = full

    def size(self) -> int:
        return self.replay_buffer.size()

    def sample(self, *args, **kwargs) -> ReplayBufferSamples:
        samples = self.replay_buffer.sample(*args, **kwargs)
        shape, device = samples.rewards.shape, samples.rewards.device
        if self._reward_th is not None:
            with th.no_grad():
                rewards_th = self._reward_th(samples.observations, samples.actions, samples.next_observations,
                                             samples.dones.reshape(-1))
            rewards_th = rewards_th.reshape(shape).to(device=device, dtype=th.float32)
        else:
            rewards = self.reward_fn(**_samples_to_reward_fn_input(samples))
            rewards_th = util.safe_to_tensor(rewards).reshape(shape).to(device=device, dtype=th.float32)
        return ReplayBufferSamples(samples.observations, samples.actions, samples.next_observations, samples.dones, rewards_th)

    def add(self, *args, **kwargs):
        self.replay_buffer.add(*args, **kwargs)

    def _get_samples(self, *args, **kwargs):
        raise NotImplementedError("_get_samples() is intentionally not implemented.")
