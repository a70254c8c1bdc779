"""Reward networks (reference: ``src/imitation/rewards/reward_nets.py``).

API parity: ``RewardNet`` (``forward`` differentiable; ``predict_th`` /
``predict`` / ``predict_processed`` numpy entry points, ``reward_nets.py:16-224``),
wrappers (``RewardNetWrapper``, ``ForwardWrapper``, ``PredictProcessedWrapper``),
``BasicRewardNet`` (hid (32, 32)), ``CnnRewardNet`` (one-hot action/done trick),
``NormalizedRewardNet`` (RunningNorm on outputs), ``ShapedRewardNet``
(``r + γ(1-d)Φ(s') - Φ(s)``), ``BasicShapedRewardNet``, ``BasicPotentialMLP``,
``BasicPotentialCNN``, ``RewardEnsemble`` (mean / ddof=1 variance),
``AddSTDRewardWrapper``, ``cnn_transpose``.

MI355X additions:

* every net also exposes ``predict_processed_th`` taking/returning **device
  tensors**, so the adversarial / preference trainers can score generator
  samples without the reference's per-step numpy->device->numpy round trip
  (``reward_wrapper.py:110-115``);
* the MLP bodies are :class:`~imitation_amd.util.networks.MLP` and run as one
  fused MFMA launch (input RunningNorm folded into the kernel prologue).
"""

from __future__ import annotations

import abc
from typing import Any, Callable, Dict, Iterable, Optional, Sequence, Tuple, Type, cast

import numpy as np
import torch as th
from torch import nn

from imitation_amd.envs import spaces
from imitation_amd.rl import preprocessing
from imitation_amd.util import networks, util
from imitation_amd.util.module_spec import SpecRecorded


class RewardNet(SpecRecorded, nn.Module, abc.ABC):
    """Minimal abstract reward network: implement ``forward(state, action, next_state, done)``."""

    def __init__(self, observation_space: spaces.Space, action_space: spaces.Space, normalize_images: bool = True):
        super().__init__()
        self.observation_space = observation_space
        self.action_space = action_space
        self.normalize_images = normalize_images

    @abc.abstractmethod
    def forward(self, state: th.Tensor, action: th.Tensor, next_state: th.Tensor, done: th.Tensor) -> th.Tensor:
        """Compute rewards for a batch of transitions, keeping gradients."""

    def preprocess(self, state, action, next_state, done) -> Tuple[th.Tensor, th.Tensor, th.Tensor, th.Tensor]:
        """numpy or tensors -> device tensors (one-hot Discrete, /255 images, float dones)."""
        dev = self.device
        state_th = util.safe_to_tensor(state).to(dev)
        action_th = util.safe_to_tensor(action).to(dev)
        next_state_th = util.safe_to_tensor(next_state).to(dev)
        done_th = util.safe_to_tensor(done).to(dev)
        state_th = cast(th.Tensor, preprocessing.preprocess_obs(state_th, self.observation_space, self.normalize_images))
        action_th = cast(th.Tensor, preprocessing.preprocess_obs(action_th, self.action_space, self.normalize_images))
        next_state_th = cast(th.Tensor, preprocessing.preprocess_obs(next_state_th, self.observation_space, self.normalize_images))
        done_th = done_th.to(th.float32)
        n_gen = len(state_th)
        assert state_th.shape == next_state_th.shape
        assert len(action_th) == n_gen
        return state_th, action_th, next_state_th, done_th

    def predict_th(self, state, action, next_state, done) -> th.Tensor:
        with networks.evaluating(self):
            s, a, ns, d = self.preprocess(state, action, next_state, done)
            with th.no_grad():
                rew_th = self(s, a, ns, d)
            assert rew_th.shape == tuple(np.shape(state)[:1]) or rew_th.shape == state.shape[:1]
            return rew_th

    def predict(self, state, action, next_state, done) -> np.ndarray:
        return self.predict_th(state, action, next_state, done).detach().cpu().numpy().flatten()

    def predict_processed(self, state, action, next_state, done, **kwargs) -> np.ndarray:
        del kwargs
        return self.predict(state, action, next_state, done)

    def predict_processed_th(self, state, action, next_state, done, **kwargs) -> th.Tensor:
        """Device-tensor version of :meth:`predict_processed` (no host round trip)."""
        del kwargs
        return self.predict_th(state, action, next_state, done)

    @property
    def device(self) -> th.device:
        try:
            return next(self.parameters()).device
        except StopIteration:
            for b in self.buffers():
                return b.device
            return th.device("cpu")

    @property
    def dtype(self) -> th.dtype:
        try:
            return next(self.parameters()).dtype
        except StopIteration:
            return th.get_default_dtype()


class RewardNetWrapper(RewardNet):
    """Abstract wrapper holding a ``base`` reward net."""

    def __init__(self, base: RewardNet):
        super().__init__(base.observation_space, base.action_space, base.normalize_images)
        self._base = base

    @property
    def base(self) -> RewardNet:
        return self._base

    @property
    def device(self) -> th.device:
        return self.base.device

    @property
    def dtype(self) -> th.dtype:
        return self.base.dtype

    def preprocess(self, state, action, next_state, done):
        return self.base.preprocess(state, action, next_state, done)


class ForwardWrapper(RewardNetWrapper):
    """Wrapper that changes ``forward`` (and therefore everything built on it)."""

    def __init__(self, base: RewardNet):
        super().__init__(base)
        if isinstance(base, PredictProcessedWrapper):
            raise ValueError("ForwardWrapper cannot be applied on top of PredictProcessedWrapper!")


class PredictProcessedWrapper(RewardNetWrapper):
    """Wrapper that only changes ``predict_processed`` (forward/predict pass through)."""

    def forward(self, state, action, next_state, done) -> th.Tensor:
        return self.base.forward(state, action, next_state, done)

    @abc.abstractmethod
    def predict_processed(self, state, action, next_state, done, **kwargs) -> np.ndarray:
        """Predict processed rewards."""

    def predict(self, state, action, next_state, done) -> np.ndarray:
        return self.base.predict(state, action, next_state, done)

    def predict_th(self, state, action, next_state, done) -> th.Tensor:
        return self.base.predict_th(state, action, next_state, done)


class RewardNetWithVariance(RewardNet):
    """Reward net that also estimates per-sample reward variance."""

    @abc.abstractmethod
    def predict_reward_moments(self, state, action, next_state, done, **kwargs) -> Tuple[np.ndarray, np.ndarray]:
        """(mean, variance), each of shape ``(batch,)``."""


class BasicRewardNet(RewardNet):
    """MLP over concat(flatten(s), flatten(a)[, flatten(s')][, d]) -> scalar."""

    def __init__(self, observation_space, action_space, use_state: bool = True, use_action: bool = True,
                 use_next_state: bool = False, use_done: bool = False, **kwargs):
        super().__init__(observation_space, action_space)
        combined = 0
        self.use_state = use_state
        if use_state:
            combined += preprocessing.get_flattened_obs_dim(observation_space)
        self.use_action = use_action
        if use_action:
            combined += preprocessing.get_flattened_obs_dim(action_space)
        self.use_next_state = use_next_state
        if use_next_state:
            combined += preprocessing.get_flattened_obs_dim(observation_space)
        self.use_done = use_done
        if use_done:
            combined += 1
        full_kwargs: Dict[str, Any] = {"hid_sizes": (32, 32), **kwargs, "in_size": combined, "out_size": 1, "squeeze_output": True}
        self.mlp = networks.build_mlp(**full_kwargs)

    def forward(self, state, action, next_state, done):
        inputs = []
        if self.use_state:
            inputs.append(th.flatten(state, 1))
        if self.use_action:
            inputs.append(th.flatten(action, 1))
        if self.use_next_state:
            inputs.append(th.flatten(next_state, 1))
        if self.use_done:
            inputs.append(th.reshape(done, [-1, 1]))
        x = th.cat(inputs, dim=1) if len(inputs) > 1 else inputs[0]
        out = self.mlp(x)
        assert out.shape == state.shape[:1]
        return out


def cnn_transpose(tens: th.Tensor) -> th.Tensor:
    """NHWC -> NCHW."""
    if len(tens.shape) == 4:
        return th.permute(tens, (0, 3, 1, 2))
    raise ValueError(f"Invalid input: len(tens.shape) = {len(tens.shape)} != 4.")


class CnnRewardNet(RewardNet):
    """CNN reward over image observations; actions/dones pick an output head (one-hot trick)."""

    def __init__(self, observation_space, action_space, use_state: bool = True, use_action: bool = True,
                 use_next_state: bool = False, use_done: bool = False, hwc_format: bool = True, **kwargs):
        super().__init__(observation_space, action_space)
        self.use_state = use_state
        self.use_action = use_action
        self.use_next_state = use_next_state
        self.use_done = use_done
        self.hwc_format = hwc_format
        if not (use_state or use_next_state):
            raise ValueError("CnnRewardNet must take current or next state as input.")
        if not preprocessing.is_image_space(observation_space):
            raise ValueError("CnnRewardNet requires observations to be images.")
        if use_action and not isinstance(action_space, spaces.Discrete):
            raise ValueError("CnnRewardNet can only use Discrete action spaces.")
        input_size, output_size = 0, 1
        if use_state:
            input_size += self.get_num_channels_obs(observation_space)
        if use_action:
            output_size = int(action_space.n)
        if use_next_state:
            input_size += self.get_num_channels_obs(observation_space)
        if use_done:
            output_size *= 2
        full_kwargs: Dict[str, Any] = {"hid_channels": (32, 32), **kwargs, "in_channels": input_size,
                                       "out_size": output_size, "squeeze_output": output_size == 1}
        self.cnn = networks.build_cnn(**full_kwargs)

    def get_num_channels_obs(self, space: spaces.Box) -> int:
        return space.shape[-1] if self.hwc_format else space.shape[0]

    def forward(self, state, action, next_state, done):
        inputs = []
        if self.use_state:
            inputs.append(cnn_transpose(state) if self.hwc_format else state)
        if self.use_next_state:
            inputs.append(cnn_transpose(next_state) if self.hwc_format else next_state)
        x = th.cat(inputs, dim=1)
        if x.is_cuda:
            x = x.contiguous(memory_format=th.channels_last)
        outputs = self.cnn(x)
        if self.use_action and not self.use_done:
            return th.sum(outputs * action, dim=1)
        if self.use_action and self.use_done:
            full_acts = th.cat((action * (1 - done[:, None]), action * done[:, None]), dim=1)
            return th.sum(outputs * full_acts, dim=1)
        if not self.use_action and self.use_done:
            return th.sum(outputs * nn.functional.one_hot(done.long(), num_classes=2), dim=1)
        return outputs


class NormalizedRewardNet(PredictProcessedWrapper):
    """Normalise processed rewards with a running normaliser (stats updated after normalising)."""

    def __init__(self, base: RewardNet, normalize_output_layer: Type[networks.BaseNorm]):
        super().__init__(base=base)
        self.normalize_output_layer = normalize_output_layer(1)

    def predict_processed(self, state, action, next_state, done, update_stats: bool = True, **kwargs) -> np.ndarray:
        """Host API: the base's ``predict_processed`` (extra kwargs forwarded, so a wrapped
        wrapper's own processing runs), then normalise; ``predict_processed_th`` is the
        device-resident variant used by the fused reward paths (reference reward_nets.py:637)."""
        with networks.evaluating(self):
            rew_th = th.as_tensor(np.asarray(self.base.predict_processed(state, action, next_state, done, **kwargs)),
                                  device=self.device).float().reshape(-1)
            with th.no_grad():
                out = self.normalize_output_layer(rew_th).detach().cpu().numpy().flatten()
        if update_stats:
            with th.no_grad():
                self.normalize_output_layer.update_stats(rew_th)
        assert out.shape == np.shape(state)[:1]
        return out

    def predict_processed_th(self, state, action, next_state, done, update_stats: bool = True, **kwargs) -> th.Tensor:
        with networks.evaluating(self):
            rew_th = self.base.predict_processed_th(state, action, next_state, done, **kwargs)
            rew_th = util.safe_to_tensor(rew_th).to(self.device).float().reshape(-1)
            with th.no_grad():
                rew = self.normalize_output_layer(rew_th).detach().reshape(-1)
        if update_stats:
            with th.no_grad():
                self.normalize_output_layer.update_stats(rew_th)
        return rew


class ShapedRewardNet(ForwardWrapper):
    """``base(s,a,s',d) + γ (1 - d) Φ(s') - Φ(s)``."""

    def __init__(self, base: RewardNet, potential: Callable[[th.Tensor], th.Tensor], discount_factor: float):
        super().__init__(base=base)
        self.potential = potential
        self.discount_factor = discount_factor

    def forward(self, state, action, next_state, done):
        base_out = self.base(state, action, next_state, done)
        new_shaping = (1 - done.float()) * self.potential(next_state).flatten()
        old_shaping = self.potential(state).flatten()
        final = base_out + self.discount_factor * new_shaping - old_shaping
        assert final.shape == state.shape[:1]
        return final


class BasicPotentialMLP(SpecRecorded, nn.Module):
    """Potential Φ(s) as a flat MLP."""

    def __init__(self, observation_space: spaces.Space, hid_sizes: Iterable[int], **kwargs):
        super().__init__()
        in_size = preprocessing.get_flattened_obs_dim(observation_space)
        self._potential_net = networks.build_mlp(in_size=in_size, hid_sizes=hid_sizes, squeeze_output=True, flatten_input=True, **kwargs)

    def forward(self, state: th.Tensor) -> th.Tensor:
        return self._potential_net(state)


class BasicPotentialCNN(SpecRecorded, nn.Module):
    """Potential Φ(s) as a CNN over image observations."""

    def __init__(self, observation_space: spaces.Space, hid_sizes: Iterable[int], hwc_format: bool = True, **kwargs):
        super().__init__()
        self.hwc_format = hwc_format
        if not preprocessing.is_image_space(observation_space):
            raise ValueError("CNN potential must be given image inputs.")
        obs_shape = observation_space.shape
        in_channels = obs_shape[-1] if hwc_format else obs_shape[0]
        self._potential_net = networks.build_cnn(in_channels=in_channels, hid_channels=hid_sizes, squeeze_output=True, **kwargs)

    def forward(self, state: th.Tensor) -> th.Tensor:
        return self._potential_net(cnn_transpose(state) if self.hwc_format else state)


class BasicShapedRewardNet(ShapedRewardNet):
    """Shaped reward: reward MLP (32,) + potential MLP (32, 32) (AIRL default)."""

    def __init__(self, observation_space, action_space, *, reward_hid_sizes: Sequence[int] = (32,),
                 potential_hid_sizes: Sequence[int] = (32, 32), use_state: bool = True, use_action: bool = True,
                 use_next_state: bool = False, use_done: bool = False, discount_factor: float = 0.99, **kwargs):
        base = BasicRewardNet(observation_space=observation_space, action_space=action_space, use_state=use_state,
                              use_action=use_action, use_next_state=use_next_state, use_done=use_done,
                              hid_sizes=reward_hid_sizes, **kwargs)
        potential = BasicPotentialMLP(observation_space=observation_space, hid_sizes=potential_hid_sizes, **kwargs)
        super().__init__(base, potential, discount_factor=discount_factor)


class RewardEnsemble(RewardNetWithVariance):
    """Ensemble of ≥ 2 reward nets: mean and unbiased variance across members."""

    def __init__(self, observation_space, action_space, members: Iterable[RewardNet]):
        super().__init__(observation_space, action_space)
        members = list(members)
        if len(members) < 2:
            raise ValueError("Must be at least 2 member in the ensemble.")
        self.members = nn.ModuleList(members)

    @property
    def num_members(self):
        return len(self.members)

    def stack(self):
        """The members as one stacked MLP (:class:`~imitation_amd.rewards.ensemble.EnsembleStack`),
        or None when they are not structurally identical ``BasicRewardNet`` MLPs."""
        if not hasattr(self, "_ia_stack"):
            from imitation_amd.rewards.ensemble import EnsembleStack

            object.__setattr__(self, "_ia_stack", EnsembleStack.build(self))
        return self._ia_stack

    def _grouped_all(self, state, action, next_state, done) -> Optional[th.Tensor]:
        """[B, M] member rewards from ONE grouped launch (GPU, stackable members), else None."""
        st = self.stack()
        if st is None or self.device.type != "cuda":
            return None
        s, a, ns, d = self.members[0].preprocess(state, action, next_state, done)
        with th.no_grad():
            return st.forward(st.features(s, a, ns, d), st.gather_params(), st.gather_norm()).T

    def predict_processed_all(self, state, action, next_state, done, **kwargs) -> np.ndarray:
        batch_size = np.shape(state)[0]
        grouped = self._grouped_all(state, action, next_state, done) if not kwargs else None
        if grouped is not None:
            rewards = grouped.cpu().numpy()
        else:
            rewards = np.stack([m.predict_processed(state, action, next_state, done, **kwargs) for m in self.members], axis=-1)
        assert rewards.shape == (batch_size, self.num_members)
        return rewards

    def predict_processed_all_th(self, state, action, next_state, done, **kwargs) -> th.Tensor:
        grouped = self._grouped_all(state, action, next_state, done) if not kwargs else None
        if grouped is not None:
            return grouped
        return th.stack([util.safe_to_tensor(m.predict_processed_th(state, action, next_state, done, **kwargs)).to(self.device).reshape(-1)
                         for m in self.members], dim=-1)

    @th.no_grad()
    def predict_reward_moments(self, state, action, next_state, done, **kwargs) -> Tuple[np.ndarray, np.ndarray]:
        batch_size = np.shape(state)[0]
        all_rewards = self.predict_processed_all(state, action, next_state, done, **kwargs)
        mean = all_rewards.mean(-1)
        var = all_rewards.var(-1, ddof=1)
        assert mean.shape == var.shape == (batch_size,)
        return mean, var

    def forward(self, *args) -> th.Tensor:
        raise NotImplementedError

    def predict_processed(self, state, action, next_state, done, **kwargs) -> np.ndarray:
        return self.predict(state, action, next_state, done, **kwargs)

    def predict_processed_th(self, state, action, next_state, done, **kwargs) -> th.Tensor:
        return self.predict_processed_all_th(state, action, next_state, done, **kwargs).mean(-1)

    def predict(self, state, action, next_state, done, **kwargs):
        mean, _ = self.predict_reward_moments(state, action, next_state, done, **kwargs)
        return mean


class AddSTDRewardWrapper(PredictProcessedWrapper):
    """``mean + alpha * std`` of a :class:`RewardNetWithVariance` (exploration bonus)."""

    def __init__(self, base: RewardNetWithVariance, default_alpha: float = 0.0):
        super().__init__(base)
        if not isinstance(base, RewardNetWithVariance):
            raise TypeError("Cannot add standard deviation to reward net that is not an instance of RewardNetWithVariance!")
        self.default_alpha = default_alpha

    def predict_processed(self, state, action, next_state, done, alpha: Optional[float] = None, **kwargs) -> np.ndarray:
        del kwargs
        if alpha is None:
            alpha = self.default_alpha
        mean, var = self.base.predict_reward_moments(state, action, next_state, done)
        return mean + alpha * np.sqrt(var)

    def predict_processed_th(self, state, action, next_state, done, alpha: Optional[float] = None, **kwargs) -> th.Tensor:
        return th.as_tensor(self.predict_processed(util.to_numpy(state), util.to_numpy(action), util.to_numpy(next_state),
                                                   util.to_numpy(done), alpha=alpha), device=self.device)
