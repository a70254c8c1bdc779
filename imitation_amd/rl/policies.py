"""Policies (SB3 ``policies`` surface: SURVEY §2.5).

* :class:`BasePolicy` -- ``predict`` (numpy in/out, clipping, single-obs support),
  ``obs_to_tensor``, ``set_training_mode``, ``save``/``load``;
* :class:`ActorCriticPolicy` -- features extractor -> :class:`MlpExtractor`
  -> ``action_net`` / ``value_net`` (+ ``log_std`` for Box), with SB3's
  ``evaluate_actions`` / ``get_distribution`` / ``predict_values`` API and
  state-dict layout;
* :class:`ActorCriticCnnPolicy`, :class:`MultiInputActorCriticPolicy`.

MI355X path: when the trunk is an MLP (the reference's FeedForward32 / [64,64]
policies) the actor head ``[norm] -> pi trunk -> action_net`` and the critic head
``[norm] -> vf trunk -> value_net`` each run as ONE fused MFMA launch
(``imitation_amd.ops.tmlp``); the features normaliser's statistics update is
the only other op. CNN trunks use MIOpen convolutions (channels-last).
"""

from __future__ import annotations

import collections
import copy
import functools
import io
import os
import pathlib
import warnings
from typing import Any, Dict, List, Optional, Tuple, Type, Union

import json

import numpy as np
import torch as th
from torch import nn

from imitation_amd import ops
from imitation_amd.envs import spaces
from imitation_amd.ops.mlp import act_code, fusable
from imitation_amd.rl.distributions import (
    BernoulliDistribution,
    CategoricalDistribution,
    DiagGaussianDistribution,
    Distribution,
    MultiCategoricalDistribution,
    make_proba_distribution,
)
from imitation_amd.rl.preprocessing import get_action_dim, is_image_space, maybe_transpose, preprocess_obs
from imitation_amd.rl.torch_layers import (
    BaseFeaturesExtractor,
    CombinedExtractor,
    FlattenExtractor,
    MlpExtractor,
    NatureCNN,
)

Schedule = Any


def get_device(device: Union[th.device, str] = "auto") -> th.device:
    if device == "auto":
        device = "cuda"
    device = th.device(device)
    if device.type == "cuda" and not th.cuda.is_available():
        return th.device("cpu")
    return device


def constant_fn(val: float):
    def func(_):
        return val

    return func


def get_schedule_fn(value_schedule) -> Any:
    if isinstance(value_schedule, (float, int)):
        return constant_fn(float(value_schedule))
    assert callable(value_schedule)
    return value_schedule


def obs_as_tensor(obs, device: th.device):
    if isinstance(obs, np.ndarray):
        return th.as_tensor(obs, device=device)
    if isinstance(obs, dict):
        return {k: th.as_tensor(v, device=device) for k, v in obs.items()}
    if isinstance(obs, th.Tensor):
        return obs.to(device)
    raise TypeError(f"Unrecognized type of observation {type(obs)}")


def is_vectorized_observation(observation, observation_space: spaces.Space) -> bool:
    if isinstance(observation_space, spaces.Dict):
        k0 = next(iter(observation_space.spaces))
        return is_vectorized_observation(observation[k0], observation_space.spaces[k0])
    obs = np.asarray(observation)
    if isinstance(observation_space, spaces.Box):
        if obs.shape == observation_space.shape:
            return False
        if obs.shape[1:] == observation_space.shape:
            return True
        raise ValueError(
            f"Error: Unexpected observation shape {obs.shape} for Box environment, please use "
            f"{observation_space.shape} or (n_env, {', '.join(map(str, observation_space.shape))}) for the observation shape."
        )
    if isinstance(observation_space, spaces.Discrete):
        if obs.shape == ():
            return False
        if len(obs.shape) == 1:
            return True
        raise ValueError(f"Unexpected observation shape {obs.shape} for Discrete environment")
    if isinstance(observation_space, spaces.MultiDiscrete):
        if obs.shape == (len(observation_space.nvec),):
            return False
        return True
    if isinstance(observation_space, spaces.MultiBinary):
        return obs.shape != observation_space.shape
    raise ValueError(f"Unsupported observation space {observation_space}")


class BaseModel(nn.Module):
    def __init__(
        self,
        observation_space: spaces.Space,
        action_space: spaces.Space,
        features_extractor_class: Type[BaseFeaturesExtractor] = FlattenExtractor,
        features_extractor_kwargs: Optional[Dict[str, Any]] = None,
        features_extractor: Optional[BaseFeaturesExtractor] = None,
        normalize_images: bool = True,
        optimizer_class: Type[th.optim.Optimizer] = th.optim.Adam,
        optimizer_kwargs: Optional[Dict[str, Any]] = None,
    ):
        super().__init__()
        self.observation_space = observation_space
        self.action_space = action_space
        self.features_extractor_class = features_extractor_class
        self.features_extractor_kwargs = features_extractor_kwargs or {}
        self.features_extractor = features_extractor
        self.normalize_images = normalize_images
        self.optimizer_class = optimizer_class
        self.optimizer_kwargs = optimizer_kwargs or {}
        self.optimizer: Optional[th.optim.Optimizer] = None

    def make_features_extractor(self) -> BaseFeaturesExtractor:
        return self.features_extractor_class(self.observation_space, **self.features_extractor_kwargs)

    def extract_features(self, obs, features_extractor: Optional[nn.Module] = None) -> th.Tensor:
        fe = features_extractor if features_extractor is not None else self.features_extractor
        if (self.normalize_images and isinstance(fe, NatureCNN) and fe.raw_frames_ok(obs)
                and is_image_space(self.observation_space)):
            # uint8 frames straight into the conv kernels, /255 folded into the first layer's
            # operand load: no float copy of the batch (== preprocess_obs then fe)
            return fe(obs, 1.0 / 255.0)
        preprocessed = preprocess_obs(obs, self.observation_space, normalize_images=self.normalize_images)
        return fe(preprocessed)

    def _get_constructor_parameters(self) -> Dict[str, Any]:
        return dict(observation_space=self.observation_space, action_space=self.action_space, normalize_images=self.normalize_images)

    @property
    def device(self) -> th.device:
        for p in self.parameters():
            return p.device
        for b in self.buffers():
            return b.device
        return th.device("cpu")

    def save(self, path) -> None:
        """Save as a tensor-only file: state dict + JSON constructor parameters + class path.

        Loadable with ``torch.load(weights_only=True)`` -- nothing is unpickled on load.
        """
        from imitation_amd.rl import save_util

        th.save(
            {
                "format": "imitation_amd.policy.v1",
                "class": f"{type(self).__module__}:{type(self).__qualname__}",
                "data": json.dumps(save_util._encode(self._get_constructor_parameters())),
                "state_dict": self.state_dict(),
            },
            path,
        )

    @classmethod
    def load(cls, path, device: Union[th.device, str] = "auto"):
        return load_policy_file(path, device=device, expected_cls=cls)

    def load_from_vector(self, vector: np.ndarray) -> None:
        th.nn.utils.vector_to_parameters(th.as_tensor(vector, dtype=th.float, device=self.device), self.parameters())

    def parameters_to_vector(self) -> np.ndarray:
        return th.nn.utils.parameters_to_vector(self.parameters()).detach().cpu().numpy()

    def set_training_mode(self, mode: bool) -> None:
        self.train(mode)

    def is_vectorized_observation(self, observation) -> bool:
        return is_vectorized_observation(maybe_transpose(observation, self.observation_space), self.observation_space)

    def obs_to_tensor(self, observation) -> Tuple[Any, bool]:
        vectorized_env = False
        if isinstance(observation, dict):
            assert isinstance(self.observation_space, spaces.Dict)
            observation = copy.deepcopy(observation)
            for key, obs in observation.items():
                sub = self.observation_space.spaces[key]
                obs_ = maybe_transpose(obs, sub) if is_image_space(sub) else np.array(obs)
                vectorized_env = vectorized_env or is_vectorized_observation(obs_, sub)
                observation[key] = obs_.reshape((-1, *self.observation_space[key].shape))
        elif isinstance(observation, th.Tensor):
            vectorized_env = observation.shape != tuple(self.observation_space.shape or ())
            if not vectorized_env:
                observation = observation.unsqueeze(0)
            return observation.to(self.device), vectorized_env
        else:
            observation = maybe_transpose(observation, self.observation_space)
            observation = np.array(observation)
            if not isinstance(observation, dict):
                vectorized_env = is_vectorized_observation(observation, self.observation_space)
                observation = observation.reshape((-1, *self.observation_space.shape))
        return obs_as_tensor(observation, self.device), vectorized_env


class BasePolicy(BaseModel):
    def __init__(self, *args, squash_output: bool = False, **kwargs):
        super().__init__(*args, **kwargs)
        self._squash_output = squash_output

    @staticmethod
    def _dummy_schedule(progress_remaining: float) -> float:
        del progress_remaining
        return 0.0

    @property
    def squash_output(self) -> bool:
        return self._squash_output

    @staticmethod
    def init_weights(module: nn.Module, gain: float = 1) -> None:
        if isinstance(module, (nn.Linear, nn.Conv2d)):
            nn.init.orthogonal_(module.weight, gain=gain)
            if module.bias is not None:
                module.bias.data.fill_(0.0)

    def forward(self, *args, **kwargs):  # pragma: no cover - abstract
        raise NotImplementedError

    def _predict(self, observation, deterministic: bool = False) -> th.Tensor:
        raise NotImplementedError

    def predict(
        self,
        observation,
        state: Optional[Tuple[np.ndarray, ...]] = None,
        episode_start: Optional[np.ndarray] = None,
        deterministic: bool = False,
    ) -> Tuple[np.ndarray, Optional[Tuple[np.ndarray, ...]]]:
        """numpy obs -> numpy actions (clipped to Box bounds), SB3 semantics."""
        self.set_training_mode(False)
        if isinstance(observation, tuple) and len(observation) == 2 and isinstance(observation[1], dict):
            raise ValueError(
                "You have passed a tuple to the predict() function instead of a Numpy array or a Dict. "
                "You are probably mixing Gym API with SB3 VecEnv API: `obs, info = env.reset()` (Gym) "
                "vs `obs = vec_env.reset()` (SB3 VecEnv)."
            )
        obs_tensor, vectorized_env = self.obs_to_tensor(observation)
        with th.no_grad():
            actions = self._predict(obs_tensor, deterministic=deterministic)
        actions = actions.cpu().numpy().reshape((-1, *self.action_space.shape))
        if isinstance(self.action_space, spaces.Box):
            if self.squash_output:
                actions = self.unscale_action(actions)
            else:
                actions = np.clip(actions, self.action_space.low, self.action_space.high)
        if not vectorized_env:
            assert isinstance(actions, np.ndarray)
            actions = actions.squeeze(axis=0)
        return actions, state

    def scale_action(self, action: np.ndarray) -> np.ndarray:
        low, high = self.action_space.low, self.action_space.high
        return 2.0 * ((action - low) / (high - low)) - 1.0

    def unscale_action(self, scaled_action: np.ndarray) -> np.ndarray:
        low, high = self.action_space.low, self.action_space.high
        return low + (0.5 * (scaled_action + 1.0) * (high - low))


def _fusable_trunk(seq: nn.Sequential) -> Optional[Tuple[List[nn.Linear], Optional[int]]]:
    """Linear/act pairs with one fusable activation type -> (linears, act code)."""
    linears: List[nn.Linear] = []
    code: Optional[int] = None
    mods = list(seq)
    i = 0
    while i < len(mods):
        lin = mods[i]
        if not isinstance(lin, nn.Linear) or lin.bias is None or i + 1 >= len(mods):
            return None
        c = act_code(mods[i + 1])
        if c is None or (code is not None and c != code):
            return None
        code = c
        linears.append(lin)
        i += 2
    return linears, code


class ActorCriticPolicy(BasePolicy):
    """Actor-critic policy with SB3's structure, state-dict layout and API."""

    def __init__(
        self,
        observation_space: spaces.Space,
        action_space: spaces.Space,
        lr_schedule: Schedule,
        net_arch: Optional[Union[List[int], Dict[str, List[int]]]] = None,
        activation_fn: Type[nn.Module] = nn.Tanh,
        ortho_init: bool = True,
        use_sde: bool = False,
        log_std_init: float = 0.0,
        full_std: bool = True,
        use_expln: bool = False,
        squash_output: bool = False,
        features_extractor_class: Type[BaseFeaturesExtractor] = FlattenExtractor,
        features_extractor_kwargs: Optional[Dict[str, Any]] = None,
        share_features_extractor: bool = True,
        normalize_images: bool = True,
        optimizer_class: Type[th.optim.Optimizer] = th.optim.Adam,
        optimizer_kwargs: Optional[Dict[str, Any]] = None,
    ):
        if optimizer_kwargs is None:
            optimizer_kwargs = {}
            if optimizer_class == th.optim.Adam:
                optimizer_kwargs["eps"] = 1e-5
        super().__init__(
            observation_space,
            action_space,
            features_extractor_class,
            features_extractor_kwargs,
            optimizer_class=optimizer_class,
            optimizer_kwargs=optimizer_kwargs,
            squash_output=squash_output,
            normalize_images=normalize_images,
        )
        if isinstance(net_arch, list) and len(net_arch) > 0 and isinstance(net_arch[0], dict):
            warnings.warn("net_arch=[dict(...)] is deprecated; use net_arch=dict(...)")
            net_arch = net_arch[0]
        if net_arch is None:
            net_arch = [] if features_extractor_class == NatureCNN else dict(pi=[64, 64], vf=[64, 64])
        self.net_arch = net_arch
        self.activation_fn = activation_fn
        self.ortho_init = ortho_init
        self.share_features_extractor = share_features_extractor
        self.features_extractor = self.make_features_extractor()
        self.features_dim = self.features_extractor.features_dim
        if self.share_features_extractor:
            self.pi_features_extractor = self.features_extractor
            self.vf_features_extractor = self.features_extractor
        else:
            self.pi_features_extractor = self.features_extractor
            self.vf_features_extractor = self.make_features_extractor()
        self.log_std_init = log_std_init
        self.use_sde = use_sde
        self.dist_kwargs = None
        self.action_dist = make_proba_distribution(action_space, use_sde=use_sde, dist_kwargs=self.dist_kwargs)
        self._build(lr_schedule)

    def _get_constructor_parameters(self) -> Dict[str, Any]:
        data = super()._get_constructor_parameters()
        data.update(
            dict(
                net_arch=self.net_arch,
                activation_fn=self.activation_fn,
                use_sde=self.use_sde,
                log_std_init=self.log_std_init,
                squash_output=self._squash_output,
                lr_schedule=self._dummy_schedule,
                ortho_init=self.ortho_init,
                optimizer_class=self.optimizer_class,
                optimizer_kwargs=self.optimizer_kwargs,
                features_extractor_class=self.features_extractor_class,
                features_extractor_kwargs=self.features_extractor_kwargs,
                share_features_extractor=self.share_features_extractor,
            )
        )
        return data

    def _build_mlp_extractor(self) -> None:
        self.mlp_extractor = MlpExtractor(self.features_dim, net_arch=self.net_arch, activation_fn=self.activation_fn)

    def _build(self, lr_schedule: Schedule) -> None:
        self._build_mlp_extractor()
        latent_dim_pi = self.mlp_extractor.latent_dim_pi
        if isinstance(self.action_dist, DiagGaussianDistribution):
            self.action_net, self.log_std = self.action_dist.proba_distribution_net(latent_dim_pi, self.log_std_init)
        elif isinstance(self.action_dist, (CategoricalDistribution, MultiCategoricalDistribution, BernoulliDistribution)):
            self.action_net = self.action_dist.proba_distribution_net(latent_dim=latent_dim_pi)
        else:
            raise NotImplementedError(f"Unsupported distribution '{self.action_dist}'.")
        self.value_net = nn.Linear(self.mlp_extractor.latent_dim_vf, 1)
        if self.ortho_init:
            module_gains = {
                self.features_extractor: np.sqrt(2),
                self.mlp_extractor: np.sqrt(2),
                self.action_net: 0.01,
                self.value_net: 1,
            }
            if not self.share_features_extractor:
                del module_gains[self.features_extractor]
                module_gains[self.pi_features_extractor] = np.sqrt(2)
                module_gains[self.vf_features_extractor] = np.sqrt(2)
            for module, gain in module_gains.items():
                module.apply(functools.partial(self.init_weights, gain=gain))
        self.optimizer = self.optimizer_class(self.parameters(), lr=lr_schedule(1), **self.optimizer_kwargs)

    # ------------------------------------------------------------------ fused heads
    def _fusion(self):
        plan = getattr(self, "_ia_fusion", None)
        if plan is not None:
            return plan
        plan = False
        fe = self.features_extractor
        if self.share_features_extractor and isinstance(fe, FlattenExtractor) and not isinstance(
            self.observation_space, spaces.Dict
        ):
            norm = getattr(fe, "normalize", None)
            from imitation_amd.util.networks import BaseNorm

            if norm is None or isinstance(norm, BaseNorm):
                pi = _fusable_trunk(self.mlp_extractor.policy_net)
                vf = _fusable_trunk(self.mlp_extractor.value_net)
                if pi is not None and vf is not None:
                    pi_l = pi[0] + [self.action_net]
                    vf_l = vf[0] + [self.value_net]
                    pi_dims = [self.features_dim] + [l.out_features for l in pi_l]
                    vf_dims = [self.features_dim] + [l.out_features for l in vf_l]
                    wide = getattr(self, "wide_bf16", None)  # opt-in bf16 wide path (ops/mlp.py)
                    if isinstance(self.action_net, nn.Linear) and fusable(pi_dims, wide) and fusable(vf_dims, wide):
                        plan = dict(
                            norm=norm,
                            pi=pi_l,
                            pi_act=pi[1] or 0,
                            vf=vf_l,
                            vf_act=vf[1] or 0,
                            wide=wide,
                        )
        object.__setattr__(self, "_ia_fusion", plan)
        return plan

    def _fused_latents(self, obs, want_pi: bool = True, want_vf: bool = True):
        """(action-net output, values) via fused MFMA kernels, or None if not applicable."""
        if not (ops.fused_enabled() and isinstance(obs, th.Tensor) and obs.is_cuda):
            return None
        plan = self._fusion()
        if not plan:
            return None
        x = preprocess_obs(obs, self.observation_space, normalize_images=self.normalize_images).flatten(1)
        if x.dtype != th.float32:
            x = x.float()
        norm = plan["norm"]
        mean = var = None
        eps = 1e-5
        if norm is not None:
            if norm.training:
                with th.no_grad():
                    norm.update_stats(x)
            mean, var, eps = norm.running_mean, norm.running_var, norm.eps
        head = vals = None
        if want_pi:
            head = ops.tmlp(x, [l.weight for l in plan["pi"]], [l.bias for l in plan["pi"]], plan["pi_act"], 0, mean, var, eps, plan["wide"])
        if want_vf:
            vals = ops.tmlp(x, [l.weight for l in plan["vf"]], [l.bias for l in plan["vf"]], plan["vf_act"], 0, mean, var, eps, plan["wide"])
        return head, vals

    def _dist_from_head(self, head: th.Tensor) -> Distribution:
        if isinstance(self.action_dist, DiagGaussianDistribution):
            return self.action_dist.proba_distribution(head, self.log_std)
        return self.action_dist.proba_distribution(action_logits=head)

    # ------------------------------------------------------------------ SB3 API
    def forward(self, obs, deterministic: bool = False) -> Tuple[th.Tensor, th.Tensor, th.Tensor]:
        fused = self._fused_latents(obs)
        if fused is not None:
            head, values = fused
            distribution = self._dist_from_head(head)
        else:
            features = self.extract_features(obs)
            if self.share_features_extractor:
                latent_pi, latent_vf = self.mlp_extractor(features)
            else:
                pi_features, vf_features = features
                latent_pi = self.mlp_extractor.forward_actor(pi_features)
                latent_vf = self.mlp_extractor.forward_critic(vf_features)
            values = self.value_net(latent_vf)
            distribution = self._get_action_dist_from_latent(latent_pi)
        actions = distribution.get_actions(deterministic=deterministic)
        log_prob = distribution.log_prob(actions)
        actions = actions.reshape((-1, *self.action_space.shape))
        return actions, values, log_prob

    def extract_features(self, obs, features_extractor: Optional[BaseFeaturesExtractor] = None):
        if self.share_features_extractor:
            return super().extract_features(obs, self.features_extractor if features_extractor is None else features_extractor)
        if features_extractor is not None:
            warnings.warn("Provided features_extractor will be ignored because the features extractor is not shared.")
        pi_features = super().extract_features(obs, self.pi_features_extractor)
        vf_features = super().extract_features(obs, self.vf_features_extractor)
        return pi_features, vf_features

    def _get_action_dist_from_latent(self, latent_pi: th.Tensor) -> Distribution:
        return self._dist_from_head(self.action_net(latent_pi))

    def _predict(self, observation, deterministic: bool = False) -> th.Tensor:
        return self.get_distribution(observation).get_actions(deterministic=deterministic)

    def evaluate_actions(self, obs, actions: th.Tensor) -> Tuple[th.Tensor, th.Tensor, Optional[th.Tensor]]:
        fused = self._fused_latents(obs)
        if fused is not None:
            head, values = fused
            distribution = self._dist_from_head(head)
        else:
            features = self.extract_features(obs)
            if self.share_features_extractor:
                latent_pi, latent_vf = self.mlp_extractor(features)
            else:
                pi_features, vf_features = features
                latent_pi = self.mlp_extractor.forward_actor(pi_features)
                latent_vf = self.mlp_extractor.forward_critic(vf_features)
            distribution = self._get_action_dist_from_latent(latent_pi)
            values = self.value_net(latent_vf)
        if isinstance(distribution, CategoricalDistribution):
            log_prob, entropy = distribution.log_prob_entropy(actions)
        else:
            log_prob = distribution.log_prob(actions)
            entropy = distribution.entropy()
        return values, log_prob, entropy

    def get_distribution(self, obs) -> Distribution:
        fused = self._fused_latents(obs, want_vf=False)
        if fused is not None:
            return self._dist_from_head(fused[0])
        features = super().extract_features(obs, self.pi_features_extractor)
        latent_pi = self.mlp_extractor.forward_actor(features)
        return self._get_action_dist_from_latent(latent_pi)

    def predict_values(self, obs) -> th.Tensor:
        fused = self._fused_latents(obs, want_pi=False)
        if fused is not None:
            return fused[1]
        features = super().extract_features(obs, self.vf_features_extractor)
        latent_vf = self.mlp_extractor.forward_critic(features)
        return self.value_net(latent_vf)


class ActorCriticCnnPolicy(ActorCriticPolicy):
    def __init__(self, observation_space, action_space, lr_schedule, net_arch=None, activation_fn=nn.Tanh, ortho_init=True,
                 use_sde=False, log_std_init=0.0, full_std=True, use_expln=False, squash_output=False,
                 features_extractor_class=NatureCNN, features_extractor_kwargs=None, share_features_extractor=True,
                 normalize_images=True, optimizer_class=th.optim.Adam, optimizer_kwargs=None):
        super().__init__(observation_space, action_space, lr_schedule, net_arch, activation_fn, ortho_init, use_sde,
                         log_std_init, full_std, use_expln, squash_output, features_extractor_class,
                         features_extractor_kwargs, share_features_extractor, normalize_images, optimizer_class,
                         optimizer_kwargs)


class MultiInputActorCriticPolicy(ActorCriticPolicy):
    def __init__(self, observation_space, action_space, lr_schedule, net_arch=None, activation_fn=nn.Tanh, ortho_init=True,
                 use_sde=False, log_std_init=0.0, full_std=True, use_expln=False, squash_output=False,
                 features_extractor_class=CombinedExtractor, features_extractor_kwargs=None,
                 share_features_extractor=True, normalize_images=True, optimizer_class=th.optim.Adam,
                 optimizer_kwargs=None):
        super().__init__(observation_space, action_space, lr_schedule, net_arch, activation_fn, ortho_init, use_sde,
                         log_std_init, full_std, use_expln, squash_output, features_extractor_class,
                         features_extractor_kwargs, share_features_extractor, normalize_images, optimizer_class,
                         optimizer_kwargs)


MlpPolicy = ActorCriticPolicy
CnnPolicy = ActorCriticCnnPolicy
MultiInputPolicy = MultiInputActorCriticPolicy


def load_policy_file(path, device: Union[th.device, str] = "auto", expected_cls=None):
    """Load a policy written by :meth:`BaseModel.save` (tensor-only file, ``weights_only=True``).

    The class is resolved by import path and restricted to this package. Classes whose
    ``__init__`` pins some constructor arguments (e.g. ``FeedForward32Policy``) are
    rebuilt through the nearest base ``__init__`` that accepts the saved arguments.
    """
    from imitation_amd.rl import save_util

    device = get_device(device)
    saved = th.load(path, map_location=device, weights_only=True)
    if not isinstance(saved, dict) or saved.get("format") != "imitation_amd.policy.v1":
        raise ValueError(f"{path} is not a policy file written by imitation_amd")
    cls_path = saved["class"]
    if not cls_path.startswith("imitation_amd."):
        raise ValueError(f"refusing to construct class outside imitation_amd: {cls_path}")
    pcls = save_util._resolve_class(cls_path)
    if expected_cls is not None and not issubclass(pcls, expected_cls):
        raise TypeError(f"{path} holds a {pcls.__name__}, not a {expected_cls.__name__}")
    data = save_util._decode(json.loads(saved["data"]))
    if "lr_schedule" in data or issubclass(pcls, ActorCriticPolicy):
        data["lr_schedule"] = _constant_zero
    data = {k: v for k, v in data.items() if v is not None or k in ("net_arch",)}
    try:
        model = pcls(**data)
    except TypeError:
        model = None
        for base in pcls.__mro__[1:]:
            if base is object or not issubclass(base, BaseModel):
                continue
            try:
                obj = pcls.__new__(pcls)
                base.__init__(obj, **data)
                model = obj
                break
            except TypeError:
                continue
        if model is None:
            raise
    model.load_state_dict(saved["state_dict"])
    model.to(device)
    return model


def _constant_zero(_progress: float) -> float:
    return 0.0

