"""RL algorithm base classes (the SB3 ``BaseAlgorithm`` surface used by the reference:
``learn(total_timesteps, reset_num_timesteps=False, callback)``, ``set_env``,
``get_env``, ``set_logger``, ``predict``, ``device``, ``save``/``load``;
``src/imitation/algorithms/adversarial/common.py:243-244, 414-419``).

Data parallel: every rank runs its own envs; gradient averaging happens inside
each algorithm's update through :class:`imitation_amd.parallel.GradBucket`
(one fused all-reduce per optimizer step). ``num_timesteps`` counts this rank's
env steps; the global count is ``num_timesteps * world_size``.
"""

from __future__ import annotations

import warnings

import collections
import pathlib
import sys
import time
from typing import Any, Dict, Iterable, List, Optional, Tuple, Type, Union

import numpy as np
import torch as th

from imitation_amd.envs import core as env_core
from imitation_amd.envs import spaces
from imitation_amd.envs.vec_env import DummyVecEnv, Monitor, VecEnv, VecNormalize
from imitation_amd.rl import logger as rl_logger
from imitation_amd.rl import save_util
from imitation_amd.rl.buffers import DictRolloutBuffer, ReplayBuffer, RolloutBuffer
from imitation_amd.rl.callbacks import BaseCallback, CallbackList, ConvertCallback, convert_callback
from imitation_amd.rl.policies import BasePolicy, get_device, get_schedule_fn, obs_as_tensor


def safe_mean(arr) -> float:
    return float("nan") if len(arr) == 0 else float(np.mean(arr))


def explained_variance(y_pred: np.ndarray, y_true: np.ndarray) -> float:
    var_y = np.var(y_true)
    return float("nan") if var_y == 0 else float(1 - np.var(y_true - y_pred) / var_y)


def set_random_seed(seed: int, using_cuda: bool = False) -> None:
    import random

    random.seed(seed)
    np.random.seed(seed)
    th.manual_seed(seed)
    if using_cuda and th.cuda.is_available():
        th.cuda.manual_seed_all(seed)


def update_learning_rate(optimizer: th.optim.Optimizer, learning_rate: float) -> None:
    for g in optimizer.param_groups:
        g["lr"] = learning_rate


def check_for_correct_spaces(env, observation_space: spaces.Space, action_space: spaces.Space) -> None:
    if observation_space != env.observation_space:
        raise ValueError(f"Observation spaces do not match: {observation_space} != {env.observation_space}")
    if action_space != env.action_space:
        raise ValueError(f"Action spaces do not match: {action_space} != {env.action_space}")


class BaseAlgorithm:
    policy_aliases: Dict[str, Type[BasePolicy]] = {}
    _EXCLUDE_SAVE = {
        "policy", "device", "env", "replay_buffer", "rollout_buffer", "_vec_normalize_env", "_episode_storage",
        "_logger", "_custom_logger", "lr_schedule", "clip_range", "clip_range_vf", "ep_info_buffer",
        "ep_success_buffer", "_last_obs", "_last_episode_starts", "_last_original_obs", "exploration_schedule",
        "q_net", "q_net_target", "actor", "critic", "critic_target", "log_ent_coef", "ent_coef_optimizer",
        "target_entropy_tensor", "_grad_bucket", "batch_norm_stats", "batch_norm_stats_target",
    }

    def __init__(
        self,
        policy: Union[str, Type[BasePolicy]],
        env,
        learning_rate,
        policy_kwargs: Optional[Dict[str, Any]] = None,
        stats_window_size: int = 100,
        tensorboard_log: Optional[str] = None,
        verbose: int = 0,
        device: Union[th.device, str] = "auto",
        support_multi_env: bool = False,
        monitor_wrapper: bool = True,
        seed: Optional[int] = None,
        use_sde: bool = False,
        sde_sample_freq: int = -1,
        supported_action_spaces: Optional[Tuple[Type[spaces.Space], ...]] = None,
    ):
        if isinstance(policy, str):
            if policy not in self.policy_aliases:
                raise ValueError(f"Policy {policy} unknown")
            self.policy_class = self.policy_aliases[policy]
        else:
            self.policy_class = policy
        self.device = get_device(device)
        self.verbose = verbose
        self.policy_kwargs = {} if policy_kwargs is None else dict(policy_kwargs)
        self.num_timesteps = 0
        self._total_timesteps = 0
        self._num_timesteps_at_start = 0
        self.seed = seed
        self.action_noise = None
        self.start_time = 0.0
        self.learning_rate = learning_rate
        self.tensorboard_log = tensorboard_log
        self._last_obs = None
        self._last_episode_starts: Optional[np.ndarray] = None
        self._last_original_obs = None
        self._episode_num = 0
        self.use_sde = use_sde
        self.sde_sample_freq = sde_sample_freq
        self._current_progress_remaining = 1.0
        self._stats_window_size = stats_window_size
        self.ep_info_buffer: Optional[collections.deque] = None
        self.ep_success_buffer: Optional[collections.deque] = None
        self._n_updates = 0
        self._custom_logger = False
        self._logger: Optional[rl_logger.Logger] = None
        self.env: Optional[VecEnv] = None
        self._vec_normalize_env: Optional[VecNormalize] = None
        self.policy: Optional[BasePolicy] = None
        self.lr_schedule = None
        self.n_envs = 1
        if env is not None:
            env = self._wrap_env(env, self.verbose, monitor_wrapper)
            self.observation_space = env.observation_space
            self.action_space = env.action_space
            self.n_envs = env.num_envs
            self.env = env
            self._vec_normalize_env = self._unwrap_vec_normalize(env)
            if supported_action_spaces is not None and not isinstance(self.action_space, supported_action_spaces):
                raise ValueError(
                    f"The algorithm only supports {supported_action_spaces} as action spaces but {self.action_space} was provided"
                )
            if not support_multi_env and self.n_envs > 1:
                raise ValueError("Error: the model does not support multiple envs; it requires a single vectorized environment.")

    @staticmethod
    def _unwrap_vec_normalize(env):
        e = env
        while e is not None:
            if isinstance(e, VecNormalize):
                return e
            e = getattr(e, "venv", None)
        return None

    @staticmethod
    def _wrap_env(env, verbose: int = 0, monitor_wrapper: bool = True) -> VecEnv:
        if isinstance(env, str):
            env = env_core.make(env)
        if not isinstance(env, VecEnv):
            if monitor_wrapper and not isinstance(env, Monitor):
                env = Monitor(env)
            env = DummyVecEnv([lambda: env])
        return env

    def _setup_model(self) -> None:
        raise NotImplementedError

    def _setup_lr_schedule(self) -> None:
        self.lr_schedule = get_schedule_fn(self.learning_rate)

    def _update_current_progress_remaining(self, num_timesteps: int, total_timesteps: int) -> None:
        self._current_progress_remaining = 1.0 - float(num_timesteps) / float(max(total_timesteps, 1))

    def _update_learning_rate(self, optimizers) -> None:
        lr = self.lr_schedule(self._current_progress_remaining)
        self.logger.record("train/learning_rate", lr)
        if not isinstance(optimizers, list):
            optimizers = [optimizers]
        for opt in optimizers:
            update_learning_rate(opt, lr)

    def _excluded_save_params(self) -> set:
        return set(self._EXCLUDE_SAVE)

    def _get_torch_save_params(self) -> Tuple[List[str], List[str]]:
        return ["policy"], []

    def _init_callback(self, callback, progress_bar: bool = False) -> BaseCallback:
        callback = convert_callback(callback)
        callback.init_callback(self)
        return callback

    def _setup_learn(self, total_timesteps: int, callback=None, reset_num_timesteps: bool = True,
                     tb_log_name: str = "run", progress_bar: bool = False):
        self.start_time = time.time_ns()
        if self.ep_info_buffer is None or reset_num_timesteps:
            self.ep_info_buffer = collections.deque(maxlen=self._stats_window_size)
            self.ep_success_buffer = collections.deque(maxlen=self._stats_window_size)
        if reset_num_timesteps:
            self.num_timesteps = 0
            self._episode_num = 0
        else:
            total_timesteps += self.num_timesteps
        self._total_timesteps = total_timesteps
        self._num_timesteps_at_start = self.num_timesteps
        if reset_num_timesteps or self._last_obs is None:
            assert self.env is not None
            self._last_obs = self.env.reset()
            self._last_episode_starts = np.ones((self.env.num_envs,), dtype=bool)
            if self._vec_normalize_env is not None:
                self._last_original_obs = self._vec_normalize_env.get_original_obs()
        if not self._custom_logger:
            self._logger = rl_logger.configure(None, ["stdout"] if self.verbose >= 1 else [])
        callback = self._init_callback(callback, progress_bar)
        return total_timesteps, callback

    def _update_info_buffer(self, infos: List[Dict[str, Any]], dones: Optional[np.ndarray] = None) -> None:
        assert self.ep_info_buffer is not None
        if dones is None:
            dones = np.array([False] * len(infos))
        for idx, info in enumerate(infos):
            ep = info.get("episode")
            ok = info.get("is_success")
            if ep is not None:
                self.ep_info_buffer.extend([ep])
            if ok is not None and dones[idx]:
                self.ep_success_buffer.append(ok)

    def get_env(self) -> Optional[VecEnv]:
        return self.env

    def get_vec_normalize_env(self) -> Optional[VecNormalize]:
        return self._vec_normalize_env

    def set_env(self, env, force_reset: bool = True) -> None:
        env = self._wrap_env(env, self.verbose)
        assert env.num_envs == self.n_envs, (
            "The number of environments to be set is different from the number of environments in the model: "
            f"({env.num_envs} != {self.n_envs}), whereas `set_env` requires them to be the same."
        )
        check_for_correct_spaces(env, self.observation_space, self.action_space)
        self._vec_normalize_env = self._unwrap_vec_normalize(env)
        if force_reset:
            self._last_obs = None
        self.n_envs = env.num_envs
        self.env = env

    def set_logger(self, logger: rl_logger.Logger) -> None:
        self._logger = logger
        self._custom_logger = True

    @property
    def logger(self) -> rl_logger.Logger:
        if self._logger is None:
            self._logger = rl_logger.configure(None, [])
        return self._logger

    def learn(self, total_timesteps: int, callback=None, log_interval: int = 100, tb_log_name: str = "run",
              reset_num_timesteps: bool = True, progress_bar: bool = False):
        raise NotImplementedError

    def predict(self, observation, state=None, episode_start=None, deterministic: bool = False):
        return self.policy.predict(observation, state, episode_start, deterministic)

    def set_random_seed(self, seed: Optional[int] = None) -> None:
        if seed is None:
            return
        set_random_seed(seed, using_cuda=self.device.type == "cuda")
        self.action_space.seed(seed)
        if self.env is not None:
            self.env.seed(seed)

    # ---------------------------------------------------------------- persistence
    def get_parameters(self) -> Dict[str, Dict]:
        state_dicts_names, _ = self._get_torch_save_params()
        params = {}
        for name in state_dicts_names:
            attr = self
            for part in name.split("."):
                attr = getattr(attr, part)
            params[name] = attr.state_dict()
        return params

    def set_parameters(self, load_path_or_dict, exact_match: bool = True, device: Union[th.device, str] = "auto") -> None:
        params = load_path_or_dict
        if not isinstance(params, dict):
            _, params, _ = save_util.load_from_zip_file(load_path_or_dict, device=device)
        objects_needing_update = set(self._get_torch_save_params()[0])
        updated = set()
        for name, sd in params.items():
            attr = self
            try:
                for part in name.split("."):
                    attr = getattr(attr, part)
            except AttributeError:
                continue
            if isinstance(attr, th.optim.Optimizer):
                try:
                    attr.load_state_dict(sd)
                except Exception:
                    continue
            else:
                attr.load_state_dict(sd, strict=exact_match)
            updated.add(name)
        if exact_match and not objects_needing_update.issubset(updated | {n for n in objects_needing_update if n.endswith("optimizer")}):
            missing = objects_needing_update - updated
            raise ValueError(f"Names of parameters do not match agents' parameters: expected {objects_needing_update}, got {updated} (missing {missing})")

    def save(self, path, exclude: Optional[Iterable[str]] = None, include: Optional[Iterable[str]] = None) -> None:
        data = {}
        excl = self._excluded_save_params() | set(exclude or [])
        if include is not None:
            excl -= set(include)
        for k, v in self.__dict__.items():
            if k in excl or isinstance(v, (th.nn.Module, th.optim.Optimizer, th.Tensor)):
                continue
            data[k] = v
        data["policy_class"] = self.policy_class
        data["algo_class"] = type(self)
        names, _ = self._get_torch_save_params()
        params = self.get_parameters()
        if self.policy is not None and getattr(self.policy, "optimizer", None) is not None:
            params["policy.optimizer"] = self.policy.optimizer.state_dict()
        save_util.save_to_zip_file(path, data=data, params=params)

    @classmethod
    def load(cls, path, env=None, device: Union[th.device, str] = "auto", custom_objects=None, print_system_info=False,
             force_reset: bool = True, **kwargs):
        device = get_device(device)
        data, params, _ = save_util.load_from_zip_file(path, device=device)
        if custom_objects:
            data.update(custom_objects)
        policy_kwargs = data.get("policy_kwargs") or {}
        if not isinstance(policy_kwargs, dict):
            policy_kwargs = {}
        policy_kwargs = {k: v for k, v in policy_kwargs.items() if v is not None}
        if "policy_kwargs" in kwargs and kwargs["policy_kwargs"] != policy_kwargs:
            policy_kwargs = kwargs.pop("policy_kwargs")
        obs_space = data.get("observation_space")
        act_space = data.get("action_space")
        if obs_space is None or act_space is None:
            raise ValueError("archive lacks decodable observation/action spaces")
        if env is not None:
            env = cls._wrap_env(env, data.get("verbose", 0))
            if (isinstance(obs_space, spaces.Box) and isinstance(env.observation_space, spaces.Box)
                    and obs_space != env.observation_space and obs_space.shape == env.observation_space.shape
                    and obs_space.dtype == env.observation_space.dtype):
                # Same layout, different declared bounds (e.g. a gymnasium CartPole expert on the
                # unbounded seals CartPole): the network is unaffected by the bounds, so adopt the env's.
                warnings.warn(f"Observation-space bounds of the archive {obs_space} differ from the env's "
                              f"{env.observation_space}; using the env's.")
                obs_space = env.observation_space
            check_for_correct_spaces(env, obs_space, act_space)
        policy_class = data.get("policy_class")
        if not isinstance(policy_class, type):
            policy_class = "MlpPolicy"
        model = cls.__new__(cls)
        model._load_init(policy_class, env, device, data, policy_kwargs, obs_space, act_space)
        for k, v in kwargs.items():
            setattr(model, k, v)
        model._setup_model()
        sd = params.get("policy")
        if sd is not None:
            model.policy.load_state_dict(sd, strict=True)
        opt = params.get("policy.optimizer")
        if opt is not None:
            try:
                model.policy.optimizer.load_state_dict(opt)
            except Exception:
                pass
        if force_reset and env is not None:
            model._last_obs = None
        return model

    def _load_init(self, policy_class, env, device, data, policy_kwargs, obs_space, act_space) -> None:
        """Minimal constructor used by :meth:`load` (attributes from the archive)."""
        BaseAlgorithm.__init__(
            self,
            policy=policy_class if isinstance(policy_class, type) else self.policy_aliases.get(policy_class, policy_class),
            env=None,
            learning_rate=data.get("learning_rate", 3e-4) if isinstance(data.get("learning_rate"), (int, float)) else 3e-4,
            policy_kwargs=policy_kwargs,
            device=device,
            verbose=data.get("verbose", 0) or 0,
            seed=data.get("seed"),
        )
        self.observation_space = obs_space
        self.action_space = act_space
        self.n_envs = int(data.get("n_envs", 1) or 1)
        for k, v in data.items():
            if k in ("policy_class", "algo_class", "observation_space", "action_space", "policy_kwargs", "learning_rate",
                     "clip_range", "lr_schedule", "device"):
                continue
            if v is None and k in self.__dict__ and self.__dict__[k] is not None:
                continue
            if isinstance(v, (int, float, str, bool, list)) or v is None:
                self.__dict__[k] = v
        if env is not None:
            self.env = env
            self.n_envs = env.num_envs
        self._post_load_init(data)

    def _post_load_init(self, data: Dict[str, Any]) -> None:
        pass

    def _dump_logs_common(self) -> None:
        assert self.ep_info_buffer is not None
        time_elapsed = max((time.time_ns() - self.start_time) / 1e9, sys.float_info.epsilon)
        fps = int((self.num_timesteps - self._num_timesteps_at_start) / time_elapsed)
        if len(self.ep_info_buffer) > 0 and len(self.ep_info_buffer[0]) > 0:
            self.logger.record("rollout/ep_rew_mean", safe_mean([ep["r"] for ep in self.ep_info_buffer]))
            self.logger.record("rollout/ep_len_mean", safe_mean([ep["l"] for ep in self.ep_info_buffer]))
        self.logger.record("time/fps", fps)
        self.logger.record("time/time_elapsed", int(time_elapsed), exclude="tensorboard")
        self.logger.record("time/total_timesteps", self.num_timesteps, exclude="tensorboard")


class OnPolicyAlgorithm(BaseAlgorithm):
    """Rollout collection into a device-resident :class:`RolloutBuffer` + abstract ``train``."""

    rollout_buffer: RolloutBuffer

    def __init__(self, policy, env, learning_rate, n_steps: int, gamma: float, gae_lambda: float, ent_coef: float,
                 vf_coef: float, max_grad_norm: float, use_sde: bool = False, sde_sample_freq: int = -1,
                 rollout_buffer_class=None, rollout_buffer_kwargs=None, stats_window_size: int = 100,
                 tensorboard_log=None, monitor_wrapper: bool = True, policy_kwargs=None, verbose: int = 0,
                 seed=None, device="auto", _init_setup_model: bool = True, supported_action_spaces=None):
        super().__init__(policy=policy, env=env, learning_rate=learning_rate, policy_kwargs=policy_kwargs,
                         verbose=verbose, device=device, use_sde=use_sde, sde_sample_freq=sde_sample_freq,
                         support_multi_env=True, monitor_wrapper=monitor_wrapper, seed=seed,
                         stats_window_size=stats_window_size, tensorboard_log=tensorboard_log,
                         supported_action_spaces=supported_action_spaces)
        self.n_steps = n_steps
        self.gamma = gamma
        self.gae_lambda = gae_lambda
        self.ent_coef = ent_coef
        self.vf_coef = vf_coef
        self.max_grad_norm = max_grad_norm
        self.rollout_buffer_class = rollout_buffer_class
        self.rollout_buffer_kwargs = rollout_buffer_kwargs or {}
        if _init_setup_model:
            self._setup_model()

    def _setup_model(self) -> None:
        self._setup_lr_schedule()
        self.set_random_seed(self.seed)
        buffer_cls = self.rollout_buffer_class or (DictRolloutBuffer if isinstance(self.observation_space, spaces.Dict)
                                                   else RolloutBuffer)
        self.rollout_buffer = buffer_cls(self.n_steps, self.observation_space, self.action_space, device=self.device,
                                         gamma=self.gamma, gae_lambda=self.gae_lambda, n_envs=self.n_envs,
                                         **self.rollout_buffer_kwargs)
        self.policy = self.policy_class(self.observation_space, self.action_space, self.lr_schedule, use_sde=self.use_sde,
                                        **self.policy_kwargs)
        self.policy = self.policy.to(self.device)
        from imitation_amd.parallel import dist as pdist

        pdist.broadcast_module(self.policy)

    def collect_rollouts(self, env: VecEnv, callback: BaseCallback, rollout_buffer: RolloutBuffer, n_rollout_steps: int) -> bool:
        assert self._last_obs is not None, "No previous observation was provided"
        self.policy.set_training_mode(False)
        n_steps = 0
        rollout_buffer.reset()
        callback.on_rollout_start()
        box = isinstance(self.action_space, spaces.Box)
        new_obs = self._last_obs
        dones = self._last_episode_starts
        while n_steps < n_rollout_steps:
            with th.no_grad():
                obs_tensor = obs_as_tensor(self._last_obs, self.device)
                actions_t, values, log_probs = self.policy(obs_tensor)
            actions = actions_t.cpu().numpy()
            clipped_actions = actions
            if box:
                if self.policy.squash_output:
                    clipped_actions = self.policy.unscale_action(clipped_actions)
                else:
                    clipped_actions = np.clip(actions, self.action_space.low, self.action_space.high)
            new_obs, rewards, dones, infos = env.step(clipped_actions)
            self.num_timesteps += env.num_envs
            callback.update_locals(locals())
            if not callback.on_step():
                return False
            self._update_info_buffer(infos, dones)
            n_steps += 1
            if isinstance(self.action_space, spaces.Discrete):
                actions = actions.reshape(-1, 1)
            # bootstrap truncated episodes with V(terminal_obs): one batched call
            trunc = [i for i, d in enumerate(dones) if d and infos[i].get("terminal_observation") is not None
                     and infos[i].get("TimeLimit.truncated", False)]
            if trunc:
                rewards = np.asarray(rewards, dtype=np.float32).copy()
                term_obs = np.stack([infos[i]["terminal_observation"] for i in trunc])
                with th.no_grad():
                    tv = self.policy.predict_values(obs_as_tensor(term_obs, self.device)).reshape(-1).cpu().numpy()
                for j, i in enumerate(trunc):
                    rewards[i] += self.gamma * tv[j]
            rollout_buffer.add(self._last_obs, actions, rewards, self._last_episode_starts, values, log_probs)
            self._last_obs = new_obs
            self._last_episode_starts = dones
        with th.no_grad():
            values = self.policy.predict_values(obs_as_tensor(new_obs, self.device))
        rollout_buffer.compute_returns_and_advantage(last_values=values, dones=dones)
        callback.update_locals(locals())
        callback.on_rollout_end()
        return True

    def train(self) -> None:
        raise NotImplementedError

    def _dump_logs(self, iteration: int) -> None:
        self.logger.record("time/iterations", iteration, exclude="tensorboard")
        self._dump_logs_common()
        self.logger.dump(step=self.num_timesteps)

    def learn(self, total_timesteps: int, callback=None, log_interval: int = 1, tb_log_name: str = "OnPolicyAlgorithm",
              reset_num_timesteps: bool = True, progress_bar: bool = False):
        iteration = 0
        total_timesteps, callback = self._setup_learn(total_timesteps, callback, reset_num_timesteps, tb_log_name, progress_bar)
        callback.on_training_start(locals(), globals())
        assert self.env is not None
        while self.num_timesteps < total_timesteps:
            cont = self.collect_rollouts(self.env, callback, self.rollout_buffer, n_rollout_steps=self.n_steps)
            if not cont:
                break
            iteration += 1
            self._update_current_progress_remaining(self.num_timesteps, total_timesteps)
            if log_interval is not None and iteration % log_interval == 0:
                self._dump_logs(iteration)
            self.train()
        callback.on_training_end()
        return self

    def _post_load_init(self, data):
        for k in ("n_steps", "gamma", "gae_lambda", "ent_coef", "vf_coef", "max_grad_norm"):
            if k in data and data[k] is not None:
                setattr(self, k, data[k])
        self.rollout_buffer_class = None
        self.rollout_buffer_kwargs = {}
