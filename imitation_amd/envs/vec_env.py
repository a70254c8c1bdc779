"""Vectorized environments (SB3 ``VecEnv`` semantics).

The reference drives every environment through SB3's ``VecEnv`` API
(``step_async``/``step_wait``/``reset``/``seed``/``env_method``, auto-reset
with ``info["terminal_observation"]``; ``src/imitation/data/rollout.py:162-167``,
``src/imitation/rewards/reward_wrapper.py:100-104``) and builds them with
``DummyVecEnv``/``SubprocVecEnv`` + ``Monitor`` (``util/util.py:144-166``).

Provided here:

* :class:`VecEnv`, :class:`VecEnvWrapper` — the abstract API;
* :class:`DummyVecEnv` — sequential Python envs in-process;
* :class:`SubprocVecEnv` — one worker process per env over pipes;
* :class:`NativeVecEnv` — all envs of the rank stepped in one C++ call
  (``csrc/runtime/vec_env.cpp``); the default for built-in environments;
* :class:`Monitor` — per-env episode stats + CSV (``info["episode"]``);
* :class:`VecNormalize` — running reward (and optionally obs) normalisation
  (used by ``scripts/train_rl.py:117-121`` in the reference).
"""

from __future__ import annotations

import abc
import csv
import json
import multiprocessing as mp
import os
import time
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple, Type, Union

import cloudpickle
import numpy as np

from imitation_amd.envs import core, spaces

VecEnvObs = Union[np.ndarray, Dict[str, np.ndarray], Tuple[np.ndarray, ...]]
VecEnvStepReturn = Tuple[VecEnvObs, np.ndarray, np.ndarray, List[Dict]]


class VecEnv(abc.ABC):
    """Abstract batched environment."""

    def __init__(self, num_envs: int, observation_space: spaces.Space, action_space: spaces.Space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space
        self.reset_infos: List[Dict[str, Any]] = [{} for _ in range(num_envs)]
        self._seeds: List[Optional[int]] = [None for _ in range(num_envs)]
        self._options: List[Dict[str, Any]] = [{} for _ in range(num_envs)]
        self.render_mode = None

    def _reset_seeds(self):
        self._seeds = [None for _ in range(self.num_envs)]

    def _reset_options(self):
        self._options = [{} for _ in range(self.num_envs)]

    @abc.abstractmethod
    def reset(self) -> VecEnvObs:
        ...

    @abc.abstractmethod
    def step_async(self, actions: np.ndarray) -> None:
        ...

    @abc.abstractmethod
    def step_wait(self) -> VecEnvStepReturn:
        ...

    def close(self) -> None:
        pass

    def get_attr(self, attr_name: str, indices=None) -> List[Any]:
        raise NotImplementedError

    def set_attr(self, attr_name: str, value: Any, indices=None) -> None:
        raise NotImplementedError

    def env_method(self, method_name: str, *method_args, indices=None, **method_kwargs) -> List[Any]:
        raise NotImplementedError

    def env_is_wrapped(self, wrapper_class, indices=None) -> List[bool]:
        return [False for _ in self._get_indices(indices)]

    def step(self, actions: np.ndarray) -> VecEnvStepReturn:
        self.step_async(actions)
        return self.step_wait()

    def get_images(self) -> Sequence[Optional[np.ndarray]]:
        return [None] * self.num_envs

    def render(self, mode: Optional[str] = None):
        return None

    def seed(self, seed: Optional[int] = None) -> Sequence[Union[None, int]]:
        if seed is None:
            seed = int(np.random.randint(0, 2**31 - 1))
        self._seeds = [seed + idx for idx in range(self.num_envs)]
        return self._seeds

    def set_options(self, options=None) -> None:
        if options is None:
            options = {}
        if isinstance(options, dict):
            self._options = [dict(options) for _ in range(self.num_envs)]
        else:
            self._options = list(options)

    @property
    def unwrapped(self) -> "VecEnv":
        return self

    def getattr_depth_check(self, name: str, already_found: bool) -> Optional[str]:
        if hasattr(self, name) and already_found:
            return f"{type(self).__module__}.{type(self).__name__}"
        return None

    def _get_indices(self, indices) -> Iterable[int]:
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices


class VecEnvWrapper(VecEnv):
    """Wraps a VecEnv; forwards everything not overridden."""

    def __init__(self, venv: VecEnv, observation_space=None, action_space=None):
        self.venv = venv
        super().__init__(
            num_envs=venv.num_envs,
            observation_space=observation_space or venv.observation_space,
            action_space=action_space or venv.action_space,
        )

    def step_async(self, actions):
        self.venv.step_async(actions)

    @abc.abstractmethod
    def reset(self):
        ...

    @abc.abstractmethod
    def step_wait(self):
        ...

    def seed(self, seed=None):
        return self.venv.seed(seed)

    def set_options(self, options=None):
        return self.venv.set_options(options)

    def close(self):
        return self.venv.close()

    def render(self, mode=None):
        return self.venv.render(mode)

    def get_images(self):
        return self.venv.get_images()

    def get_attr(self, attr_name, indices=None):
        return self.venv.get_attr(attr_name, indices)

    def set_attr(self, attr_name, value, indices=None):
        return self.venv.set_attr(attr_name, value, indices)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        return self.venv.env_method(method_name, *method_args, indices=indices, **method_kwargs)

    def env_is_wrapped(self, wrapper_class, indices=None):
        return self.venv.env_is_wrapped(wrapper_class, indices=indices)

    @property
    def unwrapped(self):
        return self.venv.unwrapped

    def __getattr__(self, name: str):
        if name.startswith("__") or name == "venv":
            raise AttributeError(name)
        return getattr(self.venv, name)


def _obs_buffer(space: spaces.Space, n: int):
    if isinstance(space, spaces.Dict):
        return {k: np.zeros((n,) + tuple(sp.shape), dtype=sp.dtype) for k, sp in space.spaces.items()}
    return np.zeros((n,) + tuple(space.shape), dtype=space.dtype)


def _copy_obs(dst, i, obs):
    if isinstance(dst, dict):
        for k in dst:
            dst[k][i] = obs[k]
    else:
        dst[i] = obs


def _copy_obs_out(buf):
    if isinstance(buf, dict):
        return {k: np.copy(v) for k, v in buf.items()}
    return np.copy(buf)


class DummyVecEnv(VecEnv):
    """Sequentially steps a list of Python :class:`~imitation_amd.envs.core.Env`."""

    def __init__(self, env_fns: List[Callable[[], core.Env]]):
        self.envs = [fn() for fn in env_fns]
        env = self.envs[0]
        super().__init__(len(env_fns), env.observation_space, env.action_space)
        self.buf_obs = _obs_buffer(self.observation_space, self.num_envs)
        self.buf_dones = np.zeros((self.num_envs,), dtype=bool)
        self.buf_rews = np.zeros((self.num_envs,), dtype=np.float32)
        self.buf_infos: List[Dict[str, Any]] = [{} for _ in range(self.num_envs)]
        self.actions = None
        self.metadata = env.metadata

    def step_async(self, actions):
        self.actions = actions

    def step_wait(self):
        for i in range(self.num_envs):
            obs, rew, term, trunc, info = self.envs[i].step(self.actions[i])
            info = dict(info)
            self.buf_dones[i] = term or trunc
            info["TimeLimit.truncated"] = bool(trunc and not term)
            if self.buf_dones[i]:
                info["terminal_observation"] = obs
                obs, self.reset_infos[i] = self.envs[i].reset()
            self.buf_rews[i] = rew
            self.buf_infos[i] = info
            _copy_obs(self.buf_obs, i, obs)
        return _copy_obs_out(self.buf_obs), np.copy(self.buf_rews), np.copy(self.buf_dones), list(self.buf_infos)

    def reset(self):
        for i in range(self.num_envs):
            kw = {}
            if self._seeds[i] is not None:
                kw["seed"] = self._seeds[i]
            if self._options[i]:
                kw["options"] = self._options[i]
            obs, self.reset_infos[i] = self.envs[i].reset(**kw)
            _copy_obs(self.buf_obs, i, obs)
        self._reset_seeds()
        self._reset_options()
        return _copy_obs_out(self.buf_obs)

    def close(self):
        for env in self.envs:
            env.close()

    def get_images(self):
        return [env.render() for env in self.envs]

    def render(self, mode=None):
        imgs = self.get_images()
        return imgs[0] if imgs else None

    def get_attr(self, attr_name, indices=None):
        return [getattr(self.envs[i], attr_name) if not hasattr(self.envs[i], "get_wrapper_attr") else self.envs[i].get_wrapper_attr(attr_name) for i in self._get_indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        for i in self._get_indices(indices):
            setattr(self.envs[i], attr_name, value)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        return [getattr(self.envs[i], method_name)(*method_args, **method_kwargs) for i in self._get_indices(indices)]

    def env_is_wrapped(self, wrapper_class, indices=None):
        out = []
        for i in self._get_indices(indices):
            env = self.envs[i]
            found = False
            while isinstance(env, core.Wrapper):
                if isinstance(env, wrapper_class):
                    found = True
                    break
                env = env.env
            out.append(found)
        return out


# --------------------------------------------------------------------------- subprocess
def _worker(remote, parent_remote, env_fn_wrapper):
    parent_remote.close()
    env = env_fn_wrapper()
    reset_info: Dict[str, Any] = {}
    try:
        while True:
            cmd, data = remote.recv()
            if cmd == "step":
                obs, rew, term, trunc, info = env.step(data)
                info = dict(info)
                done = term or trunc
                info["TimeLimit.truncated"] = bool(trunc and not term)
                if done:
                    info["terminal_observation"] = obs
                    obs, reset_info = env.reset()
                remote.send((obs, rew, done, info, reset_info))
            elif cmd == "reset":
                seed, options = data
                kw = {}
                if seed is not None:
                    kw["seed"] = seed
                if options:
                    kw["options"] = options
                obs, reset_info = env.reset(**kw)
                remote.send((obs, reset_info))
            elif cmd == "render":
                remote.send(env.render())
            elif cmd == "close":
                env.close()
                remote.close()
                break
            elif cmd == "get_spaces":
                remote.send((env.observation_space, env.action_space))
            elif cmd == "env_method":
                method = getattr(env, data[0])
                remote.send(method(*data[1], **data[2]))
            elif cmd == "get_attr":
                remote.send(env.get_wrapper_attr(data) if hasattr(env, "get_wrapper_attr") else getattr(env, data))
            elif cmd == "set_attr":
                remote.send(setattr(env, data[0], data[1]))
            elif cmd == "is_wrapped":
                e, found = env, False
                while isinstance(e, core.Wrapper):
                    if isinstance(e, data):
                        found = True
                        break
                    e = e.env
                remote.send(found)
            else:
                raise NotImplementedError(cmd)
    except EOFError:
        pass


class _CloudpickleWrapper:
    def __init__(self, fn):
        self.fn = fn

    def __getstate__(self):
        return cloudpickle.dumps(self.fn)

    def __setstate__(self, state):
        self.fn = cloudpickle.loads(state)  # noqa: pickle -- our own env factories, parent -> worker

    def __call__(self):
        return self.fn()


class SubprocVecEnv(VecEnv):
    """Each env runs in its own process (``forkserver`` by default, like the reference)."""

    def __init__(self, env_fns: List[Callable[[], core.Env]], start_method: Optional[str] = None):
        self.waiting = False
        self.closed = False
        n = len(env_fns)
        if start_method is None:
            start_method = "forkserver" if "forkserver" in mp.get_all_start_methods() else "spawn"
        ctx = mp.get_context(start_method)
        self.remotes, self.work_remotes = zip(*[ctx.Pipe() for _ in range(n)])
        self.processes = []
        for work_remote, remote, env_fn in zip(self.work_remotes, self.remotes, env_fns):
            proc = ctx.Process(target=_worker, args=(work_remote, remote, _CloudpickleWrapper(env_fn)), daemon=True)
            proc.start()
            self.processes.append(proc)
            work_remote.close()
        self.remotes[0].send(("get_spaces", None))
        obs_space, act_space = self.remotes[0].recv()
        super().__init__(n, obs_space, act_space)

    def step_async(self, actions):
        for remote, action in zip(self.remotes, actions):
            remote.send(("step", action))
        self.waiting = True

    def step_wait(self):
        results = [remote.recv() for remote in self.remotes]
        self.waiting = False
        obs, rews, dones, infos, self.reset_infos = zip(*results)
        return _stack_obs(obs, self.observation_space), np.asarray(rews, dtype=np.float32), np.asarray(dones, dtype=bool), list(infos)

    def reset(self):
        for i, remote in enumerate(self.remotes):
            remote.send(("reset", (self._seeds[i], self._options[i])))
        results = [remote.recv() for remote in self.remotes]
        obs, self.reset_infos = zip(*results)
        self._reset_seeds()
        self._reset_options()
        return _stack_obs(obs, self.observation_space)

    def close(self):
        if self.closed:
            return
        if self.waiting:
            for remote in self.remotes:
                remote.recv()
        for remote in self.remotes:
            remote.send(("close", None))
        for proc in self.processes:
            proc.join()
        self.closed = True

    def get_images(self):
        for remote in self.remotes:
            remote.send(("render", None))
        return [remote.recv() for remote in self.remotes]

    def _targets(self, indices):
        return [self.remotes[i] for i in self._get_indices(indices)]

    def get_attr(self, attr_name, indices=None):
        targets = self._targets(indices)
        for r in targets:
            r.send(("get_attr", attr_name))
        return [r.recv() for r in targets]

    def set_attr(self, attr_name, value, indices=None):
        targets = self._targets(indices)
        for r in targets:
            r.send(("set_attr", (attr_name, value)))
        for r in targets:
            r.recv()

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        targets = self._targets(indices)
        for r in targets:
            r.send(("env_method", (method_name, method_args, method_kwargs)))
        return [r.recv() for r in targets]

    def env_is_wrapped(self, wrapper_class, indices=None):
        targets = self._targets(indices)
        for r in targets:
            r.send(("is_wrapped", wrapper_class))
        return [r.recv() for r in targets]


def _stack_obs(obs_list, space):
    if isinstance(space, spaces.Dict):
        return {k: np.stack([o[k] for o in obs_list]) for k in space.spaces}
    return np.stack(obs_list)


# --------------------------------------------------------------------------- native batched env
class NativeVecEnv(VecEnv):
    """All envs of this rank in one native SoA block, stepped by one C++ call.

    Mirrors ``DummyVecEnv`` + ``Monitor`` + ``TimeLimit`` semantics exactly:
    ``dones = terminated | truncated``, ``info["TimeLimit.truncated"]``,
    ``info["terminal_observation"]``, and ``info["episode"] = {"r", "l", "t"}``
    at episode end (the reference's Monitor wrapper, ``util/util.py:150``).
    """

    def __init__(
        self,
        env_id: str,
        num_envs: int,
        seed: int = 0,
        max_episode_steps: Optional[int] = None,
        log_dir: Optional[str] = None,
    ):
        from imitation_amd import _native

        C = _native.load()
        self._impl = C.BatchedEnv(env_id, int(num_envs), int(max_episode_steps or -1), int(seed) & ((1 << 63) - 1))
        self.env_id = env_id
        obs_space, act_space = native_spaces(env_id, self._impl)
        super().__init__(num_envs, obs_space, act_space)
        self.max_episode_steps = self._impl.max_steps()
        self._is_image = self._impl.is_image()
        self._discrete = self._impl.n_actions() > 0
        self._act_dim = self._impl.act_dim()
        self._actions: Optional[np.ndarray] = None
        self._t_start = time.time()
        self._monitor_files: List[Optional[Any]] = [None] * num_envs
        self.episode_returns: List[float] = []
        self.episode_lengths: List[int] = []
        if log_dir is not None:
            os.makedirs(log_dir, exist_ok=True)
            for i in range(num_envs):
                f = open(os.path.join(log_dir, f"mon{i:03d}.monitor.csv"), "w", newline="")
                f.write("#" + json.dumps({"t_start": self._t_start, "env_id": env_id}) + "\n")
                w = csv.DictWriter(f, fieldnames=("r", "l", "t"))
                w.writeheader()
                f.flush()
                self._monitor_files[i] = (f, w)

    # The impl object is not picklable; re-create on unpickle from metadata.
    def __getstate__(self):
        raise TypeError("NativeVecEnv is not picklable; recreate it with make_vec_env")

    def seed(self, seed: Optional[int] = None):
        seeds = super().seed(seed)
        return seeds

    def seed_envs(self, seeds: Sequence[int]) -> None:
        """Reseed env i with ``seeds[i]`` immediately (per-env non-sequential seeds)."""
        assert len(seeds) == self.num_envs
        self._impl.seed([int(s) for s in seeds])

    def reset(self):
        if any(s is not None for s in self._seeds):
            self._impl.seed([int(s) if s is not None else int(np.random.randint(0, 2**31 - 1)) for s in self._seeds])
        obs = self._impl.reset().numpy()
        self._reset_seeds()
        self._reset_options()
        return obs.copy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        acts = np.asarray(self._actions)
        acts = acts.reshape(self.num_envs, -1).astype(np.float32, copy=False)
        if acts.shape[1] != self._act_dim:
            raise ValueError(f"expected actions of dim {self._act_dim}, got {acts.shape}")
        obs, rew, term, trunc, term_obs, ep_ret, ep_len = self._impl.step(np.ascontiguousarray(acts))
        obs = obs.numpy().copy()
        rew = rew.numpy().copy()
        term = term.numpy().astype(bool)
        trunc = trunc.numpy().astype(bool)
        dones = term | trunc
        infos: List[Dict[str, Any]] = [{} for _ in range(self.num_envs)]
        if dones.any():
            term_obs = term_obs.numpy()
            ep_ret = ep_ret.numpy()
            ep_len = ep_len.numpy()
            now = round(time.time() - self._t_start, 6)
            for i in np.flatnonzero(dones):
                info = infos[i]
                info["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
                info["terminal_observation"] = term_obs[i].copy()
                ep = {"r": round(float(ep_ret[i]), 6), "l": int(ep_len[i]), "t": now}
                info["episode"] = ep
                self.episode_returns.append(ep["r"])
                self.episode_lengths.append(ep["l"])
                mf = self._monitor_files[i]
                if mf is not None:
                    mf[1].writerow(ep)
                    mf[0].flush()
        return obs, rew, dones, infos

    def close(self):
        for mf in self._monitor_files:
            if mf is not None:
                mf[0].close()
        self._monitor_files = [None] * self.num_envs

    def get_attr(self, attr_name, indices=None):
        return [getattr(self, attr_name) for _ in self._get_indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        setattr(self, attr_name, value)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        raise AttributeError(f"NativeVecEnv has no per-env method {method_name}")

    def get_state(self) -> Dict[str, np.ndarray]:
        st = self._impl.get_state()
        return {k: v.numpy().copy() for k, v in st.items()}

    def set_state(self, state: Dict[str, np.ndarray]) -> None:
        import torch as th

        self._impl.set_state({k: th.as_tensor(np.asarray(v)) for k, v in state.items()})


def native_spaces(env_id: str, impl=None) -> Tuple[spaces.Space, spaces.Space]:
    if impl is None:
        from imitation_amd import _native

        impl = _native.load().BatchedEnv(env_id, 1, -1, 0)
    if impl.is_image():
        obs_space = spaces.Box(0, 255, (84, 84, 4), np.uint8)
    else:
        od = impl.obs_dim()
        if env_id.startswith("Pendulum"):
            obs_space = spaces.Box(np.array([-1, -1, -8], np.float32), np.array([1, 1, 8], np.float32))
        elif env_id.startswith("CartPole"):
            hi = np.array([4.8, np.finfo(np.float32).max, 0.41887903, np.finfo(np.float32).max], np.float32)
            obs_space = spaces.Box(-hi, hi)
        elif env_id == "seals/CartPole-v0":  # seals: fixed horizon, no termination -> unbounded box
            hi = np.full(4, np.finfo(np.float32).max, np.float32)
            obs_space = spaces.Box(-hi, hi)
        elif "MountainCar" in env_id:
            obs_space = spaces.Box(np.array([-1.2, -0.07], np.float32), np.array([0.6, 0.07], np.float32))
        else:
            obs_space = spaces.Box(-np.inf, np.inf, (od,), np.float32)
    if impl.n_actions() > 0:
        act_space = spaces.Discrete(impl.n_actions())
    elif env_id.startswith("Pendulum"):
        act_space = spaces.Box(-2.0, 2.0, (1,), np.float32)
    else:
        act_space = spaces.Box(-1.0, 1.0, (impl.act_dim(),), np.float32)
    return obs_space, act_space


class NativeEnv(core.Env):
    """Single-env gymnasium-style view over the native batched implementation."""

    def __init__(self, native_id: str):
        from imitation_amd import _native

        self._impl = _native.load().BatchedEnv(native_id, 1, 10**9, 0)
        self.native_id = native_id
        self.observation_space, self.action_space = native_spaces(native_id, self._impl)
        self._discrete = self._impl.n_actions() > 0

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._impl.seed([int(seed)])
        obs = self._impl.reset().numpy()[0].copy()
        return obs, {}

    def step(self, action):
        a = np.asarray(action, dtype=np.float32).reshape(1, -1)
        obs, rew, term, trunc, term_obs, _, _ = self._impl.step(a)
        terminated = bool(term.numpy()[0])
        o = term_obs.numpy()[0].copy() if terminated else obs.numpy()[0].copy()
        return o, float(rew.numpy()[0]), terminated, False, {}

    def render(self):
        return None


# --------------------------------------------------------------------------- Monitor / VecNormalize
class Monitor(core.Wrapper):
    """Records episode return/length/time into ``info["episode"]`` (+ optional CSV)."""

    EXT = "monitor.csv"

    def __init__(self, env: core.Env, filename: Optional[str] = None, allow_early_resets: bool = True):
        super().__init__(env)
        self.t_start = time.time()
        self.rewards: List[float] = []
        self.episode_returns: List[float] = []
        self.episode_lengths: List[int] = []
        self.episode_times: List[float] = []
        self.total_steps = 0
        self.needs_reset = True
        self._file = None
        self._writer = None
        if filename is not None:
            if not filename.endswith(self.EXT):
                filename = filename + "." + self.EXT if os.path.basename(filename) else os.path.join(filename, self.EXT)
            self._file = open(filename, "w", newline="")
            env_id = env.spec.id if env.spec is not None else None
            self._file.write("#" + json.dumps({"t_start": self.t_start, "env_id": env_id}) + "\n")
            self._writer = csv.DictWriter(self._file, fieldnames=("r", "l", "t"))
            self._writer.writeheader()
            self._file.flush()

    def reset(self, *, seed=None, options=None):
        self.rewards = []
        self.needs_reset = False
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        obs, rew, term, trunc, info = self.env.step(action)
        self.rewards.append(float(rew))
        if term or trunc:
            self.needs_reset = True
            ep_rew, ep_len = sum(self.rewards), len(self.rewards)
            ep = {"r": round(ep_rew, 6), "l": ep_len, "t": round(time.time() - self.t_start, 6)}
            self.episode_returns.append(ep_rew)
            self.episode_lengths.append(ep_len)
            self.episode_times.append(time.time() - self.t_start)
            info = dict(info)
            info["episode"] = ep
            if self._writer is not None:
                self._writer.writerow(ep)
                self._file.flush()
        self.total_steps += 1
        return obs, rew, term, trunc, info

    def get_episode_rewards(self):
        return self.episode_returns

    def get_episode_lengths(self):
        return self.episode_lengths

    def close(self):
        super().close()
        if self._file is not None:
            self._file.close()
            self._file = None


class RunningMeanStd:
    """Chan et al. parallel mean/variance (numpy)."""

    def __init__(self, epsilon: float = 1e-4, shape: Tuple[int, ...] = ()):
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon

    def update(self, arr: np.ndarray) -> None:
        batch_mean = np.mean(arr, axis=0)
        batch_var = np.var(arr, axis=0)
        batch_count = arr.shape[0]
        delta = batch_mean - self.mean
        tot = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot
        m2 = self.var * self.count + batch_var * batch_count + np.square(delta) * self.count * batch_count / tot
        self.mean, self.var, self.count = new_mean, m2 / tot, tot


class VecNormalize(VecEnvWrapper):
    """Normalise observations and/or rewards with running statistics."""

    def __init__(
        self,
        venv: VecEnv,
        training: bool = True,
        norm_obs: bool = True,
        norm_reward: bool = True,
        clip_obs: float = 10.0,
        clip_reward: float = 10.0,
        gamma: float = 0.99,
        epsilon: float = 1e-8,
    ):
        super().__init__(venv)
        self.training = training
        self.norm_obs = norm_obs
        self.norm_reward = norm_reward
        self.clip_obs = clip_obs
        self.clip_reward = clip_reward
        self.gamma = gamma
        self.epsilon = epsilon
        shape = self.observation_space.shape if isinstance(self.observation_space, spaces.Box) else ()
        self.obs_rms = RunningMeanStd(shape=shape)
        self.ret_rms = RunningMeanStd(shape=())
        self.returns = np.zeros(self.num_envs)
        self.old_obs = None
        self.old_reward = None

    def step_wait(self):
        obs, rews, dones, infos = self.venv.step_wait()
        self.old_obs = obs
        self.old_reward = rews
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        obs = self.normalize_obs(obs)
        if self.training:
            self.returns = self.returns * self.gamma + rews
            self.ret_rms.update(self.returns)
        rews = self.normalize_reward(rews)
        for i in np.flatnonzero(dones):
            if "terminal_observation" in infos[i]:
                infos[i]["terminal_observation"] = self.normalize_obs(infos[i]["terminal_observation"])
        self.returns[dones] = 0
        return obs, rews, dones, infos

    def normalize_obs(self, obs):
        if not self.norm_obs:
            return obs
        return np.clip((obs - self.obs_rms.mean) / np.sqrt(self.obs_rms.var + self.epsilon), -self.clip_obs, self.clip_obs).astype(np.float32)

    def normalize_reward(self, rew):
        if not self.norm_reward:
            return rew
        return np.clip(rew / np.sqrt(self.ret_rms.var + self.epsilon), -self.clip_reward, self.clip_reward).astype(np.float32)

    def get_original_obs(self):
        return self.old_obs

    def get_original_reward(self):
        return self.old_reward

    def reset(self):
        obs = self.venv.reset()
        self.old_obs = obs
        self.returns = np.zeros(self.num_envs)
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        return self.normalize_obs(obs)

    def save(self, path: str) -> None:
        import pickle

        with open(path, "wb") as f:
            pickle.dump({"obs_rms": self.obs_rms.__dict__, "ret_rms": self.ret_rms.__dict__, "gamma": self.gamma, "norm_obs": self.norm_obs, "norm_reward": self.norm_reward}, f)


def unwrap_vec_wrapper(venv: VecEnv, wrapper_class: Type[VecEnvWrapper]) -> Optional[VecEnvWrapper]:
    env = venv
    while isinstance(env, VecEnvWrapper):
        if isinstance(env, wrapper_class):
            return env
        env = env.venv
    return None


def is_vecenv_wrapped(venv: VecEnv, wrapper_class) -> bool:
    return unwrap_vec_wrapper(venv, wrapper_class) is not None
