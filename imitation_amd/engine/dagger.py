"""Device DAgger collection: env stepping, frame rendering, both policies and the β-mix on the GPU.

The reference collects every DAgger round through a host VecEnv wrapper
(``src/imitation/algorithms/dagger.py:151-287`` InteractiveTrajectoryCollector +
``data/rollout.py:426-554`` generate_trajectories): per step the frames cross the
host/device boundary for the expert forward, again for the learner forward, the
actions come back, the env steps on the CPU and every finished episode is pickled to
disk before BC re-reads everything. Here one round is:

* K env steps per HIP-graph replay (``chunk``): expert CNN forward (deterministic,
  as ``generate_trajectories(deterministic_policy=True)``), learner forward with
  sampling (``policy.predict`` default), ``rand > β`` mask, the executed action into
  ``dagger_env_step`` (csrc/kernels/dagger.hip: the IA_HD physics of the host env +
  in-place frame-stack rendering, TimeLimit, auto-reset with terminal frames), and the
  expert action / observation recorded into the round's device buffers;
* one pinned D2H copy of the chunk's done flags per replay, which drives the
  reference's unbiased stopping rule on the host (``sample_until`` over finished
  episodes, then each env runs out its current episode; steps of inactive envs are
  ignored);
* the round's finished episodes are gathered on the device into the flat demo
  aggregate BC trains on (:class:`DeviceDemoAggregate`, DP all-gathered over RCCL),
  and copied to the host once for the reference-format demo files, which a
  background thread writes (:class:`AsyncDemoWriter`).
"""

from __future__ import annotations

import os
import collections
import queue
import threading
import time
from typing import Callable, Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch as th

from imitation_amd.utils import graphs

from imitation_amd import ops
from imitation_amd.ops import rl as rl_ops
from imitation_amd.data import types
from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl.distributions import CategoricalDistribution, DiagGaussianDistribution
from imitation_amd.rl.policies import ActorCriticPolicy


def _unwrap_native(venv):
    from imitation_amd.envs.vec_env import NativeVecEnv

    e = venv
    while e is not None:
        if isinstance(e, NativeVecEnv):
            return e
        e = getattr(e, "venv", None)
    return None


def supports(venv, expert_policy, learner_policy) -> Tuple[bool, str]:
    """Whether :class:`DeviceDAggerCollector` can collect for this configuration."""
    if os.environ.get("IMITATION_AMD_DAGGER_DEVICE", "1") == "0":
        return False, "disabled by IMITATION_AMD_DAGGER_DEVICE=0"
    if not th.cuda.is_available():
        return False, "no GPU"
    nat = _unwrap_native(venv)
    from imitation_amd.data.wrappers import VecRolloutInfoWrapper

    # RolloutInfoWrapper only mirrors obs/rewards into infos, which device demos do not carry
    if nat is None or not (venv is nat or (isinstance(venv, VecRolloutInfoWrapper) and venv.venv is nat)):
        return False, "env is not a native vector env (optionally under RolloutInfoWrapper)"
    for name, pol in (("expert", expert_policy), ("learner", learner_policy)):
        if not isinstance(pol, ActorCriticPolicy):
            return False, f"{name} policy is not an ActorCriticPolicy"
        if pol.device.type != "cuda":
            return False, f"{name} policy is not on the GPU"
        if pol.squash_output:
            return False, f"{name} policy squashes its output"
        if type(pol.action_dist) not in (CategoricalDistribution, DiagGaussianDistribution):
            return False, f"{name} policy action distribution {type(pol.action_dist).__name__}"
    if isinstance(nat.observation_space, spaces.Dict):
        return False, "dict observations"
    if not isinstance(nat.action_space, (spaces.Discrete, spaces.Box)):
        return False, "action space"
    return True, ""


def policy_actions(policy: ActorCriticPolicy, obs: th.Tensor, deterministic: bool) -> th.Tensor:
    """``policy.predict`` on a device batch without host syncs (capturable): argmax / mean
    when deterministic, else Gumbel-max sampling of the categorical or mean + std * N(0, 1);
    Box actions are clipped to the space like ``predict`` does."""
    dist = policy.get_distribution(obs)
    if isinstance(dist, CategoricalDistribution):
        logits = dist.logits
        if deterministic:
            return logits.argmax(-1)
        u = th.rand_like(logits).clamp_(1e-20, 1.0)
        return (logits - th.log(-th.log(u))).argmax(-1)
    mean = dist.mean_actions
    a = mean if deterministic else mean + th.exp(dist.log_std) * th.randn_like(mean)
    low = th.as_tensor(policy.action_space.low, device=a.device, dtype=a.dtype)
    high = th.as_tensor(policy.action_space.high, device=a.device, dtype=a.dtype)
    return th.max(th.min(a, high), low)


class CnnActor:
    """Graph-static inference of a NatureCNN :class:`ActorCriticPolicy` with discrete actions
    (the DAgger-Pong expert and learner): three ``conv_fwd`` launches straight on the uint8
    frames (``in_scale`` = 1/255 replaces the float preprocessing), ``cnn_fc`` and the
    ``cnn_head`` action choice (csrc/kernels/cnn_infer.hip). The bf16 NHWC conv weights and
    the (h, w, c)-ordered FC weight are persistent copies refreshed by :meth:`refresh`
    (call it whenever the module's weights changed); biases and the head are read live."""

    def __init__(self, policy: ActorCriticPolicy, obs_shape: Sequence[int]):
        from torch import nn

        self.policy = policy
        fe = policy.features_extractor
        self.convs = [m for m in fe.cnn if isinstance(m, nn.Conv2d)]
        self.fc = fe.linear[0]
        self.head = policy.action_net
        H, W, C = obs_shape
        self.strides = [int(c.stride[0]) for c in self.convs]
        for c in self.convs:
            H, W, C = (H - c.kernel_size[0]) // c.stride[0] + 1, (W - c.kernel_size[1]) // c.stride[1] + 1, c.out_channels
        self.out_hwc = (H, W, C)
        dev = policy.device
        self.wb = [th.empty(c.out_channels, c.kernel_size[0], c.kernel_size[1], c.in_channels, dtype=th.bfloat16, device=dev)
                   for c in self.convs]
        self.fc_w = th.empty(self.fc.out_features, self.fc.in_features, dtype=th.bfloat16, device=dev)
        self.refresh()

    @staticmethod
    def applicable(policy: ActorCriticPolicy, obs_shape: Sequence[int]) -> bool:
        from torch import nn

        from imitation_amd.ops import conv as conv_ops
        from imitation_amd.rl.torch_layers import NatureCNN

        fe = policy.features_extractor
        if not isinstance(fe, NatureCNN) or not fe.channels_last_input or not policy.share_features_extractor:
            return False
        if not policy.normalize_images or len(list(policy.mlp_extractor.policy_net)) != 0:
            return False
        if not isinstance(policy.action_space, spaces.Discrete) or int(policy.action_space.n) > 64:
            return False
        mods = list(fe.cnn)
        convs = [m for m in mods if isinstance(m, nn.Conv2d)]
        if any(c.padding not in (0, (0, 0)) or c.stride[0] != c.stride[1] or c.dilation not in (1, (1, 1)) or c.groups != 1
               for c in convs):
            return False
        if [type(m) for m in mods] != [nn.Conv2d, nn.ReLU] * len(convs) + [nn.Flatten]:
            return False
        lin = list(fe.linear)
        if len(lin) != 2 or not isinstance(lin[0], nn.Linear) or not isinstance(lin[1], nn.ReLU):
            return False
        if lin[0].in_features % 32 or lin[0].out_features % 16:
            return False
        return conv_ops.supported((1,) + tuple(obs_shape), [c.weight for c in convs], [c.stride[0] for c in convs])

    @th.no_grad()
    def refresh(self) -> None:
        for wb, c in zip(self.wb, self.convs):
            wb.copy_(c.weight.permute(0, 2, 3, 1))
        H, W, C = self.out_hwc
        self.fc_w.copy_(self.fc.weight.view(self.fc.out_features, C, H, W).permute(0, 2, 3, 1).reshape(self.fc.out_features, -1))

    @staticmethod
    def paired(a: "CnnActor", b: "CnnActor") -> bool:
        """Whether two actors have identical shapes (then :meth:`hidden_pair` applies)."""
        return (a.strides == b.strides and a.out_hwc == b.out_hwc and [w.shape for w in a.wb] == [w.shape for w in b.wb]
                and a.fc_w.shape == b.fc_w.shape)

    @staticmethod
    def hidden_pair(a: "CnnActor", b: "CnnActor", obs_u8: th.Tensor) -> Tuple[th.Tensor, th.Tensor]:
        """Both actors' hidden features of the same frames, each layer of the two networks in
        ONE launch (``conv_fwd_pair`` / ``cnn_fc_pair``): 4 launches instead of 8 per step."""
        C = ops.native()
        x1 = x2 = obs_u8
        for i, (w1, w2, c1, c2, s) in enumerate(zip(a.wb, b.wb, a.convs, b.convs, a.strides)):
            x1, x2 = C.conv_fwd_pair(x1, x2, w1, w2, c1.bias, c2.bias, s, 1.0 / 255.0 if i == 0 else 1.0, True)
        return C.cnn_fc_pair(x1.reshape(x1.shape[0], -1), x2.reshape(x2.shape[0], -1), a.fc_w, b.fc_w, a.fc.bias, b.fc.bias)

    def hidden(self, obs_u8: th.Tensor) -> th.Tensor:
        C = ops.native()
        x = obs_u8
        for i, (wb, c, s) in enumerate(zip(self.wb, self.convs, self.strides)):
            x = C.conv_fwd(x, wb, c.bias, s, 1.0 / 255.0 if i == 0 else 1.0, True)
        return C.cnn_fc(x.reshape(x.shape[0], -1), self.fc_w, self.fc.bias)


class DeviceDemoAggregate:
    """Flat device-resident (obs, acts) of every aggregated DAgger demonstration, grown by
    capacity doubling; under DP each append is all-gathered so replicas hold the same rows
    in (round, rank) order."""

    def __init__(self, device):
        self.device = th.device(device)
        self.obs: Optional[th.Tensor] = None
        self.acts: Optional[th.Tensor] = None
        self.n = 0

    def append(self, obs: th.Tensor, acts: th.Tensor, gather: bool = True) -> int:
        if gather and pdist.world_size() > 1:
            obs, acts = pdist.all_gather_rows(obs), pdist.all_gather_rows(acts)
        k = obs.shape[0]
        if k == 0:
            return 0
        need = self.n + k
        if self.obs is None or need > self.obs.shape[0]:
            cap = max(need, 2 * (0 if self.obs is None else self.obs.shape[0]), 1024)
            if self.obs is None and self.device.type == "cuda":
                # HBM is plentiful: start with room for a whole DAgger run (up to 64K rows or
                # 2 GiB, e.g. 64K Pong frames = 1.8 GB), so the storage -- and the BC epoch
                # graphs captured on it -- never move in a typical run
                row = obs[0].numel() * obs.element_size() + acts[0].numel() * acts.element_size()
                cap = max(cap, min(1 << 16, (2 << 30) // max(1, row)))
            new_obs = th.empty((cap,) + tuple(obs.shape[1:]), dtype=obs.dtype, device=self.device)
            new_acts = th.empty((cap,) + tuple(acts.shape[1:]), dtype=acts.dtype, device=self.device)
            if self.n:
                new_obs[: self.n].copy_(self.obs[: self.n])
                new_acts[: self.n].copy_(self.acts[: self.n])
            self.obs, self.acts = new_obs, new_acts
        self.obs[self.n : need].copy_(obs)
        self.acts[self.n : need].copy_(acts)
        self.n = need
        return k

    def __len__(self) -> int:
        return self.n

    def batch_buffers(self, batch_size: int):
        """Persistent ``[obs, acts]`` minibatch buffers of ``batch_size`` rows (one pair per
        size, reused by every loader over this aggregate), flagged ``_ia_static``."""
        bufs = getattr(self, "_batch_bufs", {})
        self._batch_bufs = bufs
        if batch_size not in bufs:
            pair = [th.empty((batch_size,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
                    for t in (self.obs, self.acts)]
            for t in pair:
                t._ia_static = True
            bufs[batch_size] = pair
        return bufs[batch_size]


class DeviceTransitionsLoader:
    """Shuffled, drop-last minibatches straight from a :class:`DeviceDemoAggregate`: one
    ``perm_feistel`` launch per epoch and one two-field ``gather_rows`` per batch; yields the batch
    dict BC consumes (``obs`` / ``acts`` device tensors).

    Aliasing contract: every yielded batch is a view of the SAME persistent buffers
    (:meth:`DeviceDemoAggregate.batch_buffers`), overwritten when the next batch is produced. A
    consumer must use a batch before advancing the iterator (BC does); one that holds batches
    (``list(loader)``, prefetching, two live iterators of one batch size) must ``clone()`` them."""

    def __init__(self, agg: DeviceDemoAggregate, batch_size: int, seed: int):
        self.agg = agg
        self.batch_size = batch_size
        self._seed = int(seed)
        self._epoch = 0

    def __len__(self) -> int:
        return len(self.agg) // self.batch_size

    def next_epoch_perm(self) -> th.Tensor:
        """The int32 row order of the next epoch (advances the epoch counter exactly as iterating
        does): the BC epoch graph walks it with a device cursor."""
        from imitation_amd.ops import rl as rl_ops

        self._epoch += 1
        return rl_ops.random_permutations(1, len(self.agg), self._seed * 1000003 + self._epoch, self.agg.device)[0]

    def __iter__(self):
        n = len(self.agg)
        perm = self.next_epoch_perm().long()
        obs, acts = self.agg.obs, self.agg.acts
        bufs = self.agg.batch_buffers(self.batch_size)
        for s in range(0, n - n % self.batch_size, self.batch_size):
            # into the aggregate's persistent batch buffers: a graphed BC step captured on them
            # reads them in place (utils/graphs.py ``_ia_static``), no per-step input copies;
            # stream order keeps batch k + 1's gather behind step k's reads
            o, a = rl_ops.gather_rows([obs, acts], perm[s : s + self.batch_size], dst=bufs)
            yield {"obs": o, "acts": a}


class FrameLanding:
    """A round's frames on their way to the host: a D2H copy into pinned staging on a side
    stream (off the collector -> BC path), and :meth:`land` -- run by the demo writer thread
    before it writes the round's files, and by the trainer before ``train`` returns -- waits for
    it and fills the pageable array the round's trajectories view. Until then those host
    observation arrays are not filled in."""

    def __init__(self, dst: np.ndarray, src: th.Tensor, stream: th.cuda.Stream):
        self.dst = dst
        self._pinned = th.empty(tuple(src.shape), dtype=src.dtype, pin_memory=True)
        stream.wait_stream(th.cuda.current_stream(src.device))
        with th.cuda.stream(stream):
            self._pinned.copy_(src, non_blocking=True)
            self._ev = th.cuda.Event()
            self._ev.record()
        src.record_stream(stream)  # (allocated on the main stream; read here)
        self._lock = threading.Lock()
        self._landed = False

    def land(self) -> None:
        with self._lock:
            if self._landed:
                return
            # (polled under the capture lock: a HIP call from this thread must not fall inside
            # a capture on the training thread)
            while True:
                with graphs.CAPTURE_LOCK:
                    if self._ev.query():
                        break
                time.sleep(2e-4)
            np.copyto(self.dst, self._pinned.numpy())
            with graphs.CAPTURE_LOCK:  # (the host allocator's free may query events)
                self._pinned = None
            self._landed = True


class AsyncDemoWriter:
    """Background thread that writes demo files (``fn(trajectory, index)``) in order; the
    collector hands trajectories over and goes on. ``flush()`` waits for the queue."""

    def __init__(self):
        self._q: "queue.Queue[Optional[Tuple[Callable, tuple]]]" = queue.Queue()
        self._err: Optional[BaseException] = None
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while True:
            item = self._q.get()
            try:
                if item is None:
                    return
                fn, args = item
                if self._err is None:
                    fn(*args)
            except BaseException as e:  # surfaced by flush()
                self._err = e
            finally:
                self._q.task_done()

    def submit(self, fn: Callable, *args) -> None:
        self._q.put((fn, args))

    def flush(self) -> None:
        self._q.join()
        if self._err is not None:
            err, self._err = self._err, None
            raise err

    def close(self) -> None:
        self.flush()
        self._q.put(None)
        self._t.join(timeout=5)


class DeviceStatsVenv:
    """What :class:`~imitation_amd.algorithms.bc.RolloutStatsComputer` is handed instead of the
    host venv when DAgger collects on the device: its rollouts then run on the device too."""

    def __init__(self, collector: "DeviceDAggerCollector"):
        self.collector = collector

    def device_rollout_stats(self, policy, n_episodes: int) -> Mapping[str, float]:
        if policy is not self.collector.learner:
            raise ValueError("device rollout stats evaluate the collector's learner policy")
        return self.collector.rollout_stats(n_episodes)

    def start_rollout_stats(self, policy, n_episodes: int) -> "StatsFuture":
        """:meth:`device_rollout_stats` of the learner as it is NOW, run on a side stream by a
        worker thread while the caller goes on training it (``StatsFuture.result()``)."""
        if policy is not self.collector.learner:
            raise ValueError("device rollout stats evaluate the collector's learner policy")
        return self.collector.start_rollout_stats(n_episodes)


class StatsFuture:
    """A learner rollout-statistics run in flight (:meth:`DeviceDAggerCollector.start_rollout_stats`)."""

    def __init__(self, fn: Callable[[], Mapping[str, float]], finish: Callable[[], None]):
        self._out: Optional[Mapping[str, float]] = None
        self._err: Optional[BaseException] = None
        self._finish = finish
        self._t = threading.Thread(target=self._run, args=(fn,), daemon=True)
        self._t.start()
        self._resolved = False

    def _run(self, fn) -> None:
        try:
            with graphs.CAPTURE_LOCK:  # (no capture on the training thread while this runs)
                self._out = fn()
        except BaseException as e:  # re-raised by result()
            self._err = e

    def result(self) -> Mapping[str, float]:
        if not self._resolved:
            self._t.join()
            self._resolved = True
            if self._err is None:
                self._finish()
        if self._err is not None:
            raise self._err
        return self._out


class DeviceDAggerCollector:
    """Collects DAgger rounds on the GPU (see module docstring).

    ``collect(beta, min_timesteps=..., min_episodes=...)`` returns the round's finished
    episodes as host :class:`~imitation_amd.data.types.TrajectoryWithRew` (expert actions,
    true rewards, ``infos=None``) and leaves their flat transitions on the device in
    ``last_obs`` / ``last_acts``. The host env's state is synced back afterwards."""

    def __init__(self, venv, expert_policy: ActorCriticPolicy, learner_policy: ActorCriticPolicy,
                 rng: np.random.Generator, chunk: int = 32, use_graph: Optional[bool] = None):
        self.venv = venv
        self.nat = _unwrap_native(venv)
        self.expert = expert_policy
        self.learner = learner_policy
        self.rng = rng
        self.chunk = int(chunk)
        self.device = learner_policy.device
        self._C = ops.native()
        self.N = self.nat.num_envs
        self.img = bool(self.nat._is_image)
        self.obs_shape = tuple(self.nat.observation_space.shape)
        self.discrete = isinstance(self.nat.action_space, spaces.Discrete)
        self.act_shape = () if self.discrete else tuple(self.nat.action_space.shape)
        self.use_graph = (os.environ.get("IMITATION_AMD_DAGGER_GRAPH", "1") != "0") if use_graph is None else use_graph
        dev, N, K = self.device, self.N, self.chunk
        odt = th.uint8 if self.img else th.float32
        adt = th.int64 if self.discrete else th.float32
        st = self.nat.get_state()
        self.state = th.as_tensor(st["state"], device=dev).float().contiguous()
        self.env_rng = th.as_tensor(st["rng"].astype(np.int64), device=dev).contiguous()
        self.elapsed = th.as_tensor(st["elapsed"].astype(np.int32), device=dev).contiguous()
        self.ep_ret = th.zeros(N, device=dev)
        self.obs = th.zeros((N,) + self.obs_shape, dtype=odt, device=dev)
        # two sets of chunk step records (graph-static; double-buffered so the host reads one
        # chunk's done flags while the next chunk runs)
        def chunk_set():
            return dict(obs=th.zeros((K, N) + self.obs_shape, dtype=odt, device=dev),
                        term_obs=th.zeros((K, N) + self.obs_shape, dtype=odt, device=dev),
                        acts=th.zeros((K, N) + self.act_shape, dtype=adt, device=dev), rew=th.zeros(K, N, device=dev),
                        term=th.zeros(K, N, dtype=th.uint8, device=dev), trunc=th.zeros(K, N, dtype=th.uint8, device=dev),
                        ep_ret=th.zeros(K, N, device=dev), ep_len=th.zeros(K, N, dtype=th.int32, device=dev),
                        flags=th.zeros(2, K, N, dtype=th.uint8, pin_memory=True), graph=None, ready=None)

        self._sets = [chunk_set(), chunk_set()]
        self._rec: Dict[str, th.Tensor] = {}
        self._beta = th.ones((), device=dev)
        # fused CNN actors (both policies NatureCNN + Discrete): 7 launches per step instead of ~60
        # (each layer of the two networks shares one launch when their shapes agree)
        self.cnn = (self.img and self.discrete and CnnActor.applicable(expert_policy, self.obs_shape)
                    and CnnActor.applicable(learner_policy, self.obs_shape)
                    and os.environ.get("IMITATION_AMD_DAGGER_CNN", "1") != "0")
        if self.cnn:
            self._actors = (CnnActor(expert_policy, self.obs_shape), CnnActor(learner_policy, self.obs_shape))
            self._pair = (CnnActor.paired(*self._actors) and os.environ.get("IMITATION_AMD_DAGGER_PAIR", "1") != "0")
            self._a_exp = th.zeros(N, dtype=th.int64, device=dev)
            self._a_rob = th.zeros(N, dtype=th.int64, device=dev)
            self._a_exec = th.zeros(N, dtype=th.int64, device=dev)
            self._head_ctr = th.zeros(1, dtype=th.int64, device=dev)
            self._head_seed = int(rng.integers(0, 2**62))
        self._max_steps = int(self.nat.max_episode_steps)
        self.last_obs: Optional[th.Tensor] = None
        self.last_acts: Optional[th.Tensor] = None
        self.steps_collected = 0
        # frames to the host asynchronously (FrameLanding; the owner must land() them) -- set by
        # owners that do: SimpleDAggerTrainer; IMITATION_AMD_DAGGER_ASYNC_FRAMES=0 disables
        self.async_frames = False
        self.last_landing: Optional[FrameLanding] = None
        self.timing: Dict[str, float] = collections.defaultdict(float)  # host seconds per collect() section
        self._copy_stream: Optional[th.cuda.Stream] = None

    # -------------------------------------------------------------- device steps
    def _env_args(self, mode: int, k: int = 0, actions: Optional[th.Tensor] = None, b: Optional[Dict] = None) -> Dict:
        d = dict(env=self.nat.env_id, N=self.N, max_steps=self._max_steps, mode=mode, state=self.state, rng=self.env_rng,
                 elapsed=self.elapsed, ep_ret=self.ep_ret, obs=self.obs)
        if mode == 0:
            d.update(actions=actions, rew=b["rew"][k], term=b["term"][k], trunc=b["trunc"][k], term_obs=b["term_obs"][k],
                     ep_ret_out=b["ep_ret"][k], ep_len_out=b["ep_len"][k])
        return d

    def _step_cnn(self, k: int, b: Dict) -> None:
        C = self._C
        ea, la = self._actors
        if self._pair:
            h_e, h_l = CnnActor.hidden_pair(ea, la, self.obs)
        else:
            h_e, h_l = ea.hidden(self.obs), la.hidden(self.obs)
        if self._pair:  # both heads + the beta mix in one launch (csrc/kernels/cnn_infer.hip)
            C.cnn_head_pair(h_e, self.expert.action_net.weight, self.expert.action_net.bias, self._a_exp, b["acts"][k],
                            h_l, self.learner.action_net.weight, self.learner.action_net.bias, self._head_seed,
                            self._head_ctr, self._a_rob, self._beta, self._a_exec)
        else:
            C.cnn_head(h_e, self.expert.action_net.weight, self.expert.action_net.bias, 0, 0, None, self._a_exp,
                       rec_out=b["acts"][k])
            C.cnn_head(h_l, self.learner.action_net.weight, self.learner.action_net.bias, 1, self._head_seed,
                       self._head_ctr, self._a_rob, mix_expert=self._a_exp, beta=self._beta, exec_out=self._a_exec)
        d = self._env_args(0, k, self._a_exec, b)
        d["obs_rec"] = b["obs"][k]
        C.dagger_env_step(d)

    def _step(self, k: int, b: Dict) -> None:
        if self.cnn:
            return self._step_cnn(k, b)
        obs = self.obs
        with th.no_grad():
            a_exp = policy_actions(self.expert, obs, True)
            a_rob = policy_actions(self.learner, obs, False)
        learner_turn = th.rand(self.N, device=self.device) > self._beta
        if not self.discrete:
            learner_turn = learner_turn.reshape((self.N,) + (1,) * len(self.act_shape))
        a_exec = th.where(learner_turn, a_rob.to(a_exp.dtype), a_exp)
        b["obs"][k].copy_(obs)
        b["acts"][k].copy_(a_exp.reshape(b["acts"][k].shape))
        self._C.dagger_env_step(self._env_args(0, k, a_exec.contiguous() if self.discrete else a_exec.float().contiguous(), b))

    def _run_chunk(self, b: Dict) -> None:
        if not self.use_graph:
            for k in range(self.chunk):
                self._step(k, b)
            return
        if b["graph"] is None:
            # the first chunk of each buffer set runs eagerly (also the allocator warm-up);
            # later chunks replay
            for k in range(self.chunk):
                self._step(k, b)
            g = th.cuda.CUDAGraph()
            try:
                # capture only: nothing in this block executes until replay()
                with graphs.capture(g):
                    for k in range(self.chunk):
                        self._step(k, b)
                b["graph"] = g
            except RuntimeError as e:  # e.g. an op that syncs: stay eager
                import logging

                logging.getLogger(__name__).warning("DAgger step graph capture failed (%s); stepping eagerly", e)
                self.use_graph = False
            return
        b["graph"].replay()

    def _record(self, i: int, b: Dict) -> None:
        """Enqueue: chunk ``i``'s records -> the round buffers (grown by doubling), its done
        flags -> pinned host memory, and the event marking both."""
        K = self.chunk
        need = (i + 1) * K
        keys = ("obs", "term_obs", "acts", "rew")
        cap = self._rec["obs"].shape[0] if self._rec else 0
        if need > cap:
            new_cap = max(need, 2 * cap, 8 * K)
            for key in keys:
                src = b[key]
                t = th.empty((new_cap,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
                if cap:
                    t[: i * K].copy_(self._rec[key][: i * K])
                self._rec[key] = t
        for key in keys:
            self._rec[key][i * K : need].copy_(b[key])
        b["flags"][0].copy_(b["term"], non_blocking=True)
        b["flags"][1].copy_(b["trunc"], non_blocking=True)
        ev = th.cuda.Event()
        ev.record()
        b["ready"] = ev

    def _launch(self, i: int) -> None:
        b = self._sets[i % 2]
        self._run_chunk(b)
        self._record(i, b)

    def reset(self) -> None:
        self._C.dagger_env_step(self._env_args(1))

    # -------------------------------------------------------------- one round
    def collect(self, beta: float, *, min_timesteps: int, min_episodes: int) -> List[types.TrajectoryWithRew]:
        """One round with the reference's ``generate_trajectories`` stopping rule."""
        dev, N, K = self.device, self.N, self.chunk
        tm = self.timing
        t_a = time.perf_counter()
        self._beta.fill_(float(beta))
        if self.cnn:
            for actor in self._actors:
                actor.refresh()  # the learner changed since the last round
        self.reset()
        active = np.ones(N, dtype=bool)
        start = np.zeros(N, dtype=np.int64)
        finished: List[Tuple[int, int, int]] = []  # (env, first step, last step)
        n_steps_done = 0
        satisfied = False
        i = 0
        self._launch(0)
        while True:
            # keep the next chunk running while the host reads this one's flags
            self._launch(i + 1)
            b = self._sets[i % 2]
            b["ready"].synchronize()
            done_chunk = (b["flags"][0].numpy() | b["flags"][1].numpy()).astype(bool)
            t_base = i * K
            for k in range(K):
                t = t_base + k
                dones = done_chunk[k] & active
                for n in np.flatnonzero(dones):
                    finished.append((int(n), int(start[n]), t))
                    n_steps_done += t - int(start[n]) + 1
                    start[n] = t + 1
                if not satisfied:
                    satisfied = len(finished) >= min_episodes and n_steps_done >= min_timesteps
                if satisfied:
                    active &= ~dones
                if not active.any():
                    break
            i += 1
            if not active.any():
                break
        t_base = i * K  # chunks whose steps count (the speculative next one is discarded)
        self.steps_collected = t_base * N
        t_b = time.perf_counter()
        tm["loop"] += t_b - t_a
        obs_all, term_all, acts_all, rew_all = (self._rec[k] for k in ("obs", "term_obs", "acts", "rew"))  # [T, N, ...]
        # flat row indices (t * N + n) of every finished episode, in finishing order
        rows = np.concatenate([np.arange(s, e + 1) * N + n for (n, s, e) in finished]) if finished else np.zeros(0, np.int64)
        ends = np.asarray([e * N + n for (n, s, e) in finished], dtype=np.int64)
        ridx = th.as_tensor(rows, device=dev)
        flat = lambda x: x.reshape((-1,) + tuple(x.shape[2:]))  # noqa: E731
        self.last_obs, self.last_acts = rl_ops.gather_rows([flat(obs_all), flat(acts_all)], ridx)
        # host trajectories (demo files / stats): every episode's observations followed by its
        # terminal observation are laid out contiguously ON THE DEVICE, so ONE D2H copy lands
        # them and each trajectory's obs is a view of that array (no per-episode concatenation
        # of the frames on the host)
        lens = np.asarray([e - s + 1 for (n, s, e) in finished], dtype=np.int64)
        obs_off = np.concatenate([[0], np.cumsum(lens + 1)]).astype(np.int64)
        pos_term = obs_off[1:] - 1
        pos_step = np.delete(np.arange(int(obs_off[-1]), dtype=np.int64), pos_term)
        with_term = th.empty((int(obs_off[-1]),) + tuple(obs_all.shape[2:]), dtype=obs_all.dtype, device=dev)
        if len(finished):
            with_term.index_copy_(0, th.as_tensor(pos_step, device=dev), self.last_obs)
            with_term.index_copy_(0, th.as_tensor(pos_term, device=dev),
                                  flat(term_all).index_select(0, th.as_tensor(ends, device=dev)))
        h_obs = np.empty(tuple(with_term.shape), dtype=np.uint8 if with_term.dtype == th.uint8 else np.float32)
        self.last_landing = None
        if self.async_frames and len(finished):
            if self._copy_stream is None:
                self._copy_stream = th.cuda.Stream(device=dev)
            self.last_landing = FrameLanding(h_obs, with_term, self._copy_stream)
        else:
            th.from_numpy(h_obs).copy_(with_term)
        t_c = time.perf_counter()
        tm["tail_gather"] += t_c - t_b
        h_acts = self.last_acts.cpu().numpy()
        h_rew = flat(rew_all).index_select(0, ridx).float().cpu().numpy()
        t_d = time.perf_counter()
        tm["tail_d2h_sync"] += t_d - t_c
        trajs: List[types.TrajectoryWithRew] = []
        off = 0
        for j, (n, s, e) in enumerate(finished):
            L = e - s + 1
            trajs.append(types.TrajectoryWithRew(obs=h_obs[obs_off[j] : obs_off[j + 1]], acts=h_acts[off : off + L],
                                                 infos=None, terminal=True, rews=h_rew[off : off + L]))
            off += L
        t_e = time.perf_counter()
        self.sync_env_to_host()
        tm["tail_trajs"] += t_e - t_d
        tm["sync_env"] += time.perf_counter() - t_e
        return trajs

    # -------------------------------------------------------------- rollout stats
    _ENV_TENSORS = ("state", "env_rng", "elapsed", "ep_ret", "obs")

    def _stats_twin(self) -> "DeviceDAggerCollector":
        """A collector over a frozen copy of the learner (same expert, same host env, the
        learner head's sampling seed) whose env state is copied in before a statistics run and
        back after it, so that running the statistics on it is the same as running them here."""
        twin = getattr(self, "_twin", None)
        if twin is None:
            try:  # a fresh module of the same architecture (no training-side attributes)
                snap = type(self.learner)(**self.learner._get_constructor_parameters()).to(self.device)
                snap.load_state_dict(self.learner.state_dict())
            except Exception:  # noqa: BLE001 -- any other policy class: a deep copy
                import copy

                snap = copy.deepcopy(self.learner)
            snap.eval()
            for p in snap.parameters():
                p.requires_grad_(False)
            twin = DeviceDAggerCollector(self.venv, self.expert, snap, self.rng, chunk=self.chunk, use_graph=self.use_graph)
            if self.cnn:
                twin._head_seed = self._head_seed
            # its chunk graphs are captured here, on the calling thread (the worker thread only
            # replays them: no capture may overlap another thread's work): one eager + captured
            # chunk per buffer set, on throw-away env state (overwritten by every start)
            twin.reset()
            for b in twin._sets:
                twin._run_chunk(b)
            th.cuda.synchronize(self.device)
            self._twin = twin
            # (a high-priority stream for the statistics chain measured much slower, round 5 call AJ)
            self._twin_stream = th.cuda.Stream(device=self.device)
        return twin

    def start_rollout_stats(self, n_episodes: int) -> StatsFuture:
        """:meth:`rollout_stats` of the learner's current weights, on a worker thread and a side
        stream: the weights, the env state and the head's sampling counter are copied into the
        twin (main stream order), the twin runs the statistics, and ``result()`` copies the env
        state and counter back -- the same env / RNG sequence as the in-line call. Until
        ``result()`` returns, the caller must not step this collector's envs."""
        twin = self._stats_twin()
        main = th.cuda.current_stream(self.device)
        with th.no_grad():
            for d, s_ in zip(twin.learner.parameters(), self.learner.parameters()):
                d.copy_(s_)
            for name in self._ENV_TENSORS:
                getattr(twin, name).copy_(getattr(self, name))
            if self.cnn:
                twin._head_ctr.copy_(self._head_ctr)
        stream = self._twin_stream
        stream.wait_stream(main)

        def run():
            with th.cuda.device(self.device), th.cuda.stream(stream):
                return twin.rollout_stats(n_episodes)

        def finish():
            main.wait_stream(stream)
            with th.no_grad():
                for name in self._ENV_TENSORS:
                    getattr(self, name).copy_(getattr(twin, name))
                if self.cnn:
                    self._head_ctr.copy_(twin._head_ctr)

        return StatsFuture(run, finish)

    def rollout_stats(self, n_episodes: int) -> Mapping[str, float]:
        """BC's rollout statistics (``RolloutStatsComputer``: ``generate_trajectories`` of the
        learner alone with ``make_min_episodes(n_episodes)``, then ``rollout_stats``) on the
        device: beta 0, the same stopping rule as :meth:`collect`, and only the per-step done
        flags / finished-episode returns and lengths cross to the host -- no frame records.
        Keys match the host path over the native env (``monitor_return_*`` = the episode
        returns, which the env's monitor reports unchanged)."""
        N, K = self.N, self.chunk
        self._beta.fill_(0.0)
        if self.cnn:
            self._actors[1].refresh()
        self.reset()
        host = [dict(ret=th.zeros(K, N, pin_memory=True), len=th.zeros(K, N, dtype=th.int32, pin_memory=True))
                for _ in range(2)]

        def launch(i: int) -> None:
            b = self._sets[i % 2]
            self._run_chunk(b)
            b["flags"][0].copy_(b["term"], non_blocking=True)
            b["flags"][1].copy_(b["trunc"], non_blocking=True)
            host[i % 2]["ret"].copy_(b["ep_ret"], non_blocking=True)
            host[i % 2]["len"].copy_(b["ep_len"], non_blocking=True)
            ev = th.cuda.Event()
            ev.record()
            b["ready"] = ev

        active = np.ones(N, dtype=bool)
        rets: List[float] = []
        lens: List[int] = []
        satisfied = False
        i = 0
        launch(0)
        while active.any():
            launch(i + 1)
            b, h = self._sets[i % 2], host[i % 2]
            b["ready"].synchronize()
            done_chunk = (b["flags"][0].numpy() | b["flags"][1].numpy()).astype(bool)
            r_chunk, l_chunk = h["ret"].numpy(), h["len"].numpy()
            for k in range(K):
                dones = done_chunk[k] & active
                for n in np.flatnonzero(dones):
                    rets.append(float(r_chunk[k, n]))
                    lens.append(int(l_chunk[k, n]))
                if not satisfied:
                    satisfied = len(rets) >= n_episodes
                if satisfied:
                    active &= ~dones
                if not active.any():
                    break
            i += 1
        th.cuda.current_stream().synchronize()  # the speculative chunk
        self.sync_env_to_host()
        out: Dict[str, float] = {"n_traj": len(rets)}
        desc = {"return": np.asarray(rets, dtype=np.float64), "len": np.asarray(lens)}
        desc["monitor_return"] = desc["return"]
        out["monitor_return_len"] = len(rets)
        for name, vals in desc.items():
            for stat in ("min", "mean", "std", "max"):
                out[f"{name}_{stat}"] = getattr(np, stat)(vals).item()
        return out

    # -------------------------------------------------------------- checkpoint
    def engine_state(self) -> Dict[str, Any]:
        """Env state on the device and the learner head's sampling stream (full-trainer
        checkpoints, :func:`imitation_amd.utils.checkpoint.dagger_state`). Taken between rounds:
        nothing is in flight then."""
        st: Dict[str, Any] = {k: getattr(self, k).detach().cpu().clone() for k in self._ENV_TENSORS}
        st["steps_collected"] = int(self.steps_collected)
        if self.cnn:
            st["head_ctr"] = self._head_ctr.cpu().clone()
            st["head_seed"] = int(self._head_seed)
        return st

    def load_engine_state(self, st: Dict[str, Any]) -> None:
        with th.no_grad():
            for k in self._ENV_TENSORS:
                getattr(self, k).copy_(st[k].to(self.device))
            if self.cnn:
                self._head_ctr.copy_(st["head_ctr"].to(self.device))
        self.steps_collected = st["steps_collected"]
        if self.cnn:
            self._head_seed = st["head_seed"]
            twin = getattr(self, "_twin", None)
            if twin is not None:
                twin._head_seed = self._head_seed
        self.sync_env_to_host()

    def sync_env_to_host(self) -> None:
        st = {"state": self.state.cpu().numpy(), "rng": self.env_rng.cpu().numpy(),
              "elapsed": self.elapsed.cpu().numpy().astype(np.int64)}
        if self.img:
            st["frames"] = self.obs.cpu().numpy()
        self.nat.set_state(st)
