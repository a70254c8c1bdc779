"""Adversarial imitation core (reference: ``src/imitation/algorithms/adversarial/common.py``).

Same algorithm and API as the reference ``AdversarialTrainer``: alternate
``train_gen`` (generator RL on the learned reward; ``common.py:391-425``) and
``n_disc_updates_per_round`` × ``train_disc`` (BCE on expert=1 / generator=0,
minibatch gradient accumulation; ``:317-389``), generator replay buffer,
``compute_train_stats`` metric keys (``:27-92``), ``_get_log_policy_act_prob`` for
AIRL (``:476-519``), ``_make_disc_train_batches`` (``:521-632``).

MI355X data path (semantics unchanged):

* expert demonstrations are uploaded to the device once and minibatches are
  drawn by a device-side permutation (the reference re-collates numpy batches and
  re-uploads them every step);
* the generator replay buffer is a device ring (:class:`~imitation_amd.data.buffer.DeviceBuffer`);
* the discriminator loss is the fused BCE-with-logits kernel + fused MLP bwd;
  training statistics are reduced on the device and fetched with one sync;
* data parallel: each rank keeps its own envs and replay buffer, the
  discriminator gradient is averaged with one all-reduce per optimizer step, and
  reward-normaliser statistics are all-reduced (identical replicas).
"""

from __future__ import annotations

import abc
import dataclasses
import logging
from typing import Callable, Dict, Iterable, Iterator, Mapping, Optional, Sequence, Type

import numpy as np
import torch as th
from torch.nn import functional as F

from imitation_amd.utils import gcfreeze
from imitation_amd.algorithms import base
from imitation_amd.data import buffer, rollout, types, wrappers
from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rewards import reward_nets, reward_wrapper
from imitation_amd.rl import base as rl_base
from imitation_amd.rl import distributions
from imitation_amd.rl.policies import ActorCriticPolicy
from imitation_amd.util import logger, networks, util


def train_stats_from_sums(vec: Sequence[float], n_labels: float) -> Mapping[str, float]:
    """Statistics dict from ``[loss, acc, n_generated, n_gen_pred, n_exp_correct,
    n_gen_correct, entropy]`` (shared by the host path and the fused device update)."""
    loss, acc, n_generated, n_gen_pred, n_exp_correct, n_gen_correct, entropy = vec
    n_expert = n_labels - n_generated
    pct_expert = n_expert / n_labels if n_labels > 0 else float("NaN")
    n_expert_pred = int(n_labels - n_gen_pred)
    pct_expert_pred = n_expert_pred / n_labels if n_labels > 0 else float("NaN")
    expert_acc = float("NaN") if n_expert < 1 else n_exp_correct / n_expert
    generated_acc = n_gen_correct / float(max(1, n_generated))
    return {
        "disc_loss": float(loss),
        "disc_acc": float(acc),
        "disc_acc_expert": float(expert_acc),
        "disc_acc_gen": float(generated_acc),
        "disc_entropy": float(entropy),
        "disc_proportion_expert_true": float(pct_expert),
        "disc_proportion_expert_pred": float(pct_expert_pred),
        "n_expert": float(n_expert),
        "n_generated": float(n_generated),
    }


def compute_train_stats(disc_logits_expert_is_high: th.Tensor, labels_expert_is_one: th.Tensor, disc_loss: th.Tensor) -> Mapping[str, float]:
    """Discriminator statistics (``common.py:27-92``), reduced on-device, one host sync."""
    vec = train_stats_vec(disc_logits_expert_is_high, labels_expert_is_one, disc_loss).tolist()
    return train_stats_from_sums(vec, float(len(labels_expert_is_one)))


def train_stats_vec(disc_logits_expert_is_high: th.Tensor, labels_expert_is_one: th.Tensor, disc_loss: th.Tensor) -> th.Tensor:
    """The device-side sums behind :func:`compute_train_stats` (no host sync):
    [loss, accuracy, #gen labels, #gen predictions, #expert correct, #gen correct, entropy]."""
    with th.no_grad():
        logits = disc_logits_expert_is_high.float()
        gen_pred = logits < 0
        gen_true = labels_expert_is_one == 0
        exp_true = th.logical_not(gen_true)
        correct = th.eq(gen_pred, gen_true)
        ent = F.binary_cross_entropy_with_logits(logits, th.sigmoid(logits), reduction="none")
        return th.stack([
            th.mean(disc_loss.float()),
            th.mean(correct.float()),
            th.sum(gen_true.float()),
            th.sum(gen_pred.float()),
            th.sum(th.logical_and(exp_true, correct).float()),
            th.sum(th.logical_and(gen_true, correct).float()),
            th.mean(ent),
        ])


class _DeviceDemoSampler:
    """Endless shuffled drop-last minibatches of flat demonstrations, resident on the device."""

    def __init__(self, transitions: types.Transitions, batch_size: int, device, seed: Optional[int] = None):
        self.batch_size = batch_size
        self.device = th.device(device)
        self.n = len(transitions)
        if self.n < batch_size:
            raise ValueError(f"Number of transitions in `demonstrations` {self.n} is smaller than batch size {batch_size}.")
        self.data = {
            "obs": th.as_tensor(np.array(transitions.obs), device=self.device),
            "acts": th.as_tensor(np.array(transitions.acts), device=self.device),
            "next_obs": th.as_tensor(np.array(transitions.next_obs), device=self.device),
            "dones": th.as_tensor(np.array(transitions.dones), device=self.device),
        }
        self._gen = th.Generator(device=self.device)
        self._gen.manual_seed(int(seed if seed is not None else np.random.randint(0, 2**31 - 1)) + 104729 * pdist.rank())
        # epoch orders: one keyed Feistel permutation launch per epoch (ops.rl.random_permutations)
        # instead of torch.randperm's device radix sort (~10 launches); key = (base, epoch count)
        self._base = int(self._gen.initial_seed())
        self._epochs = 0
        self._perm = None
        self._pos = 0

    def next_indices(self) -> th.Tensor:
        """Row indices of the next batch (a contiguous slice of the epoch permutation)."""
        if self._perm is None or self._pos + self.batch_size > self.n:
            self._epochs += 1
            if self.device.type == "cuda":
                from imitation_amd.ops import rl as rl_ops

                self._perm = rl_ops.random_permutations(1, self.n, self._base * 1000003 + self._epochs, self.device)[0].long()
            else:
                self._perm = th.randperm(self.n, device=self.device, generator=self._gen)
            self._pos = 0
        idx = self._perm[self._pos : self._pos + self.batch_size]
        self._pos += self.batch_size
        return idx

    def __next__(self) -> Dict[str, th.Tensor]:
        idx = self.next_indices()
        return {k: v.index_select(0, idx) for k, v in self.data.items()}

    def __iter__(self):
        return self


class AdversarialTrainer(base.DemonstrationAlgorithm[types.Transitions]):
    """Base class for adversarial imitation learning algorithms like GAIL and AIRL."""

    def __init__(
        self,
        *,
        demonstrations: base.AnyTransitions,
        demo_batch_size: int,
        venv,
        gen_algo: rl_base.BaseAlgorithm,
        reward_net: reward_nets.RewardNet,
        demo_minibatch_size: Optional[int] = None,
        n_disc_updates_per_round: int = 2,
        log_dir: types.AnyPath = "output/",
        disc_opt_cls: Type[th.optim.Optimizer] = th.optim.Adam,
        disc_opt_kwargs: Optional[Mapping] = None,
        gen_train_timesteps: Optional[int] = None,
        gen_replay_buffer_capacity: Optional[int] = None,
        custom_logger: Optional[logger.HierarchicalLogger] = None,
        init_tensorboard: bool = False,
        init_tensorboard_graph: bool = False,
        debug_use_ground_truth: bool = False,
        allow_variable_horizon: bool = False,
    ):
        self.demo_batch_size = demo_batch_size
        self.demo_minibatch_size = demo_minibatch_size or demo_batch_size
        if self.demo_batch_size % self.demo_minibatch_size != 0:
            raise ValueError("Batch size must be a multiple of minibatch size.")
        self._demo_data_loader = None
        self._endless_expert_iterator = None
        self.gen_algo = gen_algo
        self._device = gen_algo.device
        super().__init__(demonstrations=demonstrations, custom_logger=custom_logger, allow_variable_horizon=allow_variable_horizon)
        self._global_step = 0
        self._disc_step = 0
        self.n_disc_updates_per_round = n_disc_updates_per_round
        self.debug_use_ground_truth = debug_use_ground_truth
        self.venv = venv
        self._reward_net = reward_net.to(gen_algo.device)
        pdist.broadcast_module(self._reward_net)
        self._log_dir = util.parse_path(log_dir)
        self._disc_opt_cls = disc_opt_cls
        self._disc_opt_kwargs = disc_opt_kwargs or {}
        self._init_tensorboard = init_tensorboard
        self._init_tensorboard_graph = init_tensorboard_graph
        self._disc_opt = self._disc_opt_cls(self._reward_net.parameters(), **self._disc_opt_kwargs)
        self._disc_bucket = pdist.GradBucket(self._reward_net.parameters()) if pdist.world_size() > 1 else None
        if self._init_tensorboard:
            from imitation_amd.rl.logger import TensorBoardOutputFormat

            logging.info(f"building summary directory at {self._log_dir}")
            summary_dir = self._log_dir / "summary"
            summary_dir.mkdir(parents=True, exist_ok=True)
            self._summary_writer = TensorBoardOutputFormat(str(summary_dir))
        self.venv_buffering = wrappers.BufferingWrapper(self.venv)
        if debug_use_ground_truth:
            self.venv_wrapped = self.venv_buffering
            self.gen_callback = None
        else:
            self.venv_wrapped = reward_wrapper.RewardVecEnvWrapper(self.venv_buffering, reward_fn=self.reward_train.predict_processed)
            self.gen_callback = self.venv_wrapped.make_log_callback()
        self.venv_train = self.venv_wrapped
        self.gen_algo.set_env(self.venv_train)
        self.gen_algo.set_logger(self.logger)
        if gen_train_timesteps is None:
            env = self.gen_algo.get_env()
            assert env is not None
            self.gen_train_timesteps = env.num_envs
            if isinstance(self.gen_algo, rl_base.OnPolicyAlgorithm):
                self.gen_train_timesteps *= self.gen_algo.n_steps
        else:
            self.gen_train_timesteps = gen_train_timesteps
        if gen_replay_buffer_capacity is None:
            gen_replay_buffer_capacity = self.gen_train_timesteps
        self._gen_replay_buffer = buffer.ReplayBuffer(gen_replay_buffer_capacity, self.venv)

    @property
    def policy(self):
        policy = self.gen_algo.policy
        assert policy is not None
        return policy

    @abc.abstractmethod
    def logits_expert_is_high(self, state, action, next_state, done, log_policy_act_prob: Optional[th.Tensor] = None) -> th.Tensor:
        """Discriminator logits: large positive = expert-like."""

    @property
    @abc.abstractmethod
    def reward_train(self) -> reward_nets.RewardNet:
        """Reward used to train the generator."""

    @property
    @abc.abstractmethod
    def reward_test(self) -> reward_nets.RewardNet:
        """Reward used for evaluation / transfer."""

    def set_demonstrations(self, demonstrations: base.AnyTransitions) -> None:
        if isinstance(demonstrations, Iterable) and not isinstance(demonstrations, types.TransitionsMinimal):
            first, demonstrations = util.get_first_iter_element(demonstrations)
            if isinstance(first, types.Trajectory):
                demonstrations = rollout.flatten_trajectories(list(demonstrations))
        if isinstance(demonstrations, types.Transitions) and not isinstance(demonstrations.obs, types.DictObs):
            self._demo_data_loader = None
            self._endless_expert_iterator = _DeviceDemoSampler(demonstrations, self.demo_batch_size, self._device)
            return
        self._demo_data_loader = base.make_data_loader(demonstrations, self.demo_batch_size)
        self._endless_expert_iterator = util.endless_iter(self._demo_data_loader)

    def _next_expert_batch(self) -> Mapping:
        assert self._endless_expert_iterator is not None
        return next(self._endless_expert_iterator)

    def train_disc(self, *, expert_samples: Optional[Mapping] = None, gen_samples: Optional[Mapping] = None) -> Mapping[str, float]:
        """One discriminator optimizer step over ``demo_batch_size`` expert + generator samples."""
        with self.logger.accumulate_means("disc"):
            write_summaries = self._init_tensorboard and self._global_step % 20 == 0
            self._disc_opt.zero_grad(set_to_none=self._disc_bucket is None)
            if self._disc_bucket is not None:
                self._disc_bucket.zero()
            for batch in self._make_disc_train_batches(gen_samples=gen_samples, expert_samples=expert_samples):
                disc_logits = self.logits_expert_is_high(
                    batch["state"], batch["action"], batch["next_state"], batch["done"], batch["log_policy_act_prob"]
                )
                loss = F.binary_cross_entropy_with_logits(disc_logits, batch["labels_expert_is_one"].float())
                assert len(batch["state"]) == 2 * self.demo_minibatch_size
                loss = loss * (self.demo_minibatch_size / self.demo_batch_size)
                loss.backward()
            if self._disc_bucket is not None:
                self._disc_bucket.allreduce()
            self._disc_opt.step()
            self._disc_step += 1
            with th.no_grad():
                train_stats = compute_train_stats(disc_logits, batch["labels_expert_is_one"], loss)
            self.logger.record("global_step", self._global_step)
            for k, v in train_stats.items():
                self.logger.record(k, v)
            self.logger.dump(self._disc_step)
            if write_summaries:
                self._summary_writer.write({"disc_logits_mean": float(disc_logits.mean())}, {"disc_logits_mean": None}, self._global_step)
        return train_stats

    def train_gen(self, total_timesteps: Optional[int] = None, learn_kwargs: Optional[Mapping] = None) -> None:
        """Train the generator for ``total_timesteps`` (default one round) and store its samples."""
        if total_timesteps is None:
            total_timesteps = self.gen_train_timesteps
        learn_kwargs = learn_kwargs or {}
        with self.logger.accumulate_means("gen"):
            self.gen_algo.learn(total_timesteps=total_timesteps, reset_num_timesteps=False, callback=self.gen_callback, **learn_kwargs)
            self._global_step += 1
        gen_trajs, ep_lens = self.venv_buffering.pop_trajectories()
        if pdist.world_size() > 1:
            ep_lens = [l for part in pdist.all_gather_object(list(map(int, ep_lens))) for l in part]
        self._check_fixed_horizon(ep_lens)
        gen_samples = rollout.flatten_trajectories_with_rew(gen_trajs)
        self._gen_replay_buffer.store(gen_samples)

    @gcfreeze.during
    def train(self, total_timesteps: int, callback: Optional[Callable[[int], None]] = None) -> None:
        """Alternate generator and discriminator training for ``total_timesteps // gen_train_timesteps`` rounds."""
        n_rounds = total_timesteps // self.gen_train_timesteps
        assert n_rounds >= 1, (
            f"No updates (need at least {self.gen_train_timesteps} timesteps, have only total_timesteps={total_timesteps})!"
        )
        for r in range(0, n_rounds):
            self.train_gen(self.gen_train_timesteps)
            for _ in range(self.n_disc_updates_per_round):
                with networks.training(self.reward_train):
                    self.train_disc()
            if callback:
                callback(r)
            self.logger.dump(self._global_step)

    def _torchify_array(self, ndarray):
        if ndarray is not None:
            return th.as_tensor(ndarray, device=self.reward_train.device)
        return None

    def _get_log_policy_act_prob(self, obs_th: th.Tensor, acts_th: th.Tensor) -> Optional[th.Tensor]:
        from imitation_amd.rl.sac import SACPolicy

        if isinstance(self.policy, ActorCriticPolicy):
            # evaluate_actions' log-prob without its value head and entropy (one fused MLP
            # pass fewer per discriminator minibatch; same normaliser update, same numbers)
            log_policy_act_prob_th = self.policy.get_distribution(obs_th).log_prob(acts_th)
        elif isinstance(self.policy, SACPolicy):
            actor = self.policy.actor
            mean_actions, log_std, _ = actor.get_action_dist_params(obs_th)
            dist = actor.action_dist.proba_distribution(mean_actions, log_std)
            assert self.policy.squash_output
            scaled = self.policy.scale_action(acts_th.detach().cpu().numpy())
            log_policy_act_prob_th = dist.log_prob(th.as_tensor(scaled, device=mean_actions.device))
        else:
            return None
        return log_policy_act_prob_th

    def _gen_sample(self, batch_size: int) -> Dict[str, th.Tensor]:
        if self._gen_replay_buffer.size() == 0:
            raise RuntimeError("No generator samples for training. Call `train_gen()` first.")
        return types.dataclass_quick_asdict(self._gen_replay_buffer.sample(batch_size))

    def _make_disc_train_batches(self, *, gen_samples: Optional[Mapping] = None, expert_samples: Optional[Mapping] = None) -> Iterator[Mapping[str, th.Tensor]]:
        batch_size = self.demo_batch_size
        if expert_samples is None:
            expert_samples = self._next_expert_batch()
        if gen_samples is None:
            gen_samples = self._gen_sample(batch_size)
        if not (len(gen_samples["obs"]) == len(expert_samples["obs"]) == batch_size):
            raise ValueError(
                "Need to have exactly `demo_batch_size` number of expert and generator samples, each. "
                f"(n_gen={len(gen_samples['obs'])} n_expert={len(expert_samples['obs'])} demo_batch_size={batch_size})"
            )
        dev = self._device

        def to_dev(v):
            if isinstance(v, th.Tensor):
                return v.to(dev)
            return th.as_tensor(np.asarray(v), device=dev)

        ex = {k: to_dev(expert_samples[k]) for k in ("obs", "acts", "next_obs", "dones")}
        ge = {k: to_dev(gen_samples[k]) for k in ("obs", "acts", "next_obs", "dones")}
        mb = self.demo_minibatch_size
        # constant [1]*mb + [0]*mb labels, built once per (mb, device): no fill / cat launches
        # per minibatch (nor inside a captured discriminator step)
        cache = self.__dict__.setdefault("_disc_labels", {})
        labels = cache.get((mb, dev))
        if labels is None:
            labels = cache[(mb, dev)] = th.cat([th.ones(mb, dtype=th.int64, device=dev),
                                                th.zeros(mb, dtype=th.int64, device=dev)])
        for start in range(0, batch_size, mb):
            end = start + mb
            obs = th.cat([ex["obs"][start:end], ge["obs"][start:end].to(ex["obs"].dtype)])
            acts = th.cat([ex["acts"][start:end], ge["acts"][start:end].to(ex["acts"].dtype)])
            next_obs = th.cat([ex["next_obs"][start:end], ge["next_obs"][start:end].to(ex["next_obs"].dtype)])
            dones = th.cat([ex["dones"][start:end].bool(), ge["dones"][start:end].bool()])
            with th.no_grad():
                log_policy_act_prob = self._get_log_policy_act_prob(obs, acts)
                if log_policy_act_prob is not None:
                    assert len(log_policy_act_prob) == 2 * mb
                    log_policy_act_prob = log_policy_act_prob.reshape((2 * mb,))
            obs_th, acts_th, next_obs_th, dones_th = self.reward_train.preprocess(obs, acts, next_obs, dones)
            yield {
                "state": obs_th,
                "action": acts_th,
                "next_state": next_obs_th,
                "done": dones_th,
                "labels_expert_is_one": labels,
                "log_policy_act_prob": log_policy_act_prob,
            }
