"""Behavioural cloning (reference: ``src/imitation/algorithms/bc.py``).

Loss ``-mean log π(a|s) - w_ent·H + w_l2·½‖θ‖²`` (``bc.py:94-156``), gradient
accumulation over ``batch_size / minibatch_size`` minibatches (``:482-510``),
epoch/batch iteration with end-of-epoch callbacks (``:36-77``), periodic rollout
statistics (``:171-201``) and the ``bc/*`` metric keys (``:204-247``).

:class:`MultiBC` (fork addition, ``bc.py:512-776``) concatenates the per-agent
slices ``observation_overide(i, obs)`` / ``action_overide(i, acts)`` along the
batch axis -- i.e. the agents are folded into the GEMM M dimension and the whole
homogeneous team is one fused forward/backward.

MI355X: policy heads are fused MFMA MLP kernels; minibatches come from the
vectorised transitions loader; under data parallelism the accumulated gradient is
averaged across ranks with one bucketed all-reduce right before ``optimizer.step``
(hook point SURVEY §2.4: ``bc.py:464-466``).
"""

from __future__ import annotations

import dataclasses
import itertools
import math
from typing import Any, Callable, Dict, Iterable, Iterator, List, Mapping, Optional, Tuple, Type, Union

import numpy as np
import torch as th

from imitation_amd.algorithms import base as algo_base
from imitation_amd.data import rollout, types
from imitation_amd.envs import spaces
from imitation_amd.ops import bc_cnn
from imitation_amd.ops import optim as optim_ops
from imitation_amd.parallel import dist as pdist
from imitation_amd.policies import base as policy_base
from imitation_amd.rl import torch_layers
from imitation_amd.rl.policies import ActorCriticPolicy, get_device
from imitation_amd.util import logger as imit_logger
from imitation_amd.utils import gcfreeze, graphs
from imitation_amd.util import util


@dataclasses.dataclass(frozen=True)
class BatchIteratorWithEpochEndCallback:
    """Loops through batches from a batch loader and calls a callback after every epoch."""

    batch_loader: Iterable[types.TransitionMapping]
    n_epochs: Optional[int]
    n_batches: Optional[int]
    on_epoch_end: Optional[Callable[[int], None]]

    def __post_init__(self) -> None:
        both = self.n_epochs is not None and self.n_batches is not None
        neither = self.n_epochs is None and self.n_batches is None
        if both or neither:
            raise ValueError("Must provide exactly one of `n_epochs` and `n_batches` arguments.")

    def __iter__(self) -> Iterator[types.TransitionMapping]:
        def batch_iterator() -> Iterator[types.TransitionMapping]:
            for epoch_num in itertools.islice(itertools.count(), self.n_epochs):
                yielded = False
                for batch in self.batch_loader:
                    yield batch
                    yielded = True
                if not yielded:
                    raise AssertionError(f"Data loader returned no data during epoch {epoch_num} -- did it reset correctly?")
                if self.on_epoch_end is not None:
                    self.on_epoch_end(epoch_num)

        return itertools.islice(batch_iterator(), self.n_batches)


@dataclasses.dataclass(frozen=True)
class BCTrainingMetrics:
    """Container for the different components of behavior cloning loss."""

    neglogp: th.Tensor
    entropy: Optional[th.Tensor]
    ent_loss: th.Tensor
    prob_true_act: th.Tensor
    l2_norm: th.Tensor
    l2_loss: th.Tensor
    loss: th.Tensor


@dataclasses.dataclass(frozen=True)
class BehaviorCloningLossCalculator:
    """Functor to compute the loss used in Behavior Cloning."""

    ent_weight: float
    l2_weight: float

    def __call__(self, policy: ActorCriticPolicy, obs, acts) -> BCTrainingMetrics:
        tensor_obs = types.map_maybe_dict(util.safe_to_tensor, types.maybe_unwrap_dictobs(obs))
        acts = util.safe_to_tensor(acts)
        fused = self._fused_categorical(policy, tensor_obs, acts)
        if fused is not None:
            return fused
        _, log_prob, entropy = policy.evaluate_actions(tensor_obs, acts)
        prob_true_act = th.exp(log_prob).mean()
        log_prob = log_prob.mean()
        entropy = entropy.mean() if entropy is not None else None
        params = [w for w in policy.parameters()]
        if not params:
            l2_norm = th.zeros(())
        elif self.l2_weight == 0.0:
            # only a logged metric: one multi-tensor norm launch instead of 2 kernels per tensor
            with th.no_grad():
                l2_norm = th.stack(th._foreach_norm(params)).square().sum() / 2
        else:
            l2_norm = th.stack([th.sum(th.square(w)) for w in params]).sum() / 2
        ent_loss = -self.ent_weight * (entropy if entropy is not None else th.zeros(1, device=log_prob.device))
        neglogp = -log_prob
        l2_loss = self.l2_weight * l2_norm
        loss = neglogp + ent_loss + l2_loss
        return BCTrainingMetrics(neglogp=neglogp, entropy=entropy, ent_loss=ent_loss, prob_true_act=prob_true_act,
                                 l2_norm=l2_norm, l2_loss=l2_loss, loss=loss)

    def _fused_categorical(self, policy, obs, acts) -> Optional[BCTrainingMetrics]:
        """Discrete-action policies on the GPU with their parameters in one flat bucket
        (FusedAdam): the head's logits feed one fused loss op (``ops.rl.bc_categorical_loss``:
        2 launches forward, 1 backward) and the value head is not evaluated (BC never uses
        it). Same metrics and loss as the generic path."""
        from imitation_amd.ops import rl as rl_ops
        from imitation_amd.ops import use_kernel
        from imitation_amd.rl.distributions import CategoricalDistribution

        if (self.l2_weight != 0.0 or not isinstance(policy, ActorCriticPolicy) or not isinstance(obs, th.Tensor)
                or not use_kernel(obs) or not isinstance(policy.action_dist, CategoricalDistribution)):
            return None
        params = list(policy.parameters())
        flat = rl_ops.flat_param_view(params)
        if flat is None:
            return None
        dist = policy.get_distribution(obs)
        m, loss = rl_ops.bc_categorical_loss(dist.raw_logits, acts, params, self.ent_weight, self.l2_weight, flat)
        fields = {k: m[i] for i, k in enumerate(rl_ops.BC_METRICS)}
        fields["loss"] = loss
        return BCTrainingMetrics(**fields)


def enumerate_batches(batch_it: Iterable[types.TransitionMapping]) -> Iterable[Tuple[Tuple[int, int, int], types.TransitionMapping]]:
    """Prepends batch stats before the batches of a batch iterator."""
    num_samples_so_far = 0
    for num_batches, batch in enumerate(batch_it):
        batch_size = batch["_n"] if "_n" in batch else len(batch["obs"])  # (_n: agent-concatenated batches)
        num_samples_so_far += batch_size
        yield (num_batches, batch_size, num_samples_so_far), batch


class _Done:
    def __init__(self, value):
        self.value = value

    def result(self):
        return self.value


@dataclasses.dataclass(frozen=True)
class RolloutStatsComputer:
    """Computes statistics about rollouts (for logging during BC)."""

    venv: Optional[Any]
    n_episodes: int

    def start(self, policy, rng: np.random.Generator):
        """The statistics of ``policy`` as it is now, possibly still being computed when this
        returns (a device venv runs them on a worker thread and a side stream while training
        goes on): an object whose ``result()`` gives them. IMITATION_AMD_BC_ASYNC_STATS=0: in line."""
        import os

        if (self.venv is not None and self.n_episodes > 0 and hasattr(self.venv, "start_rollout_stats")
                and os.environ.get("IMITATION_AMD_BC_ASYNC_STATS", "1") != "0"):
            return self.venv.start_rollout_stats(policy, self.n_episodes)
        return _Done(self(policy, rng))

    def __call__(self, policy, rng: np.random.Generator) -> Mapping[str, float]:
        if self.venv is not None and self.n_episodes > 0 and hasattr(self.venv, "device_rollout_stats"):
            return self.venv.device_rollout_stats(policy, self.n_episodes)  # e.g. DAgger's device collector
        if self.venv is not None and self.n_episodes > 0:
            trajs = rollout.generate_trajectories(policy, self.venv, rollout.make_min_episodes(self.n_episodes), rng=rng)
            return rollout.rollout_stats(trajs)
        return dict()


class BCLogger:
    """Utility class to help logging information relevant to Behavior Cloning."""

    def __init__(self, logger: imit_logger.HierarchicalLogger):
        self._logger = logger
        self._tensorboard_step = 0
        self._current_epoch = 0

    def reset_tensorboard_steps(self):
        self._tensorboard_step = 0

    def log_epoch(self, epoch_number):
        self._current_epoch = epoch_number

    def log_batch(self, batch_num: int, batch_size: int, num_samples_so_far: int, training_metrics: BCTrainingMetrics,
                  rollout_stats: Mapping[str, float]):
        self._logger.record("batch_size", batch_size)
        self._logger.record("bc/epoch", self._current_epoch)
        self._logger.record("bc/batch", batch_num)
        self._logger.record("bc/samples_so_far", num_samples_so_far)
        vals = {k: v for k, v in training_metrics.__dict__.items()}
        tens = [v.detach().reshape(-1)[0] for v in vals.values() if v is not None]
        host = th.stack(tens).tolist() if tens else []
        bad = [k for k, x in zip((k for k, v in vals.items() if v is not None), host) if not math.isfinite(x)]
        if bad:  # the values are on the host already: fail fast instead of logging NaN for the rest of the run
            from imitation_amd.utils.watchdog import NonFiniteError

            raise NonFiniteError(f"non-finite BC metrics at batch {batch_num} (epoch {self._current_epoch}): "
                                 f"{', '.join(bad)}")
        it = iter(host)
        for k, v in vals.items():
            self._logger.record(f"bc/{k}", float(next(it)) if v is not None else None)
        for k, v in rollout_stats.items():
            if "return" in k and "monitor" not in k:
                self._logger.record("rollout/" + k, v)
        self._logger.dump(self._tensorboard_step)
        self._tensorboard_step += 1

    def __getstate__(self):
        state = self.__dict__.copy()
        del state["_logger"]
        return state


def reconstruct_policy(policy_path: str, device: Union[th.device, str] = "auto") -> ActorCriticPolicy:
    """Reconstruct a saved policy (``util.save_policy`` / ``final.th``; weights_only load)."""
    from imitation_amd.rl.policies import load_policy_file

    policy = load_policy_file(policy_path, device=device)
    assert isinstance(policy, ActorCriticPolicy)
    return policy


class _BCBase(algo_base.DemonstrationAlgorithm):
    """Shared training loop of BC and MultiBC."""

    def _init_common(self, batch_size, minibatch_size, demonstrations, custom_logger):
        self._demo_data_loader: Optional[Iterable[types.TransitionMapping]] = None
        self.batch_size = batch_size
        self.minibatch_size = minibatch_size or batch_size
        if self.batch_size % self.minibatch_size != 0:  # pragma: no cover
            raise ValueError("Batch size must be a multiple of minibatch size.")
        algo_base.DemonstrationAlgorithm.__init__(self, demonstrations=demonstrations, custom_logger=custom_logger)
        self._bc_logger = BCLogger(self.logger)

    def _init_optimizer(self, optimizer_cls, optimizer_kwargs, ent_weight, l2_weight):
        if optimizer_kwargs and "weight_decay" in optimizer_kwargs:  # pragma: no cover
            raise ValueError("Use the parameter l2_weight instead of weight_decay.")
        pdist.broadcast_module(self._policy)
        # th.optim.Adam / AdamW on a GPU -> one-launch flat-buffer step (ops/optim.py)
        cls = optim_ops.fused_for(optimizer_cls, self.policy.device) or optimizer_cls
        self.optimizer = cls(self.policy.parameters(), **(optimizer_kwargs or {}))
        self.loss_calculator = BehaviorCloningLossCalculator(ent_weight, l2_weight)
        if pdist.world_size() <= 1:
            self._grad_bucket = None
        elif isinstance(self.optimizer, optim_ops.FusedAdam):
            self._grad_bucket = pdist.FlatGradBucket(self.optimizer)  # its gradient buffer IS the bucket
        else:
            self._grad_bucket = pdist.GradBucket(self.policy.parameters())

    @property
    def policy(self) -> ActorCriticPolicy:
        return self._policy

    def set_demonstrations(self, demonstrations: algo_base.AnyTransitions) -> None:
        self._demo_data_loader = algo_base.make_data_loader(demonstrations, self.minibatch_size)

    def _prepare_batch(self, batch) -> Tuple[Any, th.Tensor]:
        obs = types.map_maybe_dict(lambda x: util.safe_to_tensor(x, device=self.policy.device), types.maybe_unwrap_dictobs(batch["obs"]))
        acts = util.safe_to_tensor(batch["acts"], device=self.policy.device)
        return obs, acts

    def _graphed_step(self) -> Optional[graphs.GraphedTrainStep]:
        """HIP-graph minibatch step when it has the eager loop's semantics: GPU policy, no
        gradient accumulation (minibatch == batch), no DP gradient bucket, an optimiser with
        a capturable mode. Disabled with ``IMITATION_AMD_BC_GRAPH=0``."""
        if (self.minibatch_size != self.batch_size or not graphs.graphs_enabled(self.policy.device, "IMITATION_AMD_BC_GRAPH")
                or not graphs.supports_capture(self.optimizer)):
            return None
        if self._grad_bucket is not None:
            # data parallel: the fused NatureCNN step (when it applies) as two graphs around the
            # bucket all-reduce; other policies keep the eager DP loop
            g = getattr(self, "_dp_step", None)
            if g is None or g.optimizer is not self.optimizer:
                g = self._dp_step = _DPFusedStep(self)
            return g
        g = getattr(self, "_graph_step", None)
        if g is None or g.optimizer is not self.optimizer:
            fused_buckets = isinstance(self.optimizer, optim_ops.FusedAdam)
            cnn_steps: Dict[Any, Any] = {}

            def step(obs, acts):
                # NatureCNN categorical learners: the whole minibatch on the fused kernels,
                # gradients straight into the bucket (ops/bc_cnn.py)
                key = (tuple(obs.shape), obs.dtype)
                if key not in cnn_steps:
                    cnn_steps[key] = bc_cnn.FusedCnnBCStep.maybe(self.policy, self.optimizer, obs,
                                                                self.loss_calculator.ent_weight,
                                                                self.loss_calculator.l2_weight)
                fused = cnn_steps[key]
                if fused is not None:
                    m = fused(obs, acts)
                    self.optimizer.step()
                    return BCTrainingMetrics(**bc_cnn.metrics_fields(m))
                metrics = self.loss_calculator(self.policy, obs, acts)
                if fused_buckets:  # buckets are zero here: the graph runs from zero_grad / a step
                    self.optimizer.backward_into_buckets(metrics.loss)
                else:
                    metrics.loss.backward()
                self.optimizer.step()
                return metrics

            def release():
                dist = getattr(self.policy, "action_dist", None)
                if dist is not None and hasattr(dist, "detach_"):
                    dist.detach_()

            g = self._graph_step = graphs.GraphedTrainStep(step, self.optimizer, release)
        return g

    def _epoch_runner(self, graphed, on_batch_end) -> Optional["_DeviceEpochRunner"]:
        """The graph-epoch runner when the demonstrations are a device aggregate (DAgger's
        device collector, ``engine/dagger.py``) and every minibatch is the fused NatureCNN
        step: nothing per minibatch needs the host. Disabled with ``IMITATION_AMD_BC_EPOCH_GRAPH=0``."""
        import os

        loader = self._demo_data_loader
        loader = getattr(loader, "data_loader", loader)  # (make_data_loader's batch-size-checking wrapper)
        if (graphed is None or on_batch_end is not None or not hasattr(loader, "next_epoch_perm")
                or self.minibatch_size != self.batch_size or os.environ.get("IMITATION_AMD_BC_EPOCH_GRAPH", "1") == "0"):
            return None
        if self._grad_bucket is not None and _DeviceEpochRunner.dp_comm(self.optimizer) is None:
            return None  # data parallel without a capturable gradient all-reduce: _DPFusedStep per minibatch
        r = getattr(self, "_epoch_run", None)
        if r is not None and r.graphed is graphed and r.loader is not loader and getattr(loader, "agg", None) is r.agg:
            # a new loader over the same aggregate (DAgger: one per round): the captured step
            # graphs read the aggregate, the runner's perm / cursor buffers and the policy, not
            # the loader -- keep them (a recapture per round cost ~15 ms on DAgger-Pong)
            r.loader = loader
        if r is None or r.loader is not loader or r.graphed is not graphed:
            r = _DeviceEpochRunner(self, loader, graphed)
            if not r.ok:
                return None
            self._epoch_run = r
        return r

    def _zero_grad(self):
        self.optimizer.zero_grad(set_to_none=self._grad_bucket is None)
        if self._grad_bucket is not None:
            self._grad_bucket.zero()

    @gcfreeze.during
    def train(self, *, n_epochs: Optional[int] = None, n_batches: Optional[int] = None,
              on_epoch_end: Optional[Callable[[], None]] = None, on_batch_end: Optional[Callable[[], None]] = None,
              log_interval: int = 500, log_rollouts_venv=None, log_rollouts_n_episodes: int = 5,
              progress_bar: bool = True, reset_tensorboard: bool = False):
        """Train with supervised learning for ``n_epochs`` epochs or ``n_batches`` batches."""
        if reset_tensorboard:
            self._bc_logger.reset_tensorboard_steps()
        self._bc_logger.log_epoch(0)
        compute_rollout_stats = RolloutStatsComputer(log_rollouts_venv, log_rollouts_n_episodes)

        def _on_epoch_end(epoch_number: int):
            pdist.check_comm("BC epoch")
            self._bc_logger.log_epoch(epoch_number + 1)
            if on_epoch_end is not None:
                on_epoch_end()

        mini_per_batch = self.batch_size // self.minibatch_size
        n_minibatches = n_batches * mini_per_batch if n_batches is not None else None
        assert self._demo_data_loader is not None
        demonstration_batches = BatchIteratorWithEpochEndCallback(self._demo_data_loader, n_epochs, n_minibatches, _on_epoch_end)
        batches_with_stats = enumerate_batches(demonstration_batches)
        state: Dict[str, Any] = {}

        def process_batch(stepped: bool = False):
            if not stepped:
                if self._grad_bucket is not None:
                    self._grad_bucket.allreduce()
                self.optimizer.step()
                self._zero_grad()
            if state["batch_num"] % log_interval == 0:
                rollout_stats = compute_rollout_stats(self.policy, self.rng)
                self._bc_logger.log_batch(state["batch_num"], state["minibatch_size"], state["num_samples_so_far"],
                                          state["metrics"], rollout_stats)
            if on_batch_end is not None:
                on_batch_end()

        self._zero_grad()
        graphed = self._graphed_step()
        runner = self._epoch_runner(graphed, on_batch_end)
        if runner is not None:
            # device-resident demonstrations: whole runs of minibatches per HIP-graph replay
            runner.train(n_epochs, n_minibatches, _on_epoch_end, log_interval, compute_rollout_stats)
            pdist.check_comm("BC training", blocking=True)
            return
        num_samples_so_far = 0
        for (batch_num, minibatch_size, num_samples_so_far), batch in batches_with_stats:
            obs, acts = self._prepare_batch(batch)
            if graphed is not None and isinstance(obs, th.Tensor) and minibatch_size == self.batch_size:
                # whole minibatch step (fwd + bwd + optimizer) as one HIP-graph replay (data
                # parallel: two replays around the bucket all-reduce)
                metrics = graphed(obs, acts)
                if metrics is not None:
                    batch_num = batch_num * self.minibatch_size // self.batch_size
                    state.update(batch_num=batch_num, minibatch_size=minibatch_size, num_samples_so_far=num_samples_so_far,
                                 metrics=metrics)
                    process_batch(stepped=True)
                    continue
            if graphed is not None and graphed.n_captures:
                self._zero_grad()  # p.grad still holds the last replay's gradients
            metrics = self.loss_calculator(self.policy, obs, acts)
            loss = metrics.loss * minibatch_size / self.batch_size
            loss.backward()
            batch_num = batch_num * self.minibatch_size // self.batch_size
            state.update(batch_num=batch_num, minibatch_size=minibatch_size, num_samples_so_far=num_samples_so_far, metrics=metrics)
            if num_samples_so_far % self.batch_size == 0:
                process_batch()
        if num_samples_so_far % self.batch_size != 0 and state:
            state["batch_num"] += 1
            process_batch()
        # the per-epoch checks are non-blocking (they read the previous epoch's error word):
        # one blocking check makes a timed-out all-reduce in the last epoch raise here
        pdist.check_comm("BC training", blocking=True)


class _DPFusedStep:
    """Data-parallel BC minibatch on the fused NatureCNN step (``ops/bc_cnn.py``): graph G1 (the
    autograd-free forward / backward writing the local minibatch-mean gradients into the FusedAdam
    bucket), the bucket all-reduce (mean over ranks: reference ``bc.py:464-466`` hook point; RCCL,
    or gloo on one-card rehearsals), graph G2 (the optimizer step). Falls back to the eager DP loop
    (returns None from :meth:`__call__`) when the fused step does not apply to the batch."""

    def __init__(self, trainer: "_BCBase"):
        self.trainer = trainer
        self.optimizer = trainer.optimizer
        self._fused: Dict[Any, Any] = {}
        self._graphs: Dict[Any, Any] = {}
        self.n_captures = 0
        self.n_replays = 0
        self._warm: set = set()

    def __call__(self, obs: th.Tensor, acts: th.Tensor):
        t = self.trainer
        key = (tuple(obs.shape), obs.dtype)
        if key not in self._fused:
            self._fused[key] = bc_cnn.FusedCnnBCStep.maybe(t.policy, t.optimizer, obs, t.loss_calculator.ent_weight,
                                                           t.loss_calculator.l2_weight)
        f = self._fused[key]
        if f is None:
            return None
        entry = self._graphs.get(key)
        if entry is None and key not in self._warm:
            # first call for this shape: one eager step, so that lazily created library /
            # allocator state is never first made inside a capture (as GraphedTrainStep does)
            self._warm.add(key)
            f(obs, acts)
            t._grad_bucket.allreduce()
            t.optimizer.step()
            self.n_replays += 1
            return BCTrainingMetrics(**bc_cnn.metrics_fields(f.metrics))
        if entry is None:
            static = tuple(x if getattr(x, "_ia_static", False) else x.detach().clone() for x in (obs, acts))
            side = th.cuda.Stream()
            side.wait_stream(th.cuda.current_stream())
            g1, g2 = th.cuda.CUDAGraph(), th.cuda.CUDAGraph()
            with graphs.capture(g1, stream=side):
                f(*static)
            with graphs.capture(g2, stream=side):
                t.optimizer.step()
            th.cuda.current_stream().wait_stream(side)
            entry = self._graphs[key] = (static, g1, g2)
            self.n_captures += 1
        static, g1, g2 = entry
        for sx, x in zip(static, (obs, acts)):
            if sx.data_ptr() != x.data_ptr():
                sx.copy_(x, non_blocking=True)
        g1.replay()
        t._grad_bucket.allreduce()
        g2.replay()
        self.n_replays += 1
        return BCTrainingMetrics(**bc_cnn.metrics_fields(f.metrics))


class _DeviceEpochRunner:
    """BC epochs over a device demonstration aggregate as HIP-graph replays of ``K`` minibatch
    steps each: per step ``gather_rows_cursor`` (rows ``perm[cursor * B ..]`` into the
    aggregate's persistent batch buffers; run inside the step's weight-packing launch), the fused NatureCNN step (``ops/bc_cnn.py``), the
    optimizer step and ``append_at_cursor`` (the step's metrics into their row, cursor + 1).
    Per epoch the host only draws the permutation (one launch) and replays; the reference loop's
    per-batch observable effects are kept: rollout statistics + logging at every
    ``log_interval``-th batch (the replays stop at those batches), epoch-end callbacks, the
    ``n_batches`` cut-off (reference ``bc.py:443-510``). Same batches, kernels and order as the
    per-minibatch loop, so the result is bitwise the eager-graph path's."""

    K = 16  # default largest graph (minibatch steps per replay); IMITATION_AMD_BC_GRAPH_K overrides
    # the minibatch gather inside the fused step's weight-packing launch (False: its own launch;
    # test hook / A/B, bitwise the same)
    fuse_gather = True
    # the conv weight-gradient reductions inside the Adam launch (False: conv_reduce_multi's own
    # launch; test hook / A/B, bitwise the same). Not under data parallelism: the all-reduce runs
    # between them and Adam.
    fuse_reduce = True

    def __init__(self, trainer: "_BCBase", loader, graphed):
        self.trainer, self.loader, self.graphed = trainer, loader, graphed
        self.B = trainer.batch_size
        self.agg = loader.agg
        self.ok = len(self.agg) >= self.B and self._fused() is not None
        self._key = None
        import os

        opt = trainer.optimizer
        self._fold = hasattr(opt, "graph_epoch_step_ok") and opt.graph_epoch_step_ok()
        self._world = pdist.world_size()
        self._comm = _DeviceEpochRunner.dp_comm(opt) if self._world > 1 else None
        if self._world > 1 and self._comm is None:
            self.ok = False
        if self._comm is not None:
            from imitation_amd.utils.streams import shared_stream

            self._dp_side = shared_stream(self.agg.device, "bc_dp_reduce")
        kmax = max(1, int(os.environ.get("IMITATION_AMD_BC_GRAPH_K", self.K)))
        # graph sizes: the largest, then powers of two below it. A run of n steps replays the
        # largest as often as it fits and each smaller one at most once, so the remainder is
        # never a chain of relaunches of one exec (each would wait on the host for the last)
        self._sizes = [kmax] + [1 << i for i in range(kmax.bit_length() - 1, -1, -1) if (1 << i) < kmax]

    def _fused(self):
        t = self.trainer
        obs = self.agg.batch_buffers(self.B)[0]
        f = getattr(self, "_f", None)
        if f is None:
            f = bc_cnn.FusedCnnBCStep.maybe(t.policy, t.optimizer, obs, t.loss_calculator.ent_weight,
                                            t.loss_calculator.l2_weight)
            self._f = f
        return f

    @staticmethod
    def dp_comm(optimizer):
        """Under data parallelism, the one-shot communicator (``parallel/oneshot.py``: one kernel,
        capture-safe) when it can reduce the optimizer's single flat gradient bucket in chunks of
        its staging size; None otherwise (then the per-minibatch ``_DPFusedStep`` runs). Every rank
        reaches this at the same point (the communicator's creation is collective)."""
        if pdist.world_size() <= 1:
            return None
        from imitation_amd.parallel import oneshot

        comm = oneshot.get()
        if comm is None or not (hasattr(optimizer, "graph_epoch_step_ok") and optimizer.graph_epoch_step_ok()):
            return None
        flat = optimizer.flat_grads[0]
        return comm if comm.fits(flat[: min(flat.numel(), comm.stage_bytes // 4 // 4 * 4)]) else None

    def _dp_ranges(self):
        """(FC range, other ranges) of the flat gradient bucket, each split into one-shot chunks
        (<= staging size, 16-B multiples): the FC layer's gradients (6.4 of NatureCNN's 6.7 MB) are
        final right after ``fc_backward``, the conv / head ones only after the conv backward."""
        r = getattr(self, "_ranges", None)
        if r is not None:
            return r
        flat = self.trainer.optimizer.flat_grads[0]
        step = self._comm.stage_bytes // 4 // 4 * 4
        w = self._f.g_lin[0]
        lo = (w.data_ptr() - flat.data_ptr()) // 4
        hi = lo + w.numel()

        def chunks(a, b):
            return [flat[i : min(b, i + step)] for i in range(a, b, step)]

        if lo % 4 or hi % 4:
            # the early range must hold the FC weight gradient and nothing else (a neighbour's
            # gradient is not final yet) and start on a 16-B boundary: else no early reduction
            fc, rest = [], chunks(0, flat.numel())
        else:
            fc = chunks(lo, hi)
            rest = chunks(0, lo) + chunks(hi, flat.numel())
        self._ranges = r = (fc, rest)
        return r

    def _dp_allreduce(self, parts) -> None:
        """Mean over ranks, inside the captured step: one-shot kernels over ``parts`` (rank-order sum
        of grad / world per element: bitwise the eager ``FlatGradBucket.allreduce``, whatever the
        chunking)."""
        for t in parts:
            self._comm.allreduce_(t, 1.0 / self._world)

    def _one_step(self):
        C = self._f.C
        bufs = self.agg.batch_buffers(self.B)
        opt = self.trainer.optimizer
        gather = None
        if self._comm is not None or self._fold:
            # the minibatch gather and the step counter's add: inside the weight-packing launch, or
            # (``fuse_gather`` off, the test hook) a launch of its own -- bitwise the same rows
            gather = ([self.agg.obs, self.agg.acts], self.perm, self.cursor, self.B, bufs, opt.step_counter())
            if not self.fuse_gather:
                C.gather_rows_cursor(*gather[:5], inc=gather[5])
                gather = None
        if self._comm is not None:
            # data parallel, graph-resident: the bucket all-reduce is a captured one-shot kernel
            # between the fused step and Adam (reference hook point bc.py:464-466)
            fc, rest = self._dp_ranges()
            main = th.cuda.current_stream()
            side = self._dp_side

            def after_fc():
                # the FC gradients are final: reduce them on the side stream (in a captured graph: a
                # parallel branch) while the main stream runs the conv backward
                side.wait_stream(main)
                with th.cuda.stream(side):
                    self._dp_allreduce(fc)

            self._f(bufs[0], bufs[1], after_fc=after_fc, gather=gather)
            # (the one-shot calls of a rank share one staging region: the rest waits for the FC part)
            main.wait_stream(side)
            self._dp_allreduce(rest)
            opt.step(step_incremented=True, append=(self._f.metrics, self.all, self.cursor))
            return
        if self._fold:
            # the gather rides on the weight-packing launch, the conv weight-gradient reductions and
            # the metrics append on Adam's: 12 launches per step (same arithmetic)
            fold = self.fuse_reduce and self._f.reduce_foldable
            self._f(bufs[0], bufs[1], gather=gather, defer_reduce=fold)
            # zero_grad off: the fused step writes (not accumulates) every gradient slot Adam reads
            # with a nonzero value -- conv, FC and head; the value net's slots, which BC never
            # writes, stay at the zeros of the last zeroing step
            opt.step(step_incremented=True, append=(self._f.metrics, self.all, self.cursor),
                     reduce=self._f.pending_reduce if fold else None, zero_grad=False)
            return
        C.gather_rows_cursor([self.agg.obs, self.agg.acts], self.perm, self.cursor, self.B, bufs)
        self._f(bufs[0], bufs[1])
        opt.step()
        C.append_at_cursor(self._f.metrics, self.all, self.cursor)

    def _prepare(self, n: int) -> None:
        """(Re)allocate the static perm / metric buffers and capture the step graphs when the
        aggregate's storage or the epoch size outgrew them (capacity doubling: O(log) captures)."""
        dev = self.agg.device
        cap = max(n, getattr(self, "_cap", 0))
        key = (self.agg.obs.data_ptr(), self.agg.acts.data_ptr())
        if self._key == key and n <= getattr(self, "_cap", 0):
            return
        if n > getattr(self, "_cap", 0):
            # room for every row the aggregate's storage can hold: a growing aggregate then
            # recaptures only when its storage moves
            cap = max(n, 2 * getattr(self, "_cap", 0), self.agg.obs.shape[0])
            self.perm = th.zeros(cap, dtype=th.int32, device=dev)
            self.all = th.zeros(cap // self.B + 1, 8, device=dev)
            self.cursor = th.zeros(1, dtype=th.int32, device=dev)
            self._cap = cap
        self._key = key
        self.graphs = None  # captured by the next _run, after the eager warm-up step

    def _capture(self) -> None:
        """The step graphs of every size in ``_sizes``, captured once (alternating two instances per
        size, or waiting on the previous launch's event before a relaunch, measured slower on
        DAgger-Pong in round 5, ``profiles/r5_dagger.md``)."""
        self.graphs = {}
        side = getattr(self, "_capture_stream", None)
        if side is None:  # (creating a stream costs ~1 ms of host time)
            side = self._capture_stream = th.cuda.Stream()
        side.wait_stream(th.cuda.current_stream())
        for k in self._sizes:
            g = th.cuda.CUDAGraph()
            with graphs.capture(g, stream=side):
                for _ in range(k):
                    self._one_step()
            self.graphs[k] = g
        th.cuda.current_stream().wait_stream(side)

    def _replay(self, k: int) -> None:
        self.graphs[k].replay()

    def _run(self, steps: int) -> None:
        if steps > 0 and not getattr(self, "_warm", False):
            # the first step runs eagerly (same kernels, so the same result): lazily created
            # library / allocator state is never first made inside a capture
            self._one_step()
            self._warm = True
            steps -= 1
        if steps > 0 and self.graphs is None:
            self._capture()
        for k in self._sizes:
            while steps >= k:
                self._replay(k)
                steps -= k

    def _finite_flag(self, epoch: int, steps: int) -> None:
        """Fail fast on NaN/Inf BC metrics without a sync per epoch: one reduction over the epoch's
        metric rows lands in pinned memory asynchronously; it is read one epoch later (long done by
        then) and at the end of :meth:`train`."""
        self._check_finite_flag(blocking=False)
        if not hasattr(self, "_flag_host"):
            self._flag_host = th.zeros(1, dtype=th.int32, pin_memory=True)
        self._flag_host.copy_(th.isfinite(self.all[:steps]).all().to(th.int32).reshape(1), non_blocking=True)
        ev = th.cuda.Event()
        ev.record()
        self._flag_pending = (epoch, ev)

    def _check_finite_flag(self, blocking: bool) -> None:
        pend = getattr(self, "_flag_pending", None)
        if pend is None:
            return
        epoch, ev = pend
        if not blocking and not ev.query():
            return
        ev.synchronize()
        self._flag_pending = None
        if not int(self._flag_host[0]):
            from imitation_amd.utils.watchdog import NonFiniteError

            raise NonFiniteError(f"non-finite BC metrics (loss / entropy / log-prob) in epoch {epoch} of this train() call")

    def train(self, n_epochs, n_batches, on_epoch_end, log_interval: int, compute_rollout_stats) -> None:
        try:
            self._train(n_epochs, n_batches, on_epoch_end, log_interval, compute_rollout_stats)
        finally:
            self._check_finite_flag(blocking=True)

    def _train(self, n_epochs, n_batches, on_epoch_end, log_interval: int, compute_rollout_stats) -> None:
        t = self.trainer
        B = self.B
        batch_num = 0  # minibatches stepped in this call (the reference loop's batch_num)
        epoch = 0
        while (n_epochs is None or epoch < n_epochs) and (n_batches is None or batch_num < n_batches):
            n = len(self.agg)
            nb = n // B
            if nb == 0:
                raise AssertionError(f"Data loader returned no data during epoch {epoch} -- did it reset correctly?")
            perm = self.loader.next_epoch_perm()
            self._prepare(n)
            self.perm[:n].copy_(perm)
            self.cursor.zero_()
            steps = nb if n_batches is None else min(nb, n_batches - batch_num)
            done = 0
            # a logged batch's rollout statistics run beside the following minibatches (worker
            # thread + side stream, on a snapshot of the policy as of that batch); its log_batch
            # is written when they are in -- before the next logged batch and the epoch's end
            pending = None
            try:
                while done < steps:
                    nxt = -(-(batch_num + done) // log_interval) * log_interval  # next logged batch
                    j = nxt - batch_num  # its index in this epoch
                    if j >= steps:
                        self._run(steps - done)
                        break
                    self._run(j + 1 - done)
                    if pending is not None:
                        p_, pending = pending, None
                        p_[0].result()
                        p_[1]()
                    m = BCTrainingMetrics(**bc_cnn.metrics_fields(self.all[j]))
                    if self.graphs is None and done < steps:
                        # capture the step graphs now: no capture may run while the statistics'
                        # worker thread is stepping the envs
                        self._capture()
                    fut = compute_rollout_stats.start(t.policy, t.rng)
                    pending = (fut, (lambda f=fut, nb_=nxt, mm=m: t._bc_logger.log_batch(nb_, B, (nb_ + 1) * B, mm,
                                                                                        f.result())))
                    done = j + 1
            except BaseException:
                if pending is not None:  # hand the envs back before unwinding
                    try:
                        pending[0].result()
                    except BaseException:  # noqa: BLE001 -- the original error wins
                        pass
                raise
            if pending is not None:
                pending[1]()
            self._finite_flag(epoch, steps)
            batch_num += steps
            # the reference's batch iterator reaches an epoch's end callback only when it is
            # asked for a batch after the epoch's last one
            if steps == nb and (n_batches is None or batch_num < n_batches):
                on_epoch_end(epoch)
            epoch += 1


class BC(_BCBase):
    """Behavioral cloning (BC): supervised learning of the expert's actions."""

    def __init__(self, *, observation_space: spaces.Space, action_space: spaces.Space, rng: np.random.Generator,
                 policy: Optional[ActorCriticPolicy] = None, demonstrations: Optional[algo_base.AnyTransitions] = None,
                 batch_size: int = 32, minibatch_size: Optional[int] = None,
                 optimizer_cls: Type[th.optim.Optimizer] = th.optim.Adam, optimizer_kwargs: Optional[Mapping[str, Any]] = None,
                 ent_weight: float = 1e-3, l2_weight: float = 0.0, device: Union[str, th.device] = "auto",
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None):
        self._init_common(batch_size, minibatch_size, demonstrations, custom_logger)
        self.action_space = action_space
        self.observation_space = observation_space
        self.rng = rng
        if policy is None:
            extractor = torch_layers.CombinedExtractor if isinstance(observation_space, spaces.Dict) else torch_layers.FlattenExtractor
            policy = policy_base.FeedForward32Policy(observation_space=observation_space, action_space=action_space,
                                                     lr_schedule=lambda _: th.finfo(th.float32).max,
                                                     features_extractor_class=extractor)
        self._policy = policy.to(get_device(device))
        assert self.policy.observation_space == self.observation_space
        assert self.policy.action_space == self.action_space
        self._init_optimizer(optimizer_cls, optimizer_kwargs, ent_weight, l2_weight)


class MultiBC(_BCBase):
    """BC for N parameter-shared homogeneous agents (fork addition, ``bc.py:512-776``)."""

    def __init__(self, *, single_agent_observation_space, single_agent_action_space, observation_overide, action_overide,
                 num_agents, rng: np.random.Generator, policy: Optional[ActorCriticPolicy] = None,
                 demonstrations: Optional[algo_base.AnyTransitions] = None, batch_size: int = 32,
                 minibatch_size: Optional[int] = None, optimizer_cls: Type[th.optim.Optimizer] = th.optim.Adam,
                 optimizer_kwargs: Optional[Mapping[str, Any]] = None, ent_weight: float = 1e-3, l2_weight: float = 0.0,
                 device: Union[str, th.device] = "auto", custom_logger: Optional[imit_logger.HierarchicalLogger] = None):
        self._init_common(batch_size, minibatch_size, demonstrations, custom_logger)
        self.action_space = single_agent_action_space
        self.observation_space = single_agent_observation_space
        self.observation_overide = observation_overide
        self.action_overide = action_overide
        self.num_agents = num_agents
        self.rng = rng
        if policy is None:
            extractor = torch_layers.CombinedExtractor if isinstance(single_agent_observation_space, spaces.Dict) else torch_layers.FlattenExtractor
            policy = policy_base.HomogenousFeedForward32Policy(
                observation_space=self.observation_space, action_space=self.action_space,
                observation_overide=self.observation_overide, action_overide=self.action_overide,
                num_agents=self.num_agents, lr_schedule=lambda _: th.finfo(th.float32).max,
                features_extractor_class=extractor)
        self._policy = policy.to(get_device(device))
        assert self.policy.observation_space == self.observation_space
        assert self.policy.action_space == self.action_space
        self._init_optimizer(optimizer_cls, optimizer_kwargs, ent_weight, l2_weight)

    def set_demonstrations(self, demonstrations: algo_base.AnyTransitions) -> None:
        super().set_demonstrations(demonstrations)
        self._pending_demos = demonstrations  # the device agent loader is built at train() time

    def train(self, **kwargs):
        demos = getattr(self, "_pending_demos", None)
        if demos is not None:
            self._pending_demos = None
            if isinstance(demos, types.TransitionsMinimal) and self.policy.device.type == "cuda":
                loader = _AgentGatherLoader.maybe(demos, self.observation_overide, self.action_overide, self.num_agents,
                                                  self.minibatch_size, self.policy.device, int(self.rng.integers(0, 2**31 - 1)))
                if loader is not None:
                    self._demo_data_loader = loader
        return super().train(**kwargs)

    def _prepare_batch(self, batch):
        if batch.get("_agent_cat"):  # already agent-concatenated on the device (_AgentGatherLoader)
            return batch["obs"], batch["acts"]
        obs_all, acts_all = super()._prepare_batch(batch)
        obs = th.cat([self.observation_overide(i, obs_all) for i in range(self.num_agents)])
        acts = th.cat([self.action_overide(i, acts_all) for i in range(self.num_agents)])
        return obs, acts


def _column_map(fn, i: int, ncols: int, dtype, one_d: bool = False) -> Optional[Tuple[List[int], bool]]:
    """If ``fn(i, x)`` selects columns of a 2-D ``x`` (same selection for every row), the
    selected column ids and whether the result is 1-D; else None. Probed on a tiny host tensor
    whose entries encode (row, column). ``one_d``: ``x`` is 1-D (``[B]`` actions); only the
    identity selection ``fn(i, x) == x`` is folded then. The probe is a candidate only: the
    caller confirms it on real rows (:func:`_confirm_column_map`)."""
    if one_d:
        probe = th.tensor([0, 1], dtype=dtype)
        try:
            out = fn(i, probe)
        except Exception:  # noqa: BLE001 -- arbitrary user callable
            return None
        if not isinstance(out, th.Tensor) or out.shape != probe.shape or not th.equal(out.to(dtype), probe):
            return None
        return [0], True
    probe = (th.arange(ncols, dtype=th.int64)[None, :] + th.tensor([[0], [ncols]])).to(dtype)
    try:
        out = fn(i, probe)
    except Exception:  # noqa: BLE001 -- arbitrary user callable: any failure means "not a selection"
        return None
    if not isinstance(out, th.Tensor) or out.shape[:1] != (2,) or out.dim() not in (1, 2):
        return None
    o = out.to(th.int64).reshape(2, -1)
    if not th.equal(out.to(dtype).reshape(2, -1), o.to(dtype)) or not th.equal(o[1] - o[0], th.full_like(o[0], ncols)):
        return None
    cols = o[0].tolist()
    if any(c < 0 or c >= ncols for c in cols):
        return None
    return cols, out.dim() == 1


def _confirm_column_map(fn, i: int, rows: th.Tensor, m: Tuple[List[int], bool]) -> bool:
    """``fn(i, rows)`` equals the gather the column map ``m`` implies, values and shape, on real
    demonstration rows (a probe alone accepts e.g. agent-dependent in-range shifts)."""
    cols, is_1d = m
    want = rows if rows.dim() == 1 else rows[:, cols]
    if is_1d and want.dim() == 2:
        want = want.reshape(-1)
    try:
        out = fn(i, rows.clone())
    except Exception:  # noqa: BLE001
        return False
    return isinstance(out, th.Tensor) and out.shape == want.shape and th.equal(out.to(want.dtype), want)


class _AgentGatherLoader:
    """Device-resident MultiBC demonstrations with the agent concatenation folded into the row
    gather (``bc.py:752-759`` ``observation_overide`` / ``action_overide`` + ``th.cat``): when every
    override is a column selection, the per-agent column slices are laid out agent-major on the
    device once, each epoch draws one ``perm_feistel`` permutation and builds every batch's
    ``[n_agents * B]`` row ids in one launch, and a batch is ONE ``gather_rows`` launch into
    persistent buffers the graphed step reads in place -- no host-to-device copy, no concatenation
    kernels per minibatch. Shuffled, drop-last, like the host loader."""

    def __init__(self, obs_ag: th.Tensor, acts_ag: th.Tensor, n: int, n_agents: int, batch_size: int, seed: int):
        self.obs_ag, self.acts_ag = obs_ag, acts_ag
        self.n, self.n_agents, self.batch_size = n, n_agents, batch_size
        self._seed, self._epoch = seed, 0
        dev = obs_ag.device
        self._off = (th.arange(n_agents, device=dev, dtype=th.int64) * n).view(1, n_agents, 1)
        self.bufs = [th.empty((n_agents * batch_size,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
                     for t in (obs_ag, acts_ag)]
        for t in self.bufs:
            t._ia_static = True

    @staticmethod
    def maybe(demos, obs_fn, act_fn, n_agents: int, batch_size: int, device, seed: int) -> Optional["_AgentGatherLoader"]:
        import os

        if os.environ.get("IMITATION_AMD_MULTIBC_GATHER", "1") == "0":
            return None
        obs = np.asarray(demos.obs)
        acts = np.asarray(demos.acts)
        if obs.ndim != 2 or acts.ndim not in (1, 2) or len(obs) < batch_size:
            return None
        acts2 = acts.reshape(len(acts), -1)
        adt = th.int64 if np.issubdtype(acts.dtype, np.integer) else th.float32
        om = [_column_map(obs_fn, i, obs.shape[1], th.float32) for i in range(n_agents)]
        am = [_column_map(act_fn, i, acts2.shape[1], adt, one_d=acts.ndim == 1) for i in range(n_agents)]
        if any(m is None for m in om + am) or len({len(m[0]) for m in om}) != 1 or len({(len(m[0]), m[1]) for m in am}) != 1:
            return None
        if any(m[1] for m in om):
            return None
        # confirm every candidate map on real rows (the host loader is the fallback)
        k = min(len(obs), 64)
        o_rows = th.from_numpy(np.array(obs[:k], dtype=np.float32))
        a_rows = th.from_numpy(np.array(acts[:k])).to(adt)
        if not all(_confirm_column_map(obs_fn, i, o_rows, om[i]) and _confirm_column_map(act_fn, i, a_rows, am[i])
                   for i in range(n_agents)):
            return None
        o = th.as_tensor(obs, device=device).float()
        a = th.as_tensor(acts2, device=device)
        obs_ag = th.cat([o[:, m[0]] for m in om]).contiguous()
        acts_ag = th.cat([a[:, m[0]] for m in am]).contiguous()
        if am[0][1]:
            acts_ag = acts_ag.reshape(-1)
        return _AgentGatherLoader(obs_ag, acts_ag, len(obs), n_agents, batch_size, seed)

    def __len__(self) -> int:
        return self.n // self.batch_size

    def __iter__(self):
        from imitation_amd.ops import rl as rl_ops

        self._epoch += 1
        B, nb = self.batch_size, self.n // self.batch_size
        perm = rl_ops.random_permutations(1, self.n, self._seed * 1000003 + self._epoch, self.obs_ag.device)[0]
        # every batch's agent-major row ids in one launch: ids[b, a, r] = a * n + perm[b * B + r]
        ids = (perm[: nb * B].view(nb, 1, B).to(th.int64) + self._off).view(nb, -1)
        for b in range(nb):
            rl_ops.gather_rows([self.obs_ag, self.acts_ag], ids[b], dst=self.bufs)
            yield {"obs": self.bufs[0], "acts": self.bufs[1], "_agent_cat": True, "_n": B}
