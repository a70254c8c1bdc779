"""Maximum-causal-entropy IRL on tabular MDPs (reference: ``src/imitation/algorithms/mce_irl.py``).

* :func:`mce_partition_fh` -- finite-horizon soft value iteration
  ``Q_t = R + γ T V_{t+1}``, ``V_t = logsumexp_a Q_t``, ``π_t = exp(Q_t - V_t)``
  (``mce_irl.py:38-93``);
* :func:`mce_occupancy_measures` -- ``D_{t+1} = Σ_a (D_t ∘ π_t[:, a]) T[:, a, :]``
  and the discounted cumulative ``Dcum`` (``:96-144``);
* :class:`TabularPolicy` (time-indexed stochastic policy, ``:163-258``);
* :class:`MCEIRL` -- gradient ``E_π[∇r] - E_D[∇r]`` through ``dot(D_π - D_demo, r)``
  (``:264-560``), stopping on L∞ occupancy error or gradient norm.

MI355X: on the GPU each recursion is ONE fp64 HIP launch
(``csrc/kernels/tabular.hip``: a single workgroup loops over the horizon with the running
vector and the step's ``[S, A]`` table in LDS, ``T`` streamed from L2) instead of ~6
launches per timestep; larger tables and the CPU run the same recursions as batched
torch ops (``T`` is ``[S, A, S']``), which reproduce the numpy reference in float64.
"""

from __future__ import annotations

import collections
import warnings
from typing import Any, Dict, Iterable, List, Mapping, NoReturn, Optional, Tuple, Type, Union

import numpy as np
import torch as th

from imitation_amd.algorithms import base
from imitation_amd.data import rollout, types
from imitation_amd.envs import spaces
from imitation_amd.rewards import reward_nets
from imitation_amd.rl.policies import BasePolicy
from imitation_amd.util import logger as imit_logger
from imitation_amd.util import networks, util


def _dev(device):
    if device is None:
        return th.device("cpu")
    return th.device(device)


def _use_tabular_kernel(dev: th.device, S: int, A: int) -> bool:
    """The one-workgroup HIP recursions (csrc/kernels/tabular.hip) apply on the GPU when the
    running vector and one step's [S, A] table fit LDS (S * (A + 1) doubles <= 150 KB)."""
    from imitation_amd import ops

    return dev.type == "cuda" and ops.fused_enabled() and S * (A + 1) * 8 <= 150 * 1024


def mce_partition_fh(env, *, reward: Optional[np.ndarray] = None, discount: float = 1.0, device=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Soft value iteration over a finite horizon; returns ``(V [H,S], Q [H,S,A], pi [H,S,A])``."""
    horizon = env.horizon
    if horizon is None:
        raise ValueError("Only finite-horizon environments are supported.")
    dev = _dev(device)
    T = th.as_tensor(env.transition_matrix, dtype=th.float64, device=dev)
    if reward is None:
        reward = env.reward_matrix
    R = th.as_tensor(np.asarray(reward), dtype=th.float64, device=dev)
    S, A = env.state_dim, env.action_dim
    if _use_tabular_kernel(dev, S, A) and R.dim() == 1:
        from imitation_amd.ops import native

        V, Q, pi = native().soft_value_iteration(T.contiguous(), R.contiguous(), int(horizon), float(discount))
        return V.cpu().numpy(), Q.cpu().numpy(), pi.cpu().numpy()
    Q = th.zeros((horizon, S, A), dtype=th.float64, device=dev)
    V = th.full((horizon, S), -np.inf, dtype=th.float64, device=dev)
    broad_R = R[:, None]
    Q[horizon - 1] = broad_R
    V[horizon - 1] = th.logsumexp(Q[horizon - 1], dim=1)
    for t in reversed(range(horizon - 1)):
        Q[t] = broad_R + discount * (T @ V[t + 1])
        V[t] = th.logsumexp(Q[t], dim=1)
    pi = th.exp(Q - V[:, :, None])
    return V.cpu().numpy(), Q.cpu().numpy(), pi.cpu().numpy()


def mce_occupancy_measures(env, *, reward: Optional[np.ndarray] = None, pi: Optional[np.ndarray] = None,
                           discount: float = 1.0, device=None) -> Tuple[np.ndarray, np.ndarray]:
    """State occupancy per timestep ``D [H+1, S]`` and discounted total ``Dcum [S]``."""
    horizon = env.horizon
    if horizon is None:
        raise ValueError("Only finite-horizon environments are supported.")
    dev = _dev(device)
    if reward is None:
        reward = env.reward_matrix
    if pi is None:
        _, _, pi = mce_partition_fh(env, reward=reward, device=device)
    T = th.as_tensor(env.transition_matrix, dtype=th.float64, device=dev)
    P = th.as_tensor(pi, dtype=th.float64, device=dev)
    S = env.state_dim
    D0 = th.as_tensor(env.initial_state_dist, dtype=th.float64, device=dev)
    if _use_tabular_kernel(dev, S, env.action_dim) and P.shape[0] >= horizon:
        from imitation_amd.ops import native

        D = native().occupancy_measures(T.contiguous(), P[:horizon].contiguous(), D0.contiguous())
    else:
        D = th.zeros((horizon + 1, S), dtype=th.float64, device=dev)
        D[0] = D0
        for t in range(horizon):
            # sum_a (D_t * pi_t[:, a]) @ T[:, a, :]
            D[t + 1] = th.einsum("s,sa,sap->p", D[t], P[t], T)
    Dn = D.cpu().numpy()
    Dcum = rollout.discounted_sum(Dn, discount)
    assert isinstance(Dcum, np.ndarray)
    return Dn, Dcum


def squeeze_r(r_output: th.Tensor) -> th.Tensor:
    """Squeeze a reward output of shape ``(N, 1)`` to ``(N,)``."""
    if r_output.ndim == 2:
        return th.squeeze(r_output, 1)
    assert r_output.ndim == 1
    return r_output


class TabularPolicy(BasePolicy):
    """A time-indexed tabular policy ``pi[t, s, a]`` (state is the timestep)."""

    def __init__(self, state_space: spaces.Space, action_space: spaces.Space, pi: np.ndarray, rng: np.random.Generator) -> None:
        assert isinstance(state_space, spaces.Discrete), "state not tabular"
        assert isinstance(action_space, spaces.Discrete), "action not tabular"
        super().__init__(observation_space=state_space, action_space=action_space)
        self.rng = rng
        self.set_pi(pi)

    def set_pi(self, pi: np.ndarray) -> None:
        assert pi.ndim == 3, "expected three-dimensional policy"
        assert np.allclose(pi.sum(axis=2), 1), "policy not normalized"
        assert np.all(pi >= 0), "policy has negative probabilities"
        self.pi = pi

    def _predict(self, observation, deterministic: bool = False):
        raise NotImplementedError("Should never be called as predict overridden.")

    def forward(self, observation, deterministic: bool = False) -> NoReturn:
        raise NotImplementedError("Should never be called.")  # pragma: no cover

    def predict(self, observation, state=None, episode_start=None, deterministic: bool = False):
        """Actions for a batch of states from the time-indexed policy table; ``state`` carries
        each env's timestep (starts at 0, reset where ``episode_start``)."""
        obs = np.asarray(observation)
        t = np.zeros(len(obs), dtype=int) if state is None else np.asarray(state[0])
        if state is not None:
            assert len(state) == 1
        assert len(t) == len(obs), "timestep and obs batch size differ"
        if episode_start is not None:
            t[np.asarray(episode_start, dtype=bool)] = 0
        assert all(self.observation_space.contains(o) for o in obs), "illegal state"
        probs = self.pi[t, obs]  # [B, A] gathered in one indexing op
        if deterministic:
            acts = probs.argmax(axis=1)
        else:  # inverse-CDF sampling per row, one uniform draw each
            u = self.rng.random(len(obs))[:, None]
            acts = np.minimum((probs.cumsum(axis=1) < u).sum(axis=1), probs.shape[1] - 1)
        return acts.astype(int), (t + 1,)


MCEDemonstrations = Union[np.ndarray, base.AnyTransitions]


class MCEIRL(base.DemonstrationAlgorithm[types.TransitionsMinimal]):
    """Tabular MCE IRL (Ziebart 2010) with a reward network over observation features."""

    def __init__(self, demonstrations: Optional[MCEDemonstrations], env, reward_net: reward_nets.RewardNet,
                 rng: np.random.Generator, optimizer_cls: Type[th.optim.Optimizer] = th.optim.Adam,
                 optimizer_kwargs: Optional[Mapping[str, Any]] = None, discount: float = 1.0, linf_eps: float = 1e-3,
                 grad_l2_eps: float = 1e-4, log_interval: Optional[int] = 100, *,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None, device=None) -> None:
        self.discount = discount
        self.env = env
        self.demo_state_om = None
        self.device = device
        super().__init__(demonstrations=demonstrations, custom_logger=custom_logger)
        self.reward_net = reward_net
        optimizer_kwargs = optimizer_kwargs or {"lr": 1e-2}
        self.optimizer = optimizer_cls(reward_net.parameters(), **optimizer_kwargs)
        self.linf_eps = linf_eps
        self.grad_l2_eps = grad_l2_eps
        self.log_interval = log_interval
        self.rng = rng
        if self.env.horizon is None:
            raise ValueError("Only finite-horizon environments are supported.")
        uniform_pi = np.ones((self.env.horizon, self.env.state_dim, self.env.action_dim)) / self.env.action_dim
        self._policy = TabularPolicy(state_space=self.env.state_space, action_space=self.env.action_space, pi=uniform_pi, rng=self.rng)

    def _set_demo_from_trajectories(self, trajs: Iterable[types.Trajectory]) -> None:
        """Discounted state visitation counts averaged over demonstrations (one bincount
        per trajectory with weights ``discount ** t``)."""
        S = self.env.state_dim
        om = np.zeros(S)
        n = 0
        for traj in trajs:
            states = np.asarray(types.assert_not_dictobs(traj.obs)).astype(int).reshape(-1)
            om += np.bincount(states, weights=self.discount ** np.arange(len(states)), minlength=S)
            n += 1
        self.demo_state_om = om / n

    def _set_demo_from_obs(self, obses: np.ndarray, dones: Optional[np.ndarray], next_obses: Optional[np.ndarray]) -> None:
        """Undiscounted visitation counts of transition data (terminal next-states included),
        rescaled to a horizon-``H`` trajectory's total mass ``H + 1``."""
        S = self.env.state_dim
        as_int = lambda a: np.asarray(a.cpu() if isinstance(a, th.Tensor) else a).astype(int).reshape(-1)  # noqa: E731
        om = np.bincount(as_int(obses), minlength=S).astype(float)
        if dones is not None and next_obses is not None:
            done = np.asarray(dones.cpu() if isinstance(dones, th.Tensor) else dones).astype(bool).reshape(-1)
            om += np.bincount(as_int(next_obses)[done], minlength=S)
        else:
            warnings.warn("Training MCEIRL with transitions that lack next observation."
                          "This will result in systematically wrong occupancy measure estimates.")
        self.demo_state_om = om * (self.env.horizon + 1) / om.sum()

    def set_demonstrations(self, demonstrations: MCEDemonstrations) -> None:
        if isinstance(demonstrations, np.ndarray):
            assert demonstrations.ndim == 1
            self.demo_state_om = demonstrations
            return
        if isinstance(demonstrations, Iterable):
            first_item, demonstrations_it = util.get_first_iter_element(demonstrations)
            if isinstance(first_item, types.Trajectory):
                self._set_demo_from_trajectories(demonstrations_it)
                return
        if self.discount != 1.0:
            raise ValueError("Cannot compute discounted OM from timeless Transitions.")
        if isinstance(demonstrations, types.Transitions):
            self._set_demo_from_obs(types.assert_not_dictobs(demonstrations.obs), demonstrations.dones,
                                    types.assert_not_dictobs(demonstrations.next_obs))
        elif isinstance(demonstrations, types.TransitionsMinimal):
            self._set_demo_from_obs(types.assert_not_dictobs(demonstrations.obs), None, None)
        elif isinstance(demonstrations, Iterable):
            collated_list: Dict[str, List] = collections.defaultdict(list)
            for batch in demonstrations:
                assert isinstance(batch, Mapping)
                for k in ("obs", "dones", "next_obs"):
                    x = batch.get(k)
                    if x is not None:
                        assert isinstance(x, (np.ndarray, th.Tensor))
                        collated_list[k].append(util.safe_to_numpy(x))
            collated = {k: np.concatenate(v) for k, v in collated_list.items()}
            assert "obs" in collated
            for k, v in collated.items():
                assert len(v) == len(collated["obs"]), k
            self._set_demo_from_obs(collated["obs"], collated.get("dones"), collated.get("next_obs"))
        else:
            raise TypeError(f"Unsupported demonstration type {type(demonstrations)}")

    def _train_step(self, obs_mat: th.Tensor) -> Tuple[np.ndarray, np.ndarray]:
        self.optimizer.zero_grad()
        predicted_r = squeeze_r(self.reward_net(obs_mat, None, None, None))
        assert predicted_r.shape == (obs_mat.shape[0],)
        predicted_r_np = predicted_r.detach().cpu().numpy()
        _, visitations = mce_occupancy_measures(self.env, reward=predicted_r_np, discount=self.discount, device=self.device)
        weights_th = th.as_tensor(visitations - self.demo_state_om, dtype=self.reward_net.dtype, device=self.reward_net.device)
        loss = th.dot(weights_th, predicted_r)
        loss.backward()
        self.optimizer.step()
        return predicted_r_np, visitations

    def train(self, max_iter: int = 1000) -> np.ndarray:
        """Run MCE IRL until the occupancy L∞ error or the gradient norm is small."""
        obs_mat = self.env.observation_matrix
        torch_obs_mat = th.as_tensor(obs_mat, dtype=self.reward_net.dtype, device=self.reward_net.device)
        assert self.demo_state_om is not None
        assert self.demo_state_om.shape == (len(obs_mat),)
        with networks.training(self.reward_net):
            for t in range(max_iter):
                predicted_r_np, visitations = self._train_step(torch_obs_mat)
                grads = [p.grad for p in self.reward_net.parameters()]
                grad_norm = util.tensor_iter_norm(grads).item()
                linf_delta = np.max(np.abs(self.demo_state_om - visitations))
                if self.log_interval is not None and 0 == (t % self.log_interval):
                    weight_norm = util.tensor_iter_norm(self.reward_net.parameters()).item()
                    self.logger.record("iteration", t)
                    self.logger.record("linf_delta", linf_delta)
                    self.logger.record("weight_norm", weight_norm)
                    self.logger.record("grad_norm", grad_norm)
                    self.logger.dump(t)
                if linf_delta <= self.linf_eps or grad_norm <= self.grad_l2_eps:
                    break
        _, _, pi = mce_partition_fh(self.env, reward=predicted_r_np, discount=self.discount, device=self.device)
        self._policy.set_pi(pi)
        return visitations

    @property
    def policy(self) -> BasePolicy:
        return self._policy
