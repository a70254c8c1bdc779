"""PPO (clipped surrogate) -- the reference's default generator / expert trainer
(SB3 PPO via ``scripts/ingredients/rl.py:58-66``).

Same hyper-parameters and update as SB3: GAE(γ, λ), per-minibatch advantage
normalisation, ratio clip ε, optional value clip, entropy bonus,
``clip_grad_norm(max_grad_norm)``, Adam(eps=1e-5), optional ``target_kl`` stop.

MI355X specifics: the rollout buffer is device resident and shuffled on the
device; actor/critic heads run as fused MFMA MLP kernels; per-minibatch
diagnostics stay on the device (one host sync per ``train()`` instead of several
per minibatch); under data parallelism each minibatch's gradients are averaged
with ONE all-reduce of a flat bucket before clipping.
"""

from __future__ import annotations

from typing import Any, Dict, Optional, Type, Union

import numpy as np
import torch as th
from torch.nn import functional as F

from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl.base import OnPolicyAlgorithm, explained_variance
from imitation_amd.rl.policies import ActorCriticCnnPolicy, ActorCriticPolicy, BasePolicy, MultiInputActorCriticPolicy, get_schedule_fn


class PPO(OnPolicyAlgorithm):
    policy_aliases = {
        "MlpPolicy": ActorCriticPolicy,
        "CnnPolicy": ActorCriticCnnPolicy,
        "MultiInputPolicy": MultiInputActorCriticPolicy,
    }

    def __init__(
        self,
        policy: Union[str, Type[ActorCriticPolicy]],
        env,
        learning_rate=3e-4,
        n_steps: int = 2048,
        batch_size: int = 64,
        n_epochs: int = 10,
        gamma: float = 0.99,
        gae_lambda: float = 0.95,
        clip_range=0.2,
        clip_range_vf=None,
        normalize_advantage: bool = True,
        ent_coef: float = 0.0,
        vf_coef: float = 0.5,
        max_grad_norm: float = 0.5,
        use_sde: bool = False,
        sde_sample_freq: int = -1,
        rollout_buffer_class=None,
        rollout_buffer_kwargs=None,
        target_kl: Optional[float] = None,
        stats_window_size: int = 100,
        tensorboard_log: Optional[str] = None,
        policy_kwargs: Optional[Dict[str, Any]] = None,
        verbose: int = 0,
        seed: Optional[int] = None,
        device: Union[th.device, str] = "auto",
        _init_setup_model: bool = True,
    ):
        super().__init__(
            policy, env, learning_rate=learning_rate, n_steps=n_steps, gamma=gamma, gae_lambda=gae_lambda,
            ent_coef=ent_coef, vf_coef=vf_coef, max_grad_norm=max_grad_norm, use_sde=use_sde,
            sde_sample_freq=sde_sample_freq, rollout_buffer_class=rollout_buffer_class,
            rollout_buffer_kwargs=rollout_buffer_kwargs, stats_window_size=stats_window_size,
            tensorboard_log=tensorboard_log, policy_kwargs=policy_kwargs, verbose=verbose, device=device,
            seed=seed, _init_setup_model=False,
            supported_action_spaces=(spaces.Box, spaces.Discrete, spaces.MultiDiscrete, spaces.MultiBinary),
        )
        if normalize_advantage:
            assert batch_size > 1, "`batch_size` must be greater than 1."
        self.batch_size = batch_size
        self.n_epochs = n_epochs
        self.clip_range = clip_range
        self.clip_range_vf = clip_range_vf
        self.normalize_advantage = normalize_advantage
        self.target_kl = target_kl
        self._grad_bucket = None
        if _init_setup_model:
            self._setup_model()

    def _setup_model(self) -> None:
        super()._setup_model()
        self.clip_range = get_schedule_fn(self.clip_range)
        if self.clip_range_vf is not None:
            if isinstance(self.clip_range_vf, (float, int)):
                assert self.clip_range_vf > 0
            self.clip_range_vf = get_schedule_fn(self.clip_range_vf)
        self._grad_bucket = pdist.GradBucket(self.policy.parameters()) if pdist.world_size() > 1 else None

    def _post_load_init(self, data):
        super()._post_load_init(data)
        self.batch_size = int(data.get("batch_size", 64) or 64)
        self.n_epochs = int(data.get("n_epochs", 10) or 10)
        cr = data.get("clip_range")
        self.clip_range = cr if isinstance(cr, (int, float)) else 0.2
        self.clip_range_vf = None
        self.normalize_advantage = bool(data.get("normalize_advantage", True))
        self.target_kl = data.get("target_kl")
        self._grad_bucket = None

    def train(self) -> None:
        self.policy.set_training_mode(True)
        self._update_learning_rate(self.policy.optimizer)
        clip_range = self.clip_range(self._current_progress_remaining)
        clip_range_vf = self.clip_range_vf(self._current_progress_remaining) if self.clip_range_vf is not None else None
        dev = self.device
        sums = th.zeros(5, device=dev)  # entropy_loss, pg_loss, value_loss, clip_fraction, approx_kl
        n_mb = 0
        continue_training = True
        loss = th.zeros((), device=dev)
        params = list(self.policy.parameters())
        for epoch in range(self.n_epochs):
            kl_epoch = []
            for rollout_data in self.rollout_buffer.get(self.batch_size):
                actions = rollout_data.actions
                if isinstance(self.action_space, spaces.Discrete):
                    actions = rollout_data.actions.long().flatten()
                values, log_prob, entropy = self.policy.evaluate_actions(rollout_data.observations, actions)
                values = values.flatten()
                advantages = rollout_data.advantages
                if self.normalize_advantage and len(advantages) > 1:
                    advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)
                log_ratio = log_prob - rollout_data.old_log_prob
                ratio = th.exp(log_ratio)
                pl1 = advantages * ratio
                pl2 = advantages * th.clamp(ratio, 1 - clip_range, 1 + clip_range)
                policy_loss = -th.min(pl1, pl2).mean()
                if clip_range_vf is None:
                    values_pred = values
                else:
                    values_pred = rollout_data.old_values + th.clamp(values - rollout_data.old_values, -clip_range_vf, clip_range_vf)
                value_loss = F.mse_loss(rollout_data.returns, values_pred)
                entropy_loss = -th.mean(-log_prob) if entropy is None else -th.mean(entropy)
                loss = policy_loss + self.ent_coef * entropy_loss + self.vf_coef * value_loss
                with th.no_grad():
                    approx_kl = th.mean((th.exp(log_ratio) - 1) - log_ratio)
                    clip_frac = th.mean((th.abs(ratio - 1) > clip_range).float())
                    sums += th.stack([entropy_loss.detach(), policy_loss.detach(), value_loss.detach(), clip_frac, approx_kl])
                n_mb += 1
                if self.target_kl is not None:
                    kl = float(approx_kl)
                    if pdist.world_size() > 1:
                        kl = pdist.allreduce_scalars([kl], op="max")[0]
                    if kl > 1.5 * self.target_kl:
                        continue_training = False
                        if self.verbose >= 1:
                            print(f"Early stopping at step {epoch} due to reaching max kl: {kl:.2f}")
                        break
                self.policy.optimizer.zero_grad(set_to_none=self._grad_bucket is None)
                if self._grad_bucket is not None:
                    self._grad_bucket.zero()
                loss.backward()
                if self._grad_bucket is not None:
                    self._grad_bucket.allreduce()
                th.nn.utils.clip_grad_norm_(params, self.max_grad_norm)
                self.policy.optimizer.step()
            self._n_updates += 1
            if not continue_training:
                break
        stats = (sums / max(n_mb, 1)).tolist()
        ev = explained_variance(self.rollout_buffer.values.flatten().cpu().numpy(), self.rollout_buffer.returns.flatten().cpu().numpy())
        self.logger.record("train/entropy_loss", stats[0])
        self.logger.record("train/policy_gradient_loss", stats[1])
        self.logger.record("train/value_loss", stats[2])
        self.logger.record("train/approx_kl", stats[4])
        self.logger.record("train/clip_fraction", stats[3])
        self.logger.record("train/loss", float(loss.item()))
        self.logger.record("train/explained_variance", ev)
        if hasattr(self.policy, "log_std"):
            self.logger.record("train/std", th.exp(self.policy.log_std).mean().item())
        self.logger.record("train/n_updates", self._n_updates, exclude="tensorboard")
        self.logger.record("train/clip_range", clip_range)
        if clip_range_vf is not None:
            self.logger.record("train/clip_range_vf", clip_range_vf)

    def learn(self, total_timesteps: int, callback=None, log_interval: int = 1, tb_log_name: str = "PPO",
              reset_num_timesteps: bool = True, progress_bar: bool = False):
        return super().learn(total_timesteps=total_timesteps, callback=callback, log_interval=log_interval,
                             tb_log_name=tb_log_name, reset_num_timesteps=reset_num_timesteps, progress_bar=progress_bar)
