"""Device-resident AIRL -- the GAIL device engine with AIRL's reward and discriminator.

Reference: ``src/imitation/algorithms/adversarial/airl.py``. What changes
with respect to :class:`~imitation_amd.engine.gail.DeviceGAIL`:

* generator reward = ``reward_train`` = the shaped reward net itself
  (``airl.py:121-124``): the rollout kernel evaluates ``r(s, a) + gamma (1 - d) Phi(s') -
  Phi(s)`` (``reward_nets.py:701-736``, base MLP and potential MLP, both with their own
  input RunningNorm, evaluation mode) for every env step, in registers;
* ``NormalizedRewardNet`` output normalisation (``reward_nets.py:637-671``): the reference
  normalises each env step's rewards with the running statistics and then merges that
  step's batch moments -- a sequential dependency across the whole rollout. The rollout
  kernel stores the raw shaped reward and the TimeLimit bootstrap separately and one
  wave (``reward_outnorm``) replays the merge in env order: exactly the reference's
  per-step result, with the moments of each step all-reduced in ONE collective per round
  under data parallelism;
* discriminator logit ``r(s,a,s',d) - log pi(a|s)`` (``airl.py:114-119``): the generic
  discriminator update (autograd over the fused MLP kernels) -- the fused GAIL
  discriminator kernels do not apply.

PPO (MlpPolicy [64, 64], minibatch 512 in the tuned Hopper config) runs on the
cooperating-workgroup register-chained kernel.
"""

from __future__ import annotations

from typing import Any, Dict, Tuple

import torch as th
from numpy import prod as np_prod

from imitation_amd.algorithms.adversarial.airl import AIRL
from imitation_amd.engine.gail import DeviceEngineMixin, _mlp_layers, supports_generator
from imitation_amd.parallel import dist as pdist
from imitation_amd.rewards import reward_nets
from imitation_amd.util import networks


def _split(reward_net) -> Tuple[Any, Any]:
    """(output normaliser or None, ShapedRewardNet)."""
    if isinstance(reward_net, reward_nets.NormalizedRewardNet):
        return reward_net.normalize_output_layer, reward_net.base
    return None, reward_net


def supports(venv, gen_algo, reward_net) -> Tuple[bool, str]:
    ok, why = supports_generator(venv, gen_algo)
    if not ok:
        return ok, why
    out_norm, shaped = _split(reward_net)
    if out_norm is not None and type(out_norm) is not networks.RunningNorm:
        return False, "output normaliser is not RunningNorm"
    if not isinstance(shaped, reward_nets.ShapedRewardNet):
        return False, "reward net is not a ShapedRewardNet"
    if not isinstance(shaped.base, reward_nets.BasicRewardNet):
        return False, "shaped base is not a BasicRewardNet"
    if not isinstance(shaped.potential, reward_nets.BasicPotentialMLP):
        return False, "potential is not a BasicPotentialMLP"
    D = int(np_prod(venv.observation_space.shape))
    try:
        pnorm, plins, _, _ = _mlp_layers(shaped.potential._potential_net)
        if plins[0].in_features != D or plins[-1].out_features != 1:
            return False, "potential MLP shape"
        for seq in (shaped.base.mlp, shaped.potential._potential_net):
            norm, lins, _, _ = _mlp_layers(seq)
            if norm is not None and not isinstance(norm, networks.BaseNorm):
                return False, "unsupported input normaliser"
            if len(lins) > 4 or max([lins[0].in_features] + [l.out_features for l in lins]) > 64:
                return False, "reward MLP too wide / deep for the rollout kernel"
    except ValueError as e:
        return False, str(e)
    return True, ""


class OutputNormMixin:
    """``NormalizedRewardNet.predict_processed`` (update_stats=True) replayed on device after
    the rollout kernel: the kernel stores the raw learned reward and the TimeLimit
    bootstrap; ``reward_outnorm`` normalises step by step in env order and Chan-merges each
    step's moments (all-reduced once per round under DP)."""

    def _output_norm(self):
        return _split(self._reward_net)[0]

    def _rollout_extra_bufs(self) -> Dict[str, Any]:
        out_norm = self._output_norm()
        if out_norm is None:
            return {}
        if not hasattr(self, "_rew_raw"):
            self._rew_raw = th.zeros(self.T, self.N, device=self._dev)
            self._onorm_count = th.zeros(1, device=self._dev)
        return {"rew_raw": self._rew_raw}

    def _post_rollout_rewards(self) -> None:
        out_norm = self._output_norm()
        if out_norm is None:
            return
        step_stats = None
        if pdist.norm_sync_active():
            raw = self._rew_raw.double()
            msg = th.stack([th.full((self.T,), float(self.N), dtype=th.float64, device=self._dev),
                            raw.sum(1), raw.square().sum(1)], 1).contiguous()
            pdist.allreduce_sum_(msg)
            cnt = msg[:, 0]
            mean = msg[:, 1] / cnt
            var = (msg[:, 2] / cnt - mean * mean).clamp_min(0.0)
            step_stats = th.stack([cnt, mean, var], 1).float().contiguous()
        self._onorm_count.copy_(out_norm.count.reshape(1))
        self._C.engine_reward_outnorm(dict(T=self.T, N=self.N, rew_raw=self._rew_raw, boot=self._boot,
                                           rewards=self.buf["rewards"], mean=out_norm.running_mean,
                                           var=out_norm.running_var, count=self._onorm_count,
                                           eps=float(out_norm.eps), step_stats=step_stats))
        out_norm.count.copy_(self._onorm_count.to(out_norm.count.dtype).reshape(()))


class DeviceAIRL(OutputNormMixin, DeviceEngineMixin, AIRL):
    """AIRL whose generator rounds run entirely on the GPU (see module docstring)."""

    _host_cls_name = "algorithms.adversarial.airl.AIRL"

    @staticmethod
    def _supports(venv, gen_algo, reward_net):
        return supports(venv, gen_algo, reward_net)

    def _reward_spec(self) -> Dict[str, Any]:
        _, shaped = _split(self._reward_net)
        base = shaped.base
        rnorm, rl, rh, ro = _mlp_layers(base.mlp)
        pnorm, pl, ph, po = _mlp_layers(shaped.potential._potential_net)
        return dict(rew=self._wave_mlp(rl, rh, ro, rnorm), pot=self._wave_mlp(pl, ph, po, pnorm), shaped=1,
                    shaping_gamma=float(shaped.discount_factor), rew_transform=0, use_state=int(base.use_state),
                    use_action=int(base.use_action), use_next_state=int(base.use_next_state),
                    use_done=int(base.use_done))
