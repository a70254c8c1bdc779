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
* discriminator logit ``r(s,a,s',d) - log pi(a|s)`` (``airl.py:114-119``): a fused update
  (``csrc/kernels/airl_disc.hip``, :class:`AirlDiscPlan`) -- per minibatch one gather, one
  norm launch (the policy, base and potential RunningNorm merges in the reference's order:
  potential on s' then on s) and one fwd/loss/bwd launch (policy log-prob, base reward,
  both potential passes, BCE + statistics, backward of the base and potential MLPs), then
  one fixed-order Adam launch -- instead of ~60 autograd launches. Configurations outside
  the kernel's limits keep the generic (graphed autograd) update.

PPO (MlpPolicy [64, 64], minibatch 512 in the tuned Hopper config) runs on the
cooperating-workgroup register-chained kernel.
"""

from __future__ import annotations

import os
from typing import Any, Dict, List, Tuple

import torch as th

from imitation_amd.utils.streams import shared_stream
from imitation_amd.utils import profiling
from numpy import prod as np_prod

from imitation_amd.algorithms.adversarial import common
from imitation_amd.algorithms.adversarial.airl import AIRL
from imitation_amd.engine.gail import DeviceEngineMixin, _FlatParams, _mlp_layers, _policy_nets, supports_generator
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

    @profiling.traced("rollout/reward_outnorm")
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
        # an int32 module count is read / written by the kernel itself (no copies around it)
        direct = out_norm.count.dtype == th.int32
        if not direct:
            self._onorm_count.copy_(out_norm.count.reshape(1))
        self._C.engine_reward_outnorm(dict(T=self.T, N=self.N, rew_raw=self._rew_raw, boot=self._boot,
                                           rewards=self.buf["rewards"], mean=out_norm.running_mean,
                                           var=out_norm.running_var, count=self._onorm_count,
                                           count_i=out_norm.count if direct else None,
                                           eps=float(out_norm.eps), step_stats=step_stats))
        if not direct:
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

    # ------------------------------------------------------------------ fused discriminator (airl_disc.hip)
    def _fused_disc_check(self) -> Tuple[bool, str]:
        import os

        if os.environ.get("IMITATION_AMD_AIRL_FUSED", "1") == "0":
            return False, "disabled (IMITATION_AMD_AIRL_FUSED=0)"
        if type(self).logits_expert_is_high is not AIRL.logits_expert_is_high:
            return False, "custom discriminator logits"
        opt = self._disc_opt
        if type(opt) is not th.optim.Adam or len(opt.param_groups) != 1:
            return False, "discriminator optimizer is not a single-group torch.optim.Adam"
        g = opt.param_groups[0]
        if any(g.get(k) for k in ("amsgrad", "maximize", "capturable", "differentiable", "decoupled_weight_decay")):
            return False, "Adam variant not fused"
        if self._init_tensorboard:
            return False, "tensorboard summaries need per-step logits"
        if not isinstance(self._endless_expert_iterator, common._DeviceDemoSampler):
            return False, "demonstrations are not a flat device transitions set"
        _, shaped = _split(self._reward_net)
        try:
            bnorm, blins, _, bout = _mlp_layers(shaped.base.mlp)
            pnorm, plins, _, pout = _mlp_layers(shaped.potential._potential_net)
            qnorm, qlins, _, _ = _policy_nets(self.gen_algo.policy)
        except ValueError as e:
            return False, str(e)
        for norm in (bnorm, pnorm, qnorm):
            if norm is not None and type(norm) is not networks.RunningNorm:
                return False, "a normaliser is not RunningNorm"
        if bout != 0 or pout != 0 or blins[-1].out_features != 1 or plins[-1].out_features != 1:
            return False, "reward / potential MLP shape"
        if len(blins) > 4 or len(plins) > 4 or len(qlins) > 4:
            return False, "MLP deeper than 4 layers"
        widths = [l.out_features for l in blins + plins + qlins] + [blins[0].in_features, plins[0].in_features,
                                                                    qlins[0].in_features]
        if max(widths) > 64 or (self.A if not self.discrete else self.A) > 16:
            return False, "MLP wider than 64"
        mlp_params = {id(p) for l in blins + plins for p in (l.weight, l.bias)}
        if {id(p) for p in self._reward_net.parameters()} != mlp_params:
            return False, "reward net has parameters outside its MLPs"
        base = shaped.base
        din = (base.use_state + base.use_next_state) * self.D + base.use_action * self.A + base.use_done
        if din + 2 * self.D > 128:
            return False, "too many input columns"
        return True, ""

    def _setup_fused_disc(self) -> None:
        ok, why = self._fused_disc_check()
        self._fused_disc = ok
        self._fused_disc_why = why
        # log pi needs the post-PPO policy: the updates follow PPO on the main stream, but the round
        # is pipelined like GAIL's (_overlapped_round: PPO stats copied async, the updates and the
        # next rollout enqueued before the host reads anything); IMITATION_AMD_DISC_OVERLAP=0: serial
        self._overlap_disc = os.environ.get("IMITATION_AMD_DISC_OVERLAP", "1") != "0"
        self._disc_on_main = True
        self._side_stream = shared_stream(self._dev, "engine_side") if self._overlap_disc else None  # staging copies
        self._pol_defer_buf = None
        self._disc_split = False
        if not ok:
            return
        dev = self._dev
        _, shaped = _split(self._reward_net)
        base = shaped.base
        bnorm, blins, bh, _ = _mlp_layers(base.mlp)
        pnorm, plins, ph, _ = _mlp_layers(shaped.potential._potential_net)
        qnorm, qlins, _, qh = _policy_nets(self.gen_algo.policy)
        self._bnorm, self._pnorm = bnorm, pnorm
        plist = []
        for l in blins + plins:
            plist += [l.weight, l.bias]
        self._rflat = _FlatParams(plist)
        n = self._rflat.n
        self._r_m = th.zeros(n, device=dev)
        self._r_v = th.zeros(n, device=dev)
        self._adopt_disc_opt_state()
        ed = self._endless_expert_iterator.data
        ed["obs"] = ed["obs"].float().contiguous()
        ed["next_obs"] = ed["next_obs"].float().contiguous()
        ed["acts"] = (ed["acts"].long() if self.discrete else ed["acts"].float()).reshape(ed["acts"].shape[0], -1)
        ed["acts"] = ed["acts"].reshape(-1).contiguous() if self.discrete else ed["acts"].contiguous()
        ed["dones"] = ed["dones"].bool().contiguous()
        gd = self._gen_dev._arrays
        B, mb = self.demo_batch_size, self.demo_minibatch_size
        gblk, fblk = self._C.airl_plan_sizes(mb)
        din = blins[0].in_features
        D = self.D
        ncol = din + 2 * D
        z = lambda *sh, dt=th.float32: th.zeros(*sh, device=dev, dtype=dt)  # noqa: E731
        rows = 2 * mb
        self._disc_ws = dict(Xb=z(rows * din), S=z(rows * D), S2=z(rows * D), Act=z(rows * (1 if self.discrete else self.A)),
                             Done=z(rows), partials=z(gblk * 2 * ncol), sums=z(2 * ncol, dt=th.float64), nrm=z(4 * 256),
                             slab=z((B // mb) * fblk * n), stats_slab=z((B // mb) * fblk * 8), grads=z(n))
        self._disc_stats = z(max(1, self.n_disc_updates_per_round), 8)
        g = self._disc_opt.param_groups[0]
        pol = self.gen_algo.policy

        def net(lins, act):
            return dict(W=[l.weight for l in lins], b=[l.bias for l in lins], hidden_act=int(act))

        def norm_args(prefix, nm):
            if nm is None:
                return {f"{prefix}_mean": None, f"{prefix}_var": None, f"{prefix}_count": None, f"eps_{prefix}": 1e-5}
            return {f"{prefix}_mean": nm.running_mean, f"{prefix}_var": nm.running_var, f"{prefix}_count": nm.count,
                    f"eps_{prefix}": float(nm.eps)}

        d = dict(batch=B, minibatch=mb, obs_dim=D, act_dim=self.A, act_discrete=int(self.discrete),
                 use_state=int(base.use_state), use_action=int(base.use_action), use_next_state=int(base.use_next_state),
                 use_done=int(base.use_done), e_obs=ed["obs"], e_next_obs=ed["next_obs"], e_acts=ed["acts"],
                 e_dones=ed["dones"], g_obs=gd["obs"], g_next_obs=gd["next_obs"], g_acts=gd["acts"], g_dones=gd["dones"],
                 pol=net(qlins, qh), base=net(blins, bh), pot=net(plins, ph),
                 log_std=pol.log_std if self.has_log_std else None, gamma=float(shaped.discount_factor),
                 params=self._rflat.flat, exp_avg=self._r_m, exp_avg_sq=self._r_v, beta1=float(g["betas"][0]),
                 beta2=float(g["betas"][1]), eps=float(g["eps"]), weight_decay=float(g.get("weight_decay", 0.0)),
                 **norm_args("b", bnorm), **norm_args("p", pnorm), **norm_args("q", qnorm), **self._disc_ws)
        self._disc_plan = self._C.AirlDiscPlan(d)
        self._disc_stats_host = th.zeros(max(1, self.n_disc_updates_per_round), 8, pin_memory=True)
        # split rounds (single rank): the updates' gathers + norm merges are staged on the main
        # stream right after PPO, then the next rollout's step chain runs concurrently with the
        # fwd/bwd + Adam applies on the side stream (see _overlapped_round)
        # (data parallel too: the staging's normaliser all-reduces run on the main stream, the
        # applies' gradient all-reduces on the side stream, where nothing else uses the
        # communicator while they run -- the next step chain has no collectives)
        self._disc_split = (self._overlap_disc and os.environ.get("IMITATION_AMD_AIRL_SPLIT", "1") != "0")
        if self._disc_split:
            self._disc_plan.reserve(max(1, self.n_disc_updates_per_round))

    @profiling.traced("disc/stage")
    def _stage_disc_updates(self, n: int, defer_q: bool = False) -> List[Tuple[float, float]]:
        """The gathers and RunningNorm merges (policy, base, potential) of the round's ``n``
        updates, in update order (``AirlDiscPlan.stage``): everything of an update that the
        norms see, none of it dependent on the discriminator weights. Returns each update's
        Adam (step_size, sqrt(1 - beta2^t)).

        ``defer_q``: leave the policy-norm merges to ``_merge_deferred_q`` (one launch after
        PPO), so the staging can run on the side stream during the PPO update (under DP its
        normaliser all-reduces then run there too); ``self._q_deferred`` says whether there is
        anything to merge."""
        if self._gen_dev.size() == 0:
            raise RuntimeError("No generator samples for training. Call `train_gen()` first.")
        # (grows only here: the previous round's applies were waited for on the host)
        self._disc_plan.reserve(max(1, n))
        opt = self._disc_opt
        self._adopt_disc_opt_state()
        g = opt.param_groups[0]
        beta1, beta2 = g["betas"]
        t0 = float(opt.state[self._rflat.params[0]]["step"])
        B = self.demo_batch_size
        merge_b = self._bnorm is not None and self._bnorm.training
        merge_p = self._pnorm is not None and self._pnorm.training
        merge_q = self.pol_norm is not None and self.pol_norm.training
        scal = []
        world = pdist.world_size()
        defer_q = defer_q and merge_q
        self._q_deferred = defer_q
        synced = world > 1 and pdist.norm_sync_active()
        self._q_defer_rows = 2 * self.demo_minibatch_size * (world if synced else 1)
        cur = th.cuda.current_stream(self._dev)
        for i in range(n):
            e_idx = self._endless_expert_iterator.next_indices()
            # the epoch permutation may come from another stream's pool: keep its block alive
            # for this stream's reads
            e_idx.record_stream(cur)
            g_idx = th.randint(0, self._gen_dev.size(), (B,), device=self._dev)
            if world == 1 or not pdist.norm_sync_active():
                self._disc_plan.stage(i, e_idx, g_idx, merge_b, merge_p, merge_q, defer_q)
            else:  # the DP update's order: gather, moments, all-reduce, merges -- per minibatch
                mb = self.demo_minibatch_size
                for k in range(B // mb):
                    self._disc_plan.stage_part(i, k, e_idx, g_idx, 1, 0, merge_b, merge_p, merge_q)
                    pdist.allreduce_sum_(self._disc_ws["sums"])
                    self._disc_plan.stage_part(i, k, e_idx, g_idx, 2, 2 * mb * world, merge_b, merge_p, merge_q, defer_q)
            t = t0 + i + 1.0
            scal.append((float(g["lr"]) / (1.0 - beta1**t), (1.0 - beta2**t) ** 0.5))
        return scal

    def _merge_deferred_q(self, n: int) -> None:
        """The policy-norm merges ``_stage_disc_updates(n, defer_q=True)`` left (update order)."""
        if getattr(self, "_q_deferred", False):
            self._disc_plan.q_merge(n, self._q_defer_rows)
            self._q_deferred = False

    @profiling.traced("disc/apply")
    def _apply_disc_updates(self, scal: List[Tuple[float, float]], steps: List[int]) -> None:
        """The fwd/bwd passes and Adam steps of the staged updates (``AirlDiscPlan.apply``)."""
        opt = self._disc_opt
        world = pdist.world_size()
        for i, (step_size, bc2_sqrt) in enumerate(scal):
            if world == 1:
                self._disc_plan.apply(i, step_size, bc2_sqrt, self._disc_stats[i])
            else:  # mean gradient over ranks between the reduction and Adam (one-shot, in stream order)
                self._disc_plan.apply_grads(i, self._disc_stats[i])
                pdist.allreduce_grads_flat(self._disc_ws["grads"])
                self._disc_plan.adam(0, 1, step_size, bc2_sqrt, None)
            for p in self._rflat.params:
                opt.state[p]["step"] += 1
            self._disc_step += 1
            steps.append(self._disc_step)

    @profiling.traced("disc/update")
    def _fused_disc_update(self, slot: int, defer_pol: bool = False, e_idx: th.Tensor = None, g_idx: th.Tensor = None,
                           apply: bool = True) -> None:
        """One discriminator optimizer step (== AdversarialTrainer.train_disc with AIRL's logits)
        on the fused kernels, with no host sync. ``e_idx`` / ``g_idx``: explicit expert / replay
        rows (tests); ``apply=False`` stops after the gradient reduction (``_disc_ws["grads"]``)."""
        if self._gen_dev.size() == 0:
            raise RuntimeError("No generator samples for training. Call `train_gen()` first.")
        opt = self._disc_opt
        self._adopt_disc_opt_state()
        g = opt.param_groups[0]
        t = float(opt.state[self._rflat.params[0]]["step"]) + 1.0
        beta1, beta2 = g["betas"]
        step_size = float(g["lr"]) / (1.0 - beta1**t)
        bc2_sqrt = (1.0 - beta2**t) ** 0.5
        B, mb = self.demo_batch_size, self.demo_minibatch_size
        if e_idx is None:
            e_idx = self._endless_expert_iterator.next_indices()
        if g_idx is None:
            g_idx = th.randint(0, self._gen_dev.size(), (B,), device=self._dev)
        merge_b = self._bnorm is not None and self._bnorm.training
        merge_p = self._pnorm is not None and self._pnorm.training
        merge_q = self.pol_norm is not None and self.pol_norm.training
        plan = self._disc_plan
        stats_out = self._disc_stats[slot]
        if pdist.world_size() == 1 and apply:
            plan.update(e_idx, g_idx, step_size, bc2_sqrt, merge_b, merge_p, merge_q, stats_out)
        else:
            world = pdist.world_size()
            for k in range(B // mb):
                plan.gather(k, e_idx, g_idx)
                if pdist.norm_sync_active():
                    plan.norm(1, 0, merge_b, merge_p, merge_q)
                    pdist.allreduce_sum_(self._disc_ws["sums"])
                    plan.norm(2, 2 * mb * world, merge_b, merge_p, merge_q)
                else:
                    plan.norm(0, 0, merge_b, merge_p, merge_q)
                plan.fwd_bwd(k)
            plan.adam(1, 0, 0.0, 1.0, stats_out)
            if world > 1:
                pdist.allreduce_grads_flat(self._disc_ws["grads"])
            if not apply:
                return
            plan.adam(0, 1, step_size, bc2_sqrt, None)
        for p in self._rflat.params:
            opt.state[p]["step"] += 1
        self._disc_step += 1
