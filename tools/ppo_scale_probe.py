"""Time the replicated data-parallel PPO update of a headline config on ONE GPU.

At world size W every rank runs the register-chained kernel over the all-gathered rows
(W x rows) with minibatch W x batch (cooperating workgroups): emulated here with W x the
envs and W x the minibatch. Prints ms per PPO update for W = 1, 2, 4, 8.

CONFIG (env var): ``gail`` (default; HalfCheetah FeedForward32Policy, 4096 rows, mb 64, 5
epochs), ``airl`` (Hopper MlpPolicy [64, 64] ReLU, 8192 rows, mb 512, 20 epochs -- the tuned
AIRL config), ``drlhp`` (Walker2d MlpPolicy [64, 64] ReLU, 8192 rows, mb 128, 20 epochs --
the seals_walker preference-comparisons config).
"""
import sys
import time

import numpy as np
import torch as th

import os  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from imitation_amd.data import rollout
    from imitation_amd.engine.gail import DeviceGAIL
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicRewardNet, NormalizedRewardNet
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    from imitation_amd.rl.policies import ActorCriticPolicy

    cfg = os.environ.get("CONFIG", "gail")
    env_id, n_steps, mb, epochs = {"gail": ("seals/HalfCheetah-v1", 512, 64, 5), "airl": ("seals/Hopper-v1", 1024, 512, 20),
                                   "drlhp": ("seals/Walker2d-v1", 1024, 128, 20)}[cfg]
    for W in [int(w) for w in os.environ.get("WS", "1,2,4,8").split(",")]:
        rng = np.random.default_rng(0)
        venv = make_vec_env(env_id, rng=rng, n_envs=8 * W)
        demo_env = make_vec_env(env_id, rng=np.random.default_rng(7), n_envs=4)
        demos = rollout.flatten_trajectories(rollout.generate_trajectories(None, demo_env, rollout.make_min_timesteps(1024), rng=rng))
        if cfg == "gail":
            gen = PPO(FeedForward32Policy, venv, n_steps=n_steps, batch_size=mb * W, n_epochs=epochs, device="cuda",
                      policy_kwargs=dict(features_extractor_class=NormalizeFeaturesExtractor))
        else:
            gen = PPO(ActorCriticPolicy, venv, n_steps=n_steps, batch_size=mb * W, n_epochs=epochs, device="cuda",
                      policy_kwargs=dict(net_arch=dict(pi=[64, 64], vf=[64, 64]), activation_fn=th.nn.ReLU,
                                         features_extractor_class=NormalizeFeaturesExtractor))
        rn = NormalizedRewardNet(BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm), RunningNorm)
        tr = DeviceGAIL(demonstrations=demos, demo_batch_size=1024, venv=venv, gen_algo=gen, reward_net=rn,
                        n_disc_updates_per_round=1, custom_logger=logger.configure("/tmp/ia_probe", format_strs=[]))
        tr._ppo_static["rc_cw"] = int(os.environ.get("RC_CW", "0"))
        tr._ppo_static["rc_gmax"] = int(os.environ.get("RC_GMAX", "0"))  # cap on cooperating workgroups (0: plan default)
        path = tr._C.engine_ppo_path(tr._ppo_static)
        tr._rollout()
        for _ in range(2):
            tr._ppo_update()
        th.cuda.synchronize()
        # one-level vs two-level partial exchange: bitwise-equal update from one state, then timing
        pol = gen.policy
        norm = tr.pol_norm
        def snap():
            t = [q.detach().clone() for q in pol.parameters()] + [tr.exp_avg.clone(), tr.exp_avg_sq.clone(), tr.adam_step.clone()]
            if norm is not None:
                t += [norm.running_mean.clone(), norm.running_var.clone(), norm.count.clone(), tr.norm_count.clone()]
            return t, tr._perm_round
        def restore(st):
            t, pr = st
            dst = list(pol.parameters()) + [tr.exp_avg, tr.exp_avg_sq, tr.adam_step]
            if norm is not None:
                dst += [norm.running_mean, norm.running_var, norm.count, tr.norm_count]
            with th.no_grad():
                for d, v in zip(dst, t):
                    d.copy_(v)
            tr._perm_round = pr
        s0 = snap()
        res = {}
        for mode in ("0", "1"):
            os.environ["IMITATION_AMD_PPO_XCHG2"] = mode
            restore(s0)
            tr._ppo_update()
            th.cuda.synchronize()
            res[mode] = [q.detach().clone() for q in pol.parameters()]
        same = all(th.equal(a, b) for a, b in zip(res["0"], res["1"]))
        for mode in ("0", "1"):
            os.environ["IMITATION_AMD_PPO_XCHG2"] = mode
            n = 5
            t0 = time.perf_counter()
            for _ in range(n):
                tr._ppo_update()
            th.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            print(f"{cfg} W={W} path={path} rows={tr.T * tr.N} batch={mb * W} xchg2={mode}: ppo update {1e3 * dt:.3f} ms"
                  f" (two-level bitwise equal: {same})", flush=True)
        os.environ.pop("IMITATION_AMD_PPO_XCHG2")
        for mode in ("0", "1"):
            os.environ["IMITATION_AMD_PPO_XCHG2"] = mode
            prof = th.zeros(20, dtype=th.int64, device="cuda")
            tr._ppo_static["prof"] = prof
            tr._ppo_update()
            th.cuda.synchronize()
            p = prof.cpu().numpy().astype(np.float64) / tr._last_ppo_info[1]
            print(f"    xchg2={mode} cycles/minibatch (workgroup 0): chunk {p[0]:.0f} exchange+|g|^2 {p[1]:.0f} clip+adam {p[2]:.0f}"
                  f" | wave0 B1 wait {p[11]:.0f} dW {p[12]:.0f} | exchange: publish {p[13]:.0f} arrival {p[14]:.0f} loads {p[15]:.0f}"
                  f" | actor rows {p[3]:.0f} fwd {p[4]:.0f} loss {p[5]:.0f} bwd {p[6]:.0f} | critic rows {p[7]:.0f} fwd {p[8]:.0f}"
                  f" loss {p[9]:.0f} bwd {p[10]:.0f} | net-split |g|^2 hand-off {p[16]:.0f} adam {p[17]:.0f} B3 {p[18]:.0f}", flush=True)
            tr._ppo_static.pop("prof")
        os.environ.pop("IMITATION_AMD_PPO_XCHG2")


if __name__ == "__main__":
    main()
