"""Normalised imitation scores of the device engines (imitation_amd/testing/imitation_quality.py).

Usage: python tools/quality_probe.py [algo:env:steps[:seed[:replay capacity[:n_disc[:demo_batch[:norm_out]]]]] ...]  (default: the four CartPole /
Pendulum GAIL / AIRL runs). One JSON line per run on stdout (and appended to $OUT if set)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from imitation_amd.testing import imitation_quality as iq

    specs = sys.argv[1:] or ["gail:cartpole:200000", "airl:cartpole:200000", "gail:pendulum:500000", "airl:pendulum:500000"]
    for spec in specs:
        parts = spec.split(":")
        if parts[1] in iq.LOCOMOTION:  # algo:env:expert_steps:imit_steps[:seed]
            algo, env, esteps, steps = parts[0], parts[1], int(parts[2]), int(parts[3])
            seed = int(parts[4]) if len(parts) > 4 else 0
            res = iq.run_locomotion(algo, env, expert_timesteps=esteps, total_timesteps=steps, seed=seed,
                                    eval_every=max(steps // 10, 1), verbose=True)
            line = json.dumps(res)
            print(line, flush=True)
            if os.environ.get("OUT"):
                with open(os.environ["OUT"], "a") as f:
                    f.write(line + "\n")
            continue
        algo, env, steps = parts[0], parts[1], int(parts[2])
        seed = int(parts[3]) if len(parts) > 3 else 0
        cap = int(parts[4]) if len(parts) > 4 else 512
        kw = {}
        if len(parts) > 5 and parts[5]:  # Pendulum: n_disc[:demo_batch[:normalize_output]]
            kw["n_disc"] = int(parts[5])
        if len(parts) > 6 and parts[6]:
            kw["demo_batch"] = int(parts[6])
        if len(parts) > 7 and parts[7]:
            kw["normalize_output"] = parts[7] == "1"
        res = iq.run(algo, env, total_timesteps=steps, seed=seed, eval_every=max(steps // 10, 1), verbose=True, cap=cap,
                     trainer_kwargs=kw or None)
        res["trainer_kwargs"] = kw
        line = json.dumps(res)
        print(line, flush=True)
        if os.environ.get("OUT"):
            with open(os.environ["OUT"], "a") as f:
                f.write(line + "\n")


if __name__ == "__main__":
    main()
