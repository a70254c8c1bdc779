"""ms per GAIL round of the production CLI path vs bench.py.

Runs ``train_adversarial gail with gail_seals_half_cheetah`` (the reference's tuned config;
default log formats tensorboard + stdout, a checkpoint callback every ``--ckpt`` rounds) with
synthetic demonstrations, and times the rounds from the per-round callback stamps (rounds after
the first 3). ``--sync-logs``: IMITATION_AMD_LOG_ASYNC=0 (formats written on the training thread).
Prints one JSON line."""
import argparse
import contextlib
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=40)
    p.add_argument("--ckpt", type=int, default=10)
    p.add_argument("--sync-logs", action="store_true")
    p.add_argument("--no-pipeline", action="store_true", help="pipeline_callbacks=False (device idle in callbacks)")
    args = p.parse_args()
    if args.sync_logs:
        os.environ["IMITATION_AMD_LOG_ASYNC"] = "0"
    import torch as th

    from imitation_amd.data import serialize
    from imitation_amd.engine import gail as eng
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    tmp = tempfile.mkdtemp(prefix="ia_cli_speed_")
    import numpy as np

    from imitation_amd.data import rollout
    from imitation_amd.util.util import make_vec_env

    env = make_vec_env("seals/HalfCheetah-v1", rng=np.random.default_rng(12345), n_envs=16)
    demos = rollout.generate_trajectories(None, env, rollout.make_min_timesteps(16384), rng=np.random.default_rng(1))
    serialize.save(os.path.join(tmp, "demos"), demos)
    from imitation_amd.algorithms.adversarial import common

    stamps = []
    if args.no_pipeline:
        eng.DeviceEngineMixin.pipeline_callbacks = False

    def stamped(orig):
        def train(self, total, callback=None):
            def cb(r):
                stamps.append(time.perf_counter())
                if callback:
                    callback(r)
            return orig(self, total, cb)
        return train

    eng.DeviceEngineMixin.train = stamped(eng.DeviceEngineMixin.train)
    common.AdversarialTrainer.train = stamped(common.AdversarialTrainer.train)
    with open(os.path.join(tmp, "stdout.txt"), "w") as out, contextlib.redirect_stdout(out):
        run = train_adversarial_ex.run(
            command_name="gail", named_configs=["gail_seals_half_cheetah"],
            config_updates=dict(total_timesteps=4096 * args.rounds, checkpoint_interval=args.ckpt,
                                demonstrations=dict(source="local", path=os.path.join(tmp, "demos")),
                                logging=dict(log_dir=os.path.join(tmp, "log")),
                                policy_evaluation=dict(n_episodes_eval=1)))
    if th.cuda.is_available():
        th.cuda.synchronize()
    k0 = min(3, len(stamps) - 2)
    ms = 1e3 * (stamps[-1] - stamps[k0]) / (len(stamps) - 1 - k0)
    print(json.dumps({"cli_ms_per_round": round(ms, 3), "rounds": len(stamps), "engine": run.result["engine"],
                      "log_async": not args.sync_logs, "pipelined_callbacks": not args.no_pipeline,
                      "checkpoint_interval": args.ckpt, "formats": "tensorboard,stdout"}), flush=True)


if __name__ == "__main__":
    main()
