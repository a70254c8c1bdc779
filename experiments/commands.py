r"""Generate training commands for a set of named configs and seeds
(reference: experiments/commands.py). One command per (config, seed):

    python experiments/commands.py --name run0 --cfg gail_seals_walker airl_seals_walker --seeds 0 1 2 \
        --output-dir output | xargs -P 8 -I{} bash -c '{}'

``--gpus-per-run N`` emits ``torchrun --standalone --nproc-per-node N`` launches (one rank per
GPU, RCCL data parallel); ``--slurm`` wraps every command in ``sbatch --wrap``.
"""

from __future__ import annotations

import argparse
import hashlib
import pathlib
import sys
import os
from typing import List

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
from imitation_amd.scripts.config import tuned_hps  # noqa: E402

SCRIPT_FOR = {"bc": "train_imitation", "dagger": "train_imitation", "sqil": "train_imitation", "gail": "train_adversarial",
              "airl": "train_adversarial", "pc": "train_preference_comparisons", "rl": "train_rl"}


def algo_of(cfg: str) -> str:
    return cfg.split("_")[0]


def make_commands(name: str, cfgs: List[str], seeds: List[int], output_dir: str, gpus_per_run: int = 0,
                  slurm: bool = False, extra: List[str] = ()) -> List[str]:
    user = os.environ.get("USER", "user")
    out = []
    for cfg in cfgs:
        algo = algo_of(cfg)
        script = SCRIPT_FOR[algo]
        cmd_name = "" if script in ("train_rl", "train_preference_comparisons") else f" {algo}"
        for seed in seeds:
            tag = hashlib.sha1(f"{name}{cfg}{seed}".encode()).hexdigest()[:8]
            run_id = f"{user}-cmd-{name}-{algo}-{seed}-{tag}"
            launcher = (f"torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node {gpus_per_run} -m imitation_amd.scripts.{script}"
                        if gpus_per_run > 1 else f"python -m imitation_amd.scripts.{script}")
            cmd = (f"{launcher}{cmd_name} --name={name} --file_storage={output_dir}/sacred/{run_id} "
                   f"with {cfg} seed={seed} logging.log_root={output_dir}" + "".join(f" {e}" for e in extra))
            if slurm:
                g = max(gpus_per_run, 1)
                cmd = f"sbatch --job-name={run_id} --gres=gpu:{g} --wrap \"{cmd}\""
            out.append(cmd)
    return out


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--name", default="run0")
    p.add_argument("--cfg", nargs="+", default=None, help="named configs (default: every tuned config)")
    p.add_argument("--seeds", nargs="+", type=int, default=[0])
    p.add_argument("--output-dir", default="output")
    p.add_argument("--gpus-per-run", type=int, default=0)
    p.add_argument("--slurm", action="store_true")
    p.add_argument("--extra", nargs="*", default=[])
    a = p.parse_args(argv)
    cfgs = a.cfg or sorted(k for k in tuned_hps() if not k.startswith("fast"))
    print("\n".join(make_commands(a.name, cfgs, a.seeds, a.output_dir, a.gpus_per_run, a.slurm, a.extra)))


if __name__ == "__main__":
    main()
