r"""Generate training commands for a set of named configs and seeds
(reference: experiments/commands.py). One command per (config, seed):

    python experiments/commands.py --name run0 --cfg gail_seals_walker airl_seals_walker --seeds 0 1 2 \
        --output-dir output | xargs -P 8 -I{} bash -c '{}'

``--gpus-per-run N`` emits ``torchrun --standalone --nproc-per-node N`` launches (one rank per
GPU, RCCL data parallel); ``--slurm`` wraps every command in ``sbatch --wrap``.

Config-file mode, the reference's interface: ``--cfg_pattern GLOB`` of named-config JSON files
(``--export_tuned_hps DIR`` writes every tuned config as ``DIR/<name>.json``); the algorithm is
read from the file name, one command per (file, seed)::

    python experiments/commands.py --name=run0 --cfg_pattern='hps/*ai*_seals_walker*.json' --output_dir=output
    python -m imitation_amd.scripts.train_adversarial airl --capture=sys --name=run0 \
        --file_storage=output/sacred/$USER-cmd-run0-airl-0-<adler32 of the file name> \
        with hps/airl_seals_walker.json seed=0 logging.log_root=output

``--remote`` prints each command as a containerised cluster job instead (``--remote_cfg_dir``:
where the config files live inside the container; ``--container``: the image).
"""

from __future__ import annotations

import argparse
import glob
import hashlib
import json
import pathlib
import sys
import os
import zlib
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


REMOTE_TEMPLATE = ('ctl job run --name {name} --command "{command}" --container {container} '
                   '--login --force-pull --never-restart --gpu {gpus} --shared-host-dir-mount /data')


def algo_of_file(cfg_file: str) -> str:
    """The algorithm a config file is for: exactly one algorithm name among its ``_``-separated
    words (``airl_seals_walker.json`` -> airl)."""
    words = set(os.path.splitext(cfg_file)[0].split("_"))
    found = {k for k in SCRIPT_FOR if k in words}
    if not found:
        raise ValueError("Unable to find algo_name in cfg_file: " + cfg_file)
    if len(found) > 1:
        raise ValueError("algo_name is ambiguous in cfg_file: " + cfg_file)
    return found.pop()


def make_file_commands(name: str, cfg_pattern: str, seeds: List[int], output_dir: str, remote: bool = False,
                       remote_cfg_dir: str = "/data/imitation_amd/hps", container: str = "imitation-amd:rocm",
                       gpus: int = 1) -> List[str]:
    user = "$USER"
    out = []
    for rel in sorted(glob.glob(cfg_pattern)):
        cfg_file = os.path.basename(rel)
        algo = algo_of_file(cfg_file)
        script = SCRIPT_FOR[algo]
        cmd_name = "" if script in ("train_rl", "train_preference_comparisons") else f" {algo}"
        cfg_path = os.path.join(remote_cfg_dir, cfg_file) if remote else rel
        cfg_id = format(zlib.adler32(cfg_file.encode()), "x")
        for seed in seeds:
            run_id = f"{user}-cmd-{name}-{algo}-{seed}-{cfg_id}"
            cmd = (f"python -m imitation_amd.scripts.{script}{cmd_name} --capture=sys --name={name} "
                   f"--file_storage={output_dir}/sacred/{run_id} with {cfg_path} seed={seed} logging.log_root={output_dir}")
            if remote:
                cmd = REMOTE_TEMPLATE.format(name=run_id, command=cmd, container=container, gpus=gpus)
            out.append(cmd)
    return out


def export_tuned_hps(out_dir: str) -> List[str]:
    """Every tuned config as ``<out_dir>/<name>.json`` (named-config files for ``with``)."""
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for k, v in tuned_hps().items():
        path = os.path.join(out_dir, f"{k}.json")
        with open(path, "w") as f:
            json.dump(v, f, indent=2, sort_keys=True)
        paths.append(path)
    return paths


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--name", default="run0")
    p.add_argument("--cfg", nargs="+", default=None, help="named configs (default: every tuned config)")
    p.add_argument("--seeds", nargs="+", type=int, default=[0])
    p.add_argument("--output-dir", "--output_dir", dest="output_dir", default="output")
    p.add_argument("--cfg_pattern", default=None, help="glob of named-config JSON files (config-file mode)")
    p.add_argument("--remote", action="store_true", help="config-file mode: print cluster job commands")
    p.add_argument("--remote_cfg_dir", default="/data/imitation_amd/hps")
    p.add_argument("--container", default="imitation-amd:rocm")
    p.add_argument("--export_tuned_hps", default=None, metavar="DIR", help="write every tuned config to DIR/<name>.json")
    p.add_argument("--gpus-per-run", type=int, default=0)
    p.add_argument("--slurm", action="store_true")
    p.add_argument("--extra", nargs="*", default=[])
    a = p.parse_args(argv)
    if a.export_tuned_hps:
        print("\n".join(export_tuned_hps(a.export_tuned_hps)))
        return
    if a.cfg_pattern:
        print("\n".join(make_file_commands(a.name, a.cfg_pattern, a.seeds, a.output_dir, a.remote, a.remote_cfg_dir,
                                            a.container, max(1, a.gpus_per_run))))
        return
    cfgs = a.cfg or sorted(k for k in tuned_hps() if not k.startswith("fast"))
    print("\n".join(make_commands(a.name, cfgs, a.seeds, a.output_dir, a.gpus_per_run, a.slurm, a.extra)))


if __name__ == "__main__":
    main()
