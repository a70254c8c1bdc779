"""Config for ``analyze`` (reference: scripts/config/analyze.py)."""

import os.path as osp

from imitation_amd.scripts.config_engine import Experiment

analysis_ex = Experiment("analyze")


@analysis_ex.config
def config():
    source_dir_str = "output/sacred/train_adversarial"  # searched recursively for run dirs
    skip_failed_runs = True
    run_name = None
    env_name = None
    csv_output_path = None
    tex_output_path = None
    print_table = True
    split_str = ","
    table_verbosity = 1  # 0..3
    source_dirs = None


@analysis_ex.config
def convert_source_dirs(source_dir_str, split_str, source_dirs):
    if source_dirs is None:
        source_dirs = source_dir_str.split(split_str)
    source_dirs = [osp.expanduser(p) for p in source_dirs]
