"""Config for ``parallel`` (reference: scripts/config/parallel.py)."""

from imitation_amd.scripts import tune
from imitation_amd.scripts.config_engine import Experiment
from imitation_amd.util.util import make_unique_timestamp

parallel_ex = Experiment("parallel")


@parallel_ex.config
def config():
    sacred_ex_name = "train_rl"  # experiment to parallelize
    init_kwargs = {}  # accepted for config compatibility (no Ray cluster to initialise)
    run_name = f"DEFAULT_{make_unique_timestamp()}"
    resources_per_trial = {}  # {"gpu": k}: trials are pinned to k GPUs each (HIP_VISIBLE_DEVICES)
    base_named_configs = []
    base_config_updates = {}
    search_space = {"named_configs": [], "config_updates": {}}
    num_samples = 1
    repeat = 1  # run each sampled configuration with this many seeds
    experiment_checkpoint_path = ""
    # max_concurrent_trials, local_dir, seed, search_alg ("random" / "tpe"; default: tpe when
    # repeat > 1, as the reference's Repeater(OptunaSearch)), n_startup_trials (TPE)
    tune_run_kwargs = {}
    local_dir = "output/parallel"


@parallel_ex.named_config
def generate_test_data():
    sacred_ex_name = "train_rl"
    run_name = "TEST"
    repeat = 1
    search_space = {"config_updates": {"rl": {"rl_kwargs": {"learning_rate": tune.choice([3e-4 * x for x in (1 / 3, 1 / 2)])}}}}
    base_named_configs = ["cartpole", "environment.fast", "policy_evaluation.fast", "rl.fast", "fast"]
    base_config_updates = {"rollout_save_final": True}
    num_samples = 2


@parallel_ex.named_config
def example_cartpole_rl():
    sacred_ex_name = "train_rl"
    run_name = "example-cartpole"
    n_seeds = 2
    search_space = {"config_updates": {"rl": {"rl_kwargs": {"learning_rate": tune.grid_search(list(3e-4 * (2 ** i)
                                                                                               for i in range(-2, 3)))}},
                                        "seed": tune.grid_search(list(range(n_seeds)))}}
    base_named_configs = ["cartpole"]


@parallel_ex.named_config
def debug_log_root():
    search_space = {"config_updates": {"logging": {"log_root": "/tmp/output"}}}
