"""Train GAIL or AIRL (reference: src/imitation/scripts/train_adversarial.py).

    python -m imitation_amd.scripts.train_adversarial gail with seals_half_cheetah
    python -m imitation_amd.scripts.train_adversarial airl with seals_cartpole fast

``engine=auto`` (default) runs GAIL through the device engine
(``imitation_amd.engine.gail.DeviceGAIL``: rollout, learned reward, PPO update and
discriminator all on the GPU) whenever the configuration is one it supports, and
otherwise through the reference-structured host loop. ``engine=host`` forces the
host loop. Distributed: launch with ``torchrun --nproc-per-node N`` -- every rank
trains on its own envs and data shard; gradients are all-reduced over RCCL.
"""

from __future__ import annotations

import functools
import logging
import pathlib
from typing import Any, Mapping, Optional, Type

from imitation_amd.algorithms.adversarial import airl as airl_algo
from imitation_amd.algorithms.adversarial import common
from imitation_amd.algorithms.adversarial import gail as gail_algo
from imitation_amd.data import rollout
from imitation_amd.parallel import dist as pdist
from imitation_amd.utils import watchdog
from imitation_amd.policies import serialize
from imitation_amd.rewards import serialize as reward_serialize
from imitation_amd.scripts.config.train_adversarial import train_adversarial_ex
from imitation_amd.scripts.config_engine import FileStorageObserver, get_by_dotted_path, print_config
from imitation_amd.scripts.ingredients import demonstrations, environment
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients import policy_evaluation, reward, rl

logger = logging.getLogger("imitation_amd.scripts.train_adversarial")


def save(trainer: common.AdversarialTrainer, save_path: pathlib.Path) -> None:
    """Discriminator (train/test reward nets, pickle-free) and generator (model.zip)."""
    if not pdist.is_main():
        return
    save_path.mkdir(parents=True, exist_ok=True)
    reward_serialize.save_reward_net(trainer.reward_train, save_path / "reward_train.pt")
    reward_serialize.save_reward_net(trainer.reward_test, save_path / "reward_test.pt")
    serialize.save_stable_model(save_path / "gen_policy", trainer.gen_algo)


def _add_hook(ingredient) -> None:
    """Merge ``<ingredient>.algorithm_specific[<command>]`` into the ingredient's config."""

    @ingredient.config_hook
    def hook(config, command_name, logger):
        path = "" if ingredient.path == "train_adversarial" else ingredient.config_path
        cfg = get_by_dotted_path(config, path) if path else config
        return dict((cfg or {}).get("algorithm_specific", {}).get(command_name, {}))

    @ingredient.config
    def dummy_config():
        algorithm_specific = {}


for _ing in [train_adversarial_ex, *train_adversarial_ex._all_ingredients()]:
    _add_hook(_ing)


def _device_engine(algo_cls):
    """(device trainer class, eligibility check) of a host algorithm class, or None."""
    if algo_cls is gail_algo.GAIL:
        from imitation_amd.engine import gail as eng

        return eng.DeviceGAIL, eng.supports
    if algo_cls is airl_algo.AIRL:
        from imitation_amd.engine import airl as eng

        return eng.DeviceAIRL, eng.supports
    return None


def _make_trainer(algo_cls, engine: str, **kwargs) -> common.AdversarialTrainer:
    """The device engine (``DeviceGAIL`` / ``DeviceAIRL``: fused rollout + PPO + discriminator
    kernels) when ``engine`` is ``auto``/``device`` and the configuration is eligible, else the
    host-loop trainer. ``engine=device`` fails loudly when it is not eligible. The choice is
    recorded as ``trainer.engine_kind``."""
    dev = _device_engine(algo_cls) if engine in ("auto", "device") else None
    why = "no device engine for this algorithm" if dev is None else ""
    if dev is not None:
        cls, supports = dev
        ok, why = supports(kwargs["venv"], kwargs["gen_algo"], kwargs["reward_net"])
        if ok:
            try:
                trainer = cls(**kwargs)
                trainer.engine_kind = "device"
                logger.info(f"Using the device engine ({cls.__name__})")
                return trainer
            except ValueError as e:  # e.g. nets too large for the persistent PPO kernel's LDS
                why = str(e)
    if engine == "device":
        raise ValueError(f"engine=device requested but unsupported: {why}")
    if engine != "host":
        logger.info(f"Device engine not applicable ({why}); using the host loop")
    trainer = algo_cls(**kwargs)
    trainer.engine_kind = "host"
    return trainer


def train_rounds(trainer, total_timesteps: int, callback, full_checkpoint_interval: int = 0,
                 resume_from: Optional[str] = None, full_checkpoint_dir: Optional[str] = None,
                 full_checkpoint_keep: int = 3) -> int:
    """``trainer.train(total_timesteps, callback)`` with full-state checkpoints for exact resume
    (the reference snapshots only the reward net and policy,
    ``src/imitation/scripts/train_adversarial.py:25-35,157``).

    Every ``full_checkpoint_interval`` rounds the whole trainer state (parameters, optimiser
    moments, normalisers, replay ring, demo sampler, env state, RNG streams, device-engine state)
    goes to ``full_checkpoint_dir/ckpt-<rounds>`` (:class:`~imitation_amd.utils.checkpoint.CheckpointManager`:
    atomic, newest ``full_checkpoint_keep`` kept, one directory per DP rank). ``resume_from``
    restores the newest checkpoint every rank has there and trains only the remaining rounds.
    The rounds run as ``train()`` calls of at most ``full_checkpoint_interval`` rounds, which is
    bitwise the single call (the engines drain their pipeline at the end of each call); the
    callback sees the global round index. Returns the number of rounds restored."""
    from imitation_amd.utils.checkpoint import CheckpointManager

    per_round = trainer.gen_train_timesteps
    n_rounds = total_timesteps // per_round
    if full_checkpoint_interval <= 0 and not resume_from:
        trainer.train(total_timesteps, callback)
        return 0
    assert n_rounds >= 1, "No updates (need at least gen_train_timesteps transitions)"
    start = 0
    if resume_from:
        start = CheckpointManager(resume_from, keep=full_checkpoint_keep).restore_latest(trainer)
        logger.info(f"Resumed from {resume_from} after {start} rounds")
    mgr = None
    if full_checkpoint_interval > 0:
        mgr = CheckpointManager(full_checkpoint_dir or resume_from, keep=full_checkpoint_keep)
    seg = full_checkpoint_interval if full_checkpoint_interval > 0 else n_rounds
    r = start
    while r < n_rounds:
        k = min(seg - r % seg, n_rounds - r)
        trainer.train(k * per_round, None if callback is None else (lambda i, _base=r: callback(_base + i)))
        r += k
        if mgr is not None and (r % seg == 0 or r == n_rounds):
            mgr.save(trainer, r, meta=dict(total_timesteps=total_timesteps, rounds=n_rounds))
    return start


@train_adversarial_ex.capture
def train_adversarial(_run, show_config: bool, algo_cls: Type[common.AdversarialTrainer],
                      algorithm_kwargs: Mapping[str, Any], total_timesteps: int, checkpoint_interval: int,
                      agent_path: Optional[str], engine: str = "auto", full_checkpoint_interval: int = 0,
                      full_checkpoint_keep: int = 3, resume_from: Optional[str] = None) -> Mapping[str, Mapping[str, float]]:
    """Checkpoints go to ``{log_dir}/checkpoints/{round|final}/{reward_train,reward_test}.pt`` and ``gen_policy/``;
    full-state checkpoints (``full_checkpoint_interval`` > 0) to ``{log_dir}/full_checkpoints`` and
    ``resume_from=<dir>`` continues from the newest one (:func:`train_rounds`)."""
    total_timesteps = int(total_timesteps)
    checkpoint_interval = int(checkpoint_interval)
    pdist.init()
    if show_config:
        print_config(_run)
    custom_logger, log_dir = logging_ingredient.setup_logging()
    expert_trajs = demonstrations.get_expert_trajectories()
    with environment.make_venv() as venv:
        reward_net = reward.make_reward_net(venv)
        relabel_reward_fn = functools.partial(reward_net.predict_processed, update_stats=False)
        if agent_path is None:
            gen_algo = rl.make_rl_algo(venv, relabel_reward_fn=relabel_reward_fn)
        else:
            gen_algo = rl.load_rl_algo_from_path(agent_path=agent_path, venv=venv, relabel_reward_fn=relabel_reward_fn)
        logger.info(f"Using '{algo_cls}' algorithm")
        algorithm_kwargs = {k: v for k, v in dict(algorithm_kwargs).items() if k not in ("shared", "airl", "gail")}
        trainer = _make_trainer(algo_cls, engine, venv=venv, demonstrations=expert_trajs, gen_algo=gen_algo,
                                log_dir=log_dir, reward_net=reward_net, custom_logger=custom_logger, **algorithm_kwargs)

        with watchdog.cli_watchdog("train_adversarial") as wd:
            def callback(round_num: int, /) -> None:
                wd.beat()  # a round that never ends (stuck collective / kernel) aborts the run
                if checkpoint_interval > 0 and round_num % checkpoint_interval == 0:
                    save(trainer, log_dir / "checkpoints" / f"{round_num:05d}")

            resumed_rounds = train_rounds(trainer, total_timesteps, callback, int(full_checkpoint_interval),
                                          resume_from, str(log_dir / "full_checkpoints"), int(full_checkpoint_keep))
            wd.beat()
            imit_stats = policy_evaluation.eval_trainer(trainer, trainer.venv_train)
    if checkpoint_interval >= 0:
        save(trainer, log_dir / "checkpoints" / "final")
    out = {"imit_stats": imit_stats, "expert_stats": rollout.rollout_stats(expert_trajs), "engine": trainer.engine_kind}
    if resume_from:
        out["resumed_rounds"] = resumed_rounds
    return out


@train_adversarial_ex.command
def gail():
    """Generative Adversarial Imitation Learning."""
    return train_adversarial(algo_cls=gail_algo.GAIL)


@train_adversarial_ex.command
def airl():
    """Adversarial Inverse Reinforcement Learning."""
    return train_adversarial(algo_cls=airl_algo.AIRL)


def main_console(argv=None):
    observer = FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "train_adversarial")
    train_adversarial_ex.observers.append(observer)
    return train_adversarial_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
