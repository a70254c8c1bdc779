"""Full-trainer checkpoints for exact resume (SURVEY §5 "checkpoint / resume").

The reference only snapshots *artifacts* -- the reward net (``th.save(module)``,
a pickle) and the generator policy -- every ``checkpoint_interval`` rounds
(``src/imitation/scripts/train_adversarial.py:30-49``); optimizer moments,
normaliser statistics, RNG state, replay buffers and round counters are lost, so a
crashed 1e7-step run restarts from scratch. Here a checkpoint is a directory:

``state.pt``       every tensor/counter needed to continue bit-for-bit (params,
                   optimizer moments, running-norm buffers, replay ring, demo sampler
                   permutation, native env state, device-engine Adam state, RNG
                   streams); plain tensors/dicts only -> loads with
                   ``torch.load(weights_only=True)``
``meta.json``      format tag, step counters, user metadata (human-readable)
``*.npz``          bulky side data (preference dataset) in numpy's no-pickle format

:class:`CheckpointManager` writes atomically (temp dir + rename) and keeps the
newest ``keep`` checkpoints, so a restart always finds a complete one.
"""

from __future__ import annotations

import json
import os
import shutil
import tempfile
from typing import Any, Dict, List, Optional

import numpy as np
import torch as th

from imitation_amd.utils import determinism

STATE_FILE = "state.pt"
META_FILE = "meta.json"


# ----------------------------------------------------------------------------- helpers
def _to_cpu(x):
    if isinstance(x, th.Tensor):
        return x.detach().cpu().clone()
    if isinstance(x, np.ndarray):
        if x.dtype == object:
            raise TypeError("object arrays cannot be checkpointed without pickle")
        return th.as_tensor(np.ascontiguousarray(x))
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    if isinstance(x, np.generic):
        return x.item()
    return x


def _optimizers(algo) -> Dict[str, th.optim.Optimizer]:
    out: Dict[str, th.optim.Optimizer] = {}
    pol = getattr(algo, "policy", None)
    if pol is not None:
        for name, m in pol.named_modules():
            opt = getattr(m, "optimizer", None)
            if isinstance(opt, th.optim.Optimizer):
                out[f"policy.{name}" if name else "policy"] = opt
    for k, v in vars(algo).items():
        if isinstance(v, th.optim.Optimizer):
            out[k] = v
    return out


_ALGO_COUNTERS = ("num_timesteps", "_n_updates", "_episode_num", "_total_timesteps", "_num_timesteps_at_start")


def _unwrap_native(venv):
    from imitation_amd.envs.vec_env import NativeVecEnv

    e = venv
    while e is not None:
        if isinstance(e, NativeVecEnv):
            return e
        e = getattr(e, "venv", None)
    return None


_PENDING_SEEDS = "__pending_seeds__"


def env_state(venv) -> Optional[Dict[str, th.Tensor]]:
    """Native env state, plus the seeds ``venv.seed()`` queued for the next ``reset()`` (-1 =
    none): a fresh env built for the restore has its own queued seeds, which would otherwise
    override the restored RNG at the first reset."""
    nat = _unwrap_native(venv)
    if nat is None:
        return None
    st = {k: th.as_tensor(v) for k, v in nat.get_state().items()}
    st[_PENDING_SEEDS] = th.tensor([-1 if s is None else int(s) for s in nat._seeds], dtype=th.int64)
    return st


def load_env_state(venv, st: Optional[Dict[str, th.Tensor]]) -> bool:
    nat = _unwrap_native(venv)
    if nat is None or st is None:
        return False
    st = dict(st)
    pending = st.pop(_PENDING_SEEDS, None)
    nat.set_state({k: v.numpy() for k, v in st.items()})
    nat._seeds = [None] * nat.num_envs if pending is None else [None if int(s) < 0 else int(s) for s in pending]
    return True


def rl_algo_state(algo, include_replay: bool = True) -> Dict[str, Any]:
    """Policy weights, every optimizer, loose parameters (SAC ``log_ent_coef``), counters,
    the last observation (so ``learn(reset_num_timesteps=False)`` continues the episode)
    and, for off-policy algorithms, the replay buffer."""
    st: Dict[str, Any] = {
        "policy": _to_cpu(algo.policy.state_dict()),
        "optimizers": {k: _to_cpu(o.state_dict()) for k, o in _optimizers(algo).items()},
        "tensors": {k: _to_cpu(v) for k, v in vars(algo).items() if isinstance(v, th.Tensor)},
        "counters": {k: int(getattr(algo, k)) for k in _ALGO_COUNTERS if hasattr(algo, k)},
    }
    last = getattr(algo, "_last_obs", None)
    if isinstance(last, np.ndarray) and last.dtype != object:
        st["last_obs"] = _to_cpu(last)
        st["last_episode_starts"] = _to_cpu(np.asarray(getattr(algo, "_last_episode_starts")))
    st["wrappers"] = _wrapper_state(getattr(algo, "env", None))
    rb = getattr(algo, "replay_buffer", None)
    if include_replay and rb is not None:
        st["replay_buffer"] = {k: _to_cpu(v) for k, v in vars(rb).items()
                               if isinstance(v, (th.Tensor, np.ndarray)) and getattr(v, "dtype", None) != object}
        st["replay_buffer_pos"] = [int(rb.pos), bool(rb.full)]
    return st


def load_rl_algo_state(algo, st: Dict[str, Any], env_restored: bool = True) -> None:
    algo.policy.load_state_dict(st["policy"])
    opts = _optimizers(algo)
    for k, s in st["optimizers"].items():
        if k in opts:
            opts[k].load_state_dict(s)
    for k, v in st["tensors"].items():
        cur = getattr(algo, k, None)
        if isinstance(cur, th.Tensor):
            with th.no_grad():
                cur.copy_(v.to(cur.device))
    for k, v in st["counters"].items():
        setattr(algo, k, v)
    if "last_obs" in st and env_restored:
        algo._last_obs = st["last_obs"].numpy()
        algo._last_episode_starts = st["last_episode_starts"].numpy()
        _load_wrapper_state(getattr(algo, "env", None), st.get("wrappers", []), algo._last_obs)
    elif not env_restored:
        algo._last_obs = None  # env could not be restored: next learn() resets it
    rb = getattr(algo, "replay_buffer", None)
    if rb is not None and "replay_buffer" in st:
        for k, v in st["replay_buffer"].items():
            cur = getattr(rb, k, None)
            if isinstance(cur, th.Tensor):
                cur.copy_(v.to(cur.device))
            elif isinstance(cur, np.ndarray):
                cur[...] = v.numpy()
        rb.pos, rb.full = st["replay_buffer_pos"]


def _chain(venv):
    e = venv
    while e is not None:
        yield e
        e = getattr(e, "venv", None)


def _wrapper_state(venv):
    """Per-wrapper state that lives across rounds: the BufferingWrapper's running episode
    lengths (its trajectory accumulators hold only the current obs at a round boundary)."""
    from imitation_amd.data.wrappers import BufferingWrapper

    out = []
    for e in _chain(venv):
        if isinstance(e, BufferingWrapper) and e._timesteps is not None:
            out.append({"timesteps": th.as_tensor(np.asarray(e._timesteps, dtype=np.int64))})
    return out


def _load_wrapper_state(venv, states, last_obs) -> None:
    """Re-seat wrappers that cache the current observation on the restored one."""
    from imitation_amd.data import rollout
    from imitation_amd.data.wrappers import BufferingWrapper
    from imitation_amd.rewards.reward_wrapper import RewardVecEnvWrapper

    states = list(states)
    for e in _chain(venv):
        if isinstance(e, RewardVecEnvWrapper):
            e._old_obs = np.array(last_obs, copy=True)
        elif isinstance(e, BufferingWrapper) and states:
            ws = states.pop(0)
            e._init_reset = True
            e._traj_accum = rollout.TrajectoryAccumulator()
            for i, ob in enumerate(np.asarray(last_obs)):
                e._traj_accum.add_step({"obs": ob}, key=i)
            e._timesteps = ws["timesteps"].numpy().astype(int)
            e._trajectories, e._ep_lens = [], []
            e.n_transitions = 0
            e._saved_acts = None


def _py(x):
    if isinstance(x, dict):
        return {str(k): _py(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_py(v) for v in x]
    if isinstance(x, np.ndarray):
        return x.tolist()
    if isinstance(x, np.generic):
        return x.item()
    return x


def _host_buffer_state(buf) -> Dict[str, Any]:
    arrays = {}
    for k, v in buf._arrays.items():
        if isinstance(v, np.ndarray) and v.dtype == object:
            # info dicts: JSON (numpy scalars/arrays become python numbers/lists)
            arrays[k] = {"__json_objects__": json.dumps([_py(e) for e in v.tolist()])}
        else:
            arrays[k] = _to_cpu(v)
    return {"arrays": arrays, "idx": int(buf._idx), "n": int(buf._n_data)}


def _load_host_buffer_state(buf, st) -> None:
    for k, v in st["arrays"].items():
        a = buf._arrays[k]
        if isinstance(v, dict) and "__json_objects__" in v:
            for i, e in enumerate(json.loads(v["__json_objects__"])):
                a[i] = e
        elif isinstance(a, th.Tensor):
            a.copy_(v.to(a.device))
        else:
            a[...] = v.numpy()
    buf._idx, buf._n_data = st["idx"], st["n"]


# ----------------------------------------------------------------------------- trainers
def adversarial_state(trainer) -> Dict[str, Any]:
    """State of a GAIL / AIRL trainer (host loop or :class:`~imitation_amd.engine.gail.DeviceGAIL`)."""
    from imitation_amd.algorithms.adversarial import common

    if hasattr(trainer, "sync_env_to_host"):  # device engine: the host env mirrors the device env state
        trainer.sync_env_to_host()
    st: Dict[str, Any] = {
        "format": "imitation_amd.adversarial.v1",
        "global_step": int(trainer._global_step),
        "disc_step": int(trainer._disc_step),
        "reward_net": _to_cpu(trainer._reward_net.state_dict()),
        "disc_opt": _to_cpu(trainer._disc_opt.state_dict()),
        "env": env_state(trainer.venv),
        "gen": rl_algo_state(trainer.gen_algo),
        "replay": _host_buffer_state(trainer._gen_replay_buffer._buffer),
        "rng": determinism.capture_rng_state(),
    }
    sampler = trainer._endless_expert_iterator
    if isinstance(sampler, common._DeviceDemoSampler):
        st["demo_sampler"] = {"perm": None if sampler._perm is None else _to_cpu(sampler._perm), "pos": int(sampler._pos),
                              "gen": sampler._gen.get_state(), "base": int(sampler._base), "epochs": int(sampler._epochs)}
    if hasattr(trainer, "engine_state"):
        st["engine"] = trainer.engine_state()
    return st


def load_adversarial_state(trainer, st: Dict[str, Any]) -> None:
    from imitation_amd.algorithms.adversarial import common

    if st.get("format") != "imitation_amd.adversarial.v1":
        raise ValueError(f"not an adversarial trainer checkpoint: {st.get('format')}")
    trainer._reward_net.load_state_dict(st["reward_net"])
    trainer._disc_opt.load_state_dict(st["disc_opt"])
    trainer._global_step = st["global_step"]
    trainer._disc_step = st["disc_step"]
    env_ok = load_env_state(trainer.venv, st.get("env"))
    load_rl_algo_state(trainer.gen_algo, st["gen"], env_restored=env_ok)
    _load_host_buffer_state(trainer._gen_replay_buffer._buffer, st["replay"])
    sampler = trainer._endless_expert_iterator
    if "demo_sampler" in st and isinstance(sampler, common._DeviceDemoSampler):
        ds = st["demo_sampler"]
        sampler._perm = None if ds["perm"] is None else ds["perm"].to(sampler.device)
        sampler._pos = ds["pos"]
        sampler._gen.set_state(ds["gen"])
        sampler._base = int(ds.get("base", sampler._base))
        sampler._epochs = int(ds.get("epochs", 0))
    if "engine" in st and hasattr(trainer, "load_engine_state"):
        trainer.load_engine_state(st["engine"])
    determinism.restore_rng_state(st["rng"])


_PC_RNG_PATHS = ("rng", "fragmenter.rng", "fragmenter.base_fragmenter.rng", "preference_gatherer.rng",
                 "reward_trainer.rng", "trajectory_generator.rng", "trajectory_generator.exploration_wrapper.rng")


def _pc_generators(pc) -> List[Any]:
    """``(path, np.random.Generator)`` of every component of a preference-comparisons trainer
    that draws from one (the CLI shares ONE generator among them: it is saved once per path and
    restored to the same state each time)."""
    out = []
    for path in _PC_RNG_PATHS:
        obj = pc
        for part in path.split("."):
            obj = getattr(obj, part, None)
        if isinstance(obj, np.random.Generator):
            out.append((path, obj))
    for i, t in enumerate(getattr(pc.reward_trainer, "member_trainers", ()) or ()):
        if isinstance(getattr(t, "rng", None), np.random.Generator):
            out.append((f"reward_trainer.member_trainers.{i}.rng", t.rng))
    return out


def _infos_state(infos):
    return None if infos is None else {"__json_objects__": json.dumps([_py(e) for e in list(infos)])}


def _infos_load(st):
    return None if st is None else np.array(json.loads(st["__json_objects__"]) or [], dtype=object)


def traj_state(t) -> Dict[str, Any]:
    """A :class:`~imitation_amd.data.types.TrajectoryWithRew` as plain tensors (+ JSON infos)."""
    from imitation_amd.data import types

    if isinstance(t.obs, types.DictObs):
        raise TypeError("dict observations cannot be checkpointed here")
    return {"obs": _to_cpu(np.asarray(t.obs)), "acts": _to_cpu(np.asarray(t.acts)), "rews": _to_cpu(np.asarray(t.rews)),
            "terminal": bool(t.terminal), "infos": _infos_state(t.infos)}


def traj_load(st: Dict[str, Any]):
    from imitation_amd.data import types

    return types.TrajectoryWithRew(obs=st["obs"].numpy(), acts=st["acts"].numpy(), rews=st["rews"].numpy(),
                                   terminal=st["terminal"], infos=_infos_load(st["infos"]))


def _step_state(step: Dict[str, Any]) -> Dict[str, Any]:
    return {k: (_infos_state([v])) if k == "infos" else _to_cpu(np.asarray(v)) for k, v in step.items()}


def _step_load(st: Dict[str, Any]) -> Dict[str, Any]:
    return {k: (_infos_load(v)[0] if k == "infos" else v.numpy()) for k, v in st.items()}


def buffering_state(bw) -> Dict[str, Any]:
    """Everything a :class:`~imitation_amd.data.wrappers.BufferingWrapper` carries across
    ``learn()`` calls: per-env partial trajectories (step dicts), finished trajectories not yet
    popped, episode counters."""
    acc = bw._traj_accum
    return {"partial": None if acc is None else {int(k): [_step_state(d) for d in v]
                                                  for k, v in acc.partial_trajectories.items()},
            "finished": [traj_state(t) for t in bw._trajectories], "ep_lens": [int(x) for x in bw._ep_lens],
            "n_transitions": int(bw.n_transitions), "init_reset": bool(bw._init_reset),
            "timesteps": None if bw._timesteps is None else th.as_tensor(np.asarray(bw._timesteps, dtype=np.int64))}


def load_buffering_state(bw, st: Dict[str, Any]) -> None:
    from imitation_amd.data import rollout

    if st["partial"] is None:
        bw._traj_accum = None
    else:
        bw._traj_accum = rollout.TrajectoryAccumulator()
        for k, steps in st["partial"].items():
            for d in steps:
                bw._traj_accum.add_step(_step_load(d), key=int(k))
    bw._trajectories = [traj_load(t) for t in st["finished"]]
    bw._ep_lens = list(st["ep_lens"])
    bw.n_transitions = st["n_transitions"]
    bw._init_reset = st["init_reset"]
    bw._timesteps = None if st["timesteps"] is None else st["timesteps"].numpy().astype(int)
    bw._saved_acts = None


def preference_state(pc, side_dir: str) -> Dict[str, Any]:
    """State of :class:`~imitation_amd.algorithms.preference_comparisons.PreferenceComparisons`
    after a whole iteration; the comparison dataset goes to ``side_dir/dataset.npz``. The agent's
    trajectories in flight (finished ones not yet sampled, per-env partial ones) are part of it:
    the next iteration samples them. ``completed`` = iterations done (resume skips them)."""
    from imitation_amd.algorithms import preference_comparisons as pcm

    rt = pc.reward_trainer
    trainers = rt.member_trainers if isinstance(rt, pcm.EnsembleTrainer) else [rt]
    st: Dict[str, Any] = {
        "format": "imitation_amd.preference_comparisons.v1",
        "iteration": int(pc._iteration),
        "completed": int(pc._completed_iterations),
        "model": _to_cpu(pc.model.state_dict()),
        "reward_optims": [_to_cpu(t.optim.state_dict()) for t in trainers],
        "rng": determinism.capture_rng_state(),
        "pc_rng": None if pc.rng is None else determinism.generator_state(pc.rng),
        "component_rngs": {path: determinism.generator_state(g) for path, g in _pc_generators(pc)},
        "dataset_len": len(pc.dataset),
    }
    gen = pc.trajectory_generator
    if isinstance(gen, pcm.AgentTrainer):
        if hasattr(gen, "sync_env_to_host"):  # device agent: the host env mirrors the device env state
            gen.sync_env_to_host()
        st["agent"] = rl_algo_state(gen.algorithm)
        st["env"] = env_state(gen.venv)
        st["episode_rewards"] = [float(x) for x in gen.reward_venv_wrapper.episode_rewards]
        ew = getattr(gen, "exploration_wrapper", None)
        if ew is not None:
            st["explore_random"] = bool(ew.current_policy == ew._random_policy)
        if hasattr(gen, "engine_state"):  # device agent: Adam / env state on the GPU, host-side episode cutter
            st["agent_engine"] = gen.engine_state()
            st["agent_buffer"] = gen.buffer_state()
        else:
            st["agent_buffer"] = buffering_state(gen.buffering_wrapper)
    if len(pc.dataset):
        pc.dataset.save(os.path.join(side_dir, "dataset.npz"))
    return st


def load_preference_state(pc, st: Dict[str, Any], side_dir: str) -> None:
    from imitation_amd.algorithms import preference_comparisons as pcm

    if st.get("format") != "imitation_amd.preference_comparisons.v1":
        raise ValueError(f"not a preference-comparisons checkpoint: {st.get('format')}")
    pc.model.load_state_dict(st["model"])
    rt = pc.reward_trainer
    trainers = rt.member_trainers if isinstance(rt, pcm.EnsembleTrainer) else [rt]
    for t, s in zip(trainers, st["reward_optims"]):
        t.optim.load_state_dict(s)
    pc._iteration = st["iteration"]
    pc._completed_iterations = st.get("completed", st["iteration"])
    pc._resume_at = pc._completed_iterations  # the next train() continues the interrupted schedule
    gen = pc.trajectory_generator
    if "agent" in st and isinstance(gen, pcm.AgentTrainer):
        env_ok = load_env_state(gen.venv, st.get("env"))
        load_rl_algo_state(gen.algorithm, st["agent"], env_restored=env_ok)
        if "episode_rewards" in st:
            er = gen.reward_venv_wrapper.episode_rewards
            er.clear()
            er.extend(st["episode_rewards"])
        ew = getattr(gen, "exploration_wrapper", None)
        if ew is not None and "explore_random" in st:
            ew.current_policy = ew._random_policy if st["explore_random"] else ew.wrapped_policy
        if "agent_engine" in st and hasattr(gen, "load_engine_state"):
            gen.load_engine_state(st["agent_engine"])
            gen.load_buffer_state(st["agent_buffer"])
        elif "agent_buffer" in st:
            load_buffering_state(gen.buffering_wrapper, st["agent_buffer"])
    if st["dataset_len"]:
        ds = pcm.PreferenceDataset.load(os.path.join(side_dir, "dataset.npz"))
        ds.max_size = pc.dataset.max_size
        pc.dataset = ds
    if pc.rng is not None and st["pc_rng"] is not None:
        determinism.set_generator_state(pc.rng, st["pc_rng"])
    saved = st.get("component_rngs", {})
    for path, g in _pc_generators(pc):
        if path in saved:
            determinism.set_generator_state(g, saved[path])
    determinism.restore_rng_state(st["rng"])


AGGREGATE_FILE = "dagger_aggregate.pt"


def dagger_state(tr, side_dir: str) -> Dict[str, Any]:
    """State of a DAgger trainer between rounds (reference ``dagger.py:521-552`` saves the
    trainer object; this is the pickle-free full state): the learner and its optimiser moments,
    the round, the beta schedule's input, every RNG stream, the env state, BC's log counters.

    Demonstrations: the host path re-reads the round files of its scratch dir (as the
    reference's ``reconstruct_trainer`` does); the device path's aggregate -- its rows in append
    order, which the BC loader's permutations index -- goes to ``side_dir/dagger_aggregate.pt``,
    with the device collector's env state and sampling counter."""
    bct = tr.bc_trainer
    st: Dict[str, Any] = {
        "format": "imitation_amd.dagger_full.v1",
        "round_num": int(tr.round_num),
        "rng": determinism.generator_state(tr.rng),
        "bc_rng": determinism.generator_state(bct.rng) if isinstance(getattr(bct, "rng", None), np.random.Generator) else None,
        "policy": _to_cpu(bct.policy.state_dict()),
        "optimizer": _to_cpu(bct.optimizer.state_dict()),
        "bc_log": [int(bct._bc_logger._tensorboard_step), int(bct._bc_logger._current_epoch)],
        "env": env_state(tr.venv),
        "global_rng": determinism.capture_rng_state(),
    }
    col = getattr(tr, "_device_collector", None)
    if col is not None:
        tr.flush_demos()
        agg = tr._device_agg
        th.save({"obs": agg.obs[: agg.n].cpu(), "acts": agg.acts[: agg.n].cpu()} if agg.n else {},
                os.path.join(side_dir, AGGREGATE_FILE))
        st["device"] = {"n": int(agg.n), "counts": {str(k): int(v) for k, v in tr._device_counts.items()},
                        "collector": col.engine_state(), "loaded_through": int(tr._store.loaded_through)}
    return st


def load_dagger_state(tr, st: Dict[str, Any], side_dir: str) -> None:
    if st.get("format") != "imitation_amd.dagger_full.v1":
        raise ValueError(f"not a DAgger checkpoint: {st.get('format')}")
    bct = tr.bc_trainer
    bct.policy.load_state_dict(st["policy"])
    bct.optimizer.load_state_dict(st["optimizer"])
    tr.round_num = st["round_num"]
    determinism.set_generator_state(tr.rng, st["rng"])
    if st["bc_rng"] is not None and isinstance(getattr(bct, "rng", None), np.random.Generator):
        determinism.set_generator_state(bct.rng, st["bc_rng"])
    bct._bc_logger._tensorboard_step, bct._bc_logger._current_epoch = st["bc_log"]
    load_env_state(tr.venv, st.get("env"))
    dev = st.get("device")
    col = getattr(tr, "_device_collector", None)
    if dev is not None:
        if col is None:
            raise ValueError("checkpoint of a device-collector DAgger run; this trainer collects on the host")
        from imitation_amd.engine import dagger as dagger_engine

        agg = dagger_engine.DeviceDemoAggregate(tr._device_agg.device)
        if dev["n"]:
            rows = th.load(os.path.join(side_dir, AGGREGATE_FILE), map_location="cpu", weights_only=True)
            agg.append(rows["obs"].to(agg.device), rows["acts"].to(agg.device), gather=False)
        tr._device_agg = agg
        tr._device_counts = {int(k): v for k, v in dev["counts"].items()}
        tr._store.loaded_through = dev["loaded_through"]
        col.load_engine_state(dev["collector"])
    else:  # host path: the next update re-reads every round's demo files from the scratch dir
        tr._store.trajectories, tr._store._flat, tr._store.loaded_through = [], None, -1
    # demo files of the round that was in progress (and any later one) when the run stopped are
    # stale: that round is collected again
    r = tr.round_num
    while tr._store.round_dir(r).is_dir():
        shutil.rmtree(tr._store.round_dir(r))
        r += 1
    determinism.restore_rng_state(st["global_rng"])


def trainer_state(trainer, side_dir: str) -> Dict[str, Any]:
    from imitation_amd.algorithms import preference_comparisons as pcm
    from imitation_amd.algorithms.adversarial import common

    if isinstance(trainer, common.AdversarialTrainer):
        return adversarial_state(trainer)
    if isinstance(trainer, pcm.PreferenceComparisons):
        return preference_state(trainer, side_dir)
    from imitation_amd.rl.base import BaseAlgorithm

    if isinstance(trainer, BaseAlgorithm):
        return {"format": "imitation_amd.rl.v1", "algo": rl_algo_state(trainer), "env": env_state(trainer.env),
                "rng": determinism.capture_rng_state()}
    from imitation_amd.algorithms import dagger

    if isinstance(trainer, dagger.DAggerTrainer):
        return dagger_state(trainer, side_dir)
    raise TypeError(f"no checkpoint support for {type(trainer).__name__}")


def load_trainer_state(trainer, st: Dict[str, Any], side_dir: str) -> None:
    fmt = st.get("format")
    if fmt == "imitation_amd.adversarial.v1":
        load_adversarial_state(trainer, st)
    elif fmt == "imitation_amd.preference_comparisons.v1":
        load_preference_state(trainer, st, side_dir)
    elif fmt == "imitation_amd.dagger_full.v1":
        load_dagger_state(trainer, st, side_dir)
    elif fmt == "imitation_amd.rl.v1":
        env_ok = load_env_state(trainer.env, st.get("env"))
        load_rl_algo_state(trainer, st["algo"], env_restored=env_ok)
        determinism.restore_rng_state(st["rng"])
    else:
        raise ValueError(f"unknown checkpoint format {fmt!r}")


# ----------------------------------------------------------------------------- files
def save_checkpoint(trainer, path: str, meta: Optional[Dict[str, Any]] = None) -> str:
    """Write ``trainer``'s full state into directory ``path`` (atomically replaced)."""
    parent = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(parent, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix=".ckpt-", dir=parent)
    try:
        st = trainer_state(trainer, tmp)
        th.save(st, os.path.join(tmp, STATE_FILE))
        m = {"format": st["format"]}
        for k in ("global_step", "disc_step", "iteration", "round_num"):
            if k in st:
                m[k] = st[k]
        m.update(meta or {})
        with open(os.path.join(tmp, META_FILE), "w") as f:
            json.dump(m, f, indent=2, sort_keys=True)
        old = None
        if os.path.exists(path):  # move the previous copy aside: `path` is never missing
            old = tempfile.mkdtemp(prefix=".ckpt-old-", dir=parent)
            os.rmdir(old)
            os.replace(path, old)
        os.replace(tmp, path)
        if old is not None:
            shutil.rmtree(old, ignore_errors=True)
    except BaseException:
        shutil.rmtree(tmp, ignore_errors=True)
        raise
    return path


def load_checkpoint(trainer, path: str) -> Dict[str, Any]:
    """Restore ``trainer`` from a directory written by :func:`save_checkpoint`; returns meta."""
    st = th.load(os.path.join(path, STATE_FILE), map_location="cpu", weights_only=True)
    load_trainer_state(trainer, st, path)
    with open(os.path.join(path, META_FILE)) as f:
        return json.load(f)


class CheckpointManager:
    """Numbered checkpoints ``<root>/ckpt-<step>`` keeping the newest ``keep``.

    >>> mgr = CheckpointManager("out/ckpts", keep=3)
    >>> start = mgr.restore_latest(trainer)  # 0 when starting fresh
    >>> for r in range(start, rounds):
    ...     trainer.train(trainer.gen_train_timesteps)
    ...     if (r + 1) % 10 == 0:
    ...         mgr.save(trainer, r + 1)
    """

    def __init__(self, root: str, keep: int = 3, rank: Optional[int] = None):
        from imitation_amd.parallel import dist as pdist

        self.root = root
        self.keep = keep
        self.rank = pdist.rank() if rank is None else rank
        os.makedirs(root, exist_ok=True)

    def _rank_dir(self, step: int) -> str:
        suffix = "" if self.rank == 0 else f"-rank{self.rank}"
        return os.path.join(self.root, f"ckpt-{step:010d}{suffix}")

    def list(self) -> List[int]:
        suffix = "" if self.rank == 0 else f"-rank{self.rank}"
        steps = []
        for n in os.listdir(self.root):
            if not n.startswith("ckpt-"):
                continue
            body = n[5:]
            if suffix:
                if not body.endswith(suffix):
                    continue
                body = body[: -len(suffix)]
            elif "-rank" in body:
                continue
            if body.isdigit() and os.path.exists(os.path.join(self.root, n, META_FILE)):
                steps.append(int(body))
        return sorted(steps)

    def save(self, trainer, step: int, meta: Optional[Dict[str, Any]] = None) -> str:
        """Every rank saves its own shard of env / replay / RNG state (DP ranks differ there);
        replicated parameters are identical across ranks."""
        p = save_checkpoint(trainer, self._rank_dir(step), dict(meta or {}, step=step, rank=self.rank))
        for old in self.list()[: -self.keep] if self.keep > 0 else []:
            shutil.rmtree(self._rank_dir(old), ignore_errors=True)
        return p

    def latest(self) -> Optional[int]:
        s = self.list()
        return s[-1] if s else None

    def agreed_step(self) -> Optional[int]:
        """Newest step that EVERY rank has saved (MIN over ranks of each rank's latest, then
        checked present everywhere): a rank that died between the others' saves must not
        make the replicas restore different steps."""
        from imitation_amd.parallel import dist as pdist

        mine = self.list()
        if pdist.world_size() <= 1:
            return mine[-1] if mine else None
        lo = int(pdist.allreduce_scalars([float(mine[-1]) if mine else -1.0], op="min")[0])
        if lo < 0:
            return None
        have = pdist.allreduce_scalars([1.0 if lo in mine else 0.0], op="min")[0]
        if have < 1.0:
            raise RuntimeError(f"checkpoint step {lo} is missing on some rank; cannot restore consistently")
        return lo

    def restore_latest(self, trainer) -> int:
        step = self.agreed_step()
        if step is None:
            return 0
        load_checkpoint(trainer, self._rank_dir(step))
        return step
