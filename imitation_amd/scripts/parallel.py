"""Run many configurations of another experiment in parallel (reference:
src/imitation/scripts/parallel.py, which drives Ray Tune).

Trials are expanded from ``search_space`` (see ``scripts.tune``) and executed in a
local process pool, one process per trial (``spawn``), each attaching a
FileStorageObserver under ``{local_dir}/{run_name}/sacred``. On a multi-GPU node,
``resources_per_trial={"gpu": k}`` pins every trial to its own k GPUs through
``HIP_VISIBLE_DEVICES`` so up to ``num_gpus // k`` trials run concurrently.
"""

from __future__ import annotations

import collections.abc
import copy
import importlib
import multiprocessing as mp
import os
import pathlib
from typing import Any, Dict, List, Mapping, Optional, Sequence

import numpy as np

from imitation_amd.scripts import tune
from imitation_amd.scripts.config.parallel import parallel_ex
from imitation_amd.scripts.config_engine import FileStorageObserver, recursive_update

EXPERIMENTS = {
    "train_rl": ("imitation_amd.scripts.train_rl", "train_rl_ex"),
    "train_adversarial": ("imitation_amd.scripts.train_adversarial", "train_adversarial_ex"),
    "train_imitation": ("imitation_amd.scripts.train_imitation", "train_imitation_ex"),
    "train_preference_comparisons": ("imitation_amd.scripts.train_preference_comparisons",
                                     "train_preference_comparisons_ex"),
    "eval_policy": ("imitation_amd.scripts.eval_policy", "eval_policy_ex"),
}


def _get_experiment(name: str):
    if ":" in name:  # "module:attr" -- any experiment (or, for tests, a plain trial function)
        mod, attr = name.split(":", 1)
        return getattr(importlib.import_module(mod), attr)
    mod, attr = EXPERIMENTS[name]
    return getattr(importlib.import_module(mod), attr)


def _num_gpus() -> int:
    """GPUs on this node, counted without initialising HIP in this (parent) process: the
    children are the ones that must see ``HIP_VISIBLE_DEVICES`` before their runtime starts."""
    from imitation_amd.parallel.launch import count_gpus

    try:
        return int(count_gpus())
    except Exception:  # pragma: no cover
        return 0


def _run_trial(ex_name: str, run_kwargs: Dict[str, Any], observer_dir: str, run_name: str, gpus: str = "") -> Dict[str, Any]:
    if gpus:
        os.environ["HIP_VISIBLE_DEVICES"] = gpus
    ex = _get_experiment(ex_name)
    if not hasattr(ex, "run"):  # plain trial function (tests)
        return ex(run_kwargs, observer_dir, run_name)
    ex.observers = [FileStorageObserver(observer_dir)]
    ex.path = ex.path  # keep experiment name
    run = ex.run(command_name=run_kwargs.get("command_name"), named_configs=run_kwargs.get("named_configs", []),
                 config_updates=run_kwargs.get("config_updates", {}))
    result = run.result
    return {"result": result, "config_updates": run_kwargs.get("config_updates", {}),
            "named_configs": run_kwargs.get("named_configs", []), "status": run.status}


def _trial_process(idx: int, ex_name: str, run_kwargs: Dict[str, Any], observer_dir: str, run_name: str, gpus: str,
                   results) -> None:
    """Entry point of one trial's fresh process (spawned with ``HIP_VISIBLE_DEVICES`` = its slot
    already in its environment, so the GPU runtime starts pinned)."""
    try:
        rec = _run_trial(ex_name, run_kwargs, observer_dir, run_name, gpus)
    except BaseException as e:  # noqa: BLE001 -- reported as a FAILED trial, as Ray Tune does
        rec = {"result": None, "config_updates": run_kwargs.get("config_updates", {}),
               "named_configs": run_kwargs.get("named_configs", []), "status": "FAILED", "error": repr(e)}
    results.put((idx, rec))


def _metric(result: Any, key: str = "imit_stats/monitor_return_mean") -> float:
    cur = result
    for part in key.split("/"):
        if isinstance(cur, Mapping) and part in cur:
            cur = cur[part]
        else:
            alt = result.get("monitor_return_mean", result.get("return_mean")) if isinstance(result, Mapping) else None
            return float("nan") if alt is None else float(alt)
    return float(cur)


@parallel_ex.main
def parallel(sacred_ex_name: str, run_name: str, num_samples: int, search_space: Mapping[str, Any],
             base_named_configs: Sequence[str], base_config_updates: Mapping[str, Any],
             resources_per_trial: Mapping[str, Any], init_kwargs: Mapping[str, Any], repeat: int,
             experiment_checkpoint_path: str, tune_run_kwargs: Dict[str, Any], local_dir: str) -> List[Dict[str, Any]]:
    """Returns one record per trial: its search-space sample, status and result."""
    if not isinstance(base_named_configs, collections.abc.Sequence):
        raise TypeError("base_named_configs must be a Sequence")
    if not isinstance(base_config_updates, collections.abc.Mapping):
        raise TypeError("base_config_updates must be a Mapping")
    del init_kwargs, experiment_checkpoint_path
    rng = np.random.default_rng(tune_run_kwargs.get("seed", 0))
    observer_dir = str(pathlib.Path(tune_run_kwargs.get("local_dir", local_dir)) / run_name / "sacred")
    # the reference defaults to OptunaSearch (TPE) wrapped in a Repeater when repeat > 1, and
    # to Ray's random variant generator otherwise (scripts/parallel.py:114-125)
    search_alg = str(tune_run_kwargs.get("search_alg") or ("tpe" if int(repeat) > 1 else "random")).lower()
    if search_alg not in ("random", "tpe"):
        raise ValueError(f"search_alg must be 'random' or 'tpe', got {search_alg!r}")
    if search_alg == "tpe":
        return _parallel_tpe(sacred_ex_name, run_name, int(num_samples), search_space, base_named_configs,
                             base_config_updates, resources_per_trial, int(repeat), tune_run_kwargs, observer_dir, rng)
    samples = tune.generate_trials(search_space, int(num_samples), rng)
    trials = _expand(samples, base_named_configs, base_config_updates, int(repeat), rng)
    records = run_trials(sacred_ex_name, trials, observer_dir, run_name, resources_per_trial,
                         tune_run_kwargs.get("max_concurrent_trials"))
    for r, t in zip(records, trials):
        r["sample"] = t["sample"]
    return records


def _expand(samples, base_named_configs, base_config_updates, repeat: int, rng) -> List[Dict[str, Any]]:
    """Trials of sampled configurations: each sample ``repeat`` times (fresh seeds when > 1)."""
    trials = []
    for s in samples:
        # (checked per sampled trial, as the reference's trainable does: search-space values
        # may be samplers that only resolve here)
        if not isinstance(s.get("named_configs", []), collections.abc.Sequence):
            raise TypeError("search_space['named_configs'] must resolve to a Sequence")
        if not isinstance(s.get("config_updates", {}), collections.abc.Mapping):
            raise TypeError("search_space['config_updates'] must resolve to a Mapping")
        for rep in range(int(repeat)):
            updates = recursive_update(copy.deepcopy(dict(base_config_updates)), s.get("config_updates") or {})
            if repeat > 1:
                updates.setdefault("seed", int(rng.integers(0, 2**31 - 1)))
            trials.append(dict(command_name=s.get("command_name"),
                               named_configs=list(base_named_configs) + list(s.get("named_configs") or []),
                               config_updates=updates, sample=s))
    return trials


def _parallel_tpe(ex_name: str, run_name: str, num_samples: int, search_space, base_named_configs, base_config_updates,
                  resources_per_trial, repeat: int, tune_run_kwargs, observer_dir: str, rng) -> List[Dict[str, Any]]:
    """Model-based search (``tune.TPESearch``, the reference's ``Repeater(OptunaSearch())``): batches
    of suggestions -- as many as can run concurrently -- each run ``repeat`` times; a sample's
    metric is the mean over its repeats (Repeater semantics) and feeds the model before the next
    batch is suggested."""
    searcher = tune.TPESearch(search_space, rng, n_startup=int(tune_run_kwargs.get("n_startup_trials", 10)))
    conc = tune_run_kwargs.get("max_concurrent_trials")
    if conc is None:
        conc = max(1, len(_gpu_slots(resources_per_trial)))
    per_batch = max(1, int(conc) // max(1, repeat))
    records: List[Dict[str, Any]] = []
    done = 0
    while done < num_samples:
        k = min(per_batch, num_samples - done)
        samples = [searcher.suggest() for _ in range(k)]
        for s in samples:
            if not isinstance(s.get("named_configs", []), collections.abc.Sequence):
                raise TypeError("search_space['named_configs'] must resolve to a Sequence")
            if not isinstance(s.get("config_updates", {}), collections.abc.Mapping):
                raise TypeError("search_space['config_updates'] must resolve to a Mapping")
        trials = _expand(samples, base_named_configs, base_config_updates, repeat, rng)
        recs = run_trials(ex_name, trials, observer_dir, run_name, resources_per_trial, conc)
        for r, t in zip(recs, trials):
            r["sample"] = t["sample"]
        for j, s in enumerate(samples):
            ms = [r["metric"] for r in recs[j * repeat:(j + 1) * repeat]]
            searcher.observe(s, float(np.nanmean(ms)) if any(m == m for m in ms) else float("nan"))
        records += recs
        done += k
    return records


def _gpu_slots(resources_per_trial: Mapping[str, Any]) -> List[str]:
    """``HIP_VISIBLE_DEVICES`` strings of the disjoint k-GPU slots (k = ``resources_per_trial["gpu"]``)."""
    gpus_per_trial = int(resources_per_trial.get("gpu", 0) or 0)
    n_gpus = _num_gpus() if gpus_per_trial > 0 else 0
    if gpus_per_trial > 0 and n_gpus >= gpus_per_trial:
        return [",".join(str(g) for g in range(i, i + gpus_per_trial))
                for i in range(0, n_gpus - gpus_per_trial + 1, gpus_per_trial)]
    return []


def run_trials(ex_name: str, trials: List[Dict[str, Any]], observer_dir: str, run_name: str,
               resources_per_trial: Mapping[str, Any], max_concurrent: Any = None,
               gpu_slots: Optional[Sequence[str]] = None) -> List[Dict[str, Any]]:
    """Run ``trials`` (dicts of command_name / named_configs / config_updates) of experiment ``ex_name``.

    With GPU slots (``resources_per_trial={"gpu": k}`` on a node with >= k GPUs, or explicit
    ``gpu_slots``), every trial runs in a FRESH ``spawn`` process whose environment carries
    ``HIP_VISIBLE_DEVICES`` = a slot that is free at its start; the slot returns to the pool when
    the process ends. No process that may already have initialised HIP is ever re-pinned (a
    reused pool worker would keep its first trial's GPU), and no slot hosts two running trials
    (Ray Tune's per-trial GPU resources, reference ``scripts/parallel.py:114-148``)."""
    if gpu_slots is None:
        gpu_slots = _gpu_slots(resources_per_trial)
    slots = list(gpu_slots)
    max_conc = int(max_concurrent if max_concurrent is not None else (len(slots) if slots else 1))
    if slots:
        max_conc = min(max_conc, len(slots))
    if max_conc <= 1 and not slots:
        records = [_run_trial(ex_name, t, observer_dir, run_name, "") for t in trials]
    else:
        records = _schedule(ex_name, trials, observer_dir, run_name, slots or [""] * max_conc, max_conc)
    for r in records:
        r["metric"] = _metric(r["result"]) if r["status"] == "COMPLETED" else float("nan")
    return records


def _schedule(ex_name: str, trials: List[Dict[str, Any]], observer_dir: str, run_name: str, slots: List[str],
              max_conc: int) -> List[Dict[str, Any]]:
    """Free-slot queue: start a trial whenever a slot is free, one fresh process per trial."""
    import queue as queue_mod

    ctx = mp.get_context("spawn")
    results = ctx.Queue()
    free = list(range(len(slots)))
    running: Dict[int, Any] = {}  # trial index -> (process, slot index)
    records: List[Optional[Dict[str, Any]]] = [None] * len(trials)
    pending = list(range(len(trials)))
    while pending or running:
        while pending and free and len(running) < max_conc:
            i, si = pending.pop(0), free.pop(0)
            gpus = slots[si]
            saved = os.environ.get("HIP_VISIBLE_DEVICES")
            if gpus:  # inherited by the spawned interpreter before anything in it starts HIP
                os.environ["HIP_VISIBLE_DEVICES"] = gpus
            try:
                p = ctx.Process(target=_trial_process, args=(i, ex_name, trials[i], observer_dir, run_name, gpus, results))
                p.start()
            finally:
                if gpus:
                    if saved is None:
                        os.environ.pop("HIP_VISIBLE_DEVICES", None)
                    else:
                        os.environ["HIP_VISIBLE_DEVICES"] = saved
            running[i] = (p, si)
        try:
            i, rec = results.get(timeout=0.5)
        except queue_mod.Empty:
            for i, (p, si) in list(running.items()):  # a trial process that died without a result
                if not p.is_alive() and records[i] is None:
                    p.join()
                    # its result may still be in flight on the queue: drain before declaring it lost
                    try:
                        while True:
                            j, rj = results.get_nowait()
                            records[j] = rj
                            if j in running and j != i:
                                pj, sj = running.pop(j)
                                pj.join()
                                free.append(sj)
                    except queue_mod.Empty:
                        pass
                    if records[i] is None:
                        records[i] = {"result": None, "config_updates": trials[i].get("config_updates", {}),
                                      "named_configs": trials[i].get("named_configs", []), "status": "FAILED",
                                      "error": f"trial process exited with code {p.exitcode}"}
                    running.pop(i, None)
                    free.append(si)
            continue
        records[i] = rec  # (a late real result overwrites a FAILED record)
        entry = running.pop(i, None)
        if entry is not None:
            p, si = entry
            p.join()
            free.append(si)
    return [r for r in records if r is not None]


def main_console(argv=None):
    parallel_ex.observers.append(FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "parallel"))
    return parallel_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
