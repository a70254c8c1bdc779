"""Experiment definitions (config scopes + named configs) for the scripts
(reference: src/imitation/scripts/config/)."""

import json
import pathlib
from typing import Iterable

TUNED_HPS_PATH = pathlib.Path(__file__).with_name("tuned_hps.json")


def tuned_hps() -> dict:
    """Tuned hyper-parameter configs (reference ``config/tuned_hps/*.json``), keyed by name."""
    return json.loads(TUNED_HPS_PATH.read_text())


def register_tuned(experiment, names: Iterable[str]) -> None:
    table = tuned_hps()
    for name in names:
        if name not in table:
            raise KeyError(f"tuned config {name} missing from {TUNED_HPS_PATH}")
        experiment.add_named_config(name, table[name])
