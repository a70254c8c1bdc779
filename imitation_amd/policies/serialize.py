"""Policy loading/saving by type key (reference: src/imitation/policies/serialize.py).

``policy_registry`` keys: ``random``, ``zero``, ``ppo``, ``sac``, ``dqn`` (from a
``model.zip`` path or a directory holding one) and ``<algo>-huggingface``. There is
no network access on MI355X training nodes, so the ``-huggingface`` loaders resolve
the reference's hub naming (``{organization}/{algo}-{env}``) against LOCAL model
directories: ``$IMITATION_AMD_HUB`` (default ``~/.cache/imitation_amd/hub``). A
model is ``<hub>/<organization>/<algo>-<env-name-with-slashes-as-dashes>/<same>.zip``
or ``.../model.zip`` -- the layout ``huggingface_sb3`` downloads produce.
SB3 ``model.zip`` archives load through ``imitation_amd.rl.save_util`` (JSON + tensors
with ``weights_only=True``; no pickle execution).
"""

from __future__ import annotations

import logging
import os
import pathlib
from typing import Callable, Type

from imitation_amd.policies import base
from imitation_amd.rl import callbacks
from imitation_amd.util import registry, util

PolicyLoaderFn = Callable[..., "object"]

policy_registry: registry.Registry[PolicyLoaderFn] = registry.Registry()


def load_stable_baselines_model(cls: Type, path, venv, **kwargs):
    """Load an RL algorithm from a ``model.zip`` (or a directory containing one)."""
    logging.info(f"Loading policy for '{cls}' from '{path}'")
    path_obj = util.parse_path(path)
    if path_obj.is_dir():
        path_obj = path_obj / "model.zip"
        if not path_obj.exists():
            raise FileNotFoundError(f"Expected '{path}' to be a directory containing a 'model.zip' file.")
    if (path_obj.parent / "vec_normalize.pkl").exists():
        raise FileExistsError(
            "Outdated policy format: we do not support restoring normalization statistics from "
            f"'{path_obj.parent / 'vec_normalize.pkl'}'"
        )
    return cls.load(path_obj, env=venv, **kwargs)


def _load_from_file(cls: Type) -> PolicyLoaderFn:
    def f(venv, path: str):
        return load_stable_baselines_model(cls, path, venv).policy

    return f


def env_name_to_hub(env_name: str) -> str:
    """``seals/CartPole-v0`` -> ``seals-CartPole-v0`` (huggingface_sb3 EnvironmentName)."""
    return env_name.replace("/", "-")


_BUNDLED_HUB = pathlib.Path(__file__).resolve().parents[2] / "experts"


def hub_dir() -> pathlib.Path:
    return pathlib.Path(os.environ.get("IMITATION_AMD_HUB", os.path.expanduser("~/.cache/imitation_amd/hub")))


def hub_dirs():
    """Search order: ``$IMITATION_AMD_HUB`` (or ``~/.cache/imitation_amd/hub``), then the
    experts bundled in the repository (``experts/``: the CartPole expert of the test data)."""
    return [hub_dir(), _BUNDLED_HUB]


def resolve_hub_model(algo_name: str, env_name: str, organization: str = "HumanCompatibleAI") -> pathlib.Path:
    model_name = f"{algo_name}-{env_name_to_hub(env_name)}"
    for hub in hub_dirs():
        root = hub / organization / model_name
        for cand in (root / f"{model_name}.zip", root / "model.zip", hub / f"{model_name}.zip"):
            if cand.exists():
                return cand
    raise FileNotFoundError(
        f"No local copy of hub model {organization}/{model_name} under {[str(h) for h in hub_dirs()]} "
        "(training nodes have no network access; place the model.zip there or set IMITATION_AMD_HUB)."
    )


def _load_from_hub(algo_name: str, cls: Type) -> PolicyLoaderFn:
    def f(venv, env_name: str, organization: str = "HumanCompatibleAI"):
        return load_stable_baselines_model(cls, resolve_hub_model(algo_name, env_name, organization), venv).policy

    return f


policy_registry.register("random", value=registry.build_loader_fn_require_space(base.RandomPolicy))
policy_registry.register("zero", value=registry.build_loader_fn_require_space(base.ZeroPolicy))

_ALGOS = {"ppo": "imitation_amd.rl.ppo:PPO", "sac": "imitation_amd.rl.sac:SAC", "dqn": "imitation_amd.rl.dqn:DQN",
          "td3": "imitation_amd.rl.td3:TD3", "ddpg": "imitation_amd.rl.td3:DDPG"}


def _lazy(loader_factory, *args):
    def f(venv, *a, **kw):
        return loader_factory(*args)(venv, *a, **kw)

    return f


for _k, _cls_name in _ALGOS.items():
    policy_registry.register(_k, value=_lazy(lambda n=_cls_name: _load_from_file(registry.load_attr(n))))
    policy_registry.register(
        f"{_k}-huggingface", value=_lazy(lambda k=_k, n=_cls_name: _load_from_hub(k, registry.load_attr(n)))
    )


def load_policy(policy_type: str, venv, **kwargs):
    """Load a policy of type ``policy_type`` for ``venv`` (kwargs go to the loader)."""
    return policy_registry.get(policy_type)(venv, **kwargs)


def save_stable_model(output_dir, model, filename: str = "model.zip") -> None:
    """Save ``model`` as ``output_dir/filename`` (reference layout)."""
    output_dir = util.parse_path(output_dir)
    os.makedirs(output_dir, exist_ok=True)
    model.save(output_dir / filename)
    logging.info("Saved policy to %s", output_dir)


class SavePolicyCallback(callbacks.EventCallback):
    """Saves the policy under ``policy_dir/{num_timesteps:012d}`` on each event trigger."""

    def __init__(self, policy_dir, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.policy_dir = util.parse_path(policy_dir)

    def _on_step(self) -> bool:
        output_dir = self.policy_dir / f"{self.num_timesteps:012d}"
        save_stable_model(output_dir, self.model)
        return True
