"""One-off: fold the reference's tuned-HP JSON files into one table keyed by name,
translating class references to this package (stable_baselines3.* / imitation.*)."""

import json
import pathlib
import sys

MAP = {
    "stable_baselines3.ppo.ppo.PPO": "imitation_amd.rl.ppo:PPO",
    "stable_baselines3.sac.sac.SAC": "imitation_amd.rl.sac:SAC",
    "stable_baselines3.dqn.dqn.DQN": "imitation_amd.rl.dqn:DQN",
    "stable_baselines3.common.policies.ActorCriticPolicy": "imitation_amd.rl.policies:ActorCriticPolicy",
    "stable_baselines3.common.policies.ActorCriticCnnPolicy": "imitation_amd.rl.policies:ActorCriticCnnPolicy",
}


def tr(path: str) -> str:
    if path in MAP:
        return MAP[path]
    if path.startswith("imitation."):
        mod, _, name = path.rpartition(".")
        return "imitation_amd." + mod[len("imitation."):] + ":" + name
    mod, _, name = path.rpartition(".")
    return f"{mod}:{name}"


def walk(v):
    if isinstance(v, dict):
        if set(v) == {"py/type"}:
            return {"py/type": tr(v["py/type"])}
        return {k: walk(x) for k, x in v.items()}
    if isinstance(v, list):
        return [walk(x) for x in v]
    return v


src = pathlib.Path(sys.argv[1])
out = {}
for f in sorted(src.glob("*.json")):
    name = f.stem.replace("_best_hp_eval", "")
    out[name] = walk(json.loads(f.read_text()))
pathlib.Path(sys.argv[2]).write_text(json.dumps(out, indent=1, sort_keys=True))
print(f"{len(out)} configs -> {sys.argv[2]}")
