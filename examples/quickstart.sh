#!/usr/bin/env bash
# CLI quickstart (reference examples/quickstart.sh): an RL expert on Pendulum, then GAIL and
# AIRL from its rollouts. Add `engine=device` to the adversarial runs to require the GPU engine.
set -e
python -m imitation_amd.scripts.train_rl with pendulum environment.fast policy_evaluation.fast rl.fast fast logging.log_dir=quickstart/rl/
python -m imitation_amd.scripts.train_adversarial gail with pendulum environment.fast demonstrations.fast policy_evaluation.fast rl.fast fast demonstrations.path=quickstart/rl/rollouts/final.npz demonstrations.source=local
python -m imitation_amd.scripts.train_adversarial airl with pendulum environment.fast demonstrations.fast policy_evaluation.fast rl.fast fast demonstrations.path=quickstart/rl/rollouts/final.npz demonstrations.source=local
