"""Interactive (human-in-the-loop) policies (reference: tests/policies/test_interactive.py).

The key prompts are answered by a scripted ``input`` that interleaves invalid keys (which
must be re-asked) with the requested action keys; rendering is stubbed out."""

import collections
from unittest import mock

import numpy as np
import pytest

from imitation_amd.policies import interactive
from imitation_amd.util.util import make_vec_env


class _QuietDiscretePolicy(interactive.DiscreteInteractivePolicy):
    def _render(self, obs):
        return None


class _QuietAtariPolicy(interactive.AtariInteractivePolicy):
    def _render(self, obs):
        return None

    def _clean_up(self, context):
        pass


class _ScriptedKeys:
    """``input()`` stand-in: cycles through the action keys, with an invalid key before
    every other answer."""

    def __init__(self, keys, rng):
        self.keys, self.rng, self.i, self.asked = list(keys), rng, 0, 0

    def __call__(self, prompt=""):
        self.asked += 1
        if self.rng.uniform() < 0.5:
            return "not-a-key"
        k = self.keys[self.i]
        self.i = (self.i + 1) % len(self.keys)
        return k


@pytest.mark.parametrize("env_name", ["seals/CartPole-v0", "PongNoFrameskip-v4"])
def test_interactive_policy_follows_keys(env_name):
    venv = make_vec_env(env_name, rng=np.random.default_rng(0), n_envs=1, max_episode_steps=20)
    if env_name.startswith("Pong"):
        pol = _QuietAtariPolicy(venv, clear_screen_on_query=False)
        assert list(pol.action_keys_names.values()) == interactive.PONG_ACTION_MEANINGS
    else:
        n = venv.action_space.n
        pol = _QuietDiscretePolicy(venv.observation_space, venv.action_space,
                                   collections.OrderedDict((f"k{i}", f"n{i}") for i in range(n)),
                                   clear_screen_on_query=False)
    keys = list(pol.action_keys_names)
    script = _ScriptedKeys(keys, np.random.default_rng(1))
    obs = venv.reset()
    with mock.patch("builtins.input", script), mock.patch("builtins.print"):
        for step in range(20):
            action, _ = pol.predict(obs)
            assert isinstance(action, np.ndarray) and action.shape == (1,)
            assert venv.action_space.contains(action[0])
            assert action[0] == step % len(keys)  # invalid keys were re-asked, not taken
            obs, _, _, _ = venv.step(action)
    assert script.asked > 20


def test_interactive_policy_rejects_bad_key_maps():
    venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(0), n_envs=1)
    with pytest.raises(AssertionError):
        _QuietDiscretePolicy(venv.observation_space, venv.action_space, collections.OrderedDict(a="x"))
