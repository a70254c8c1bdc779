"""Toy-text grid worlds with discrete observations (gymnasium's ``FrozenLake-v1``
semantics; the reference's tests build reward nets and rollouts on it because its
observation space is ``Discrete``). Host-side numpy: these are test / tutorial envs."""

from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np

from imitation_amd.envs import core, spaces

MAPS = {
    "4x4": ["SFFF", "FHFH", "FFFH", "HFFG"],
    "8x8": ["SFFFFFFF", "FFFFFFFF", "FFFHFFFF", "FFFFFHFF", "FFFHFFFF", "FHHFFFHF", "FHFFHFHF", "FFFHFFFG"],
}
# actions: 0 left, 1 down, 2 right, 3 up
_MOVES = ((0, -1), (1, 0), (0, 1), (-1, 0))


class FrozenLakeEnv(core.Env):
    """Walk from S to G over frozen tiles F without falling into a hole H. Observation: the
    cell index ``row * ncol + col`` (Discrete); reward 1 on reaching G; an episode ends on G
    or H. ``is_slippery``: the intended move happens with probability 1/3, each of the two
    perpendicular moves with 1/3."""

    metadata = {"render_modes": ["ansi"]}

    def __init__(self, desc: Optional[Sequence[str]] = None, map_name: str = "4x4", is_slippery: bool = True,
                 render_mode: Optional[str] = None):
        rows = list(desc) if desc is not None else MAPS[map_name]
        self.desc = np.asarray([list(r) for r in rows])
        self.nrow, self.ncol = self.desc.shape
        self.is_slippery = bool(is_slippery)
        self.render_mode = render_mode
        self.observation_space = spaces.Discrete(self.nrow * self.ncol)
        self.action_space = spaces.Discrete(4)
        self.reward_range = (0, 1)
        starts = np.argwhere(self.desc == "S")
        self._start = int(starts[0][0] * self.ncol + starts[0][1])
        self.s = self._start

    def _move(self, s: int, a: int) -> int:
        r, c = divmod(s, self.ncol)
        dr, dc = _MOVES[a]
        r = min(max(r + dr, 0), self.nrow - 1)
        c = min(max(c + dc, 0), self.ncol - 1)
        return int(r * self.ncol + c)

    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None) -> Tuple[int, dict]:
        super().reset(seed=seed)
        self.s = self._start
        return self.s, {"prob": 1.0}

    def step(self, action):
        a = int(action)
        if self.is_slippery:
            a = (a + int(self.np_random.integers(-1, 2))) % 4
        self.s = self._move(self.s, a)
        tile = self.desc.flat[self.s]
        terminated = tile in ("G", "H")
        reward = 1.0 if tile == "G" else 0.0
        return self.s, reward, terminated, False, {"prob": 1.0 / 3.0 if self.is_slippery else 1.0}

    def render(self):
        out = self.desc.copy().astype("<U1")
        r, c = divmod(self.s, self.ncol)
        out[r, c] = "@"
        return "\n".join("".join(row) for row in out)


core.register("FrozenLake-v1", entry_point=FrozenLakeEnv, max_episode_steps=100)
core.register("FrozenLake8x8-v1", entry_point=FrozenLakeEnv, max_episode_steps=200, kwargs={"map_name": "8x8"})
