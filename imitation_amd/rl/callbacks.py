"""Training callbacks (SB3 ``callbacks`` surface used by the reference:
``BaseCallback``/``EventCallback``/``EveryNTimesteps``/``CallbackList``,
``src/imitation/rewards/reward_wrapper.py:15-37``, ``scripts/train_rl.py:129-138``)."""

from __future__ import annotations

import os
from typing import Any, Callable, Dict, List, Optional, Union


class BaseCallback:
    def __init__(self, verbose: int = 0):
        self.model = None
        self.n_calls = 0
        self.num_timesteps = 0
        self.verbose = verbose
        self.locals: Dict[str, Any] = {}
        self.globals: Dict[str, Any] = {}
        self.parent: Optional["BaseCallback"] = None

    @property
    def training_env(self):
        return self.model.get_env()

    @property
    def logger(self):
        return self.model.logger

    def init_callback(self, model) -> None:
        self.model = model
        self._init_callback()

    def _init_callback(self) -> None:
        pass

    def on_training_start(self, locals_: Dict[str, Any], globals_: Dict[str, Any]) -> None:
        self.locals = locals_
        self.globals = globals_
        self.num_timesteps = self.model.num_timesteps
        self._on_training_start()

    def _on_training_start(self) -> None:
        pass

    def on_rollout_start(self) -> None:
        self._on_rollout_start()

    def _on_rollout_start(self) -> None:
        pass

    def _on_step(self) -> bool:
        return True

    def on_step(self) -> bool:
        self.n_calls += 1
        self.num_timesteps = self.model.num_timesteps
        return self._on_step()

    def on_training_end(self) -> None:
        self._on_training_end()

    def _on_training_end(self) -> None:
        pass

    def on_rollout_end(self) -> None:
        self._on_rollout_end()

    def _on_rollout_end(self) -> None:
        pass

    def update_locals(self, locals_: Dict[str, Any]) -> None:
        self.locals.update(locals_)
        self.update_child_locals(locals_)

    def update_child_locals(self, locals_: Dict[str, Any]) -> None:
        pass


class EventCallback(BaseCallback):
    def __init__(self, callback: Optional[BaseCallback] = None, verbose: int = 0):
        super().__init__(verbose=verbose)
        self.callback = callback
        if callback is not None:
            self.callback.parent = self

    def init_callback(self, model) -> None:
        super().init_callback(model)
        if self.callback is not None:
            self.callback.init_callback(self.model)

    def _on_training_start(self) -> None:
        if self.callback is not None:
            self.callback.on_training_start(self.locals, self.globals)

    def _on_event(self) -> bool:
        if self.callback is not None:
            return self.callback.on_step()
        return True

    def _on_step(self) -> bool:
        return True

    def update_child_locals(self, locals_: Dict[str, Any]) -> None:
        if self.callback is not None:
            self.callback.update_locals(locals_)


class CallbackList(BaseCallback):
    def __init__(self, callbacks: List[BaseCallback]):
        super().__init__()
        assert isinstance(callbacks, list)
        self.callbacks = callbacks

    def _init_callback(self) -> None:
        for c in self.callbacks:
            c.init_callback(self.model)

    def _on_training_start(self) -> None:
        for c in self.callbacks:
            c.on_training_start(self.locals, self.globals)

    def _on_rollout_start(self) -> None:
        for c in self.callbacks:
            c.on_rollout_start()

    def _on_step(self) -> bool:
        cont = True
        for c in self.callbacks:
            cont = c.on_step() and cont
        return cont

    def _on_rollout_end(self) -> None:
        for c in self.callbacks:
            c.on_rollout_end()

    def _on_training_end(self) -> None:
        for c in self.callbacks:
            c.on_training_end()

    def update_child_locals(self, locals_: Dict[str, Any]) -> None:
        for c in self.callbacks:
            c.update_locals(locals_)


class ConvertCallback(BaseCallback):
    """Wrap ``fn(locals, globals) -> bool`` as a callback."""

    def __init__(self, callback: Callable[[Dict[str, Any], Dict[str, Any]], bool], verbose: int = 0):
        super().__init__(verbose)
        self.callback = callback

    def _on_step(self) -> bool:
        if self.callback is not None:
            return self.callback(self.locals, self.globals)
        return True


class EveryNTimesteps(EventCallback):
    def __init__(self, n_steps: int, callback: BaseCallback):
        super().__init__(callback)
        self.n_steps = n_steps
        self.last_time_trigger = 0

    def _on_step(self) -> bool:
        if (self.num_timesteps - self.last_time_trigger) >= self.n_steps:
            self.last_time_trigger = self.num_timesteps
            return self._on_event()
        return True


class CheckpointCallback(BaseCallback):
    def __init__(self, save_freq: int, save_path: str, name_prefix: str = "rl_model", verbose: int = 0):
        super().__init__(verbose)
        self.save_freq = save_freq
        self.save_path = save_path
        self.name_prefix = name_prefix

    def _init_callback(self) -> None:
        os.makedirs(self.save_path, exist_ok=True)

    def _on_step(self) -> bool:
        if self.n_calls % self.save_freq == 0:
            self.model.save(os.path.join(self.save_path, f"{self.name_prefix}_{self.num_timesteps}_steps"))
        return True


class StopTrainingOnMaxEpisodes(BaseCallback):
    def __init__(self, max_episodes: int, verbose: int = 0):
        super().__init__(verbose)
        self.max_episodes = max_episodes
        self.n_episodes = 0

    def _on_step(self) -> bool:
        dones = self.locals.get("dones")
        if dones is not None:
            self.n_episodes += int(sum(dones))
        return self.n_episodes < self.max_episodes


def convert_callback(callback) -> BaseCallback:
    if isinstance(callback, list):
        callback = CallbackList(callback)
    if not isinstance(callback, BaseCallback):
        callback = ConvertCallback(callback) if callback is not None else CallbackList([])
    return callback
