"""Episode video recording (reference: src/imitation/util/video_wrapper.py -- the fork
comments the whole module out; upstream records one video per episode).

Frames come from ``env.render()`` (rgb_array). Videos are written as numbered PNG
frame directories plus an ``.npz`` of the frame stack (no ffmpeg on the training
nodes); ``single_video`` keeps one growing video across episodes.
"""

from __future__ import annotations

import os
import pathlib
from typing import List, Optional

import numpy as np

from imitation_amd.envs import core


class VideoWrapper(core.Wrapper):
    def __init__(self, env: core.Env, directory: pathlib.Path, single_video: bool = True, delete_on_close: bool = True):
        super().__init__(env)
        self.directory = pathlib.Path(directory)
        self.directory.mkdir(parents=True, exist_ok=True)
        self.single_video = single_video
        self.delete_on_close = delete_on_close
        self.episode_id = 0
        self._frames: List[np.ndarray] = []
        self.output_paths: List[pathlib.Path] = []

    def _capture(self) -> None:
        try:
            frame = self.env.render()
        except Exception:
            frame = None
        if frame is not None:
            self._frames.append(np.asarray(frame))

    def _flush(self) -> Optional[pathlib.Path]:
        if not self._frames:
            return None
        path = self.directory / f"video.{self.episode_id:06}.npz"
        np.savez_compressed(path, frames=np.stack(self._frames))
        self.output_paths.append(path)
        self._frames = []
        return path

    def reset(self, **kwargs):
        if not self.single_video:
            self._flush()
        self.episode_id += 1
        out = self.env.reset(**kwargs)
        self._capture()
        return out

    def step(self, action):
        out = self.env.step(action)
        self._capture()
        return out

    def close(self) -> None:
        self._flush()
        if self.delete_on_close:
            for p in self.output_paths:
                if p.exists():
                    os.remove(p)
        super().close()
