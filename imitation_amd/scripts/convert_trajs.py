"""Convert legacy ``.npz`` trajectory files to the HF-dataset directory format
(reference: src/imitation/scripts/convert_trajs.py). ``A.npz`` -> ``A/``.

Legacy pickles are only converted with ``--allow-pickle`` (they execute code on load);
``.npz`` files are read with ``allow_pickle=False`` (their ``infos`` are then dropped).
"""

from __future__ import annotations

import argparse
import pathlib
import warnings

from imitation_amd.data import huggingface_utils, serialize, types
from imitation_amd.util import util


def update_traj_file_in_place(path_str: types.AnyPath, /, allow_pickle: bool = False) -> pathlib.Path:
    path = util.parse_path(path_str)
    trajs = serialize.load(path, allow_pickle=allow_pickle)
    if isinstance(trajs, huggingface_utils.TrajectoryDatasetSequence):
        warnings.warn(f"File {path} is already in the new format. Skipping.")
        return path
    converted = path.with_suffix("")
    serialize.save(converted, trajs)
    return converted


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("paths", nargs="+")
    p.add_argument("--allow-pickle", action="store_true", help="also convert legacy .pkl files (trusted input only)")
    args = p.parse_args(argv)
    for path in args.paths:
        print(update_traj_file_in_place(path, allow_pickle=args.allow_pickle))


if __name__ == "__main__":  # pragma: no cover
    main()
