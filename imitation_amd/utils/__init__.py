"""Runtime utilities around training: tracing (:mod:`.profiling`), failure detection
(:mod:`.watchdog`), full-trainer checkpoints (:mod:`.checkpoint`) and seeding /
deterministic mode (:mod:`.determinism`). See SURVEY §5."""

from imitation_amd.utils import checkpoint, determinism, profiling, watchdog
from imitation_amd.utils.checkpoint import CheckpointManager, load_checkpoint, save_checkpoint
from imitation_amd.utils.profiling import StepTimer
from imitation_amd.utils.watchdog import NonFiniteError, Watchdog, check_finite

__all__ = ["checkpoint", "determinism", "profiling", "watchdog", "CheckpointManager", "load_checkpoint",
           "save_checkpoint", "StepTimer", "NonFiniteError", "Watchdog", "check_finite"]
