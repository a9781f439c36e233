"""Minimal SpeechBrain-0.5-compatible training runtime for the VAE recipe.

The reference subclasses speechbrain.Brain (un-vendored, unpinned: SURVEY.md 8(c)); this
package re-creates only what the recipe touches: Brain (fit / evaluate / fit_batch /
evaluate_batch / check_gradients / stage hooks / update_average), Stage, EpochCounter,
Checkpointer, InputNormalization (global), FileTrainLogger, PaddedBatch-style batches,
parse_arguments and create_experiment_directory.  Behaviour is restated from SpeechBrain
0.5 semantics; no reference test pins it ("parity unpinned").
"""
from .core import Brain, Stage  # noqa: F401
from .epoch_loop import EpochCounter  # noqa: F401
from .checkpoints import Checkpointer  # noqa: F401
from .features import InputNormalization  # noqa: F401
from .train_logger import FileTrainLogger  # noqa: F401
from .cli import parse_arguments, create_experiment_directory  # noqa: F401
from .dataio import PaddedBatch, length_to_mask  # noqa: F401
