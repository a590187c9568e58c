"""Train/eval loops (reference-compatible), whole-step hipGraph capture, part entry points."""
from .trainer import train_model, test_model, CrossEntropyLoss  # noqa: F401
from .step import TrainStep, SegmentedDDPStep  # noqa: F401
