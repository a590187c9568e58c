"""CLI contract, seeding, device selection, metrics, checkpoints, watchdog, roctx tracing."""
from .cli import get_rank, parse_arguments, parse_all, build_parser  # noqa: F401
from .misc import (seed_everything, pick_device, local_rank_of, MetricsSink,  # noqa: F401
                   save_checkpoint, load_checkpoint, Watchdog, fault_point)
from . import ladder  # noqa: F401
from .trace import trace_range, enable as enable_tracing  # noqa: F401
