"""Optimizers and flat parameter/gradient arenas."""
from .arena import ParamArena, arena_for  # noqa: F401
from .sgd import FusedSGD  # noqa: F401
