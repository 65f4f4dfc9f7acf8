"""Postprocessors (re-exported; implementations live next to their clients)."""
from .base_postprocess import Postprocess  # noqa: F401
