"""Synthetic gradient sets of the BASELINE.json model configs (shapes only, random init)."""
from .grad_sets import GRAD_SETS, gradient_shapes  # noqa: F401
