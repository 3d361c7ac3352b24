"""Small shared utilities (timing, stats)."""
from .timing import percentile, summarize  # noqa: F401
