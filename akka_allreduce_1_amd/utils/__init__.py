"""Shared utilities: timing statistics, metrics registry / exporters, tracing dump."""
from .metrics import MetricsRegistry, NodeMetricsSampler, node_metrics, write_trace  # noqa: F401
from .timing import busbw, percentile, summarize  # noqa: F401
