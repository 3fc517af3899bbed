"""Data-parallel runtime: process-group bootstrap, bucketed overlapped all-reduce, native RCCL engine."""
from .dist import DistInfo, init_distributed  # noqa: F401
