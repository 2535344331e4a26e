"""Mirror of kaolin/metrics (the DIB-R silhouette loss only)."""
from . import render  # noqa: F401
