"""Operators backed by hand-written gfx950 HIP kernels (GPU tensors) and the
OpenMP C references (CPU tensors) of libmpx."""

from .classify import class_stats, classify_
from .classify import plan as classify_plan
from .edge import ConvLauncher, conv, conv_rows, roberts, roberts_rgb
from .filters import Filter, get_filter, list_filters
from .sort import sort_
from .stencil import jacobi_sweep
from .vector import vsub

__all__ = [
    "class_stats",
    "classify_",
    "classify_plan",
    "conv",
    "ConvLauncher",
    "conv_rows",
    "roberts",
    "roberts_rgb",
    "Filter",
    "get_filter",
    "list_filters",
    "jacobi_sweep",
    "sort_",
    "vsub",
]
