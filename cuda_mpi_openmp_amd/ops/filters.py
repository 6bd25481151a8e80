"""Convolution filters of the lab2 family.

The named table lives in native code (``native/include/mpx/filters.h``) so the
CLIs and Python always agree; :func:`get_filter` reads it through libmpx.
``Filter.custom`` builds any K x K (K <= 7) filter for the generic kernels.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Sequence

from .. import _native

MAX_K = 7
MODE_MAG2, MODE_ABS1, MODE_LIN1 = 0, 1, 2
MODE_NAMES = {"mag2": MODE_MAG2, "abs1": MODE_ABS1, "lin1": MODE_LIN1}


@dataclass(frozen=True)
class Filter:
    """K x K taps (row-major [dy][dx]) applied at (y + dy - anchor, x + dx - anchor)."""

    name: str
    k: int
    anchor: int
    mode: int
    wx: tuple
    wy: tuple = field(default=())

    @property
    def halo_up(self) -> int:
        """Rows above an output row that the window reads."""
        return self.anchor

    @property
    def halo_down(self) -> int:
        """Rows below an output row that the window reads."""
        return self.k - 1 - self.anchor

    def c_taps(self):
        wy = self.wy if self.wy else (0.0,) * (self.k * self.k)
        return _native.f32_array(self.wx), _native.f32_array(wy)

    @staticmethod
    def custom(k: int, wx: Sequence[float], wy: Sequence[float] = (), anchor: int | None = None,
               mode: str | int = "mag2", name: str = "custom") -> "Filter":
        if not 1 <= k <= MAX_K:
            raise ValueError(f"k must be in [1, {MAX_K}]")
        m = MODE_NAMES[mode] if isinstance(mode, str) else int(mode)
        if anchor is None:
            anchor = (k - 1) // 2
        if len(wx) != k * k or (m == MODE_MAG2 and len(wy) != k * k):
            raise ValueError("need k*k taps per filter")
        return Filter(name, k, int(anchor), m, tuple(float(v) for v in wx), tuple(float(v) for v in wy))


_cache: dict = {}


def get_filter(name: str) -> Filter:
    if isinstance(name, Filter):
        return name
    if name in _cache:
        return _cache[name]
    L = _native.lib()
    k, a, m = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    wx = (ctypes.c_float * (MAX_K * MAX_K))()
    wy = (ctypes.c_float * (MAX_K * MAX_K))()
    _native.check(L.mpx_filter_lookup(name.encode(), ctypes.byref(k), ctypes.byref(a), ctypes.byref(m), wx, wy))
    n = k.value * k.value
    f = Filter(name, k.value, a.value, m.value, tuple(wx[:n]), tuple(wy[:n]) if m.value == MODE_MAG2 else ())
    _cache[name] = f
    return f


def list_filters() -> List[str]:
    L = _native.lib()
    out, i = [], 0
    while True:
        nm = L.mpx_filter_name(i)
        if not nm:
            return out
        out.append(nm.decode())
        i += 1
