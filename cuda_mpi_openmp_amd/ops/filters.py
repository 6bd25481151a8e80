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
MODE_SEP = 16  # flag: wx / wy hold separable factors (native/include/mpx/common.h)
MODE_NAMES = {"mag2": MODE_MAG2, "abs1": MODE_ABS1, "lin1": MODE_LIN1}


@dataclass(frozen=True)
class Filter:
    """K x K taps (row-major [dy][dx]) applied at (y + dy - anchor, x + dx - anchor).

    Separable filters (``mode & MODE_SEP``) store ``wx = hx + vx + (sx,)`` (and
    ``wy`` alike): gx = sx * sum_dy vx[dy] * sum_dx hx[dx] * Y, horizontal pass
    first, each sum a sequential fp32 fma chain.
    """

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

    @property
    def separable(self) -> bool:
        return bool(self.mode & MODE_SEP)

    @property
    def base_mode(self) -> int:
        return self.mode & 3

    @property
    def ntaps(self) -> int:
        return 2 * self.k + 1 if self.separable else self.k * self.k

    def dense(self) -> tuple:
        """(wx, wy) as K x K row-major taps (the outer products for separable filters)."""
        if not self.separable:
            return self.wx, self.wy
        k = self.k

        def outer(t):
            if not t:
                return ()
            h, v, s = t[:k], t[k:2 * k], t[2 * k]
            return tuple(float(v[i]) * float(h[j]) * float(s) for i in range(k) for j in range(k))

        return outer(self.wx), outer(self.wy)

    def c_taps(self):
        wy = self.wy if self.wy else (0.0,) * self.ntaps
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

    @staticmethod
    def separable_custom(hx: Sequence[float], vx: Sequence[float], scale_x: float = 1.0,
                         hy: Sequence[float] = (), vy: Sequence[float] = (), scale_y: float = 1.0,
                         anchor: int | None = None, mode: str | int = "mag2", name: str = "custom_sep") -> "Filter":
        """Separable filter gx = scale_x * (vx outer hx) (and gy alike for ``mag2``)."""
        k = len(hx)
        if not 1 <= k <= MAX_K or len(vx) != k:
            raise ValueError(f"need hx, vx of one length in [1, {MAX_K}]")
        m = MODE_NAMES[mode] if isinstance(mode, str) else int(mode)
        if m == MODE_MAG2 and (len(hy) != k or len(vy) != k):
            raise ValueError("mag2 needs hy, vy of length k")
        if anchor is None:
            anchor = (k - 1) // 2
        wx = tuple(float(v) for v in (*hx, *vx, scale_x))
        wy = tuple(float(v) for v in (*hy, *vy, scale_y)) if m == MODE_MAG2 else ()
        return Filter(name, k, int(anchor), m | MODE_SEP, wx, wy)


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
    n = 2 * k.value + 1 if m.value & MODE_SEP else k.value * k.value
    two = (m.value & 3) == MODE_MAG2
    f = Filter(name, k.value, a.value, m.value, tuple(wx[:n]), tuple(wy[:n]) if two else ())
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
