"""roctx ranges for rocprofv3 timelines (SURVEY §5 "tracing / profiling").

``MPX_ROCTX=1`` turns the ranges on; otherwise :func:`range` is a no-op
context manager, so the hot loops pay nothing. Ranges appear under
``rocprofv3 --marker-trace`` next to the kernel trace, e.g. one
``edge.step`` range per step with ``halo`` and ``conv`` children.

libroctx64 is bound with ctypes from /opt/rocm (or ``MPX_ROCTX_LIB``).
"""

from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Iterator, Optional

_lib: Optional[ctypes.CDLL] = None
_enabled: Optional[bool] = None


def enabled() -> bool:
    global _enabled, _lib
    if _enabled is None:
        _enabled = False
        if os.environ.get("MPX_ROCTX", "0") not in ("", "0"):
            path = os.environ.get("MPX_ROCTX_LIB", "/opt/rocm/lib/libroctx64.so")
            try:
                _lib = ctypes.CDLL(path)
                _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _lib.roctxRangePushA.restype = ctypes.c_int
                _lib.roctxRangePop.restype = ctypes.c_int
                _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _enabled = True
            except (OSError, AttributeError):
                _enabled = False
    return _enabled


@contextlib.contextmanager
def range(name: str) -> Iterator[None]:  # noqa: A001 - mirrors roctx naming
    if not enabled():
        yield
        return
    _lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if enabled():
        _lib.roctxMarkA(name.encode())
