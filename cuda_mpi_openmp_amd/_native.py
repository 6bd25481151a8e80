"""ctypes binding of ``libmpx.so`` — the single native library (HIP kernels for
gfx950, OpenMP CPU references, host statistics) shared with the lab CLIs.

Import order matters on ROCm: PyTorch ships its own ``libamdhip64.so.7``. Loading
torch first makes the dynamic loader resolve libmpx's ``libamdhip64.so.7``
dependency to torch's already-loaded runtime (same SONAME), so device pointers,
streams and contexts are shared between torch tensors and mpx kernels.

The library is built in-tree (``make lib`` or ``__graft_entry__.build()``). On a
GPU path a missing library is an error, never a silent fallback.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from pathlib import Path

import torch  # noqa: F401  (must be loaded before libmpx; see module docstring)

_PKG_DIR = Path(__file__).resolve().parent
REPO_ROOT = _PKG_DIR.parent
# MPX_LIB_PATH: load another build of libmpx (kernel A/B runs: tools/*_ab.py)
LIB_PATH = Path(os.environ["MPX_LIB_PATH"]) if os.environ.get("MPX_LIB_PATH") else _PKG_DIR / "_lib" / "libmpx.so"

_lib = None
_lock = threading.Lock()

c_int, c_i64, c_size, c_vp = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p
c_char_p = ctypes.c_char_p
_dp = ctypes.POINTER(ctypes.c_double)
_fp = ctypes.POINTER(ctypes.c_float)
_ip = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes)
_SIGNATURES = {
    "mpx_last_error": (c_char_p, []),
    "mpx_version": (c_char_p, []),
    "mpx_device_count": (c_int, [_ip]),
    "mpx_device_report": (c_int, [c_int, ctypes.c_char_p, c_size]),
    "mpx_stream_sync": (c_int, [c_vp]),
    "mpx_vsub_f64": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp]),
    "mpx_vsub_f32": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp]),
    "mpx_roberts": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "mpx_conv": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _fp, _fp, c_vp]),
    "mpx_conv_direct": (
        c_int,
        [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _fp, _fp, c_vp],
    ),
    "mpx_conv_set_band_min": (ctypes.c_longlong, [ctypes.c_longlong]),
    "mpx_conv_set_band_mode": (c_int, [c_int]),
    "mpx_conv_peer": (
        c_int,
        [c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _fp, _fp, c_vp],
    ),
    "mpx_ipc_handle_size": (c_int, []),
    "mpx_ipc_get_handle": (c_int, [c_vp, c_vp, ctypes.POINTER(c_i64)]),
    "mpx_ipc_open": (c_int, [c_vp, ctypes.POINTER(c_vp)]),
    "mpx_ipc_open_dev": (c_int, [c_int, c_vp, ctypes.POINTER(c_vp)]),
    "mpx_ipc_close": (c_int, [c_vp]),
    "mpx_memcpy_d2d": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "mpx_filter_lookup": (c_int, [c_char_p, _ip, _ip, _ip, _fp, _fp]),
    "mpx_filter_name": (c_char_p, [c_int]),
    "mpx_class_stats": (c_int, [c_vp, c_int, c_int, c_int, _ip, _ip, _dp, _dp]),
    "mpx_classify": (c_int, [c_vp, c_i64, c_int, _dp, _dp, c_int, c_int, c_int, c_vp]),
    "mpx_comm_load": (c_int, [ctypes.c_char_p]),
    "mpx_comm_version": (c_int, []),
    "mpx_comm_unique_id": (c_int, [c_vp, c_int]),
    "mpx_comm_init": (c_int, [ctypes.POINTER(c_vp), c_int, c_int, c_vp, c_int, c_int]),
    "mpx_comm_destroy": (c_int, [c_vp]),
    "mpx_comm_rank": (c_int, [c_vp]),
    "mpx_comm_size": (c_int, [c_vp]),
    "mpx_comm_p2p_start": (c_int, [c_vp, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_vp),
                                   ctypes.POINTER(c_i64), ctypes.POINTER(c_int), c_vp]),
    "mpx_comm_p2p_wait": (c_int, [c_vp, c_vp]),
    "mpx_comm_p2p": (c_int, [c_vp, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_vp),
                             ctypes.POINTER(c_i64), ctypes.POINTER(c_int), c_vp]),
    "mpx_comm_allreduce": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp]),
    "mpx_comm_check": (c_int, [c_vp]),
    "mpx_comm_abort": (c_int, [c_vp]),
    "mpx_comm_stream": (c_vp, [c_vp]),
    "mpx_classify_ex": (c_int, [c_vp, c_i64, c_int, _dp, _dp, c_int, c_int, c_int, c_vp, c_vp]),
    "mpx_classify_plan": (c_int, [c_int, _dp, _dp, c_int, ctypes.POINTER(ctypes.c_float)]),
    "mpx_classify_i8_params": (c_int, [c_int, _dp, _dp, c_vp, c_vp, c_vp, c_vp]),
    "mpx_classify_f16_params": (c_int, [c_int, _dp, _dp, c_vp, c_vp, c_vp]),
    "mpx_jacobi_f64": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "mpx_jacobi_sync_bytes": (c_int, []),
    "mpx_jacobi_peer_sweep": (c_int, [c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "mpx_jacobi_f32": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "mpx_cpu_threads": (c_int, []),
    "mpx_cpu_vsub_f64": (None, [c_vp, c_vp, c_vp, c_i64]),
    "mpx_cpu_vsub_f32": (None, [c_vp, c_vp, c_vp, c_i64]),
    "mpx_cpu_roberts": (None, [c_vp, c_vp, c_int, c_int]),
    "mpx_cpu_roberts_rgb": (None, [c_vp, c_vp, c_int, c_int]),
    "mpx_roberts_rgb": (c_int, [c_vp, c_vp, c_int, c_int, c_vp]),
    "mpx_cpu_conv": (None, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _fp, _fp]),
    "mpx_cpu_classify": (None, [c_vp, c_i64, c_int, _dp, _dp]),
    "mpx_cpu_jacobi_f64": (ctypes.c_double, [c_vp, c_vp, c_int, c_int, c_int, c_int]),
    "mpx_sort": (c_int, [c_vp, c_i64, c_int, c_vp]),
    "mpx_sort_workspace_bytes": (c_i64, [c_i64, c_int]),
    "mpx_sort_ws": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_vp]),
    "mpx_sort_ws_status": (c_int, [c_vp, c_i64, c_int]),
    "mpx_sort_lane_order_ok": (c_int, [c_vp]),
    "mpx_cpu_sort": (None, [c_vp, c_i64, c_int]),
    "mpx_rows_checksum": (c_int, [c_vp, c_i64, c_int, c_i64, c_int, c_vp, c_vp]),
    "mpx_peer_probe_run": (c_int, [c_vp, c_vp]),
    "mpx_halo_fetch_run": (c_int, [c_vp, c_vp]),
    "mpx_conv_stream_peer_ok": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "mpx_conv_stream_peer_run": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _fp,
                                         _fp, c_vp, c_vp]),
    "mpx_sync_alloc": (c_int, [c_i64, ctypes.POINTER(c_vp), _ip]),
    "mpx_sync_free": (c_int, [c_vp]),
    "mpx_sync_write": (c_int, [c_vp, c_int, ctypes.c_uint]),
    "mpx_sync_read": (c_int, [c_vp, c_int, ctypes.POINTER(ctypes.c_uint)]),
    "mpx_sync_clear": (c_int, [c_vp, c_i64]),
}

# tuning-only entry points (kernel variants, copy probes, the exhaustive
# fast-sqrt self-test): libmpx_tune.so, built from native/tune/ and loaded only
# by tools/kbench.py and its tests, never by the production paths
TUNE_PATH = _PKG_DIR / "_lib" / "libmpx_tune.so"
_TUNE_SIGNATURES = {
    "mpx_conv_variant": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _fp, _fp, c_vp]),
    "mpx_selftest_fast_sqrt": (c_int, [c_vp, c_int, c_vp]),
    "mpx_strip_copy_probe": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp]),
    # lab5 radix variants / scatter probe (native/tune/sort_variants.hip)
    "mpx_sort_variant": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_int, c_vp]),
    "mpx_sort_scatter_probe": (c_int, [c_vp, c_i64, c_vp, c_i64, c_int, c_vp]),
    # lab1 / Jacobi tuning variants (native/tune/{vsub,jacobi}_variants.hip)
    "mpx_vsub_variant": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp]),
    "mpx_jacobi_variant": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp]),
}
_tune = None


class MpxError(RuntimeError):
    """A libmpx entry point returned a non-zero status."""


def build(quiet: bool = True) -> None:
    """Build libmpx.so in-tree with the repository Makefile (gfx950 cross-compile)."""
    jobs = str(min(8, os.cpu_count() or 1))
    res = subprocess.run(
        ["make", "-C", str(REPO_ROOT), "-j", jobs, "lib"],
        capture_output=quiet,
        text=True,
    )
    if res.returncode != 0:
        raise MpxError(f"building libmpx failed:\n{res.stdout}\n{res.stderr}")


def lib(auto_build: bool = True) -> ctypes.CDLL:
    """Return the loaded library, building it first if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            if not auto_build:
                raise MpxError(f"{LIB_PATH} not built; run `make lib`")
            build()
        handle = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def tune_lib() -> ctypes.CDLL:
    """The tuning library (after libmpx, whose error state and runtime it shares)."""
    global _tune
    lib()
    with _lock:
        if _tune is None:
            if not TUNE_PATH.exists():
                raise MpxError(f"{TUNE_PATH} not built; run `make tune`")
            handle = ctypes.CDLL(str(TUNE_PATH), mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in _TUNE_SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _tune = handle
    return _tune


def available() -> bool:
    try:
        lib()
        return True
    except (OSError, MpxError):
        return False


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().mpx_last_error()
        raise MpxError(msg.decode() if msg else f"libmpx error {rc}")


def ptr(t: "torch.Tensor") -> int:
    return t.data_ptr()


def stream_of(t: "torch.Tensor") -> int:
    """hipStream_t of the current torch stream on t's device (0 for CPU)."""
    if t.is_cuda:
        return torch.cuda.current_stream(t.device).cuda_stream
    return 0


def f32_array(values) -> ctypes.Array:
    vals = list(values)
    return (ctypes.c_float * max(1, len(vals)))(*vals)


def f64_array(values) -> ctypes.Array:
    vals = list(values)
    return (ctypes.c_double * max(1, len(vals)))(*vals)


def i32_array(values) -> ctypes.Array:
    vals = list(values)
    return (ctypes.c_int * max(1, len(vals)))(*vals)
