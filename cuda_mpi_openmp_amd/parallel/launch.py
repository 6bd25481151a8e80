"""Self-launch of N ranks (one process per GPU) for scripts run as ``python X --gpus N``.

A benchmark started without a torchrun environment but asked for N > 1 GPUs
must not quietly measure one GPU: :func:`relaunch_if_needed` re-runs the same
script under ``torch.distributed.run`` with N local ranks and returns the
child's exit code, *before* anything in this process initialises HIP (the
launcher only counts devices, which does not create a HIP context on this
image). Inside a rank, :func:`check_world` refuses a WORLD_SIZE that differs
from the requested N.

One-GPU rehearsal: with ``MPX_DIST_BACKEND=gloo`` several ranks may share a
device (control plane over gloo, halos over IPC-mapped peer memory); with
``MPX_DIST_CONTRACT=nccl`` they share it through the framework's RCCL code
paths (``parallel/contract.py``); every other GPU run needs N usable devices
or fails with exit code 2 — here, and again inside each rank
(``parallel/dist.py``).

The reference has no multi-process code at all; this is the
north-star "1/2/4/8 MI355X" launch path.
"""

from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List, Optional, Sequence

EXIT_BAD_WORLD = 2


def in_rank_env() -> bool:
    """True when this process is already one rank of a launched job."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


DRI = "/dev/dri"


def _kfd_gpu_count(root: str = KFD_NODES, dri: str = DRI) -> Optional[int]:
    """GPU agents in the KFD topology (nodes whose gfx_target_version is set;
    CPU nodes report 0) that this process can actually open — read from sysfs,
    no HIP runtime involved. Containers do not namespace sysfs, so a lease of
    one render node still lists every GPU of the host: a node counts only when
    its ``/dev/dri/renderD<drm_render_minor>`` is readable and writable here
    (ADVICE r3). None when the topology is unreadable."""
    try:
        names = os.listdir(root)
    except OSError:
        return None
    n = 0
    for d in names:
        props = {}
        try:
            with open(os.path.join(root, d, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        try:
            if int(props.get("gfx_target_version") or 0) == 0:
                continue
            minor = int(props.get("drm_render_minor", "-1"))
        except ValueError:
            continue
        if minor >= 0 and not os.access(os.path.join(dri, f"renderD{minor}"), os.R_OK | os.W_OK):
            continue
        n += 1
    return n


def _visible_filter(n: int) -> int:
    """Apply the runtime's device-visibility variables to n physical GPUs."""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        toks = [t for t in v.split(",") if t.strip() != ""]
        n = min(n, len(toks)) if v.strip() else 0
    return n


def visible_devices() -> int:
    """GPUs this process would see, counted from the KFD sysfs topology and the
    visibility variables — the launcher never loads or initialises HIP before
    spawning its ranks. Falls back to torch's count only when
    sysfs is unreadable."""
    n = _kfd_gpu_count()
    if n is None:
        import torch

        return int(torch.cuda.device_count())
    return _visible_filter(n)


def launcher_cmd(script: str, argv: Sequence[str], nproc: int, port: Optional[int] = None) -> List[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()), script, *argv]


def relaunch_if_needed(script: str, argv: Sequence[str], gpus: int, device: str) -> Optional[int]:
    """None when this process should run the work itself (already a rank, or
    N == 1); otherwise launch N ranks of ``script argv`` and return their exit
    code (non-zero when N devices are not available)."""
    if in_rank_env() or gpus <= 1:
        return None
    rehearsal = os.environ.get("MPX_DIST_BACKEND") == "gloo" or os.environ.get("MPX_DIST_CONTRACT") == "nccl"
    if device != "cpu" and not rehearsal:
        ndev = visible_devices()
        if device == "cuda" and ndev == 0:
            print("[launch] --device cuda but no GPU is visible", file=sys.stderr)
            return EXIT_BAD_WORLD
        if ndev and ndev < gpus:
            print(f"[launch] --gpus {gpus} requested but only {ndev} GPU(s) are visible; refusing to run fewer "
                  f"ranks (set MPX_DIST_BACKEND=gloo to rehearse {gpus} ranks on shared devices)", file=sys.stderr)
            return EXIT_BAD_WORLD
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // gpus)))
    r = subprocess.run(launcher_cmd(script, argv, gpus), env=env)
    return r.returncode


def check_world(gpus: int, world: int) -> None:
    """Inside a rank: the launched world must be exactly the requested one."""
    if gpus != world:
        print(f"[launch] --gpus {gpus} but WORLD_SIZE={world}; refusing to report a different GPU count",
              file=sys.stderr)
        raise SystemExit(EXIT_BAD_WORLD)
