"""Process-group bootstrap: one process per GPU over torch.distributed.

On ROCm the ``nccl`` backend IS RCCL, which moves halo rows and reductions
over the xGMI point-to-point links between MI355X GPUs. CPU runs (tests, the
container without a GPU) use ``gloo`` with the same code path. Rendezvous comes
from the standard torchrun environment (RANK, WORLD_SIZE, LOCAL_RANK,
MASTER_ADDR, MASTER_PORT); there is no MPI anywhere (the reference has none
either — its name promises MPI, its code has none: SURVEY §0).
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, Optional

import torch
import torch.distributed as dist

from . import contract as _contract


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    native: Optional[Any] = None  # NativeComm (libmpx RCCL tier) when every rank could create it

    @property
    def is_distributed(self) -> bool:
        return self.world > 1 and dist.is_available() and dist.is_initialized()

    @property
    def up(self) -> Optional[int]:
        """Neighbour holding the rows above this rank's slab."""
        return self.rank - 1 if self.rank > 0 else None

    @property
    def down(self) -> Optional[int]:
        """Neighbour holding the rows below this rank's slab."""
        return self.rank + 1 if self.rank + 1 < self.world else None

    def barrier(self) -> None:
        if self.is_distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


_CTX: Optional[DistContext] = None

VISIBILITY_VARS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def select_device(local_rank: int, local_world: Optional[int], ndev: int, env=None) -> Optional[int]:
    """The device index this rank drives, or None when node-local ranks would
    silently share GPUs (decide on node-local values, never on the
    global WORLD_SIZE, so multi-node jobs pass).

    * local_world <= ndev (or unknown and local_rank < ndev): device local_rank;
    * the launcher isolated devices per rank (a visibility variable set and
      fewer devices than node-local ranks, e.g. HIP_VISIBLE_DEVICES=<rank>):
      every rank sees its own GPU(s) from index 0 — device local_rank % ndev
      (0 for one GPU per rank). Ranks that were all handed the SAME GPU (a
      job-level restriction such as ROCR_VISIBLE_DEVICES=0,1,2,3 under 8
      local ranks) are caught by :func:`init` itself, which gathers every
      rank's (host, PCI id) and refuses duplicates;
    * otherwise (not isolated, more node-local ranks than devices): None.
    """
    env = os.environ if env is None else env
    if ndev <= 0:
        return None
    lw = local_world if local_world is not None else local_rank + 1
    if lw <= ndev:
        return local_rank
    if any(env.get(v, "").strip() for v in VISIBILITY_VARS):
        return local_rank % ndev
    return None


def init(device: str = "auto", backend: Optional[str] = None, timeout_s: float = 300.0) -> DistContext:
    """Initialise (once) from the torchrun environment.

    device: "cuda", "cpu" or "auto" (cuda when available). A single process
    without RANK/WORLD_SIZE in the environment gets a world of one and no
    process group.
    """
    global _CTX
    if _CTX is not None:
        return _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_cuda = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
    contract = _contract.active()
    rehearsal = contract or (backend or os.environ.get("MPX_DIST_BACKEND")) == "gloo"
    if use_cuda:
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError("device='cuda' requested but no GPU is visible")
        lw_env = os.environ.get("LOCAL_WORLD_SIZE")
        idx = select_device(local_rank, int(lw_env) if lw_env else None, ndev)
        if idx is None:
            if not rehearsal:
                # node-local ranks would silently share devices: refuse, as the
                # launcher does before spawning
                import sys

                print(f"[dist] {lw_env or local_rank + 1} ranks on this node (LOCAL_RANK={local_rank}) but only "
                      f"{ndev} GPU(s) are usable in this process; refusing to put several ranks on one device "
                      f"(MPX_DIST_CONTRACT=nccl or MPX_DIST_BACKEND=gloo rehearse that)", file=sys.stderr)
                raise SystemExit(2)
            idx = local_rank % ndev
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
        # the compute stream pair before any communicator creates its streams:
        # they get hardware queues of their own (utils/streams.py)
        from ..utils.streams import compute_streams, host_wait_policy

        host_wait_policy(dev)  # MPX_HIP_WAIT: how host syncs detect completion
        compute_streams(dev, 2)
    else:
        dev = torch.device("cpu")
    if backend is None:
        # MPX_DIST_BACKEND=gloo: control plane over gloo, e.g. to rehearse several
        # ranks on one GPU (RCCL refuses two ranks per device);
        # MPX_DIST_CONTRACT=nccl: the same rehearsal through the nccl code paths
        # (parallel/contract.py)
        backend = "nccl" if contract else (os.environ.get("MPX_DIST_BACKEND") or ("nccl" if use_cuda else "gloo"))
    ctx = DistContext(rank=rank, world=world, local_rank=local_rank, device=dev, backend=backend)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend="gloo" if contract else backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if use_cuda and backend == "nccl" and not contract:
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    if world > 1 and use_cuda and not rehearsal:
        check_distinct_devices(ctx)
    if world > 1 and contract:
        _contract.install(dev)
        ctx.native = _contract.ContractNativeComm.create(ctx) if use_cuda else None
    elif world > 1 and use_cuda and backend == "nccl":
        from .native_comm import NativeComm  # collective: every rank runs init()

        ctx.native = NativeComm.create(ctx)
    _CTX = ctx
    return ctx


def device_pci(dev: torch.device) -> str:
    """PCI location of a GPU ("dddd:bb:dd"), or "cpu"."""
    if dev.type != "cuda":
        return "cpu"
    p = torch.cuda.get_device_properties(dev)
    bus = getattr(p, "pci_bus_id", None)
    if bus is None:
        return f"cuda:{dev.index}"
    return f"{getattr(p, 'pci_domain_id', 0):04x}:{bus:02x}:{getattr(p, 'pci_device_id', 0):02x}"


def check_distinct_devices(ctx: DistContext) -> None:
    """Collective: every rank's (host, GPU PCI id); SystemExit(2) on every
    rank when two ranks of one host drive the same GPU — whatever the backend
    or caller (RCCL would refuse later, gloo never)."""
    import socket
    import sys

    mine = (socket.gethostname(), device_pci(ctx.device))
    every = [None] * ctx.world
    dist.all_gather_object(every, mine)
    seen: dict = {}
    dups = []
    for r, key in enumerate(every):
        if key in seen:
            dups.append((seen[key], r, key))
        seen.setdefault(key, r)
    if dups:
        if ctx.rank == 0:
            print(f"[dist] ranks share a GPU: {', '.join(f'{a} and {b} on {k[0]} {k[1]}' for a, b, k in dups)}; "
                  f"refusing (MPX_DIST_BACKEND=gloo or MPX_DIST_CONTRACT=nccl rehearse several ranks per GPU)",
                  file=sys.stderr)
        dist.destroy_process_group()
        raise SystemExit(2)


def shutdown() -> None:
    global _CTX
    if _CTX is not None and _CTX.native is not None:
        if _CTX.device.type == "cuda":
            torch.cuda.synchronize(_CTX.device)
        _CTX.native.close()
        _CTX.native = None
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _contract.uninstall()
    _CTX = None


def context() -> DistContext:
    return _CTX if _CTX is not None else DistContext()
