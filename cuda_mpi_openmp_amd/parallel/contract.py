"""nccl-contract mode: rehearse the RCCL code paths with ranks sharing one GPU.

RCCL refuses two ranks on one device, so every one-GPU multi-rank rehearsal
used to run with ``MPX_DIST_BACKEND=gloo`` — and then every ``backend ==
"nccl"`` branch of the framework (device-resident scalars, ``barrier(device_ids=…)``,
``broadcast_object_list(device=…)``, the native RCCL tier) stayed unexecuted
until the first real multi-GPU run (missing #1 / weak #3).

``MPX_DIST_CONTRACT=nccl`` closes that gap. The process group is gloo
underneath, but :class:`~.dist.DistContext` reports ``backend = "nccl"``, so
the framework takes exactly the branches it takes on an 8-GPU node, and a thin
wrapper installed over ``torch.distributed`` enforces RCCL's device contract on
every collective of the default group:

* every tensor handed to ``all_reduce`` / ``all_gather`` / ``broadcast`` /
  ``batch_isend_irecv`` must live on the rank's own GPU — a host tensor (or one
  on another device) raises :class:`ContractError` naming the call site;
* ``barrier`` must name the rank's device in ``device_ids`` and the object
  collectives must pass ``device=`` the rank's device when they pass one;
* the checked tensors are then forwarded host-staged to gloo (D2H, gloo op,
  H2D), so results are the ones RCCL would produce.

The native RCCL tier is replaced by :class:`ContractNativeComm`, which runs the
same plans (grouped send/recv lists, in-place all-reduce) with the same checks:
a host tensor reaching a native-comm call fails too.

Subgroups (the gloo control-plane group of ``parallel/peer.py``) are CPU by
design and pass through untouched. There is no reference counterpart (the
reference has no distributed code: SURVEY §2.6); SURVEY §7.4 item 7 asks for a
fake comm backend that makes the multi-GPU tier testable without the GPUs.
"""

from __future__ import annotations

import os
import traceback
from typing import List, Optional

import torch
import torch.distributed as dist

ENV = "MPX_DIST_CONTRACT"


class ContractError(RuntimeError):
    """A collective received a tensor RCCL could not take."""


def active() -> bool:
    return os.environ.get(ENV, "").lower() == "nccl"


_DEV: Optional[torch.device] = None
_ORIG: dict = {}
_HERE = os.path.abspath(__file__)


def _callsite() -> str:
    """First stack frame outside this module and outside torch."""
    tdir = os.path.dirname(torch.__file__)
    for fr in reversed(traceback.extract_stack()[:-1]):
        f = os.path.abspath(fr.filename)
        if f == _HERE or f.startswith(tdir):
            continue
        return f"{fr.filename}:{fr.lineno} in {fr.name}"
    return "<unknown>"


def _default(group) -> bool:
    return group is None or group is dist.GroupMember.WORLD


def check_tensor(t, what: str) -> None:
    if not isinstance(t, torch.Tensor):
        raise ContractError(f"[nccl contract] {what}: expected a tensor, got {type(t).__name__} "
                            f"(call site {_callsite()})")
    if _DEV is not None and t.device != _DEV:
        raise ContractError(f"[nccl contract] {what}: {tuple(t.shape)} {t.dtype} tensor on {t.device}, but RCCL "
                            f"needs it on this rank's device {_DEV} (call site {_callsite()})")


class _Done:
    """Work handle of an already-completed host-staged op (runs ``post`` once on wait)."""

    def __init__(self, inner=None, post=None):
        self._inner, self._post = inner, post

    def wait(self, timeout=None) -> bool:  # noqa: ARG002 - torch Work signature
        if self._inner is not None:
            self._inner.wait()
            self._inner = None
        if self._post is not None:
            self._post()
            self._post = None
        return True

    def is_completed(self) -> bool:
        return self._inner is None and self._post is None


def _all_reduce(tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):
    if not _default(group):
        return _ORIG["all_reduce"](tensor, op=op, group=group, async_op=async_op)
    check_tensor(tensor, "all_reduce")
    h = tensor.cpu()
    _ORIG["all_reduce"](h, op=op)
    tensor.copy_(h)
    return _Done() if async_op else None


def _all_gather(tensor_list, tensor, group=None, async_op=False):
    if not _default(group):
        return _ORIG["all_gather"](tensor_list, tensor, group=group, async_op=async_op)
    check_tensor(tensor, "all_gather (input)")
    for i, t in enumerate(tensor_list):
        check_tensor(t, f"all_gather (output {i})")
    hl = [torch.empty(t.shape, dtype=t.dtype) for t in tensor_list]
    _ORIG["all_gather"](hl, tensor.cpu())
    for t, h in zip(tensor_list, hl):
        t.copy_(h)
    return _Done() if async_op else None


def _broadcast(tensor, src=None, group=None, async_op=False, **kw):
    if not _default(group):
        return _ORIG["broadcast"](tensor, src=src, group=group, async_op=async_op, **kw)
    check_tensor(tensor, "broadcast")
    h = tensor.cpu()
    _ORIG["broadcast"](h, src=src, **kw)
    tensor.copy_(h)
    return _Done() if async_op else None


def _check_obj_device(device, what: str) -> None:
    if device is not None and _DEV is not None and torch.device(device) != _DEV:
        raise ContractError(f"[nccl contract] {what}: device={device}, but RCCL serialises objects through "
                            f"this rank's device {_DEV} (call site {_callsite()})")


def _broadcast_object_list(object_list, src=None, group=None, device=None, **kw):
    if not _default(group):
        return _ORIG["broadcast_object_list"](object_list, src=src, group=group, device=device, **kw)
    _check_obj_device(device, "broadcast_object_list")
    return _ORIG["broadcast_object_list"](object_list, src=src, **kw)


def _all_gather_object(object_list, obj, group=None):
    return _ORIG["all_gather_object"](object_list, obj, group=group)


def _barrier(group=None, async_op=False, device_ids=None):
    if not _default(group):
        return _ORIG["barrier"](group=group, async_op=async_op)
    if _DEV is not None and _DEV.type == "cuda" and device_ids != [_DEV.index]:
        raise ContractError(f"[nccl contract] barrier: device_ids={device_ids}, expected [{_DEV.index}] so RCCL "
                            f"synchronises on this rank's device (call site {_callsite()})")
    return _ORIG["barrier"](async_op=async_op)


def _batch_isend_irecv(p2p_op_list):
    if not p2p_op_list or not all(_default(o.group) for o in p2p_op_list):
        return _ORIG["batch_isend_irecv"](p2p_op_list)
    host, posts = [], []
    for i, o in enumerate(p2p_op_list):
        send = o.op in (dist.isend, getattr(dist, "send", None))
        check_tensor(o.tensor, f"batch_isend_irecv ({'send' if send else 'recv'} #{i}, peer {o.peer})")
        h = o.tensor.cpu() if send else torch.empty(o.tensor.shape, dtype=o.tensor.dtype)
        host.append(dist.P2POp(o.op, h, o.peer))
        posts.append(None if send else (lambda d=o.tensor, h=h: d.copy_(h)))
    works = _ORIG["batch_isend_irecv"](host)
    return [_Done(w, p) for w, p in zip(works, posts)]


_WRAPPERS = {"all_reduce": _all_reduce, "all_gather": _all_gather, "broadcast": _broadcast,
             "broadcast_object_list": _broadcast_object_list, "all_gather_object": _all_gather_object,
             "barrier": _barrier, "batch_isend_irecv": _batch_isend_irecv}


def install(device: torch.device) -> None:
    """Wrap the torch.distributed collectives (idempotent; the device is the rank's own)."""
    global _DEV
    _DEV = torch.device(device)
    for name, fn in _WRAPPERS.items():
        if name not in _ORIG:
            _ORIG[name] = getattr(dist, name)
            setattr(dist, name, fn)


def uninstall() -> None:
    global _DEV
    for name, fn in _ORIG.items():
        setattr(dist, name, fn)
    _ORIG.clear()
    _DEV = None


class ContractNativeComm:
    """Stand-in for :class:`~.native_comm.NativeComm` under the contract: the
    same plan / all-reduce interface, every tensor checked, host-staged over
    the gloo group (the native RCCL tier cannot exist with ranks sharing a GPU)."""

    def __init__(self, rank: int, world: int, device: torch.device):
        self.rank, self.world, self.device = rank, world, device
        self.handle = True

    @classmethod
    def create(cls, ctx) -> Optional["ContractNativeComm"]:
        if os.environ.get("MPX_NATIVE_COMM", "1") == "0":
            return None
        return cls(ctx.rank, ctx.world, ctx.device)

    def size(self) -> int:
        return self.world

    def _run(self, plan) -> None:
        ops: List = []
        for i in range(plan.n):
            t = plan.keep[i]
            check_tensor(t, f"native p2p ({'send' if plan.kind[i] == 0 else 'recv'} #{i}, peer {plan.peer[i]})")
            ops.append(dist.P2POp(dist.isend if plan.kind[i] == 0 else dist.irecv, t, int(plan.peer[i])))
        for w in _batch_isend_irecv(ops):
            w.wait()

    def p2p_start(self, plan, stream=None) -> None:  # noqa: ARG002 - NativeComm signature
        self._run(plan)

    def p2p(self, plan, stream=None) -> None:  # noqa: ARG002
        self._run(plan)

    def p2p_wait(self, stream=None) -> None:  # noqa: ARG002
        pass

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        check_tensor(t, "native all_reduce_")
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        return _all_reduce(t, op=rop) or t

    def check(self) -> None:
        pass

    def comm_stream(self):
        return torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None

    def abort(self) -> None:
        self.handle = None

    def close(self) -> None:
        self.handle = None
