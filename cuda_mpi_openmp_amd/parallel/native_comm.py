"""Native RCCL communicator of libmpx (``native/src/core/comm.cpp``).

torch.distributed pays per operation for Work objects, CUDA events and
Python dispatch — 60-90 us of host time per halo exchange on MI355X, more
than a whole 4096^2 convolution. The native tier does the same RCCL calls
from C: ``p2p`` queues a grouped send/recv list in order on the caller's
stream; ``p2p_start``/``p2p_wait`` fork it onto a comm stream and join it back
for overlap with independent work.

Creation is collective and defensive, because a communicator that fails on
one rank would hang the others in ``ncclCommInitRank``:

1. every rank binds the RCCL torch loaded (``mpx_comm_load``);
2. a torch all-reduce(MIN) agrees that every rank could — otherwise all ranks
   stay on torch.distributed;
3. rank 0's unique id is broadcast over torch.distributed, all ranks init;
4. a ring self-test (send own rank to both neighbours, receive theirs) runs on
   the new communicator and a second agreement keeps it only if every rank
   received the right values.

``MPX_NATIVE_COMM=0`` disables the tier.
"""

from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import _native

_DTYPES = {torch.float64: 0, torch.float32: 1, torch.int32: 2, torch.uint64: 3}
_OPS = {"sum": 0, "max": 1, "min": 2}


def rccl_path() -> str:
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


class P2PPlan:
    """A fixed list of (kind, tensor view, peer) ops as C arrays (kind 0 send, 1 recv)."""

    def __init__(self, ops: Sequence[Tuple[int, torch.Tensor, int]]):
        n = len(ops)
        for _, t, _ in ops:
            if not t.is_contiguous():
                raise ValueError("p2p buffers must be contiguous")
        self.n = n
        self.kind = (ctypes.c_int * max(n, 1))(*[k for k, _, _ in ops])
        self.ptr = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for _, t, _ in ops])
        self.bytes = (ctypes.c_int64 * max(n, 1))(*[t.numel() * t.element_size() for _, t, _ in ops])
        self.peer = (ctypes.c_int * max(n, 1))(*[p for _, _, p in ops])
        self.keep = [t for _, t, _ in ops]  # views keep their storage alive


class NativeComm:
    def __init__(self, handle: ctypes.c_void_p, rank: int, world: int, device: torch.device):
        self.handle = handle
        self.rank = rank
        self.world = world
        self.device = device
        self._L = _native.lib()

    def size(self) -> int:
        """World size as the RCCL communicator itself reports it (ncclCommCount)."""
        return int(self._L.mpx_comm_size(self.handle))

    # ------------------------------------------------------------ creation
    @classmethod
    def create(cls, ctx) -> Optional["NativeComm"]:
        """Collective: every rank of ``ctx`` must call it. None -> stay on torch."""
        if os.environ.get("MPX_NATIVE_COMM", "1") == "0":
            return None
        if ctx.device.type != "cuda" or ctx.backend != "nccl" or not dist.is_initialized():
            return None
        L = _native.lib()
        ok = L.mpx_comm_load(rccl_path().encode()) == 0
        if not _agree(ok, ctx):
            return None
        idbuf = ctypes.create_string_buffer(512)
        if ctx.rank == 0:
            nb = L.mpx_comm_unique_id(idbuf, 512)
            payload = idbuf.raw[:nb] if nb > 0 else b""
        else:
            payload = None
        box = [payload]
        dist.broadcast_object_list(box, src=0, device=ctx.device)
        uid = box[0]
        if not _agree(bool(uid), ctx):
            return None
        h = ctypes.c_void_p()
        ok = L.mpx_comm_init(ctypes.byref(h), ctx.world, ctx.rank, uid, len(uid), ctx.device.index) == 0
        if not _agree(ok, ctx):
            if ok:
                L.mpx_comm_destroy(h)
            return None
        comm = cls(h, ctx.rank, ctx.world, ctx.device)
        good = comm.self_test()
        if not _agree(good, ctx):
            comm.close()
            return None
        return comm

    def self_test(self) -> bool:
        """Ring exchange of rank ids with both neighbours (self when world == 1)."""
        try:
            r, w = self.rank, self.world
            nxt, prv = (r + 1) % w, (r - 1) % w
            send = torch.full((2,), r, dtype=torch.int32, device=self.device)
            recv = torch.full((2,), -1, dtype=torch.int32, device=self.device)
            plan = P2PPlan([(0, send[0:1], nxt), (0, send[1:2], prv), (1, recv[0:1], prv), (1, recv[1:2], nxt)])
            s = torch.cuda.current_stream(self.device)
            self.p2p_start(plan, s)          # forked onto the comm stream
            self.p2p_wait(s)
            got_forked = recv.clone()
            recv.fill_(-1)
            self.p2p(plan, s)                # in order on the caller's stream
            red = torch.tensor([r + 1.0], dtype=torch.float64, device=self.device)
            self.all_reduce_(red, "sum")
            torch.cuda.synchronize(self.device)
            return (got_forked.tolist() == [prv, nxt] and recv.tolist() == [prv, nxt]
                    and red.item() == w * (w + 1) / 2)
        except Exception:  # noqa: BLE001 - any failure means "do not use"
            return False

    # ------------------------------------------------------------ operations
    def p2p_start(self, plan: P2PPlan, stream: Optional[torch.cuda.Stream] = None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _native.check(self._L.mpx_comm_p2p_start(self.handle, plan.n, plan.kind, plan.ptr, plan.bytes, plan.peer,
                                                 s.cuda_stream))

    def p2p(self, plan: P2PPlan, stream: Optional[torch.cuda.Stream] = None) -> None:
        """The exchange in order on ``stream`` (no second queue, no events)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _native.check(self._L.mpx_comm_p2p(self.handle, plan.n, plan.kind, plan.ptr, plan.bytes, plan.peer,
                                           s.cuda_stream))

    def p2p_wait(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _native.check(self._L.mpx_comm_p2p_wait(self.handle, s.cuda_stream))

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if not t.is_contiguous() or t.dtype not in _DTYPES:
            raise ValueError("all_reduce_ needs a contiguous f64/f32/i32/u64 tensor")
        s = torch.cuda.current_stream(self.device)
        _native.check(self._L.mpx_comm_allreduce(self.handle, t.data_ptr(), t.data_ptr(), t.numel(),
                                                 _DTYPES[t.dtype], _OPS[op], s.cuda_stream))
        return t

    def check(self) -> None:
        _native.check(self._L.mpx_comm_check(self.handle))

    def comm_stream(self) -> torch.cuda.Stream:
        """The communicator's own (highest-priority) stream as a torch stream."""
        if getattr(self, "_cs", None) is None:
            self._cs = torch.cuda.ExternalStream(self._L.mpx_comm_stream(self.handle), device=self.device)
        return self._cs

    def abort(self) -> None:
        """ncclCommAbort: unblock and free a communicator whose peers are gone."""
        if self.handle:
            self._L.mpx_comm_abort(self.handle)

    def close(self) -> None:
        if self.handle:
            self._L.mpx_comm_destroy(self.handle)
            self.handle = None


def _agree(ok: bool, ctx) -> bool:
    """True only if every rank passes ``ok`` (all-reduce MIN over torch.distributed)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def plan_from_p2p_ops(ops: List[dist.P2POp]) -> P2PPlan:
    """Convert torch P2POp descriptors into a native plan (same semantics)."""
    out = []
    for o in ops:
        kind = 0 if o.op in (dist.isend, getattr(dist, "send", None)) else 1
        out.append((kind, o.tensor, o.peer))
    return P2PPlan(out)
