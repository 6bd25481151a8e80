"""Time bounds of the one-sided transports' set-up (parallel/peer.py; VERDICT r2
#1): every IPC open and every set-up collective has a deadline, and a stall
turns into an exception that names its phase instead of a hang. CPU only
(gloo); the GPU fallback paths are in tests/test_peer_halo.py."""

import os
import socket
import time
import traceback

import pytest
import torch.multiprocessing as mp

from cuda_mpi_openmp_amd import parallel
from cuda_mpi_openmp_amd.parallel import peer


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_open_bounded_times_out(monkeypatch, tmp_path):
    monkeypatch.setenv("MPX_PEER_INJECT", "open_stall@0")
    monkeypatch.setenv("MPX_PEER_OPEN_TIMEOUT", "0.5")
    monkeypatch.setenv("MPX_PEER_LOG_DIR", str(tmp_path))
    ctx = parallel.DistContext()
    t0 = time.monotonic()
    with pytest.raises(TimeoutError, match="did not return within"):
        peer._open_bounded(ctx, b"\0" * 64, 0, "up")
    assert time.monotonic() - t0 < 3.0
    log = (tmp_path / "peer_rank0.log").read_text()
    assert "ipc open up: start" in log and "TIMED OUT" in log


def test_injection_parser(monkeypatch):
    monkeypatch.setenv("MPX_PEER_INJECT", "open_stall@1, probe_corrupt@3")
    assert peer._injected("open_stall", 1) and peer._injected("probe_corrupt", 3)
    assert not peer._injected("open_stall", 0) and not peer._injected("verify_corrupt", 1)


def _late_worker(rank, world, port, logdir, errq, resq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), MPX_PEER_SETUP_TIMEOUT="2", MPX_PEER_LOG_DIR=logdir)
        ctx = parallel.init(device="cpu")
        peer._setup_group(ctx)  # collective creation, on time
        if rank == 1:
            time.sleep(8.0)     # a rank that stops answering
        t0 = time.monotonic()
        try:
            peer._allgather(ctx, rank, "test: handles")
            resq.put((rank, "ok", time.monotonic() - t0))
        except peer.PeerSetupError as e:
            resq.put((rank, str(e), time.monotonic() - t0))
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


def test_setup_collective_deadline(tmp_path):
    """Rank 1 arrives 8 s late to a set-up exchange with a 2 s deadline: rank 0
    gets a PeerSetupError naming the step within the deadline (no hang)."""
    ctx = mp.get_context("spawn")
    errq, resq = ctx.Queue(), ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_late_worker, args=(r, 2, port, str(tmp_path), errq, resq)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 90
    while len(res) < 2 and time.monotonic() < deadline and errq.empty():
        try:
            r, msg, dt = resq.get(timeout=1.0)
            res[r] = (msg, dt)
        except Exception:  # noqa: BLE001 - queue.Empty
            pass
    for p in procs:
        p.join(15)
        if p.is_alive():
            p.kill()
    assert errq.empty(), errq.get()
    assert 0 in res, res
    msg, dt = res[0]
    assert "test: handles" in msg and "timed out" in msg, msg
    assert dt < 6.0, dt
    assert "all_gather FAILED" in (tmp_path / "peer_rank0.log").read_text()


class _FakeOwn:
    """Stands in for a CUDA slab: try_peer_halo's control plane only asks
    these questions before it maps anything."""
    is_cuda = True

    def is_contiguous(self):
        return True

    def __getitem__(self, i):
        import torch
        return torch.zeros(16, 4, dtype=torch.uint8)

    def element_size(self):
        return 1


class _FakeMailbox:
    kind, nbytes = "fake", 64

    def __init__(self, *a):
        self.freed = False

    def export(self):
        return {"handle": b"x"}

    def free(self):
        self.freed = True


class _FakePeerHalo:
    def __init__(self, ctx, slab, own, mb, every):
        assert len(every) == ctx.world and all(e is not None for e in every)
        self.closed = False

    def publish(self):
        pass

    def verify(self):
        return True

    def close(self, collective=True):
        self.closed = True


def _fallback_vote_worker(rank, world, port, inject, errq, resq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), MPX_PEER_INJECT=inject, MPX_PEER_SETUP_TIMEOUT="20")
        ctx = parallel.init(device="cpu")
        peer.Mailbox, peer.PeerHalo = _FakeMailbox, _FakePeerHalo
        from types import SimpleNamespace

        ph = peer.try_peer_halo(ctx, SimpleNamespace(halo_down=2, halo_up=2), _FakeOwn())
        resq.put((rank, "peer" if ph is not None else "rccl"))
        parallel.shutdown()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


@pytest.mark.parametrize("world,inject,want", [(2, "map_fail@1", "rccl"), (3, "map_fail@0", "rccl"),
                                               (3, "", "peer")])
def test_peer_map_failure_on_one_rank_every_rank_takes_rccl(world, inject, want):
    """VERDICT r5 Next #7: the peer set-up's collective vote (parallel/peer.py
    try_peer_halo) on CPU/gloo with fake mailboxes: one rank whose mapping
    fails (MPX_PEER_INJECT=map_fail@R) makes EVERY rank agree on the RCCL
    fallback; without the fault every rank takes the peer path."""
    ctx = mp.get_context("spawn")
    errq, resq = ctx.Queue(), ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_vote_worker, args=(r, world, port, inject, errq, resq))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 120
    while len(res) < world and time.monotonic() < deadline and errq.empty():
        try:
            r, path = resq.get(timeout=1.0)
            res[r] = path
        except Exception:  # noqa: BLE001 - queue.Empty
            pass
    for p in procs:
        p.join(15)
        if p.is_alive():
            p.kill()
    assert errq.empty(), errq.get()
    assert res == {r: want for r in range(world)}, res
