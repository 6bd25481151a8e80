"""Native RCCL tier (native/src/core/comm.cpp).

Multi-rank RCCL needs one GPU per rank (RCCL refuses two ranks on one
device), so on a one-GPU box the communicator is exercised as a world of one:
creation + ring self-test, grouped send/recv to self (the same code path a
neighbour exchange takes), stream fork/join ordering and all-reduce. The
halo op lists themselves are produced by HaloExchange._ops, which the gloo
multi-process tests (test_distributed_cpu.py) cover at world sizes 2 and 3.
"""

import os
import socket
import time
import types

import pytest
import torch
import torch.distributed as dist

from cuda_mpi_openmp_amd import parallel
from cuda_mpi_openmp_amd.parallel.native_comm import NativeComm, P2PPlan, plan_from_p2p_ops


def test_plan_from_p2p_ops_cpu():
    buf = torch.arange(64, dtype=torch.uint8).reshape(16, 4)
    # P2POp needs a process group; the converter only reads .op/.tensor/.peer
    op = lambda f, t, p: types.SimpleNamespace(op=f, tensor=t, peer=p)  # noqa: E731
    ops = [op(dist.isend, buf[2:4], 1), op(dist.irecv, buf[0:2], 1), op(dist.irecv, buf[14:16], 3)]
    plan = plan_from_p2p_ops(ops)
    assert plan.n == 3
    assert list(plan.kind)[:3] == [0, 1, 1]
    assert list(plan.peer)[:3] == [1, 1, 3]
    assert list(plan.bytes)[:3] == [8, 8, 8]
    assert plan.ptr[0] == buf[2:4].data_ptr() and plan.ptr[2] == buf[14:16].data_ptr()
    with pytest.raises(ValueError):
        P2PPlan([(0, buf[:, 1], 0)])  # non-contiguous view


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def world1(gpu):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    ctx = parallel.DistContext(rank=0, world=1, local_rank=0, device=gpu, backend="nccl")
    comm = NativeComm.create(ctx)
    yield ctx, comm
    if comm is not None:
        torch.cuda.synchronize(gpu)
        comm.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_create_and_self_test(world1):
    ctx, comm = world1
    assert comm is not None, "native RCCL tier unavailable: %r" % parallel.native_comm._native.lib().mpx_last_error()
    assert comm.self_test()
    assert comm._L.mpx_comm_version() > 0
    comm.check()


@pytest.mark.gpu
def test_p2p_self_exchange_rows(world1, gpu):
    """Send two row blocks of a slab buffer to self into the halo rows: the
    same grouped send/recv a neighbour exchange issues."""
    _, comm = world1
    w = 4096
    buf = torch.randint(0, 256, (4 + 100, w, 4), dtype=torch.uint8, device=gpu)
    top, bot = buf[2:4].clone(), buf[100:102].clone()
    plan = P2PPlan([(0, buf[2:4], 0), (1, buf[102:104], 0), (0, buf[100:102], 0), (1, buf[0:2], 0)])
    comm.p2p_start(plan)
    comm.p2p_wait()
    torch.cuda.synchronize(gpu)
    assert torch.equal(buf[102:104], top) and torch.equal(buf[0:2], bot)


@pytest.mark.gpu
def test_p2p_orders_after_queued_work(world1, gpu):
    """start() must see writes queued on the stream before it; work queued
    between start() and wait() overlaps; wait() orders later work after it."""
    _, comm = world1
    n = 1 << 22
    src = torch.zeros(n, dtype=torch.float32, device=gpu)
    dst = torch.empty_like(src)
    src.fill_(3.0)                      # queued before start: must be sent
    plan = P2PPlan([(0, src, 0), (1, dst, 0)])
    comm.p2p_start(plan)
    other = torch.ones(n, device=gpu) * 2  # independent work in the overlap window
    comm.p2p_wait()
    dst.mul_(other)                     # after wait: sees the received values
    torch.cuda.synchronize(gpu)
    assert torch.all(dst == 6.0)


@pytest.mark.gpu
def test_allreduce_world1(world1, gpu):
    _, comm = world1
    t = torch.tensor([1.5, -2.0, 7.0], dtype=torch.float64, device=gpu)
    comm.all_reduce_(t, "max")
    comm.all_reduce_(t, "sum")
    i = torch.arange(5, dtype=torch.int32, device=gpu)
    comm.all_reduce_(i, "min")
    torch.cuda.synchronize(gpu)
    assert t.tolist() == [1.5, -2.0, 7.0] and i.tolist() == list(range(5))


@pytest.mark.gpu
def test_p2p_rejects_bad_peer(world1, gpu):
    _, comm = world1
    x = torch.zeros(4, device=gpu)
    with pytest.raises(parallel.native_comm._native.MpxError):
        comm.p2p_start(P2PPlan([(0, x, 5)]))
    comm.p2p_wait()


@pytest.mark.gpu
def test_p2p_host_overhead(world1, gpu):
    """Host cost of one native exchange (start + wait): the per-step budget of
    the distributed benchmark. Reported, loosely bounded."""
    _, comm = world1
    buf = torch.zeros((8, 4096, 4), dtype=torch.uint8, device=gpu)
    plan = P2PPlan([(0, buf[0:2], 0), (1, buf[4:6], 0), (0, buf[2:4], 0), (1, buf[6:8], 0)])
    for _ in range(20):
        comm.p2p_start(plan)
        comm.p2p_wait()
    torch.cuda.synchronize(gpu)
    n = 500
    t0 = time.perf_counter()
    for _ in range(n):
        comm.p2p_start(plan)
        comm.p2p_wait()
    host_us = (time.perf_counter() - t0) * 1e6 / n
    torch.cuda.synchronize(gpu)
    print(f"native p2p start+wait host cost: {host_us:.1f} us")
    assert host_us < 500


@pytest.mark.gpu
def test_slab_edge_pipelined_world1(world1, gpu):
    """Pipelined SlabEdgeDetector on a world-of-one native communicator: the
    double-buffer / event protocol must give the same image every step."""
    from cuda_mpi_openmp_amd import ops
    from cuda_mpi_openmp_amd.models import SlabEdgeDetector

    ctx, comm = world1
    ctx = parallel.DistContext(rank=0, world=1, local_rank=0, device=gpu, backend="nccl", native=comm)
    det = SlabEdgeDetector(ctx, 512, 384, "sobel5", overlap="pipeline")
    assert det.pipeline and len(det.bufs) == 2
    det.fill_random(seed=3)
    ref = ops.conv(det.own.contiguous(), "sobel5")
    for _ in range(5):
        out = det.step()
        det.finish()
        torch.cuda.synchronize(gpu)
        assert torch.equal(out, ref)
    img = torch.randint(0, 256, (512, 384, 4), dtype=torch.uint8, device=gpu)
    det.load(img)  # drains the comm stream first
    out = det.step()
    det.finish()
    torch.cuda.synchronize(gpu)
    assert torch.equal(out, ops.conv(img, "sobel5"))
