"""One-sided halo transports (parallel/peer.py): neighbour slabs IPC-mapped
and read by the kernels over xGMI — the conv (static inputs) and the Jacobi
sweep (device-signalled: per-iteration order from completed-iteration words,
no host round trip).

The GPU tests run 2, 3, 4 and 8 ranks as separate processes on ONE MI355X
(IPC works between processes on the same device; RCCL would refuse two ranks
on one GPU, so the control plane is gloo): interior ranks map both
neighbours, as at N = 8 on a node. Global row counts 8k+5 leave uneven slabs.
Decomposed results must be bit-identical to the single-process run.
"""

import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

from cuda_mpi_openmp_amd import ops, parallel
from cuda_mpi_openmp_amd.models import SlabEdgeDetector
from cuda_mpi_openmp_amd.parallel.peer import try_peer_halo


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _img(h, w, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (h, w, 4), dtype=torch.uint8, generator=g)


def _peer_worker(rank, world, port, h, w, filt, errq, band=False):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        if band:  # the band kernel on these small slabs (its halo rows then come over IPC)
            from cuda_mpi_openmp_amd import _native

            _native.lib().mpx_conv_set_band_min(0)
        ctx = parallel.init(device="cuda", backend="gloo")
        det = SlabEdgeDetector(ctx, h, w, filt, halo="peer")
        assert det.transport == "xgmi-peer", det.transport
        s = det.slab
        for seed in (1, 2):  # a second load must be picked up by the neighbours' next step
            full = _img(h, w, seed)
            det.load(full[s.row0:s.row0 + s.rows].to(ctx.device))
            for _ in range(3):
                out = det.step()
            torch.cuda.synchronize()
            got = parallel.gather_slabs(out.cpu(), s, ctx)
            if ctx.rank == 0:
                assert torch.equal(got, ops.conv(full, filt)), f"peer-halo conv differs ({filt}, seed {seed})"
            # the halo rows the kernel read, copied in: CPU reference on the same buffer
            buf = det.halo_filled().cpu()
            ref = torch.empty((s.rows, w, 4), dtype=torch.uint8)
            ops.conv_rows(buf, ref, det.filter, src_row0=s.own_offset, out_row0=0, oy0=0, oy1=s.rows,
                          y_lo=s.y_lo, y_hi=s.y_hi)
            assert torch.equal(ref, out.cpu())
            ctx.barrier()
        det.close()
        parallel.shutdown()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


def _jacobi_peer_worker(rank, world, port, rows, cols, iters, fp64, errq, graph=False):
    try:
        from cuda_mpi_openmp_amd.models import SlabJacobi

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        ctx = parallel.init(device="cuda", backend="gloo")
        dt = torch.float64 if fp64 else torch.float32
        g = torch.Generator().manual_seed(3)
        field = torch.rand((rows, cols - 2), generator=g, dtype=torch.float64).to(dt)

        def setup(sol):
            sol.set_boundary(top=1.0, left=0.5, right=0.25)
            s = sol.slab
            sol.u[1:1 + s.rows, 1:-1] = field[s.row0:s.row0 + s.rows].to(sol.u.device)
            sol.un.copy_(sol.u)
            sol._halos_valid = False

        sol = SlabJacobi(ctx, rows, cols, dtype=dt, check_every=10, halo="peer")
        assert sol.transport == "xgmi-peer-signalled", sol.transport
        setup(sol)
        sol.run(iters, graph=graph)  # graph: replays of one captured residual cycle
        torch.cuda.synchronize()
        sol.check_peer()
        got = sol.gather()
        res = sol.last_residual
        # a restart from the gathered state must continue seamlessly (re-publish)
        sol.run(10)
        got2 = sol.gather()
        sol.close()
        if ctx.rank == 0:
            ref = SlabJacobi(parallel.DistContext(device=ctx.device), rows, cols, dtype=dt, check_every=10)
            setup(ref)
            ref.run(iters)
            assert torch.equal(got.cpu(), ref.owned.cpu()), "peer-signalled Jacobi differs from one rank"
            assert res == ref.last_residual
            ref.run(10)
            assert torch.equal(got2.cpu(), ref.owned.cpu())
        parallel.shutdown()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


def _run_ranks(target, world, *args, timeout=240, **kwargs):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, errq), kwargs=kwargs) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.gpu
@pytest.mark.parametrize("world,filt", [(2, "sobel5"), (3, "roberts"), (3, "sobel5_dense"), (4, "sobel5"),
                                        (8, "sobel5")])
def test_peer_halo_ranks_share_one_gpu(gpu, world, filt):
    h = 301 if world <= 3 else 8 * 37 + 5  # 8k+5: uneven slabs at 4 and 8 ranks
    _run_ranks(_peer_worker, world, h, 258, filt)


@pytest.mark.gpu
@pytest.mark.parametrize("world,filt", [(2, "sobel5"), (3, "roberts"), (4, "sobel3"), (8, "sobel5_dense")])
def test_peer_halo_band_kernel(gpu, world, filt):
    """Aligned width (260 = one full 256-column strip + a partial one): the band
    kernel reads its neighbours' halo rows over IPC (RowSrc), boundary segments
    dispatched first."""
    h = 301 if world <= 3 else 8 * 37 + 5
    _run_ranks(_peer_worker, world, h, 260, filt, band=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world,fp64", [(2, True), (3, False), (4, True), (8, True)])
def test_jacobi_peer_signalled_equals_one_rank(gpu, world, fp64):
    """100 iterations of the device-signalled one-sided halo sweep (plus a
    10-iteration restart) are bit-identical to a single-rank run, residual
    included; 8k+5 global rows."""
    _run_ranks(_jacobi_peer_worker, world, 8 * 9 + 5, 132 if fp64 else 136, 100, fp64)


def test_peer_halo_not_for_single_rank_or_cpu():
    ctx = parallel.DistContext()
    s = parallel.Slab(10, 1, 0, 2, 2)
    assert try_peer_halo(ctx, s, torch.zeros((10, 4, 4), dtype=torch.uint8)) is None


@pytest.mark.gpu
def test_jacobi_peer_signalled_hip_graph(gpu):
    """The peer sweep reads its iteration from device memory, so replays of one
    captured residual cycle stay correct: bit-identical to one rank."""
    _run_ranks(_jacobi_peer_worker, 2, 8 * 9 + 5, 132, 100, True, graph=True)
