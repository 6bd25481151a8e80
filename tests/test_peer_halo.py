"""One-sided halo transport (parallel/peer.py): neighbour slabs IPC-mapped and
read by the conv kernel over xGMI.

The GPU tests run 2 and 3 ranks as separate processes on ONE MI355X (IPC works
between processes on the same device; RCCL would refuse two ranks on one GPU,
so the control plane is gloo). The decomposed result must be bit-identical to
the single-process convolution of the whole image.
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


def _peer_worker(rank, world, port, h, w, filt, errq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
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


@pytest.mark.gpu
@pytest.mark.parametrize("world,filt", [(2, "sobel5"), (3, "roberts"), (3, "sobel5_dense")])
def test_peer_halo_ranks_share_one_gpu(gpu, world, filt):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    h, w = 301, 258
    procs = [ctx.Process(target=_peer_worker, args=(r, world, port, h, w, filt, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_peer_halo_not_for_single_rank_or_cpu():
    ctx = parallel.DistContext()
    s = parallel.Slab(10, 1, 0, 2, 2)
    assert try_peer_halo(ctx, s, torch.zeros((10, 4, 4), dtype=torch.uint8)) is None
