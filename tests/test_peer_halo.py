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


def _jacobi_peer_ckpt_worker(rank, world, port, rows, cols, ckdir, errq):
    """Graph replays, then a checkpoint reload that flips the u/u_new parity
    (saved at an odd iteration, reloaded while u is the even-iteration
    buffer), then graph replays again: a cycle graph captured before the
    reload must not be replayed with the old neighbour-parity descriptor."""
    try:
        from cuda_mpi_openmp_amd.models import SlabJacobi

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        ctx = parallel.init(device="cuda", backend="gloo")
        g = torch.Generator().manual_seed(5)
        field = torch.rand((rows, cols - 2), generator=g, dtype=torch.float64)

        def setup(sol):
            sol.set_boundary(top=1.0, left=0.5, right=0.25)
            s = sol.slab
            sol.u[1:1 + s.rows, 1:-1] = field[s.row0:s.row0 + s.rows].to(sol.u.device)
            sol.un.copy_(sol.u)
            sol._halos_valid = False

        sol = SlabJacobi(ctx, rows, cols, dtype=torch.float64, check_every=5, halo="peer")
        assert sol.transport == "xgmi-peer-signalled", sol.transport
        setup(sol)
        sol.run(10, graph=True)      # captures the cycle graph starting at an even iteration
        sol.run(3)
        prefix = os.path.join(ckdir, "ck")
        sol.save_checkpoint(prefix)  # iteration 13
        sol.run(13)                  # iteration 26: u is the even-iteration buffer
        sol.load_checkpoint(prefix)  # back to 13 with the parity flipped
        sol.run(12, graph=True)      # 2 eager steps, then cycle graphs again
        torch.cuda.synchronize()
        sol.check_peer()
        got = sol.gather()
        sol.close()
        if ctx.rank == 0:
            ref = SlabJacobi(parallel.DistContext(device=ctx.device), rows, cols, dtype=torch.float64, check_every=5)
            setup(ref)
            ref.run(25)
            assert torch.equal(got.cpu(), ref.owned.cpu()), "graph replay after a parity-flipping reload differs"
        parallel.shutdown()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


def _stream_peer_worker(rank, world, port, h, w, filt, steps, errq, fused=True):
    """Streaming conv on GPU ranks sharing one device: the halo exchange fused
    into the band kernel (edge waves wait, read the neighbours' mailboxes,
    publish; one launch per step) for aligned widths, else the device-signalled
    fetch kernel; N ranks == one device running the same frame sequence on the
    whole image."""
    try:
        from cuda_mpi_openmp_amd.models.edge import stream_reference

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        if not fused:
            os.environ["MPX_STREAM_FUSED"] = "0"
        ctx = parallel.init(device="cuda", backend="gloo")
        det = SlabEdgeDetector(ctx, h, w, filt, halo="peer", stream=True)
        want = "xgmi-peer-fused" if (fused and w % 4 == 0) else "xgmi-peer-signalled-fetch"
        assert det.transport == want, (det.transport, want)
        s = det.slab
        for seed, k in ((21, steps), (22, steps + 3)):
            full = _img(h, w, seed)
            det.load(full[s.row0:s.row0 + s.rows].to(ctx.device))
            for _ in range(k):
                det.step()
            torch.cuda.synchronize()
            det.check_stream()
            got = parallel.gather_slabs(det.stream_out.contiguous(), s, ctx)
            if ctx.rank == 0:
                ref = stream_reference(full.to(ctx.device), filt, k).cpu()
                assert torch.equal(got.cpu(), ref), f"streaming peer conv differs ({filt}, {k} steps)"
            # this rank's last step against the CPU reference on the halo rows it read
            buf = det.halo_filled().cpu()
            exp = torch.empty((s.rows, w, 4), dtype=torch.uint8)
            ops.conv_rows(buf, exp, det.filter, src_row0=s.own_offset, out_row0=0, oy0=0, oy1=s.rows,
                          y_lo=s.y_lo, y_hi=s.y_hi)
            assert torch.equal(exp, det.stream_out.cpu()), "last step differs from the CPU on its halo rows"
            ctx.barrier()
        det.close()
        parallel.shutdown()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


def _fallback_worker(rank, world, port, kind, env, errq):
    """An injected set-up fault on one rank: every rank must fall back to the
    two-sided transport (here torch.distributed over gloo) and still produce
    the single-process result."""
    try:
        from cuda_mpi_openmp_amd.models import SlabJacobi

        os.environ.update(env)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        ctx = parallel.init(device="cuda", backend="gloo")
        if kind == "conv":
            h, w = 61, 64
            det = SlabEdgeDetector(ctx, h, w, "sobel5", halo="auto")
            assert det.transport == "torch.distributed", det.transport
            full = _img(h, w, 3)
            s = det.slab
            det.load(full[s.row0:s.row0 + s.rows].to(ctx.device))
            got = parallel.gather_slabs(det.step().cpu(), s, ctx)
            if ctx.rank == 0:
                assert torch.equal(got, ops.conv(full, "sobel5"))
            det.close()
        else:
            sol = SlabJacobi(ctx, 8 * 4 + 5, 132, dtype=torch.float64, check_every=5, halo="auto")
            assert sol.transport == "torch.distributed", sol.transport
            sol.fill(seed=4)
            sol.run(10)
            got = sol.gather()
            if ctx.rank == 0:
                assert got is not None and torch.isfinite(got).all()
        parallel.shutdown()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


def _run_ranks(target, world, *args, timeout=150, **kwargs):
    """Run `world` rank processes; bounded by `timeout` seconds in total. Each
    rank logs its peer set-up phases (MPX_PEER_LOG_DIR); on a timeout the
    ranks are killed and their last phases are reported."""
    import tempfile
    import time

    logdir = tempfile.mkdtemp(prefix="mpx_peer_log_")
    os.environ["MPX_PEER_LOG_DIR"] = logdir  # inherited by the spawned ranks
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, errq), kwargs=kwargs) for r in range(world)]
    for p in procs:
        p.start()
    errs = []
    deadline = time.monotonic() + timeout
    while any(p.is_alive() for p in procs) and time.monotonic() < deadline:
        while not errq.empty():  # drain while waiting: a child blocks at exit until its queue is read
            errs.append(errq.get())
        time.sleep(0.2)
    hung = [r for r, p in enumerate(procs) if p.is_alive()]
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join(10)
    time.sleep(0.2)
    while not errq.empty():
        errs.append(errq.get())

    def tails():
        out = []
        for r in range(world):
            fn = os.path.join(logdir, f"peer_rank{r}.log")
            last = open(fn).read().splitlines()[-3:] if os.path.exists(fn) else ["(no peer phase logged)"]
            out.append(f"rank {r}: " + " | ".join(last))
        return "\n".join(out)

    assert not hung, f"ranks {hung} still running after {timeout} s; last peer phases:\n{tails()}"
    assert not errs, "\n".join(errs) + "\nlast peer phases:\n" + tails()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return logdir


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


@pytest.mark.gpu
def test_jacobi_peer_graph_after_parity_flipping_reload(gpu, tmp_path):
    """re-publishing the peer descriptor drops the captured cycle
    graphs, so replays after a reload read the neighbours' current buffers."""
    _run_ranks(_jacobi_peer_ckpt_worker, 3, 8 * 9 + 5, 132, str(tmp_path))


@pytest.mark.gpu
@pytest.mark.parametrize("world,filt", [(2, "sobel5"), (3, "roberts"), (4, "sobel5_dense"), (8, "sobel5"),
                                        (4, "roberts"), (3, "gauss5")])
def test_stream_peer_equals_one_device(gpu, world, filt):
    """each step's input is the previous step's output,
    so the halo rows change every step; the fused band kernel (aligned widths:
    64, 260) or the signalled fetch kernel (unaligned: 62) orders them on the
    device. Slabs of a few rows up to a few segments."""
    w = {3: 62}.get(world, 64) if filt != "gauss5" else 260
    h = 8 * 6 + 5 if filt != "gauss5" else 8 * 37 + 5
    _run_ranks(_stream_peer_worker, world, h, w, filt, 5)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_stream_peer_fetch_kernel_aligned(gpu, world):
    """The fetch-kernel form (MPX_STREAM_FUSED=0) on an aligned width: the A/B
    partner of the fused form, over the same mailboxes."""
    _run_ranks(_stream_peer_worker, world, 8 * 6 + 5, 64, "sobel5", 5, fused=False)


@pytest.mark.gpu
def test_jacobi_peer_slabs_beyond_2gib(gpu):
    """per-rank u / u_new slabs of 20,000 x 16,384 fp64 (2.6 GB
    each, past the 2 GiB size whose IPC open hung in round 2) keep the
    one-sided transport — only the mailboxes are exported — and stay
    bit-identical to one device."""
    _run_ranks(_jacobi_peer_worker, 2, 40000, 16384, 20, True, timeout=400)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,inject", [("conv", "open_stall@1"), ("conv", "verify_corrupt@0"),
                                         ("jacobi", "probe_corrupt@1"), ("jacobi", "open_stall@0")])
def test_peer_setup_fault_falls_back(gpu, kind, inject):
    """a stalled IPC open (deadline 3 s) or a failing
    kernel-path check on ONE rank makes EVERY rank fall back to the two-sided
    transport within the deadline; results stay exact; the phase log names
    the failure."""
    import time

    t0 = time.monotonic()
    env = {"MPX_PEER_INJECT": inject, "MPX_PEER_OPEN_TIMEOUT": "3"}
    logdir = _run_ranks(_fallback_worker, 3, kind, env, timeout=120)
    assert time.monotonic() - t0 < 110
    logs = "".join(open(os.path.join(logdir, f)).read() for f in os.listdir(logdir))
    want = {"open_stall": "TIMED OUT", "verify_corrupt": "DIFFER", "probe_corrupt": "probe failed"}[inject.split("@")[0]]
    assert want in logs, logs[-2000:]
