"""Multi-process decomposition tests on CPU (gloo backend, world sizes 2, 3, 4
and 8): every distributed workload must reproduce the single-process result
exactly. At 8 ranks every interior rank has both neighbours (the N = 8 node
topology); global row counts of 8k+5 leave uneven slabs."""

import os
import socket
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from cuda_mpi_openmp_amd import ops, parallel
from cuda_mpi_openmp_amd.models import SlabEdgeDetector, SlabJacobi, SlabPixelClassifier, ShardedVectorSub
from cuda_mpi_openmp_amd.models.classifier import class_points_for, split_rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn_name, args, errq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        torch.set_num_threads(1)
        ctx = parallel.init(device="cpu")
        globals()[fn_name](ctx, *args)
        parallel.shutdown()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")


def run_world(world, fn_name, *args):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn_name, args, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _img(h, w, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (h, w, 4), dtype=torch.uint8, generator=g)


# ---------------------------------------------------------------- workers
def conv_worker(ctx, h, w, filt, overlap, outdir):
    full = _img(h, w, 5)
    det = SlabEdgeDetector(ctx, h, w, filt, overlap=overlap)
    s = det.slab
    det.load(full[s.row0:s.row0 + s.rows])
    out = det.step()
    got = parallel.gather_slabs(out, s, ctx)
    if ctx.rank == 0:
        ref = ops.conv(full, filt)
        assert torch.equal(got, ref), "decomposed conv differs from the single-process result"
        torch.save(got, os.path.join(outdir, f"conv_{filt}.pt"))


def stream_worker(ctx, h, w, filt, steps):
    """Streaming conv (input = previous step's output): N ranks == one device
    running the same frame sequence on the whole image; then a reload."""
    from cuda_mpi_openmp_amd.models.edge import stream_reference

    det = SlabEdgeDetector(ctx, h, w, filt, stream=True)
    s = det.slab
    for seed, k in ((11, steps), (12, steps + 1)):
        full = _img(h, w, seed)
        det.load(full[s.row0:s.row0 + s.rows])
        for _ in range(k):
            det.step()
        got = parallel.gather_slabs(det.stream_out.contiguous(), s, ctx)
        if ctx.rank == 0:
            assert torch.equal(got, stream_reference(full, filt, k)), f"streaming conv differs ({filt}, {k} steps)"
    det.close()


def jacobi_worker(ctx, rows, cols, iters, outdir, tag):
    sol = SlabJacobi(ctx, rows, cols, check_every=5)
    sol.set_boundary(top=1.0, left=0.5)
    sol.fill(seed=3)
    # the initial field must not depend on the decomposition: rebuild from the global one
    g = torch.Generator().manual_seed(3)
    field = torch.rand((rows, cols - 2), generator=g, dtype=torch.float64)
    sol.u[1:1 + sol.slab.rows, 1:-1] = field[sol.slab.row0:sol.slab.row0 + sol.slab.rows]
    sol.sync_halos()
    sol.run(iters)
    full = sol.gather()
    if ctx.rank == 0:
        torch.save({"u": full, "res": sol.last_residual}, os.path.join(outdir, f"jacobi_{tag}.pt"))


def jacobi_ckpt_worker(ctx, rows, cols, outdir):
    a = SlabJacobi(ctx, rows, cols, check_every=4)
    a.set_boundary(top=2.0)
    a.fill(seed=1)
    a.run(8)
    a.save_checkpoint(os.path.join(outdir, "ck"))
    a.run(8)
    b = SlabJacobi(ctx, rows, cols, check_every=4)
    b.set_boundary(top=2.0)
    b.load_checkpoint(os.path.join(outdir, "ck"))
    b.run(8)
    assert b.iteration == a.iteration == 16
    assert torch.equal(a.u, b.u) and a.last_residual == b.last_residual


def classify_worker(ctx, h, w, nc):
    full = _img(h, w, 9)
    pts = class_points_for(h, w, nc, 25, seed=2)
    clf = SlabPixelClassifier(ctx, h, w, path="direct")
    clf.img.copy_(split_rows(full, clf.slab))
    clf.fit(pts)
    mu, inv = ops.class_stats(full, pts)
    assert np.array_equal(mu, clf.mu) and np.array_equal(inv, clf.inv)
    clf.classify()
    got = parallel.gather_slabs(clf.img, clf.slab, ctx)
    if ctx.rank == 0:
        ref = full.clone()
        ops.classify_(ref, mu, inv)
        assert torch.equal(got, ref)


def vsub_worker(ctx, n):
    m = ShardedVectorSub(ctx, n)
    m.fill_random(seed=4)
    m.step()
    assert torch.equal(m.c, m.a - m.b)
    got = m.gather()
    if ctx.rank == 0:
        assert got.shape == (n,)


def collectives_worker(ctx):
    t = torch.tensor([float(ctx.rank + 1)])
    parallel.all_reduce_max(t, ctx)
    assert t.item() == ctx.world
    assert parallel.max_over_ranks(ctx.rank * 2.0, ctx) == 2.0 * (ctx.world - 1)
    obj = parallel.broadcast_object({"r": ctx.rank} if ctx.rank == 0 else None, ctx)
    assert obj == {"r": 0}
    s = parallel.Slab(10, ctx.world, ctx.rank)
    full = torch.arange(40, dtype=torch.float32).reshape(10, 4) if ctx.rank == 0 else None
    mine = parallel.scatter_rows(full, s, ctx, like=torch.empty(0, 4))
    assert torch.equal(mine, torch.arange(40, dtype=torch.float32).reshape(10, 4)[s.row0:s.row0 + s.rows])


def all_workloads_worker(ctx, k):
    """conv (sobel5 overlapped + roberts in order), classifier, vsub and Jacobi
    on 8k+5-row problems, each compared bit-exactly with one process."""
    h, w = 8 * k + 5, 29
    full = _img(h, w, 17)
    for filt, overlap in (("sobel5", True), ("roberts", False)):
        det = SlabEdgeDetector(ctx, h, w, filt, overlap=overlap)
        s = det.slab
        det.load(full[s.row0:s.row0 + s.rows])
        got = parallel.gather_slabs(det.step(), s, ctx)
        if ctx.rank == 0:
            assert torch.equal(got, ops.conv(full, filt)), f"{filt} at world {ctx.world}"
    # classifier
    pts = class_points_for(h, w, 5, 20, seed=4)
    clf = SlabPixelClassifier(ctx, h, w, path="direct")
    clf.img.copy_(split_rows(full, clf.slab))
    clf.fit(pts)
    clf.classify()
    got = parallel.gather_slabs(clf.img, clf.slab, ctx)
    if ctx.rank == 0:
        ref = full.clone()
        mu, inv = ops.class_stats(full, pts)
        ops.classify_(ref, mu, inv)
        assert torch.equal(got, ref), f"classifier at world {ctx.world}"
    # vsub
    m = ShardedVectorSub(ctx, 8 * 1000 + 5)
    m.fill_random(seed=6)
    m.step()
    assert torch.equal(m.c, m.a - m.b)
    # Jacobi: 25 iterations, residual every 5
    rows, cols = 8 * k + 5, 19
    g = torch.Generator().manual_seed(8)
    field = torch.rand((rows, cols - 2), generator=g, dtype=torch.float64)

    def setup(sol):
        sol.set_boundary(top=1.0, left=0.5)
        sol.u[1:1 + sol.slab.rows, 1:-1] = field[sol.slab.row0:sol.slab.row0 + sol.slab.rows]
        sol._halos_valid = False

    sol = SlabJacobi(ctx, rows, cols, check_every=5)
    setup(sol)
    sol.run(25)
    got = sol.gather()
    if ctx.rank == 0:
        ref = SlabJacobi(parallel.DistContext(), rows, cols, check_every=5)
        setup(ref)
        ref.run(25)
        assert torch.equal(got, ref.owned) and sol.last_residual == ref.last_residual, f"jacobi at {ctx.world}"


# ---------------------------------------------------------------- tests
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_all_workloads_decomposed_uneven(world):
    run_world(world, "all_workloads_worker", 3)

@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("filt", ["sobel5", "roberts", "sobel3"])
def test_slab_conv_equals_single(world, filt, tmp_path):
    run_world(world, "conv_worker", 37, 29, filt, True, str(tmp_path))


@pytest.mark.parametrize("world,filt", [(2, "sobel5"), (3, "roberts"), (8, "sobel5_dense")])
def test_slab_conv_stream_equals_one_device(world, filt):
    run_world(world, "stream_worker", 8 * 5 + 5, 21, filt, 4)


@pytest.mark.parametrize("mode", [False, "pipeline"])
def test_slab_conv_no_overlap(mode, tmp_path):
    run_world(2, "conv_worker", 20, 16, "sobel5", mode, str(tmp_path))


def test_slab_jacobi_equals_single(tmp_path):
    run_world(1, "jacobi_worker", 23, 17, 20, str(tmp_path), "w1")
    run_world(3, "jacobi_worker", 23, 17, 20, str(tmp_path), "w3")
    a = torch.load(tmp_path / "jacobi_w1.pt", weights_only=True)
    b = torch.load(tmp_path / "jacobi_w3.pt", weights_only=True)
    assert torch.equal(a["u"], b["u"]) and a["res"] == b["res"] and a["res"] is not None


def test_slab_jacobi_checkpoint_resume(tmp_path):
    run_world(2, "jacobi_ckpt_worker", 16, 12, str(tmp_path))


@pytest.mark.parametrize("world", [2, 3])
def test_slab_classifier(world):
    run_world(world, "classify_worker", 31, 23, 4)


def test_sharded_vsub_and_collectives():
    run_world(3, "vsub_worker", 1001)
    run_world(2, "collectives_worker")


def test_slab_math():
    s = [parallel.Slab(10, 3, r, 2, 2) for r in range(3)]
    assert [x.rows for x in s] == [4, 3, 3] and [x.row0 for x in s] == [0, 4, 7]
    assert s[0].y_lo == 0 and s[0].y_hi == 5 and s[1].y_lo == -2 and s[2].y_hi == 2
    assert s[0].interior() == (0, 2) and s[0].boundary() == [(2, 4)]
    assert s[1].interior() == (2, 2) and s[1].boundary() == [(0, 2), (2, 3)]
    with pytest.raises(ValueError):
        parallel.Slab(5, 3, 0, 2, 2)
    assert parallel.min_ranks_for(16384 * 8, 16384 * 8, buffers=2) == 1
    assert parallel.max_rows_per_gpu(16384 * 8, buffers=2) > 16384 * 50  # a 16384-wide fp64 grid: ~930k rows per GPU


def test_fault_injection_raises(monkeypatch):
    from cuda_mpi_openmp_amd.models.jacobi import FaultInjected

    monkeypatch.setenv("MPX_FAULT_INJECT", "0:3")
    sol = SlabJacobi(parallel.DistContext(), 8, 8)
    sol.fill()
    with pytest.raises(FaultInjected):
        sol.run(10)
    assert sol.iteration == 3


def test_select_device_uses_node_local_values():
    """the same-device refusal is decided on node-local values
    (LOCAL_WORLD_SIZE, LOCAL_RANK), never on the global WORLD_SIZE."""
    from cuda_mpi_openmp_amd.parallel.dist import select_device

    # one node of 8 GPUs, 8 ranks: rank k drives GPU k
    assert [select_device(r, 8, 8, env={}) for r in range(8)] == list(range(8))
    # a multi-node job (WORLD_SIZE 16, 8 ranks per node): node-local values pass
    assert select_device(7, 8, 8, env={}) == 7
    # per-rank isolation (HIP_VISIBLE_DEVICES=<rank>): one visible GPU, index 0
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        assert [select_device(r, 8, 1, env={var: str(r)}) for r in range(8)] == [0] * 8
    # not isolated, more node-local ranks than devices: refused (None)
    assert select_device(1, 2, 1, env={}) is None
    assert select_device(3, None, 2, env={}) is None
    assert select_device(0, None, 1, env={}) == 0
    assert select_device(0, 1, 0, env={}) is None


def test_span_per_rank_clock_when_multi_node():
    """ranks on different hosts read unrelated monotonic clocks —
    the job time is then the slowest rank's own span, never max(t1) - min(t0)
    across clocks, and the skews are not reported."""
    from cuda_mpi_openmp_amd.parallel.timing import Span

    s = Span([0.0, 5e17], [2e6, 5e17 + 3e6], shared=False)
    assert s.job_s == 3e-3 and s.fields(1)["clock"] == "per-rank" and s.fields(1)["start_skew_ms"] is None
    one = Span([0.0, 1e6], [2e6, 3e6])
    assert one.job_s == 3e-3 and one.fields(1)["clock"] == "shared-monotonic"
