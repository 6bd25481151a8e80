"""HIP-graph replay of launch-bound loops (utils/graphs.py): a replayed step
must do exactly what the eager step does — same pixels, same Jacobi field and
residuals, bit for bit."""

import pytest
import torch

from cuda_mpi_openmp_amd import ops, parallel
from cuda_mpi_openmp_amd.models import SlabEdgeDetector, SlabJacobi
from cuda_mpi_openmp_amd.utils.graphs import StepGraph, try_step_graph

from .helpers import rand_img


def test_graphs_need_a_gpu():
    assert try_step_graph(lambda: None, 3, torch.device("cpu")) is None
    with pytest.raises(ValueError):
        StepGraph(lambda: None, 0, torch.device("cpu"))


@pytest.mark.gpu
def test_conv_step_graph_matches_eager(gpu):
    ctx = parallel.DistContext(device=gpu)
    det = SlabEdgeDetector(ctx, 300, 256, "sobel5")
    det.fill_random(seed=5)
    g = StepGraph(det.step, 4, gpu)
    det.out.zero_()
    g.replay()
    torch.cuda.synchronize(gpu)
    assert torch.equal(det.out.cpu(), ops.conv(det.own.cpu().contiguous(), "sobel5"))


@pytest.mark.gpu
@pytest.mark.parametrize("check_every", [4, 5])
def test_jacobi_graph_run_matches_eager(gpu, check_every):
    ctx = parallel.DistContext(device=gpu)
    a = SlabJacobi(ctx, 130, 97, check_every=check_every)
    b = SlabJacobi(ctx, 130, 97, check_every=check_every)
    for s in (a, b):
        s.set_boundary(top=1.0, left=0.25)
        s.fill(seed=2)
    ra = a.run(43)
    rb = b.run(43, graph=True)
    torch.cuda.synchronize(gpu)
    assert ra == rb == 43
    assert torch.equal(a.u, b.u)
    assert a.last_residual == b.last_residual
    # tolerance stop lands on the same iteration
    c = SlabJacobi(ctx, 130, 97, check_every=check_every)
    d = SlabJacobi(ctx, 130, 97, check_every=check_every)
    for s in (c, d):
        s.set_boundary(top=1.0)
        s.fill(seed=3)
    tol = 0.05
    assert c.run(400, tol=tol) == d.run(400, tol=tol, graph=True)
    assert torch.equal(c.u, d.u)
