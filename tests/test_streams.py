"""utils/streams.py: the process-wide compute stream set (created once,
shared by every caller, distinct streams), the detector's twin-output step the
bench's cache-resident pass runs on it, and the host wait policy."""

import pytest
import torch



@pytest.mark.gpu
def test_compute_streams_are_shared_and_distinct(gpu):
    from cuda_mpi_openmp_amd.utils.streams import compute_streams

    a = compute_streams(gpu, 2)
    b = compute_streams(gpu, 3)
    assert [s.cuda_stream for s in a] == [s.cuda_stream for s in b[:2]]
    assert len({s.cuda_stream for s in b}) == 3
    assert all(s.device == gpu for s in b)
    # work queued on both overlaps with nothing shared: a join is enough
    x = torch.ones(1 << 20, device=gpu)
    main = torch.cuda.current_stream(gpu)
    outs = []
    for st in a:
        st.wait_stream(main)
        with torch.cuda.stream(st):
            outs.append(x * 2)
    for st in a:
        main.wait_stream(st)
    assert all(torch.equal(o, torch.full_like(x, 2.0)) for o in outs)


@pytest.mark.gpu
def test_step_twin_matches_step(gpu):
    """bench.py's cache-resident pass: step and step_twin of one input on two
    streams write identical slabs (resident hint on and off)."""
    from cuda_mpi_openmp_amd import ops, parallel
    from cuda_mpi_openmp_amd.models.edge import SlabEdgeDetector
    from cuda_mpi_openmp_amd.utils.streams import compute_streams

    ctx = parallel.DistContext(device=gpu)
    d = SlabEdgeDetector(ctx, 512, 384, "sobel5")
    d.fill_random(seed=3)
    s0, s1 = compute_streams(gpu, 2)
    main = torch.cuda.current_stream(gpu)
    for flag in (False, True):
        d.cache_resident(flag)
        s0.wait_stream(main)
        s1.wait_stream(main)
        a = d.step(s0.cuda_stream)
        b = d.step_twin(s1.cuda_stream)
        main.wait_stream(s0)
        main.wait_stream(s1)
        assert a.data_ptr() != b.data_ptr()
        assert torch.equal(a, b)
        # bit for bit against the native CPU conv (the plain fp32 PyTorch
        # reference is within 1 of both: test_gpu_kernels.py)
        assert torch.equal(a.cpu(), ops.conv(d.own.cpu().contiguous(), "sobel5"))


def test_host_wait_policy_names():
    from cuda_mpi_openmp_amd.utils.streams import host_wait_policy

    assert host_wait_policy(torch.device("cpu"), "spin") == "auto"  # CPU: nothing to set
    with pytest.raises(ValueError):
        host_wait_policy(torch.device("cpu"), "busy")


@pytest.mark.gpu
def test_host_wait_policy_sets_and_restores(gpu):
    from cuda_mpi_openmp_amd.utils.streams import host_wait_policy, wait_policy_in_force

    assert host_wait_policy(gpu, "spin") == "spin"
    assert wait_policy_in_force(gpu) == "spin"
    x = torch.ones(1 << 20, device=gpu) * 3  # a wait under the policy
    torch.cuda.synchronize(gpu)
    assert float(x[0]) == 3.0
    assert host_wait_policy(gpu, "auto") == "auto"
    assert wait_policy_in_force(gpu) == "auto"
