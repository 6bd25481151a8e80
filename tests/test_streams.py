"""The process-wide compute stream set (utils/streams.py): created once,
shared by every caller, distinct streams."""

import pytest
import torch

pytestmark = pytest.mark.gpu


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
