"""One rank of tests/test_contract.py's collective checks (run under torchrun
with MPX_DIST_CONTRACT=nccl; argv[1] = cpu | cuda)."""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cuda_mpi_openmp_amd import parallel  # noqa: E402
from cuda_mpi_openmp_amd.parallel import contract  # noqa: E402
from cuda_mpi_openmp_amd.parallel.halo import HaloExchange  # noqa: E402
from cuda_mpi_openmp_amd.parallel.slab import Slab  # noqa: E402


def main() -> int:
    ctx = parallel.init(device=sys.argv[1])
    r, w = ctx.rank, ctx.world
    assert ctx.backend == "nccl" and ctx.is_distributed
    assert (ctx.native is not None) == (ctx.device.type == "cuda")
    ctx.barrier()
    assert parallel.max_over_ranks(float(r), ctx) == w - 1
    assert parallel.all_gather_floats(r * 1.5, ctx) == [i * 1.5 for i in range(w)]
    assert parallel.all_reduce_sum_host(1.0, ctx) == w
    assert parallel.broadcast_object(("cfg", r), ctx) == ("cfg", 0)
    x = torch.full((4,), float(r), device=ctx.device)
    parallel.all_reduce_max(x, ctx)
    assert x.tolist() == [w - 1.0] * 4
    # a slab's halo rows through the default-group p2p path (native stand-in on GPU)
    s = Slab(global_rows=6 * w, world=w, rank=r, halo_up=2, halo_down=1)
    buf = torch.full((s.buffer_rows, 5), -1.0, device=ctx.device)
    buf[s.own_offset:s.own_offset + s.rows] = torch.arange(s.row0, s.row0 + s.rows, dtype=torch.float32,
                                                           device=ctx.device)[:, None]
    HaloExchange(s, ctx).exchange(buf)
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    if r > 0:
        assert buf[0:2, 0].tolist() == [s.row0 - 2.0, s.row0 - 1.0]
    if r + 1 < w:
        assert buf[s.own_offset + s.rows, 0].item() == s.row0 + s.rows
    got = parallel.gather_slabs(buf[s.own_offset:s.own_offset + s.rows].contiguous(), s, ctx)
    if r == 0:
        assert got[:, 0].tolist() == [float(i) for i in range(6 * w)]
    # a host tensor where RCCL needs a device one is refused, naming this file
    if ctx.device.type == "cuda":
        try:
            torch.distributed.all_reduce(torch.zeros(1))
        except contract.ContractError as e:
            assert "contract_worker.py" in str(e), str(e)
        else:
            raise AssertionError("host tensor passed the nccl contract")
        try:
            ctx.native.all_reduce_(torch.zeros(1), "sum")
        except contract.ContractError:
            pass
        else:
            raise AssertionError("host tensor passed the native-comm contract")
    ctx.barrier()
    parallel.shutdown()
    print(f"contract worker ok rank {r}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
