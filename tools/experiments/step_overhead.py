#!/usr/bin/env python3
"""Host (CPU) cost per step of the flagship pipeline on one GPU.

A step is GPU-bound only while the host enqueues it faster than the GPU runs
it (~40 us for a 4096^2 sobel5 image). This measures, without synchronising:
  * N = 1 step: one pre-validated conv launch;
  * the N > 1 step shape on a world-of-one native communicator: halo start
    (grouped send/recv to self) + interior conv + halo wait + 2 boundary convs;
  * the same exchange through torch.distributed batch_isend_irecv (self).
and the GPU time of each (events), as JSON lines.
"""

import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops, parallel  # noqa: E402
from cuda_mpi_openmp_amd.parallel.native_comm import NativeComm, P2PPlan  # noqa: E402


def host_and_gpu_us(fn, n=400):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t0) * 1e6 / n
    e.record()
    e.synchronize()
    return host, s.elapsed_time(e) * 1e3 / n


def main():
    only_native = "--native-only" in sys.argv  # short run for a kernel timeline
    dev = torch.device("cuda:0")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ctx = parallel.DistContext(rank=0, world=1, local_rank=0, device=dev, backend="nccl")
    comm = NativeComm.create(ctx)
    size, f = 4096, ops.get_filter("sobel5")
    hu, hd = f.halo_up, f.halo_down
    buf = torch.randint(0, 256, (size + hu + hd, size, 4), dtype=torch.uint8, device=dev)
    out = torch.empty((size, size, 4), dtype=torch.uint8, device=dev)
    L = lambda a, b, lo, hi: ops.ConvLauncher(buf, out, f, src_row0=hu, out_row0=0, oy0=a, oy1=b,  # noqa: E731
                                              y_lo=lo, y_hi=hi)
    full = L(0, size, 0, size - 1)
    interior = L(hd, size - hu, -hu, size - 1 + hd)
    b_top, b_bot = L(0, hd, -hu, size - 1 + hd), L(size - hu, size, -hu, size - 1 + hd)
    st = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731

    def step1():
        full(st())

    if not only_native:
        h, g = host_and_gpu_us(step1)
        print(json.dumps({"what": "step N=1 (one conv launch)", "host_us": round(h, 2), "gpu_us": round(g, 2)}))

    # self "neighbours": my first hd rows -> my bottom halo, my last hu rows -> my top halo
    plan = P2PPlan([(0, buf[hu:hu + hd], 0), (1, buf[hu + size:hu + size + hd], 0),
                    (0, buf[size:size + hu], 0), (1, buf[0:hu], 0)])

    def step_native():
        s = st()
        comm.p2p_start(plan)
        interior(s)
        comm.p2p_wait()
        b_top(s)
        b_bot(s)

    def step_inline():
        s = st()
        comm.p2p(plan)
        full(s)

    # software-pipelined: two input buffers; during step k the comm stream
    # refreshes the halos of buffer (k+1)%2 while the compute stream convolves
    # buffer k%2 (its halos arrived during step k-1)
    buf2 = buf.clone()
    plans = [plan, P2PPlan([(0, buf2[hu:hu + hd], 0), (1, buf2[hu + size:hu + size + hd], 0),
                            (0, buf2[size:size + hu], 0), (1, buf2[0:hu], 0)])]
    convs = [full, ops.ConvLauncher(buf2, out, f, src_row0=hu, out_row0=0, oy0=0, oy1=size, y_lo=0,
                                    y_hi=size - 1)]
    ev_recv = [torch.cuda.Event(), torch.cuda.Event()]
    ev_conv = [torch.cuda.Event(), torch.cuda.Event()]
    cs = comm.comm_stream() if comm is not None else None
    pstate = {"k": 0}

    def step_pipelined():
        k = pstate["k"]
        cur, nxt = k % 2, (k + 1) % 2
        compute = torch.cuda.current_stream(dev)
        # comm: halos of the next buffer, after the conv that last read it
        cs.wait_event(ev_conv[nxt])
        comm.p2p(plans[nxt], cs)
        ev_recv[nxt].record(cs)
        # compute: this step's buffer (its exchange completed a step ago)
        compute.wait_event(ev_recv[cur])
        convs[cur](compute.cuda_stream)
        ev_conv[cur].record(compute)
        pstate["k"] = k + 1

    if comm is not None and only_native:
        for _ in range(15):
            step_native()
        for _ in range(15):
            step_inline()
        ev_conv[0].record()
        ev_conv[1].record()
        comm.p2p(plans[0])
        ev_recv[0].record()
        for _ in range(15):
            step_pipelined()
        torch.cuda.synchronize()
        comm.close()
        dist.destroy_process_group()
        return
    if comm is not None:
        h, g = host_and_gpu_us(step_native)
        print(json.dumps({"what": "step N>1 shape, native RCCL fork/join overlap (self exchange)",
                          "host_us": round(h, 2), "gpu_us": round(g, 2)}))
        h, g = host_and_gpu_us(step_inline)
        print(json.dumps({"what": "step N>1 shape, native RCCL in-order + one launch (self exchange)",
                          "host_us": round(h, 2), "gpu_us": round(g, 2)}))
        h, g = host_and_gpu_us(lambda: comm.p2p(plan))
        print(json.dumps({"what": "native p2p in-order only", "host_us": round(h, 2), "gpu_us": round(g, 2)}))
        ev_conv[0].record()
        ev_conv[1].record()
        comm.p2p(plans[0])
        ev_recv[0].record()
        h, g = host_and_gpu_us(step_pipelined)
        print(json.dumps({"what": "step N>1 shape, native RCCL software-pipelined (exchange k+1 during conv k)",
                          "host_us": round(h, 2), "gpu_us": round(g, 2)}))
        h, g = host_and_gpu_us(lambda: (comm.p2p_start(plan), comm.p2p_wait()))
        print(json.dumps({"what": "native p2p start+wait only", "host_us": round(h, 2), "gpu_us": round(g, 2)}))
    else:
        print(json.dumps({"what": "native comm unavailable"}))

    def torch_exchange():
        p2p = [dist.P2POp(dist.isend, buf[hu:hu + hd], 0), dist.P2POp(dist.irecv, buf[hu + size:hu + size + hd], 0),
               dist.P2POp(dist.isend, buf[size:size + hu], 0), dist.P2POp(dist.irecv, buf[0:hu], 0)]
        for w in dist.batch_isend_irecv(p2p):
            w.wait()

    try:
        h, g = host_and_gpu_us(torch_exchange, n=200)
        print(json.dumps({"what": "torch batch_isend_irecv start+wait (self)", "host_us": round(h, 2),
                          "gpu_us": round(g, 2)}))
    except Exception as exc:  # noqa: BLE001
        print(json.dumps({"what": "torch batch_isend_irecv (self)", "error": str(exc)[:200]}))
    torch.cuda.synchronize()
    if comm is not None:
        comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
