import json, os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cuda_mpi_openmp_amd import ops
from cuda_mpi_openmp_amd.models.classifier import class_points_for
dev = torch.device('cuda:0'); size = 8192
img = torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev)
host = img.cpu()
for nc in (2, 4, 6, 8, 16, 32):
    pts = class_points_for(size, size, nc, 64, seed=nc)
    mu, inv = ops.class_stats(host, pts)
    ref = ops.classify_(host.clone(), mu, inv)
    work = img.clone()
    ops.classify_(work, mu, inv, path="fast")
    ok = torch.equal(work.cpu(), ref)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2): ops.classify_(work, mu, inv, path="fast")
    torch.cuda.synchronize(); s.record()
    for _ in range(10): ops.classify_(work, mu, inv, path="fast")
    e.record(); torch.cuda.synchronize()
    print(json.dumps({"nc": nc, "us": round(s.elapsed_time(e) * 100, 1), "verified": ok}), flush=True)
