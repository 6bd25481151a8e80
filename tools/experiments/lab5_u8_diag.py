"""Diagnose the uint8 counting sort: CLI with 0/1 warm-ups and the in-place
re-sort through the Python binding. Prints one line per case."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

a = np.random.default_rng(7).integers(0, 256, 50_000).astype(np.uint8)
want = np.sort(a)
data = np.int32(a.size).tobytes() + a.tobytes()
for warm in ("0", "1", "3"):
    env = dict(os.environ, MPX_WARMUP=warm)
    r = subprocess.run([os.path.join(ROOT, "labs/lab5/src/hip_exe"), "uchar"], input=data, capture_output=True,
                       timeout=60, env=env)
    got = np.frombuffer(r.stdout, dtype=np.uint8)
    bad = np.flatnonzero(got != want) if got.size == want.size else np.array([-1])
    print(f"cli warmup={warm}: rc={r.returncode} ok={bad.size == 0} first_bad={bad[:3].tolist()} "
          f"hist_got={np.bincount(got, minlength=256)[:6].tolist()} hist_want={np.bincount(want, minlength=256)[:6].tolist()}",
          flush=True)
import torch  # noqa: E402

from cuda_mpi_openmp_amd import ops  # noqa: E402

d = torch.from_numpy(a.copy()).cuda()
for i in range(3):
    ops.sort_(d)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    print(f"python pass {i}: ok={np.array_equal(got, want)} hist_got={np.bincount(got, minlength=256)[:6].tolist()}",
          flush=True)
s = torch.from_numpy(want.copy()).cuda()
ops.sort_(s)
print("python sorted input:", np.array_equal(s.cpu().numpy(), want), flush=True)
