#!/bin/bash
# Empty-workgroup elision for caller geometries: geometry GPU tests, then the
# reference-methodology harness comparison (lab2 buckets, lab1 sizes).
# SKIP_TESTS=1 runs only the comparison.
set -o pipefail
O=gpurun_out/r2/geom; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "geometry or roberts or vsub or classify_matches" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
rc=0
timeout -k 10 1000 bash tools/harness_compare.sh > $O/harness.log 2>&1 || rc=$?
# keep the CSVs and logs only: the copied binaries would exceed gpurun_out's 64 MiB
find gpurun_out/harness_cmp -type f ! -name '*.csv' ! -name '*.log' -delete
[ $rc -eq 0 ] || { tail -30 $O/harness.log; exit 1; }
tail -3 $O/harness.log
