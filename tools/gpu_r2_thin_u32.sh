#!/bin/bash
# vsub very thin launches: 16 (default) vs 32 vectors per operand in flight (MPX_VSUB_U32=1, blocks <= 64).
set -o pipefail
O=gpurun_out/r2/thin_u32; mkdir -p $O
MPX_VSUB_U32=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "vsub" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python tools/thin_geom_bench.py > $O/u16_$r.jsonl 2>&1 || { tail -20 $O/u16_$r.jsonl; exit 1; }
  MPX_VSUB_U32=1 timeout -k 10 300 python tools/thin_geom_bench.py > $O/u32_$r.jsonl 2>&1 || { tail -20 $O/u32_$r.jsonl; exit 1; }
done
for f in $O/*.jsonl; do echo "== $f"; grep '"lab": 1' $f; done
