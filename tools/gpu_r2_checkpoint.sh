#!/bin/bash
# Round checkpoint: full GPU suite, smoke(), bench.py N=1 (driver defaults).
set -o pipefail
O=gpurun_out/r2/checkpoint; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
