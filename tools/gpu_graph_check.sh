set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_graphs.py -x -v --timeout 120 > gpurun_out/graphs.log 2>&1; tail -6 gpurun_out/graphs.log
for g in 0 10; do timeout -k 10 120 python bench.py --graph $g > gpurun_out/bench_g$g.log 2>&1 || exit 3; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"graph_steps": [0-9]*' gpurun_out/bench_g$g.log | tr '\n' ' '; echo; done
for sz in 1024 2048 16384; do for g in "" "--graph"; do timeout -k 10 120 python tools/bench_jacobi.py --size $sz --iters 200 --warmup 20 $g > gpurun_out/jac.log 2>&1 || exit 4; grep -o '"value": [0-9.]*\|"grid": \[[0-9, ]*\]\|"hip_graph": [a-z]*' gpurun_out/jac.log | tr '\n' ' '; echo; done; done
