#!/bin/bash
# Round-6 second-session GPU checkpoints (gpurun: bash tools/checkpoints/r6_s2.sh <name>).
# Every GPU step has its own time limit; the first failing step ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
name=$1
out=$R/gpurun_out/${OUTNAME:-$name}
mkdir -p "$out"
pmc() {  # pmc <tag> <counters...>: one counter pass over a short bench
    local tag=$1; shift
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$out/pmc_$tag" -o pmc -- \
        python3 "$R/bench.py" --steps 5 --warmup 2 > "$out/pmc_$tag.log" 2>&1)
}
case "$name" in
g1)  # sobel5 band-kernel VALU cut: lab2 GPU tests, bench, VALU counters
    timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
        tests/test_gpu_kernels.py tests/test_gpu_headline.py -m gpu > "$out/tests.log" 2>&1 \
        || { tail -40 "$out/tests.log"; exit 1; }
    tail -3 "$out/tests.log"
    timeout -k 10 200 python bench.py > "$out/bench1.log" 2>&1 || { tail -20 "$out/bench1.log"; exit 1; }
    tail -1 "$out/bench1.log" | cut -c1-700
    pmc valu SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU; echo "pmc rc=$?"
    ;;
edges)  # the band-kernel strip-edge cases only, every filter and width
    timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
        "tests/test_gpu_kernels.py::test_conv_band_kernel_strip_edges" -m gpu > "$out/tests.log" 2>&1
    grep -E "passed|failed|FAILED" "$out/tests.log" | tail -60
    ;;
probe)  # band-kernel edge debug probe
    PYTHONPATH=$R timeout -k 10 200 python -u tools/experiments/band_edge_probe.py > "$out/probe.log" 2>&1; rc=$?
    tail -80 "$out/probe.log"; exit $rc
    ;;
full)  # the whole GPU suite and smoke on the current tree
    O=$out bash tools/gpu.sh tests && O=$out bash tools/gpu.sh smoke
    ;;
g2)  # g1 plus a second bench and a kernel trace of the bench
    OUTNAME=g2 bash "$0" g1 || exit 1
    timeout -k 10 200 python bench.py > "$out/bench2.log" 2>&1 || { tail -20 "$out/bench2.log"; exit 1; }
    tail -1 "$out/bench2.log" | cut -c1-300
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace -- \
        python3 "$R/bench.py" --steps 20 --warmup 5 > "$out/trace.log" 2>&1); echo "trace rc=$?"
    ;;
ab)  # same-box A/B of the driver bench over library builds (cuda_mpi_openmp_amd/_lib/ab/libmpx_<v>.so;
    # "new" = this tree), alternated: AB_VARIANTS="r6a mid new", AB_ROUNDS=3
    for k in $(seq 1 ${AB_ROUNDS:-3}); do
        for v in ${AB_VARIANTS:-r6a new}; do
            if [ $v = new ]; then lib=$R/cuda_mpi_openmp_amd/_lib/libmpx.so; else lib=$R/cuda_mpi_openmp_amd/_lib/ab/libmpx_$v.so; fi
            MPX_LIB_PATH=$lib timeout -k 10 200 python bench.py > "$out/bench_${v}_$k.log" 2>&1 \
                || { tail -20 "$out/bench_${v}_$k.log"; exit 1; }
            python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['steady_clocks'][0]; print(sys.argv[2], sys.argv[3], d['value'], d['value_sustained'], d['value_steady'], d['value_streaming'], d['value_warm_cache'], c.get('gfxclk_mhz'), c.get('power_w'))" "$out/bench_${v}_$k.log" $v $k
        done
    done
    ;;
final)  # smoke, the driver bench, and the per-kernel profile (prof_all) of the current tree
    export O=$out
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py &&
    python tools/experiments/kprof_table.py "$O" > "$O/kernels_table.md" &&
    python tools/pmc_median.py "$O"/kfinal.pmc* > "$O/medians.md" &&
    python tools/experiments/trace_db.py "$O/kfinal" --top 40 > "$O/trace.md" &&
    find "$O" -name "*.db" -delete && du -sh "$O"
    ;;
g3)  # band-kernel change check: edge probe, lab2 GPU tests, VALU counters, then the bench A/B
    PYTHONPATH=$R timeout -k 10 200 python -u tools/experiments/band_edge_probe.py > "$out/probe.log" 2>&1 \
        || { tail -30 "$out/probe.log"; exit 1; }
    tail -3 "$out/probe.log"
    timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
        tests/test_gpu_kernels.py tests/test_gpu_headline.py -m gpu > "$out/tests.log" 2>&1 \
        || { tail -40 "$out/tests.log"; exit 1; }
    tail -1 "$out/tests.log"
    pmc valu SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS; echo "pmc rc=$?"
    OUTNAME=$name AB_VARIANTS="${AB_VARIANTS:-r6a alp new}" bash "$0" ab
    ;;
multi)  # the driver's N-rank command rehearsed on one GPU (ranks share it), weak and strong
    export O=$out
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run drv2 300 python bench.py --gpus 2 --steps 20 --warmup 5 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run drv4s 300 python bench.py --gpus 4 --steps 20 --warmup 5 --layout strong
    for f in "$O"/drv*.log; do echo "$f"; grep '^{' "$f" | tail -1 | cut -c1-420; done
    ;;
*) echo "unknown checkpoint $name"; exit 2 ;;
esac
