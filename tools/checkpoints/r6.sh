# Round-6 GPU checkpoints: bash tools/gpu.sh checkpoint r6_<x>
# (each a chain of time-bounded gpu.sh steps; outputs under gpurun_out/r6/<x>).

# lab3 final: classifier GPU tests after the AUTO rule change (mfma16 from 2
# classes), three alternated 8192^2 sweeps of auto / mfma16 / mfma8 / fast,
# the kernel trace and two counter passes (VALU per pair, MFMA busy).
ckpt_r6_lab3() {
    export O=${O:-gpurun_out/r6/lab3}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    for r in 1 2 3; do
        LAB3_NCS=1,2,3,4,5,8,12,16,24,32 LAB3_PATHS=auto,mfma16,mfma8,fast LAB3_TAG=r$r \
            bash tools/gpu.sh run lab3_$r 300 python -u tools/experiments/lab3_m16.py || return 1
    done &&
    LAB3_PROF=1 LAB3_NCS=4,16,32 LAB3_PATHS=auto,mfma8,fast \
        bash tools/gpu.sh prof lab3_trace -- python tools/experiments/lab3_m16.py &&
    local i=0 grp
    for grp in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
               "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
               "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
        i=$((i + 1))
        LAB3_PROF=1 LAB3_NCS=4,16,32 LAB3_PATHS=auto,mfma8,fast \
            bash tools/gpu.sh pmc lab3_pmc$i "$grp" -- python tools/experiments/lab3_m16.py || return 1
    done
}

# lab3 in-wave exact fallback of the one-shot mfma16 kernel (no fix-up launch)
# against the device deferral list: A = libmpx (list), B = $LIB (in-wave up to
# 16 classes); classifier GPU tests on B first.
ckpt_r6_inwave() {
    export O=${O:-gpurun_out/r6/inwave}
    mkdir -p "$O"
    local lib=${LIB:-abtmp/libmpx.so}
    MPX_LIB_PATH=$lib bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "classify" &&
    LAB3_NCS=1,2,3,4,5,6,8,12,16 LAB3_PATHS=mfma16,fast \
        bash tools/gpu.sh ab lab3 "$lib" 3 -- python -u tools/experiments/lab3_m16.py
}

# lab3 one-shot mfma16 kernel occupancy (amdgpu_waves_per_eu for the 1-set
# instantiations up to 16 classes): A = libmpx, B = abtmp/w5 (5 waves per
# SIMD, no scratch) and abtmp/w6 (6, a few spill slots in the rare paths).
ckpt_r6_wpe() {
    export O=${O:-gpurun_out/r6/wpe}
    mkdir -p "$O"
    MPX_LIB_PATH=abtmp/w5/libmpx.so bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "classify_mfma16" &&
    LAB3_NCS=2,3,4,5,8,12,16 LAB3_PATHS=mfma16 \
        bash tools/gpu.sh ab w5 abtmp/w5/libmpx.so 3 -- python -u tools/experiments/lab3_m16.py &&
    LAB3_NCS=2,3,4,5,8,12,16 LAB3_PATHS=mfma16 \
        bash tools/gpu.sh ab w6 abtmp/w6/libmpx.so 3 -- python -u tools/experiments/lab3_m16.py
}

# Multi-GPU rehearsal on one GPU (VERDICT r5 Next #2 / #7): the conv jobs of
# tools/scale.py at 1/2/4 ranks sharing the GPU (gloo control plane, peer
# halos), weak and strong; the driver bench with rank 1's peer mapping failing
# (every rank must take the fallback, verified, rc 0) and with rank 1's
# streaming phase timing out (value_streaming null, status records it, rc 0).
ckpt_r6_multi() {
    export O=${O:-gpurun_out/r6/multi}
    mkdir -p "$O"
    bash tools/gpu.sh run scale 900 python -u tools/scale.py --gpus 1,2,4 --rehearse --only conv --quick \
        --out "$O/scale" &&
    MPX_DIST_BACKEND=gloo MPX_PEER_INJECT=map_fail@1 bash tools/gpu.sh run inject_map 300 \
        python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline &&
    MPX_DIST_BACKEND=gloo MPX_BENCH_INJECT_STREAM_TIMEOUT=1 bash tools/gpu.sh run inject_stream 300 \
        python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
}

# The reference-methodology harness rows VERDICT r5 Next #5 asks for: the
# literal [[16,16],[1024,1024]] grid in every lab2 bucket, and cold runs that
# include HIP's lazy code-object load (no preload).
ckpt_r6_hcmp() {
    export O=${O:-gpurun_out/r6/hcmp}
    mkdir -p "$O"
    timeout -k 10 1000 bash tools/harness_compare.sh literal lazy > "$O/hcmp.log" 2>&1 || { tail -20 "$O/hcmp.log"; return 1; }
    tail -30 "$O/hcmp.log"
}

# The driver's bench command twice after the steady-window changes (one
# untimed window after each settle loop, clock sampler in a child process).
ckpt_r6_bench() {
    export O=${O:-gpurun_out/r6/bench}
    mkdir -p "$O"
    for r in 1 2; do
        bash tools/gpu.sh run bench$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || return 1
    done
}

# Strong-scaling per-rank floor: one rank's slab of a 4096^2 frame at
# 4096..512 rows, with and without its resident halo rows, and the whole
# frame cut into 1..8 launches (tools/experiments/strong_floor.py).
ckpt_r6_floor() {
    export O=${O:-gpurun_out/r6/floor}
    mkdir -p "$O"
    bash tools/gpu.sh run floor 300 python -u tools/experiments/strong_floor.py
}

# The new GPU tests (fallback records, cold-lazy policy) then the harness rows.
ckpt_r6_newtests() {
    export O=${O:-gpurun_out/r6/newtests}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_bench_launch.py tests/test_cli_programs.py -k "bench or timing"
}

# Final-tree kernel profile (kernels_r6.md): smoke, the driver's bench, the lab3
# AUTO sweep, then one trace + the counter groups over every production kernel
# at the BASELINE sizes (tools/prof_all.py), summarised on the box.
ckpt_r6_final() {
    export O=${O:-gpurun_out/r6/final}
    mkdir -p "$O"
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    LAB3_NCS=1,2,3,4,5,8,12,16,24,32 LAB3_PATHS=auto LAB3_TAG=auto \
        bash tools/gpu.sh run lab3_auto 400 python -u tools/experiments/lab3_m16.py &&
    bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py &&
    python tools/experiments/kprof_table.py "$O" > "$O/kernels_table.md" &&
    python tools/pmc_median.py "$O"/kfinal.pmc* > "$O/medians.md" &&
    python tools/experiments/trace_db.py "$O/kfinal" --top 40 > "$O/trace.md" &&
    du -sh "$O" && find "$O" -name "*.db" -delete && du -sh "$O"
}

# lab3 one-shot mfma16 kernel: 2 / 8 vectors per thread against 4 (A/B libs
# abtmp/t2, abtmp/t8; small class counts), and the kernel trace of the
# rotating nc = 4 loop (where the 121 µs per call go).
ckpt_r6_trips() {
    export O=${O:-gpurun_out/r6/trips}
    mkdir -p "$O"
    LAB3_NCS=4 LAB3_PATHS=mfma16,fast bash tools/gpu.sh prof rot_trace -- python tools/experiments/lab3_m16.py &&
    for t in t2 t8; do
        MPX_LIB_PATH=abtmp/$t/libmpx.so bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "classify_mfma16" &&
        LAB3_NCS=3,4,5,8 LAB3_PATHS=mfma16 \
            bash tools/gpu.sh ab $t abtmp/$t/libmpx.so 3 -- python -u tools/experiments/lab3_m16.py || return 1
    done
}

# Short-slab segment sweep of the band kernel (strong-scaling per-rank floor).
ckpt_r6_seg() {
    export O=${O:-gpurun_out/r6/seg}
    mkdir -p "$O"
    bash tools/gpu.sh run seg 300 python -u tools/experiments/small_slab_seg.py
}

# lab3 mfma16: class constants pinned in VGPRs (no per-pixel re-copy from
# SGPRs) — B = abtmp/pin against libmpx, classifier GPU tests on B first.
ckpt_r6_pin() {
    export O=${O:-gpurun_out/r6/pin}
    mkdir -p "$O"
    MPX_LIB_PATH=abtmp/pin/libmpx.so bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=2,3,4,5,8,12,16,24,32 LAB3_PATHS=mfma16 \
        bash tools/gpu.sh ab pin abtmp/pin/libmpx.so 3 -- python -u tools/experiments/lab3_m16.py
}

# The whole -m gpu suite on the final tree.
ckpt_r6_tests() {
    export O=${O:-gpurun_out/r6/tests}
    mkdir -p "$O"
    bash tools/gpu.sh tests
}

# The conv jobs of the scaling driver on the final tree (one GPU, ranks share it).
ckpt_r6_multi2() {
    export O=${O:-gpurun_out/r6/multi2}
    mkdir -p "$O"
    bash tools/gpu.sh run scale 900 python -u tools/scale.py --gpus 1,2,4 --rehearse --only conv --quick \
        --out "$O/scale" &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run drv2 300 python bench.py --gpus 2 --steps 20 --warmup 5
}

# Sort bench on the final tree, three runs (VERDICT r5 Next #3: within ±1 % of
# round 5's 0.689-0.697 / 0.722-0.730 ms at 2^26).
ckpt_r6_sort() {
    export O=${O:-gpurun_out/r6/sort}
    mkdir -p "$O"
    for r in 1 2 3; do
        LAB5_DTYPES=int32,float32 LAB5_LOGN=24,26 LAB5_VARIANTS=22 LAB5_ITERS=9 \
            bash tools/gpu.sh run sort$r 300 python -u tools/experiments/lab5_bench.py || return 1
    done
}

# lab3 mfma16 with the fix-up fused into the one-shot kernel (the last block
# of each sub-list re-ranks it; no fix-up launch): B = abtmp/fused against
# libmpx, classifier GPU tests on B first.
ckpt_r6_fused() {
    export O=${O:-gpurun_out/r6/fused}
    mkdir -p "$O"
    MPX_LIB_PATH=abtmp/fused/libmpx.so bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=2,3,4,5,8,12,16,24,32 LAB3_PATHS=mfma16 \
        bash tools/gpu.sh ab fused abtmp/fused/libmpx.so 3 -- python -u tools/experiments/lab3_m16.py
}

# After the Jacobi / vsub variants moved to the tune library.
ckpt_r6_tunemove() {
    export O=${O:-gpurun_out/r6/tunemove}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_peer_halo.py \
        -k "jacobi or vsub or tune" &&
    JBENCH_R=8 JBENCH_AUX=18 bash tools/gpu.sh run jbench 300 python -u tools/experiments/jbench.py 8192
}

# The driver's bench command under the kernel trace (per-kernel stats of the
# flagship step), summarised for profiles/.
ckpt_r6_benchprof() {
    export O=${O:-gpurun_out/r6/benchprof}
    mkdir -p "$O"
    bash tools/gpu.sh prof bench_trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 &&
    python tools/prof_summary.py trace "$O/bench_trace" > "$O/bench_trace.md" &&
    find "$O" -name "*.db" -delete
}

# Last look at the committed tree: smoke and the driver's bench command.
ckpt_r6_last() {
    export O=${O:-gpurun_out/r6/last}
    mkdir -p "$O"
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh run bench_default 300 python bench.py
}
