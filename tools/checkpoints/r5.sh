# Round-5 GPU checkpoints: bash tools/gpu.sh checkpoint r5_<x>
# (each a chain of time-bounded gpu.sh steps; outputs under gpurun_out/r5/<x>).

# A: the full -m gpu suite after the job-span / acq_rel changes, the driver's
# bench command twice (plain, then with the clock sampler), and the
# sustained-load attribution run (copy / vsub / roberts / sobel5 + clocks).
ckpt_r5_a() {
    export O=${O:-gpurun_out/r5/a}
    mkdir -p "$O"
    bash tools/gpu.sh tests &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh run bench_clk 300 python bench.py --gpus 1 --steps 20 --warmup 5 --clocks 200 \
        --no-cpu-baseline &&
    bash tools/gpu.sh run sustain 300 python -u tools/experiments/sustain_clocks.py --out "$O/sustain"
}

# B: sustained-load attribution only (quick re-run after a kernel change)
ckpt_r5_sustain() {
    export O=${O:-gpurun_out/r5/sustain}
    mkdir -p "$O"
    bash tools/gpu.sh run sustain 300 python -u tools/experiments/sustain_clocks.py --out "$O/sustain" "$@"
}

# C: lab3 small class counts on the 4x4x4 int8 MFMA form (VERDICT r4 Next #4):
# the layout probe, the classifier GPU tests, then 8192^2 timings alternated
# (fast32 / mfma8s / the 32x32 mfma8 form) and the MFMA counters of the new path.
ckpt_r5_lab3() {
    export O=${O:-gpurun_out/r5/lab3}
    mkdir -p "$O"
    timeout -k 10 60 bin/mfma4_layout > "$O/mfma4_layout.json" &&
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    for r in 1 2; do
        LAB3_NCS=2,4,6,8,12,16 LAB3_PATHS=fast,mfma8 LAB3_TAG=small$r \
            bash tools/gpu.sh run lab3_new$r 300 python -u tools/experiments/lab3_ab.py &&
        MPX_CLS_MFMA8_SMALL=0 LAB3_NCS=2,4,8 LAB3_PATHS=mfma8 LAB3_TAG=old$r \
            bash tools/gpu.sh run lab3_old$r 300 python -u tools/experiments/lab3_ab.py || return 1
    done &&
    LAB3_NCS=4 LAB3_PATHS=mfma8 bash tools/gpu.sh prof lab3_trace -- python tools/experiments/lab3_ab.py &&
    LAB3_NCS=4 LAB3_PATHS=mfma8 bash tools/gpu.sh pmc lab3_pmc \
        "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" -- \
        python tools/experiments/lab3_ab.py
}

# D: after the tighter int8 bound and the per-trip deferral: classifier +
# sort GPU tests, lab3 8192^2 fast vs mfma8 alternated, the AUTO sweep.
ckpt_r5_lab3b() {
    export O=${O:-gpurun_out/r5/lab3b}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_lab5_sort.py \
        -k "classify or sort" &&
    for r in 1 2; do
        LAB3_NCS=2,3,4,5,6,8,12,16,20,24,32 LAB3_PATHS=fast,mfma8 LAB3_TAG=r$r \
            bash tools/gpu.sh run lab3_$r 300 python -u tools/experiments/lab3_ab.py || return 1
    done &&
    LAB3_NCS=4 LAB3_PATHS=mfma8 bash tools/gpu.sh pmc lab3_pmc \
        "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" -- \
        python tools/experiments/lab3_ab.py
}

# E: the per-dispatch shader clock (GRBM_GUI_ACTIVE / duration) along the
# sustain protocol, sobel5 vs roberts vs copy (one counter, kernel trace only).
ckpt_r5_dclk() {
    export O=${O:-gpurun_out/r5/dclk}
    mkdir -p "$O"
    timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d "$O/dclk" -o "dclk_%pid%" -- \
        python tools/experiments/sustain_clocks.py --workloads sobel5,roberts,copy --rounds 1 --sustain-ms 1500 \
        --hz 50 --out "$O/sustain" > "$O/dclk.log" 2>&1 &&
    for k in conv_band4 conv_wave linear_copy; do
        python tools/experiments/dispatch_clock.py "$(ls "$O"/dclk/*_results.db | head -1)" --grep "$k" \
            --csv "$O/dispatch_$k.csv" > "$O/dispatch_$k.md" || return 1
    done
}

# F: the value_streaming gap (VERDICT r4 Next #5): layouts and data in one
# process, interleaved rounds, then the same under a kernel trace.
ckpt_r5_gap() {
    export O=${O:-gpurun_out/r5/gap}
    mkdir -p "$O"
    bash tools/gpu.sh run stream_gap 300 python -u tools/experiments/stream_gap.py &&
    GAP_ROUNDS=4 bash tools/gpu.sh prof gap_trace -- python tools/experiments/stream_gap.py
}

# G (final tree): smoke, the driver's bench, and the per-kernel profile
# (kernel trace + the standard counter passes over tools/prof_all.py),
# summarised on the box (the rocpd databases exceed gpurun's 64 MiB return).
ckpt_r5_final() {
    export O=${O:-gpurun_out/r5/final}
    mkdir -p "$O"
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py &&
    python tools/experiments/kprof_table.py "$O" > "$O/kernels_table.md" &&
    python tools/pmc_median.py "$O"/kfinal.pmc* > "$O/medians.md" &&
    python tools/experiments/trace_db.py "$O/kfinal" --top 40 > "$O/trace.md" &&
    du -sh "$O" && find "$O" -name "*.db" -delete && du -sh "$O"
}

# H: the same-methodology harness comparison (VERDICT r4 Next #3), lab2 + the
# 4096^2 synthetic bucket in one call, lab1 in another
ckpt_r5_hcmp2() {
    timeout -k 10 1100 bash tools/harness_compare.sh lab2 lab2xl
}
ckpt_r5_hcmp1() {
    timeout -k 10 1100 bash tools/harness_compare.sh lab1
}

# I: lab3 A/B after the host parameter cache (the uncached int8 bound search
# made the back-to-back timing host-bound), then the stream-gap and the
# per-dispatch clock experiments (E, F) in the same call.
ckpt_r5_b2() {
    export O=${O:-gpurun_out/r5/b2}
    mkdir -p "$O"
    for r in 1 2; do
        LAB3_NCS=2,3,4,6,8,12,16,20,24,32 LAB3_PATHS=fast,mfma8 LAB3_TAG=r$r \
            bash tools/gpu.sh run lab3_$r 300 python -u tools/experiments/lab3_ab.py || return 1
    done &&
    MPX_CLS_MFMA8_SMALL=0 LAB3_NCS=4,8 LAB3_PATHS=mfma8 LAB3_TAG=old \
        bash tools/gpu.sh run lab3_old 300 python -u tools/experiments/lab3_ab.py &&
    O=$O/gap ckpt_r5_gap &&
    O=$O/dclk ckpt_r5_dclk
}

# J: the streaming layout: output row alignment against the input's
ckpt_r5_gap2() {
    export O=${O:-gpurun_out/r5/gap2}
    mkdir -p "$O"
    GAP_MODES=static,pingpong,static_outpad,pingpong_skew1,pingpong_skew2,pingpong_skew3,pingpong_skew4,pingpong_skew8 \
        bash tools/gpu.sh run stream_gap 300 python -u tools/experiments/stream_gap.py
}

# K: the streaming gap vs the load policy (NT interior loads vs plain)
ckpt_r5_gap3() {
    export O=${O:-gpurun_out/r5/gap3}
    mkdir -p "$O"
    GAP_MODES=static,pingpong,static_plain,pingpong_plain,static_m1,pingpong_m1 \
        bash tools/gpu.sh run stream_gap 300 python -u tools/experiments/stream_gap.py
}

# L: the job-span accounting on the one-GPU rehearsal (VERDICT r4 Next #1):
# the driver's bench command at 2 and 4 ranks sharing the GPU (gloo control
# plane, peer halos), Jacobi and lab1 at 2 / 4 ranks; every JSON carries
# job_span_ms, max_rank_span_ms and the start / end skews.
ckpt_r5_scale() {
    export O=${O:-gpurun_out/r5/scale}
    mkdir -p "$O"
    export MPX_DIST_BACKEND=gloo
    for n in 2 4; do
        bash tools/gpu.sh run bench$n 400 python bench.py --gpus $n --steps 20 --warmup 5 --no-cpu-baseline &&
        bash tools/gpu.sh run jacobi$n 300 python -u tools/bench_jacobi.py --gpus $n --halo peer --iters 200 \
            --warmup 20 &&
        bash tools/gpu.sh run vsub$n 300 python -u tools/bench_workloads.py --workload vsub --gpus $n --steps 50 \
            --warmup 5 || return 1
    done
}

# M: frames in flight — the driver's bench command with 2 / 3 / 6 streams,
# alternated twice (is 2 still the best overlap?)
ckpt_r5_streams() {
    export O=${O:-gpurun_out/r5/streams}
    mkdir -p "$O"
    for r in 1 2; do
        for s in 2 3 6; do
            bash tools/gpu.sh run bench_s${s}_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --streams $s \
                --no-cpu-baseline --no-stream --no-warm || return 1
        done
    done
}

# N: mfma8s loads in flight: one vs two trips ahead (MPX_CLS_MFMA8S_PF), nc 2-8
ckpt_r5_pf() {
    export O=${O:-gpurun_out/r5/pf}
    mkdir -p "$O"
    for r in 1 2; do
        for pf in 1 2; do
            MPX_CLS_MFMA8S_PF=$pf LAB3_NCS=2,3,4,6,8 LAB3_PATHS=mfma8 LAB3_TAG=pf${pf}_$r \
                bash tools/gpu.sh run lab3_pf${pf}_$r 300 python -u tools/experiments/lab3_ab.py || return 1
        done
    done
}

# O: sort hot digits (VERDICT r4 Next #6): RANK 3 / 4 rank up to four / two
# hot digits per pass by ballot. Sort GPU tests, variants 12 / 18 / 20 and
# 13 / 19 / 21 (SORT_AB) in one process on uniform and skewed data, twice, then
# one kernel trace and one LDS counter pass (SORT_PROF) on 2^26 uniform int32
# and normal floats (the skewed last pass).
ckpt_r5_sort() {
    export O=${O:-gpurun_out/r5/sort}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_lab5_sort.py &&
    for r in 1 2; do
        SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=${SORT_AB:-12,18,20,13,19,21} SORT_PROBE_LOGN=24,26 \
            bash tools/gpu.sh run probe$r 400 python -u tools/experiments/sort_probe.py || return 1
    done &&
    export SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=${SORT_PROF:-12,18,20} SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 \
        SORT_PROBE_CASES=float32_normal,int32_uniform SORT_PROBE_ITERS=3 &&
    bash tools/gpu.sh prof sort_trace -- python tools/experiments/sort_probe.py &&
    bash tools/gpu.sh pmc sort_lds "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" -- \
        python tools/experiments/sort_probe.py &&
    python tools/experiments/kprof_table.py "$O" --grep radix > "$O/kernels_table.md" &&
    python tools/pmc_median.py "$O"/sort_lds > "$O/medians.md" &&
    find "$O" -name "*.db" -delete
}

# P: mfma8s feature pairs by v_perm sign-extension (two VALU fewer per pixel):
# classifier GPU tests, then the new library against the previous classify
# kernel (abl/libmpx_old.so, built from HEAD's classify.hip) alternated 3x.
ckpt_r5_lab3c() {
    export O=${O:-gpurun_out/r5/lab3c}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=2,3,4,6,8 LAB3_PATHS=mfma8 bash tools/gpu.sh ab lab3 abl/libmpx_old.so 3 -- \
        python -u tools/experiments/lab3_ab.py
}

# Q: the lab3 in-place floor on the same box: the linear 16-B copy with source
# == destination (plain / non-temporal) beside mfma8 / fast32 at nc = 2 / 4
ckpt_r5_floor() {
    export O=${O:-gpurun_out/r5/floor}
    mkdir -p "$O"
    for r in 1 2; do
        LAB3_FLOOR=1 LAB3_NCS=2,4 LAB3_PATHS=mfma8,fast LAB3_TAG=r$r \
            bash tools/gpu.sh run lab3_floor$r 300 python -u tools/experiments/lab3_ab.py || return 1
    done
}

# R: mfma8s memory policy (MPX_CLS_MFMA8S_MEM: 1 NT loads, 2 NT stores, 3 both)
# against the in-place copy floor, alternated twice
ckpt_r5_mem() {
    export O=${O:-gpurun_out/r5/mem}
    mkdir -p "$O"
    for r in 1 2; do
        for m in 0 1 2 3; do
            MPX_CLS_MFMA8S_MEM=$m LAB3_FLOOR=$([ $m = 0 ] && echo 1 || echo 0) LAB3_NCS=2,4,8 LAB3_PATHS=mfma8 \
                LAB3_TAG=m${m}_$r bash tools/gpu.sh run lab3_m${m}_$r 300 python -u tools/experiments/lab3_ab.py || return 1
        done
    done
}

# S: where the mfma8s time goes: the same loop without the ranking (MEM=4),
# the default, and larger grids (MPX_CLS_MFMA8S_GRID blocks per CU), twice
ckpt_r5_grid() {
    export O=${O:-gpurun_out/r5/grid}
    mkdir -p "$O"
    for r in 1 2; do
        for k in 8 32 256; do
            for m in 0 4; do
                MPX_CLS_MFMA8S_GRID=$k MPX_CLS_MFMA8S_MEM=$m LAB3_FLOOR=$([ $k$m = 80 ] && echo 1 || echo 0) \
                    LAB3_NCS=2,4 LAB3_PATHS=mfma8 LAB3_TAG=g${k}m${m}_$r \
                    bash tools/gpu.sh run lab3_g${k}m${m}_$r 300 python -u tools/experiments/lab3_ab.py || return 1
            done
        done
    done
}

# T: mfma8s grid sweep (blocks per CU: trips per thread = 256 / k) with one or
# two trips of loads in flight, nc = 2 / 4 / 8, twice
ckpt_r5_grid2() {
    export O=${O:-gpurun_out/r5/grid2}
    mkdir -p "$O"
    for r in 1 2; do
        for k in 16 32 64; do
            for pf in 1 2; do
                MPX_CLS_MFMA8S_GRID=$k MPX_CLS_MFMA8S_PF=$pf LAB3_NCS=2,4,8 LAB3_PATHS=mfma8 LAB3_TAG=g${k}pf${pf}_$r \
                    bash tools/gpu.sh run lab3_g${k}pf${pf}_$r 300 python -u tools/experiments/lab3_ab.py || return 1
            done
        done
    done
}

# U: launch grids of the other classify paths (explicit grids through the
# public API: 2048 = the default 8 blocks per CU, up to 16384), nc = 12 (fast32
# in AUTO), 16 and 32 (mfma8), plus the new mfma8s default at nc = 2 / 4 / 8
ckpt_r5_grid3() {
    export O=${O:-gpurun_out/r5/grid3}
    mkdir -p "$O"
    LAB3_NCS=12,16,32 LAB3_GRIDS=2048,4096,8192,16384 \
        bash tools/gpu.sh run grid_sweep 600 python -u tools/experiments/lab3_grid_sweep.py &&
    LAB3_NCS=2,4,8 LAB3_PATHS=mfma8 LAB3_TAG=g16 \
        bash tools/gpu.sh run lab3_g16 300 python -u tools/experiments/lab3_ab.py
}

# V: mfma8 (32x32) feature bytes from packed 16-bit products: classifier GPU
# tests, then new vs previous classify kernel (abl/libmpx_old.so) alternated
# 3x at nc = 16 / 32 (mfma8) and 4 (mfma8s)
ckpt_r5_lab3d() {
    export O=${O:-gpurun_out/r5/lab3d}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=4,16,32 LAB3_PATHS=mfma8 bash tools/gpu.sh ab lab3 abl/libmpx_old.so 3 -- \
        python -u tools/experiments/lab3_ab.py
}

# W (final tree, after the late lab3 / sort changes): smoke, the driver's
# bench, the per-kernel profile, and AUTO at nc = 2 .. 32 over three rotated
# images; the full GPU suite runs in its own call (checkpoint r5_tests)
ckpt_r5_final2() {
    export O=${O:-gpurun_out/r5/final2}
    mkdir -p "$O"
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    LAB3_NCS=2,3,4,6,8,12,16,20,24,32 LAB3_PATHS=auto LAB3_TAG=auto \
        bash tools/gpu.sh run lab3_auto 400 python -u tools/experiments/lab3_ab.py &&
    bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py &&
    python tools/experiments/kprof_table.py "$O" > "$O/kernels_table.md" &&
    python tools/pmc_median.py "$O"/kfinal.pmc* > "$O/medians.md" &&
    python tools/experiments/trace_db.py "$O/kfinal" --top 40 > "$O/trace.md" &&
    du -sh "$O" && find "$O" -name "*.db" -delete && du -sh "$O"
}
ckpt_r5_tests() {
    export O=${O:-gpurun_out/r5/tests2}
    mkdir -p "$O"
    bash tools/gpu.sh tests
}

# X: mfma8s with per-wave deferral lists (no block barriers): classifier GPU
# tests; new vs previous kernel (abl/libmpx_old.so) at the default grid, then
# the new kernel at 16 / 32 / 64 / 128 blocks per CU, nc = 2 / 4 / 8, twice
ckpt_r5_lab3e() {
    export O=${O:-gpurun_out/r5/lab3e}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=2,4,8 LAB3_PATHS=mfma8 bash tools/gpu.sh ab lab3 abl/libmpx_old.so 2 -- \
        python -u tools/experiments/lab3_ab.py &&
    for r in 1 2; do
        for k in 16 32 64 128; do
            MPX_CLS_MFMA8S_GRID=$k LAB3_NCS=2,4,8 LAB3_PATHS=mfma8 LAB3_TAG=g${k}_$r \
                bash tools/gpu.sh run lab3_g${k}_$r 300 python -u tools/experiments/lab3_ab.py || return 1
        done
    done
}

# Y: non-temporal count-pass loads (MPX_SORT_COUNT_NT) for the 16384-key
# tiles, alternated three times at 2^26 (variant 22 = AUTO there)
ckpt_r5_cnt() {
    export O=${O:-gpurun_out/r5/cnt}
    mkdir -p "$O"
    for r in 1 2 3; do
        for nt in 0 1; do
            MPX_SORT_COUNT_NT=$nt SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=22 SORT_PROBE_LOGN=26 \
                SORT_PROBE_SMALL=0 bash tools/gpu.sh run probe_nt${nt}_$r 300 python -u tools/experiments/sort_probe.py \
                || return 1
        done
    done
}

# Z: the final tree as the driver will see it: smoke, the driver's bench
# command, the full GPU suite
ckpt_r5_last() {
    export O=${O:-gpurun_out/r5/last}
    mkdir -p "$O"
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh tests
}

# AA: fast32 with per-wave deferral lists: classifier GPU tests, then new vs
# previous kernel (abl/libmpx_old.so) alternated 3x at nc = 12 / 16 / 32
ckpt_r5_fast() {
    export O=${O:-gpurun_out/r5/fast}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=12,16,32 LAB3_PATHS=fast bash tools/gpu.sh ab lab3 abl/libmpx_old.so 3 -- \
        python -u tools/experiments/lab3_ab.py
}

# AB: mfma8 (32x32) with per-wave deferral lists: classifier GPU tests, then
# new vs previous kernel (abl/libmpx_old.so) alternated 3x at nc = 16 / 24 / 32
ckpt_r5_m8w() {
    export O=${O:-gpurun_out/r5/m8w}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=16,24,32 LAB3_PATHS=mfma8 bash tools/gpu.sh ab lab3 abl/libmpx_old.so 3 -- \
        python -u tools/experiments/lab3_ab.py
}

# AC: the 4x4x4 one-pixel-per-lane form at 9-16 classes (MPX_CLS_MFMA8S_MAX=16,
# row sets 5-8) against the 32x32 form and fast32, nc = 10 / 12 / 14 / 16, twice
ckpt_r5_small16() {
    export O=${O:-gpurun_out/r5/small16}
    mkdir -p "$O"
    for r in 1 2; do
        MPX_CLS_MFMA8S_MAX=16 LAB3_NCS=10,12,14,16 LAB3_PATHS=mfma8 LAB3_TAG=small_$r \
            bash tools/gpu.sh run small_$r 300 python -u tools/experiments/lab3_ab.py &&
        LAB3_NCS=10,12,14,16 LAB3_PATHS=mfma8,fast LAB3_TAG=base_$r \
            bash tools/gpu.sh run base_$r 300 python -u tools/experiments/lab3_ab.py || return 1
    done
}

# AD: AUTO with the 4x4x4 form up to 14 classes: classifier GPU tests (nc 1-14
# on the small form), then AUTO over nc = 2 .. 32 on three rotated images
ckpt_r5_auto14() {
    export O=${O:-gpurun_out/r5/auto14}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py -k "classify" &&
    LAB3_NCS=2,4,8,9,10,11,12,13,14,15,16,20,32 LAB3_PATHS=auto LAB3_TAG=auto \
        bash tools/gpu.sh run lab3_auto 400 python -u tools/experiments/lab3_ab.py
}

# AE: AUTO at nc = 15 (now the 32x32 form) and its neighbours, twice
ckpt_r5_auto15() {
    export O=${O:-gpurun_out/r5/auto15}
    mkdir -p "$O"
    for r in 1 2; do
        LAB3_NCS=14,15,16,17 LAB3_PATHS=auto,fast LAB3_TAG=r$r \
            bash tools/gpu.sh run lab3_auto_$r 300 python -u tools/experiments/lab3_ab.py || return 1
    done
}

# AF: 11-14 classes, the three forms side by side on one box, alternated
# twice: 4x4x4 (mfma8 path, default), 32x32 (MPX_CLS_MFMA8S_MAX=8), fast32
ckpt_r5_mid() {
    export O=${O:-gpurun_out/r5/mid}
    mkdir -p "$O"
    for r in 1 2; do
        LAB3_NCS=11,12,13,14 LAB3_PATHS=mfma8,fast LAB3_TAG=small_$r \
            bash tools/gpu.sh run small_$r 300 python -u tools/experiments/lab3_ab.py &&
        MPX_CLS_MFMA8S_MAX=8 LAB3_NCS=11,12,13,14 LAB3_PATHS=mfma8 LAB3_TAG=big_$r \
            bash tools/gpu.sh run big_$r 300 python -u tools/experiments/lab3_ab.py || return 1
    done
}

# AG: the final AUTO rule: classifier GPU tests, AUTO at nc = 2 .. 32 once
ckpt_r5_autofinal() {
    export O=${O:-gpurun_out/r5/autofinal}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_cpu_reference.py -k "classify" &&
    LAB3_NCS=2,4,8,9,12,14,15,16,20,32 LAB3_PATHS=auto LAB3_TAG=auto \
        bash tools/gpu.sh run lab3_auto 400 python -u tools/experiments/lab3_ab.py
}

# AH: the 2^26-key AUTO sort tests
ckpt_r5_sort26() {
    export O=${O:-gpurun_out/r5/sort26}
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_lab5_sort.py -k "auto_at_2_26 or lane_order"
}

# AI: uint8 counting sort at 2^26: kernel trace (hist vs fill split)
ckpt_r5_u8() {
    export O=${O:-gpurun_out/r5/u8}
    mkdir -p "$O"
    LAB5_DTYPES=uint8 LAB5_LOGN=26 LAB5_VARIANTS=0 bash tools/gpu.sh prof u8_trace -- python tools/experiments/lab5_bench.py &&
    python tools/experiments/kprof_table.py "$O" --grep u8 > "$O/kernels_table.md" && find "$O" -name "*.db" -delete
}

ckpt_r5_u8b() {
    export O=${O:-gpurun_out/r5/u8b}
    mkdir -p "$O"
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lab5_sort.py -m gpu -k "u8 or uchar" > "$O/tests.log" 2>&1 &&
    LAB5_DTYPES=uint8 LAB5_LOGN=26 LAB5_VARIANTS=0 bash tools/gpu.sh prof u8_trace -- python tools/experiments/lab5_bench.py &&
    python tools/experiments/kprof_table.py "$O" --grep u8 > "$O/kernels_table.md" && find "$O" -name "*.db" -delete
}

# AJ: uint8 counting sort at 2^26 after the bank-spread histogram: trace + counters
ckpt_r5_u8p() {
    export O=${O:-gpurun_out/r5/u8p}
    mkdir -p "$O"
    LAB5_DTYPES=uint8 LAB5_LOGN=26 LAB5_VARIANTS=0 bash tools/gpu.sh profile u8 -- python tools/experiments/lab5_bench.py &&
    python tools/experiments/kprof_table.py "$O" --grep u8 > "$O/kernels_table.md" && find "$O" -name "*.db" -delete
}

# AK: AUTO without onesweep (21 from 2^14 keys): lab5 GPU tests + small-n bench
ckpt_r5_small() {
    export O=${O:-gpurun_out/r5/small}
    mkdir -p "$O"
    timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lab5_sort.py tests/test_gpu_kernels.py -m gpu > "$O/tests.log" 2>&1 &&
    LAB5_DTYPES=int32,float32 LAB5_LOGN=12,14,16,17,18,19,20 LAB5_VARIANTS=1,21 LAB5_ITERS=30 timeout -k 10 300 python tools/experiments/lab5_bench.py > "$O/bench.log" 2>&1
}
