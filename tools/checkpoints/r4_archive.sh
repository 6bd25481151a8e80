# Round-4 GPU checkpoints, folded into one file (VERDICT r4 Next #7).
# Each former tools/checkpoints/gpu_r4_<x>.sh is the function ckpt_r4_<x>;
# run one with:  bash tools/gpu.sh checkpoint r4_<x>
# (the profiles/ pages cite their outputs under profiles/raw/r4/<x>/).

ckpt_r4_a() {
    # Round-4 checkpoint A on one MI355X: burst-tile copy probes,
    # then the mailbox / fused-streaming peer tests, the nccl-contract tests and
    # the headline torch oracles. Each step time-bounded, chained with &&.
    O=${O:-gpurun_out/r4/a}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run kbench_copy 300 python -u tools/kbench.py --only copy/ --rotate 6 --rounds 5 --iters 20 &&
    bash tools/gpu.sh tests tests/test_peer_halo.py -k "stream or beyond or jacobi_peer_signalled_equals" &&
    cp "$O/pytest.log" "$O/pytest_peer.log" &&
    bash tools/gpu.sh tests tests/test_contract.py &&
    cp "$O/pytest.log" "$O/pytest_contract.log" &&
    bash tools/gpu.sh tests tests/test_gpu_headline.py tests/test_gpu_kernels.py -k "oracle or fast_sqrt"
}

ckpt_r4_aa() {
    # Round-4 checkpoint AA: the driver's bench command three times on one box and
    # a kernel trace of it (hardware queue of each phase's streams).
    O=${O:-gpurun_out/r4/aa}
    export O
    mkdir -p "$O"
    for r in 1 2 3; do
      bash tools/gpu.sh run bench_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    done &&
    bash tools/gpu.sh prof trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
    python tools/experiments/trace_db.py "$O/trace" --top 5 > "$O/trace.md" && find "$O" -name "*.db" -size +20M -delete
}

ckpt_r4_b() {
    # Round-4 checkpoint B: more copy probes (band copies with NT loads, burst
    # tiles with a one-workgroup-per-CU residency cap), then the peer / contract /
    # oracle GPU tests. Each step time-bounded, chained with &&.
    O=${O:-gpurun_out/r4/b}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run kbench_copy2 300 python -u tools/kbench.py --only copy/ --rotate 6 --rounds 5 --iters 20 &&
    bash tools/gpu.sh tests tests/test_peer_halo.py &&
    cp "$O/pytest.log" "$O/pytest_peer.log" &&
    bash tools/gpu.sh tests tests/test_contract.py &&
    cp "$O/pytest.log" "$O/pytest_contract.log" &&
    bash tools/gpu.sh tests tests/test_gpu_headline.py tests/test_gpu_kernels.py -k "oracle or fast_sqrt"
}

ckpt_r4_bb() {
    # Round-4 checkpoint BB (final tree): the full GPU suite and smoke.
    O=${O:-gpurun_out/r4/bb}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh tests && bash tools/gpu.sh smoke
}

ckpt_r4_c() {
    # Round-4 checkpoint C: bench.py A/B of the 2-stream alternation and of the
    # time-based warm-up (driver command: --steps 20 --warmup 5), alternated
    # twice, then a kernel trace of the default bench. Time-bounded steps.
    O=${O:-gpurun_out/r4/c}
    export O
    mkdir -p "$O"
    B="python bench.py --gpus 1 --steps 20 --warmup 5"
    bash tools/gpu.sh run bench_default 300 $B &&
    for r in 1 2; do
      bash tools/gpu.sh run ab_s2_w30_$r 200 $B --no-cpu-baseline --no-stream &&
      bash tools/gpu.sh run ab_s1_w30_$r 200 $B --no-cpu-baseline --no-stream --streams 1 &&
      bash tools/gpu.sh run ab_s2_w0_$r 200 $B --no-cpu-baseline --no-stream --warmup-ms 0 &&
      bash tools/gpu.sh run ab_s1_w0_$r 200 $B --no-cpu-baseline --no-stream --streams 1 --warmup-ms 0 || exit 1
    done &&
    bash tools/gpu.sh prof bench_trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh run lab3_grid 400 python -u tools/experiments/lab3_grid_sweep.py
}

ckpt_r4_cc() {
    # Round-4 checkpoint CC: lean onesweep at 1 block per CU (variant 15) vs 2 (14)
    # vs the AUTO reduce-then-scan (12).
    O=${O:-gpurun_out/r4/cc}
    export O
    mkdir -p "$O"
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14,15 SORT_PROBE_SMALL=1 bash tools/gpu.sh run sort_os1 300 \
      python -u tools/experiments/sort_probe.py
}

ckpt_r4_d() {
    # Round-4 checkpoint D: the vertical-halo-sharing band kernel (conv_band16v)
    # against production and the copy floors, its GPU test, then checkpoint C
    # (bench A/B of streams / warm-up, kernel trace, lab3 grid sweep).
    O=${O:-gpurun_out/r4/d}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run kbench_vs 300 python -u tools/kbench.py --rotate 6 --rounds 7 --iters 20 \
        --only "band16v,sobel5/production,gauss5/production,band4/seg0/w34000,copy/band-seg16-f106,copy/band-seg16-f74,copy/linear" &&
    bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "vertical_share or strip_edges or fast_sqrt" &&
    cp "$O/pytest.log" "$O/pytest_vs.log" &&
    O=gpurun_out/r4/c bash tools/gpu_r4_c.sh
}

ckpt_r4_dd() {
    # Round-4 checkpoint DD: lean onesweep with a static tile order (variant 16,
    # no tile counter) vs the counter form (14) and AUTO (12); its GPU tests.
    O=${O:-gpurun_out/r4/dd}
    export O
    mkdir -p "$O"
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,16,14 bash tools/gpu.sh run sort_os_static 300 \
      python -u tools/experiments/sort_probe.py &&
    bash tools/gpu.sh tests tests/test_lab5_sort.py -k "variants and 16"
}

ckpt_r4_e() {
    # Round-4 checkpoint E: bench.py over the stream count (2 / 3 / 6) and band
    # modes under 2 streams, alternated; lab3 grid sweep with larger grids.
    O=${O:-gpurun_out/r4/e}
    export O
    mkdir -p "$O"
    B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-stream"
    bash tools/gpu.sh run bench_default 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    for r in 1 2; do
      bash tools/gpu.sh run s2_$r 200 $B &&
      bash tools/gpu.sh run s3_$r 200 $B --streams 3 &&
      bash tools/gpu.sh run s6_$r 200 $B --streams 6 &&
      MPX_CONV_BAND=4 bash tools/gpu.sh run s2_band4_$r 200 $B &&
      MPX_CONV_BAND=2 bash tools/gpu.sh run s2_band2_$r 200 $B || exit 1
    done &&
    LAB3_NCS=2,4,32 LAB3_GRIDS=0,2048,4096,8192,16384 bash tools/gpu.sh run lab3_grid 400 python -u tools/experiments/lab3_grid_sweep.py &&
    bash tools/gpu.sh prof bench_trace -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
}

ckpt_r4_ee() {
    # Round-4 checkpoint EE: stream-set test and the driver's bench command.
    O=${O:-gpurun_out/r4/ee}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_streams.py tests/test_lab5_sort.py -k "streams or variants" &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
}

ckpt_r4_f() {
    # Round-4 checkpoint F: radix scatter attribution (knock-out probes, times and
    # LDS counters) and the returning-add ranking (variant 9) vs production.
    O=${O:-gpurun_out/r4/f}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run sort_probe 300 python -u tools/experiments/sort_probe.py &&
    SORT_PROBE_ITERS=1 SORT_PROBE_PARTS=knock bash tools/gpu.sh pmc probe_lds \
      "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES" -- python3 tools/experiments/sort_probe.py &&
    SORT_PROBE_ITERS=1 SORT_PROBE_PARTS=knock bash tools/gpu.sh prof probe_trace -- python3 tools/experiments/sort_probe.py &&
    bash tools/gpu.sh tests tests/test_lab5_sort.py
}

ckpt_r4_ff() {
    # Round-4 checkpoint FF: step_twin test; bench with the two-stream
    # cache-resident pass (value_warm_cache) beside the one-stream one.
    O=${O:-gpurun_out/r4/ff}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_streams.py &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh run bench50 300 python bench.py --gpus 1 --steps 50 --warmup 5
}

ckpt_r4_g() {
    # Round-4 checkpoint G: sort ranking variants (7 production, 9 returning-add,
    # 10 = 9 on 4096-key tiles, 11 = 9 at 3 blocks/CU) timed, traced and counted;
    # lab3 fast32 memory-policy variants and the mfma8 windowed fix-ups A/B'd,
    # mfma8 write bytes; the lab3 / lab5 GPU suites on the new kernels.
    O=${O:-gpurun_out/r4/g}
    export O
    mkdir -p "$O"
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=7,8,9,10,11 bash tools/gpu.sh run sort_variants 300 \
      python -u tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=2 \
      bash tools/gpu.sh prof sort_v9_trace -- python3 tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=7,9 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
      bash tools/gpu.sh pmc sort_v79_lds "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES" \
      -- python3 tools/experiments/sort_probe.py &&
    for r in 1 2; do
      for o in 0 1 2 3 4 7; do
        MPX_CLS_OPT=$o LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run lab3_fast_o${o}_r$r 200 \
          python -u tools/experiments/lab3_ab.py || exit 1
      done
      for wv in 0 1; do
        MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=8,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_w${wv}_r$r 200 \
          python -u tools/experiments/lab3_ab.py || exit 1
      done
    done &&
    for wv in 0 1; do
      MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=32 LAB3_PATHS=mfma8 bash tools/gpu.sh pmc lab3_mfma8_w${wv}_bytes "WRITE_SIZE" \
        -- python3 tools/experiments/lab3_ab.py || exit 1
    done &&
    bash tools/gpu.sh tests tests/test_lab5_sort.py tests/test_classify_i8.py tests/test_gpu_kernels.py tests/test_gpu_headline.py
}

ckpt_r4_gg() {
    # Round-4 checkpoint GG: bench.py with 2 vs 3 compute streams, alternated
    # (3 streams were last measured before the process-wide stream pool).
    O=${O:-gpurun_out/r4/gg}
    export O
    mkdir -p "$O"
    for i in 1 2; do
      bash tools/gpu.sh run s2_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --streams 2 &&
      bash tools/gpu.sh run s3_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --streams 3 || exit 1
    done
}

ckpt_r4_h() {
    # Round-4 checkpoint H: bench.py (streaming phase now on 2 streams) and the
    # stream count A/B; mfma8 windowed fix-ups with a single chunk body; lab5 with
    # the new AUTO (returning-add ranking); kernel trace of the bench; GPU tests.
    O=${O:-gpurun_out/r4/h}
    export O
    mkdir -p "$O"
    B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-stream"
    bash tools/gpu.sh run bench_default 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    for r in 1 2; do
      bash tools/gpu.sh run s1_$r 200 $B --streams 1 &&
      bash tools/gpu.sh run s2_$r 200 $B &&
      bash tools/gpu.sh run s3_$r 200 $B --streams 3 || exit 1
      for wv in 0 1; do
        MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=8,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_w${wv}_r$r 200 \
          python -u tools/experiments/lab3_ab.py || exit 1
      done
    done &&
    LAB5_DTYPES=int32,float32 LAB5_LOGN=20,24,26 LAB5_VARIANTS=7,9,10 bash tools/gpu.sh run lab5 300 \
      python -u tools/experiments/lab5_bench.py &&
    bash tools/gpu.sh prof bench_trace -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh tests tests/test_lab5_sort.py tests/test_gpu_kernels.py -k "sort or radix or classify"
}

ckpt_r4_hh() {
    # Round-4 checkpoint HH: checkpoint Z again after the clock moved before the closing
    # barrier (each rank stops at its own device sync); bench launch and contract tests.
    O=${O:-gpurun_out/r4/hh}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n2 300 python bench.py --gpus 2 --steps 20 --warmup 5 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n4 300 python bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh tests tests/test_gpu_bench_launch.py tests/test_contract.py
}

ckpt_r4_i() {
    # Round-4 checkpoint I: the streaming phase on 1 vs 2 streams (N = 1, both
    # phases), the fused streaming halo rehearsed at 2 and 4 ranks on one GPU
    # (retained vs N = 1) with a kernel trace of the 2-rank run (one dispatch per
    # streaming step), and the radix scatter's HBM bytes for 8192- vs 4096-key tiles.
    O=${O:-gpurun_out/r4/i}
    export O
    mkdir -p "$O"
    B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
    for r in 1 2; do
      bash tools/gpu.sh run n1_s1_$r 200 $B --gpus 1 --streams 1 &&
      bash tools/gpu.sh run n1_s2_$r 200 $B --gpus 1 || exit 1
    done &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n2 300 $B --gpus 2 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n4 300 $B --gpus 4 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh prof n2_trace -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --gpus 2 &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
      bash tools/gpu.sh pmc sort_wr "WRITE_SIZE" -- python3 tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
      bash tools/gpu.sh pmc sort_rd "FETCH_SIZE" -- python3 tools/experiments/sort_probe.py &&
    bash tools/gpu.sh jpeer 2 4 && bash tools/gpu.sh mgpu jacobi --halo peer --shared --gpus 2 --size 16384
    [ $? -eq 0 ] || exit 1
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,12,10,13 bash tools/gpu.sh run sort_pf2 300 \
      python -u tools/experiments/sort_probe.py
}

ckpt_r4_ii() {
    # Round-4 checkpoint II: host wait policy A/B (MPX_HIP_WAIT=auto, the HIP
    # default, vs spin) on the driver's bench command, alternated twice.
    O=${O:-gpurun_out/r4/ii}
    export O
    mkdir -p "$O"
    for i in 1 2; do
      MPX_HIP_WAIT=auto bash tools/gpu.sh run auto_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
      MPX_HIP_WAIT=spin bash tools/gpu.sh run spin_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    done
}

ckpt_r4_j() {
    # Round-4 checkpoint J: streaming-phase stream count at 2 ranks (rehearsal),
    # N = 1 default bench (streaming back on one stream), radix 2-deep prefetch
    # variants and HBM bytes, Jacobi peer cost with mailboxes.
    O=${O:-gpurun_out/r4/j}
    export O
    mkdir -p "$O"
    B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
    bash tools/gpu.sh run n1 200 $B --gpus 1 &&
    for r in 1 2; do
      MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n2_ss1_$r 300 $B --gpus 2 --stream-streams 1 &&
      MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n2_ss2_$r 300 $B --gpus 2 --stream-streams 2 || exit 1
    done &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,12,10,13 bash tools/gpu.sh run sort_pf2 300 \
      python -u tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10,12 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
      bash tools/gpu.sh pmc sort_wr "WRITE_SIZE" -- python3 tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10,12 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
      bash tools/gpu.sh pmc sort_rd "FETCH_SIZE" -- python3 tools/experiments/sort_probe.py &&
    bash tools/gpu.sh jpeer 2 4 &&
    bash tools/gpu.sh mgpu jacobi --halo peer --shared --gpus 2 --size 16384
}

ckpt_r4_jj() {
    # Round-4 checkpoint JJ: kernel trace of bench.py (N = 1, no sustain / warm
    # passes) to compare the static and streaming phases burst by burst.
    O=${O:-gpurun_out/r4/jj}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh prof bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --sustain-ms 0 --no-warm --no-cpu-baseline &&
    python3 tools/experiments/phase_trace.py "$O/bench" > "$O/phases.md" &&
    python3 tools/experiments/trace_db.py "$O/bench" > "$O/kernels.md" &&
    find "$O/bench" -name "*.db" -delete
}

ckpt_r4_k() {
    # Round-4 checkpoint K: the lean onesweep (variant 14) against the PF-2 lean
    # scatters (12 / 13, the new AUTO): times on every stability case, HBM bytes,
    # kernel trace; the sort GPU suite.
    O=${O:-gpurun_out/r4/k}
    export O
    mkdir -p "$O"
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14,13 bash tools/gpu.sh run sort_os 300 \
      python -u tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=14 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=2 \
      bash tools/gpu.sh prof sort_os_trace -- python3 tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
      bash tools/gpu.sh pmc sort_os_wr "WRITE_SIZE" -- python3 tools/experiments/sort_probe.py &&
    bash tools/gpu.sh tests tests/test_lab5_sort.py
}

ckpt_r4_kk() {
    # Round-4 checkpoint KK: does value_streaming trail value because its phase
    # runs after ~50 ms of sustained load and the warm passes? The driver's bench
    # command with and without those passes, alternated.
    O=${O:-gpurun_out/r4/kk}
    export O
    mkdir -p "$O"
    for i in 1 2; do
      bash tools/gpu.sh run full_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
      bash tools/gpu.sh run bare_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --no-warm || exit 1
    done
}

ckpt_r4_l() {
    # Round-4 checkpoint L: lean onesweep look-back window 8 / 16 / 32 vs the PF-2
    # lean scatter (AUTO); sort GPU suite.
    O=${O:-gpurun_out/r4/l}
    export O
    mkdir -p "$O"
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14,15,16 SORT_PROBE_SMALL=0 bash tools/gpu.sh run sort_lbw 300 \
      python -u tools/experiments/sort_probe.py &&
    bash tools/gpu.sh tests tests/test_lab5_sort.py -k "radix_variants"
}

ckpt_r4_ll() {
    # Round-4 checkpoint LL: is the conv's time data dependent (value_streaming
    # trails value by ~6 %; its kernels ran ~6 % longer in trace JJ)?
    O=${O:-gpurun_out/r4/ll}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run datadep 300 python tools/experiments/conv_data_dep.py
}

ckpt_r4_m() {
    # Round-4 checkpoint M: fast32 with interleaved FMA chains (MPX_CLS_OPT=8)
    # against the default, alternated twice; mfma8's fp32 re-rank stage on/off;
    # the classify env-variant tests.
    O=${O:-gpurun_out/r4/m}
    export O
    mkdir -p "$O"
    for r in 1 2; do
      for o in 0 8 10; do
        MPX_CLS_OPT=$o LAB3_NCS=2,4,8,16,32 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run lab3_fast_o${o}_r$r 200 \
          python -u tools/experiments/lab3_ab.py || exit 1
      done
      for f in 1 0; do
        MPX_CLS_MFMA8_FP32=$f LAB3_NCS=16,24,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_fp32_${f}_r$r 200 \
          python -u tools/experiments/lab3_ab.py || exit 1
      done
    done &&
    bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "classify"
}

ckpt_r4_mm() {
    # Round-4 checkpoint MM: host enqueue time per step (static vs streaming
    # phase) beside the step time; the driver's bench command twice.
    O=${O:-gpurun_out/r4/mm}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run b1 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh run b2 300 python bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu-baseline
}

ckpt_r4_n() {
    # Round-4 checkpoint N: mfma8 windowed fix-ups (now with the fp32 stage) vs
    # after-loop, with write bytes; then the full GPU suite.
    O=${O:-gpurun_out/r4/n}
    export O
    mkdir -p "$O"
    for r in 1 2; do
      for wv in 0 1; do
        MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=16,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_w${wv}_r$r 200 \
          python -u tools/experiments/lab3_ab.py || exit 1
      done
    done &&
    for wv in 0 1; do
      MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=32 LAB3_PATHS=mfma8 bash tools/gpu.sh pmc lab3_mfma8_w${wv}_bytes "WRITE_SIZE" \
        -- python3 tools/experiments/lab3_ab.py || exit 1
    done &&
    bash tools/gpu.sh tests
}

ckpt_r4_nn() {
    # Round-4 checkpoint NN (checkpoint X again, after the clock change): the scaling driver's one-GPU rehearsal (ranks share the
    # GPU) at 1 / 2 / 4 ranks over every multi-GPU workload.
    O=${O:-gpurun_out/r4/nn}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run scale 1000 python -u tools/scale.py --gpus 1,2,4 --rehearse --out "$O/scaling" --timeout 300
}

ckpt_r4_o() {
    # Round-4 checkpoint O (final tree): smoke, bench, and the per-kernel profile
    # (kernel trace + the standard counter passes over tools/prof_all.py),
    # summarised on the box (the rocpd databases exceed gpurun's 64 MiB return).
    O=${O:-gpurun_out/r4/o}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py &&
    bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py &&
    python tools/experiments/kprof_table.py "$O" > "$O/kernels_table.md" &&
    python tools/experiments/kprof_table.py "$O" --grep "<" > /dev/null &&
    python tools/pmc_median.py "$O"/kfinal.pmc* > "$O/medians.md" &&
    python tools/experiments/trace_db.py "$O/kfinal" --top 40 > "$O/trace.md" &&
    du -sh "$O" && find "$O" -name "*.db" -delete && du -sh "$O"
}

ckpt_r4_oo() {
    # Round-4 checkpoint OO (final tree): the full GPU suite, smoke, and the
    # driver's bench command.
    O=${O:-gpurun_out/r4/oo}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh tests && bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
}

ckpt_r4_p() {
    # Round-4 checkpoint P: copy floors and conv schedules with launches
    # overlapped on 2 streams (the bench's regime) vs one stream.
    O=${O:-gpurun_out/r4/p}
    export O
    mkdir -p "$O"
    V="copy/linear,copy/band-seg16-f106,copy/band-seg16-f74,copy/band-seg16-f10,copy/burst-r16-t512-f7,copy/burst-r8-t256-f4,copy/burst-r16-t1024-f15,sobel5/production,copy/torch"
    bash tools/gpu.sh run kb_s2 300 python -u tools/kbench.py --rotate 6 --streams 2 --rounds 5 --only "$V" &&
    bash tools/gpu.sh run kb_s1 300 python -u tools/kbench.py --rotate 6 --streams 1 --rounds 5 --only "$V" &&
    bash tools/gpu.sh run kb_s3 300 python -u tools/kbench.py --rotate 6 --streams 3 --rounds 5 --only "$V"
}

ckpt_r4_pp() {
    # Round-4 checkpoint PP: the timed region's fixed cost, T(K) for K = 0..50.
    O=${O:-gpurun_out/r4/pp}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run timed_k 300 python tools/experiments/timed_k.py
}

ckpt_r4_q() {
    # Round-4 checkpoint Q: fast32 with two trips of loads in flight (OPT 24 / 26)
    # against the default (8), alternated twice; classify tests.
    O=${O:-gpurun_out/r4/q}
    export O
    mkdir -p "$O"
    for r in 1 2; do
      for o in 8 24 26; do
        MPX_CLS_OPT=$o LAB3_NCS=2,4,8,16,32 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run lab3_fast_o${o}_r$r 200 \
          python -u tools/experiments/lab3_ab.py || exit 1
      done
    done &&
    bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "classify"
}

ckpt_r4_qq() {
    # Round-4 checkpoint QQ: kernel trace of the T(K) probe (queues and per-burst
    # overlap of the K-step runs).
    O=${O:-gpurun_out/r4/qq}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh prof tk -- python3 tools/experiments/timed_k.py &&
    python3 tools/experiments/phase_trace.py "$O/tk" --gap 3 > "$O/phases.md"
}

ckpt_r4_r() {
    # Round-4 checkpoint R: fast32 vs mfma8 over nc (AUTO re-derived with the
    # fp32 re-rank stage), two rounds.
    O=${O:-gpurun_out/r4/r}
    export O
    mkdir -p "$O"
    for r in 1 2; do
      LAB3_NCS=6,8,10,12,13,14,15,16,17,18,19,20,21,22,23,24,28,32 LAB3_PATHS=fast,mfma8 LAB3_TAG=r$r \
        bash tools/gpu.sh run lab3_nc_sweep_r$r 400 python -u tools/experiments/lab3_ab.py || exit 1
    done
}

ckpt_r4_rr() {
    # Round-4 checkpoint RR (final tree): the one-GPU benchmark suite, every
    # workload at its BASELINE size, verified.
    O=${O:-gpurun_out/r4/rr}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run suite 600 python tools/bench_suite.py
}

ckpt_r4_s() {
    # Round-4 checkpoint S: load policy per regime — band mode 3 (NT interior
    # loads, default) vs 2 (plain loads) on all three bench numbers (streaming
    # from HBM, streaming iterated frames, one cache-resident pair).
    O=${O:-gpurun_out/r4/s}
    export O
    mkdir -p "$O"
    B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --gpus 1"
    for r in 1 2; do
      bash tools/gpu.sh run m3_$r 200 $B &&
      MPX_CONV_BAND=2 bash tools/gpu.sh run m2_$r 200 $B || exit 1
    done
}

ckpt_r4_ss() {
    # Round-4 checkpoint SS: variant 17 (a counter row per half-wave) — the sort
    # variant tests, then 12 vs 17 alternated at 2^24 / 2^26 int32 / float32.
    O=${O:-gpurun_out/r4/ss}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh tests tests/test_lab5_sort.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,17 SORT_PROBE_SMALL=1 \
      bash tools/gpu.sh run probe1 300 python tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=17,12 SORT_PROBE_SMALL=0 \
      bash tools/gpu.sh run probe2 300 python tools/experiments/sort_probe.py
}

ckpt_r4_tt() {
    # Round-4 checkpoint TT (final tree, after the sort variant-17 rebuild): the full GPU suite, smoke, and the
    # driver's bench command.
    O=${O:-gpurun_out/r4/tt}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh tests && bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
}

ckpt_r4_u() {
    # Round-4 checkpoint U: fast32 at 4 pixels per thread (5 waves per SIMD) with
    # interleaved chains and two trips in flight, small nc, alternated twice.
    O=${O:-gpurun_out/r4/u}
    export O
    mkdir -p "$O"
    for r in 1 2; do
      LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run nq2_o8_r$r 200 python -u tools/experiments/lab3_ab.py &&
      MPX_CLS_NQ=1 MPX_CLS_OPT=8 LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run nq1_o8_r$r 200 python -u tools/experiments/lab3_ab.py &&
      MPX_CLS_NQ=1 MPX_CLS_OPT=24 LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run nq1_o24_r$r 200 python -u tools/experiments/lab3_ab.py || exit 1
    done
}

ckpt_r4_uu() {
    # Round-4 checkpoint UU (final tree, checkpoint O again after the last native rebuild): smoke, bench, and the per-kernel profile
    # (kernel trace + the standard counter passes over tools/prof_all.py),
    # summarised on the box (the rocpd databases exceed gpurun's 64 MiB return).
    O=${O:-gpurun_out/r4/uu}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py &&
    bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py &&
    python tools/experiments/kprof_table.py "$O" > "$O/kernels_table.md" &&
    python tools/experiments/kprof_table.py "$O" --grep "<" > /dev/null &&
    python tools/pmc_median.py "$O"/kfinal.pmc* > "$O/medians.md" &&
    python tools/experiments/trace_db.py "$O/kfinal" --top 40 > "$O/trace.md" &&
    du -sh "$O" && find "$O" -name "*.db" -delete && du -sh "$O"
}

ckpt_r4_v() {
    # Round-4 checkpoint V (final tree): full GPU suite, smoke, the driver's bench
    # command, and the 2-rank rehearsal bench.
    O=${O:-gpurun_out/r4/v}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh tests &&
    bash tools/gpu.sh smoke &&
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n2 300 python bench.py --gpus 2 --steps 20 --warmup 5
}

ckpt_r4_vv() {
    # Round-4 checkpoint VV (final tree): lab3 on three rotated 8192^2 images
    # (the lab3_classify.md methodology) for the README's figures, and the
    # driver's bench command twice more.
    O=${O:-gpurun_out/r4/vv}
    export O
    mkdir -p "$O"
    LAB3_NCS=4,16,32 LAB3_PATHS=fast,mfma8,auto bash tools/gpu.sh run lab3 300 python tools/experiments/lab3_ab.py &&
    bash tools/gpu.sh run bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh run bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
}

ckpt_r4_w() {
    # Round-4 checkpoint W: float32's skewed last pass on the peer-mask ranking
    # (variant 15) vs the returning add (12, AUTO); the sort GPU suite.
    O=${O:-gpurun_out/r4/w}
    export O
    mkdir -p "$O"
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,15 SORT_PROBE_ITERS=9 bash tools/gpu.sh run sort_v15 300 \
      python -u tools/experiments/sort_probe.py &&
    SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=15,12 SORT_PROBE_ITERS=9 SORT_PROBE_SMALL=0 bash tools/gpu.sh run sort_v15b 300 \
      python -u tools/experiments/sort_probe.py &&
    bash tools/gpu.sh tests tests/test_lab5_sort.py
}

ckpt_r4_x() {
    # Round-4 checkpoint X: the scaling driver's one-GPU rehearsal (ranks share the
    # GPU) at 1 / 2 / 4 ranks over every multi-GPU workload.
    O=${O:-gpurun_out/r4/x}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run scale 1000 python -u tools/scale.py --gpus 1,2,4 --rehearse --out "$O/scaling" --timeout 300
}

ckpt_r4_y() {
    # Round-4 checkpoint Y: the streaming phase on the static phase's two streams
    # (one process-wide stream set) vs one stream, N = 1, alternated; trace.
    O=${O:-gpurun_out/r4/y}
    export O
    mkdir -p "$O"
    B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
    for r in 1 2; do
      bash tools/gpu.sh run ss1_$r 200 $B --stream-streams 1 &&
      bash tools/gpu.sh run ss2_$r 200 $B --stream-streams 2 || exit 1
    done &&
    bash tools/gpu.sh prof ss2_trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --stream-streams 2 &&
    python tools/experiments/trace_db.py "$O/ss2_trace" --top 5 > "$O/ss2_trace.md" && find "$O" -name "*.db" -size +20M -delete
}

ckpt_r4_z() {
    # Round-4 checkpoint Z: the driver's bench command and the 2-rank rehearsal
    # on the stream-pool tree, with a trace of the N = 1 run (queue ids); bench
    # launch tests.
    O=${O:-gpurun_out/r4/z}
    export O
    mkdir -p "$O"
    bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n2 300 python bench.py --gpus 2 --steps 20 --warmup 5 &&
    MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n4 300 python bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh tests tests/test_gpu_bench_launch.py tests/test_contract.py
}
