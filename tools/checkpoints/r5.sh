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
