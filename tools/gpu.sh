#!/bin/bash
# One driver for every GPU-box step (run through gpurun; each step under its
# own time limit, output under $O = gpurun_out/<tag>, exit non-zero on the
# first failure so a calling `&&` chain stops there):
#
#   O=gpurun_out/r3/x bash tools/gpu.sh tests [pytest args...]     # -m gpu suite (or a subset)
#   O=...             bash tools/gpu.sh smoke                       # __graft_entry__.smoke()
#   O=...             bash tools/gpu.sh bench [bench.py args...]    # one JSON line -> $O/bench.json
#   O=...             bash tools/gpu.sh prof NAME -- CMD...         # rocprofv3 kernel trace + stats
#   O=...             bash tools/gpu.sh pmc NAME "C1 C2 ..." -- CMD...   # one counter pass
#   O=...             bash tools/gpu.sh jpeer [N...]                # device-signalled Jacobi: peer vs no-exchange
#   O=...             bash tools/gpu.sh run NAME SECONDS CMD...     # any command, logged, time-bounded
#   O=...             bash tools/gpu.sh checkpoint                  # tests + smoke + bench
set -o pipefail
O=${O:-gpurun_out/scratch}
mkdir -p "$O"
cd /tmp 2>/dev/null && cd - >/dev/null
export TMPDIR=/tmp
cmd=$1; shift

fail() { echo "[gpu.sh] $1 failed (rc $2); tail of $3:"; tail -30 "$3"; exit "$2"; }

case "$cmd" in
  tests)
    args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests)
    timeout -k 10 1000 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu "${args[@]}" \
        > "$O/pytest.log" 2>&1 || fail tests $? "$O/pytest.log"
    grep -E "passed|failed" "$O/pytest.log" | tail -1 ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || fail smoke $? "$O/smoke.log"
    tail -1 "$O/smoke.log" ;;
  bench)
    timeout -k 10 400 python bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" || fail bench $? "$O/bench.err"
    grep '^{' "$O/bench.json" | tail -1 | cut -c1-400 ;;
  prof)
    name=$1; shift; [ "$1" = "--" ] && shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/$name" -o "$name" -- "$@" > "$O/$name.log" 2>&1 \
        || fail "prof $name" $? "$O/$name.log"
    find "$O/$name" -name "*kernel_stats.csv" | head -1 | xargs -r head -12 ;;
  pmc)
    name=$1; ctrs=$2; shift 2; [ "$1" = "--" ] && shift
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$O/$name" -o "$name" -- "$@" > "$O/$name.log" 2>&1 \
        || fail "pmc $name" $? "$O/$name.log"
    echo "pmc $name done" ;;
  jpeer)
    ns=("$@"); [ ${#ns[@]} -eq 0 ] && ns=(2 4)
    for n in "${ns[@]}"; do
      for h in peer none; do
        MPX_DIST_BACKEND=gloo timeout -k 10 200 python -u tools/bench_jacobi.py --gpus "$n" --halo "$h" \
            --iters 400 --warmup 40 > "$O/j_${h}${n}.json" 2>&1 || fail "jpeer $h$n" $? "$O/j_${h}${n}.json"
        echo "jacobi16384 $h n=$n $(grep -o '"ms_per_iter": [0-9.]*' "$O/j_${h}${n}.json")"
        MPX_DIST_BACKEND=gloo timeout -k 10 200 python -u tools/bench_jacobi.py --gpus "$n" --halo "$h" \
            --rows $((64 * n)) --iters 2000 --warmup 100 > "$O/js_${h}${n}.json" 2>&1 \
            || fail "jpeer small $h$n" $? "$O/js_${h}${n}.json"
        echo "jacobi64rows $h n=$n $(grep -o '"ms_per_iter": [0-9.]*' "$O/js_${h}${n}.json")"
      done
    done ;;
  run)
    name=$1; secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1 || fail "$name" $? "$O/$name.log"
    tail -3 "$O/$name.log" ;;
  checkpoint)
    bash "$0" tests && bash "$0" smoke && bash "$0" bench ;;
  *)
    sed -n 2,14p "$0"; exit 2 ;;
esac
