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
#   O=...             bash tools/gpu.sh profile NAME -- CMD...      # trace + the standard counter groups
#   O=...             bash tools/gpu.sh ab NAME LIB ROUNDS -- CMD...  # CMD alternately on libmpx / LIB
#   O=...             bash tools/gpu.sh mgpu [ARGS...]              # native runtime: N-rank == one-device
#   O=...             bash tools/gpu.sh jpeer [N...]                # device-signalled Jacobi: peer vs no-exchange
#   O=...             bash tools/gpu.sh run NAME SECONDS CMD...     # any command, logged, time-bounded
#   O=...             bash tools/gpu.sh checkpoint [NAME]           # tests + smoke + bench, or ckpt_NAME
#                                                                   # of tools/checkpoints/*.sh
#
# Counter groups respect the per-block limits (<= 8 SQ, 4 TCC, 2 GRBM per pass);
# FETCH_SIZE / WRITE_SIZE get passes of their own. tools/pmc_median.py merges
# the passes (median per kernel); tools/prof_summary.py writes the tables.
set -o pipefail
O_GIVEN=${O:-}
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
    # one result file per process (%pid%): ranks launched as children would
    # otherwise finalise into the same sqlite file (disk I/O error, abort, hang)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/$name" -o "${name}_%pid%" -- "$@" > "$O/$name.log" 2>&1 \
        || fail "prof $name" $? "$O/$name.log"
    find "$O/$name" -name "*kernel_stats.csv" | head -1 | xargs -r head -12 ;;
  pmc)
    name=$1; ctrs=$2; shift 2; [ "$1" = "--" ] && shift
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$O/$name" -o "${name}_%pid%" -- "$@" > "$O/$name.log" 2>&1 \
        || fail "pmc $name" $? "$O/$name.log"
    echo "pmc $name done" ;;
  profile)
    name=$1; shift; [ "$1" = "--" ] && shift
    bash "$0" prof "$name" -- "$@" || exit $?
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
               "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
               "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" \
               "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
               "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
      i=$((i + 1))
      bash "$0" pmc "$name.pmc$i" "$grp" -- "$@" || exit $?
    done ;;
  ab)
    name=$1; lib=$2; rounds=$3; shift 3; [ "$1" = "--" ] && shift
    for r in $(seq 1 "$rounds"); do
      timeout -k 10 300 "$@" > "$O/$name.a$r.log" 2>&1 || fail "ab $name a$r" $? "$O/$name.a$r.log"
      MPX_LIB_PATH="$lib" timeout -k 10 300 "$@" > "$O/$name.b$r.log" 2>&1 || fail "ab $name b$r" $? "$O/$name.b$r.log"
    done
    echo "ab $name: $rounds rounds in $O/$name.{a,b}N.log" ;;
  mgpu)
    args=("$@"); [ ${#args[@]} -eq 0 ] && args=(jacobi --halo peer --shared --gpus 2 --size 4096)
    timeout -k 10 200 bin/mpx_mgpu "${args[@]}" > "$O/mgpu.json" 2> "$O/mgpu.err"; rc=$?
    echo "mpx_mgpu ${args[*]}: rc=$rc $(grep -o '"verified": [a-z]*\|"one_device_equal": [a-z]*' "$O/mgpu.json" | tr '\n' ' ')"
    head -c 900 "$O/mgpu.err"
    [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc ;;
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
    # no name: tests + smoke + bench; NAME: the function ckpt_NAME of the
    # checkpoint table (tools/checkpoints/*.sh: r5.sh this round, r4_archive.sh)
    if [ $# -eq 0 ]; then
      bash "$0" tests && bash "$0" smoke && bash "$0" bench
    else
      here=$(dirname "$0")
      for f in "$here"/checkpoints/*.sh; do . "$f"; done
      declare -F "ckpt_$1" >/dev/null || { echo "[gpu.sh] no checkpoint $1"; exit 2; }
      [ -n "$O_GIVEN" ] || unset O  # the checkpoint's own default output directory
      name=$1; shift
      "ckpt_$name" "$@"
    fi ;;
  *)
    sed -n 2,21p "$0"; exit 2 ;;
esac
