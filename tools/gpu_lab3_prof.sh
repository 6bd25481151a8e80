#!/bin/bash
# lab3: tests, suite, kernel-trace stats and PMC counters per classifier path.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
mkdir -p gpurun_out/lab3prof
if [ "$1" != "--prof-only" ]; then
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k classify > gpurun_out/pytest_cls.log 2>&1 || { tail -30 gpurun_out/pytest_cls.log; exit 1; }
tail -2 gpurun_out/pytest_cls.log
timeout -k 10 300 python tools/bench_suite.py --only lab3 > gpurun_out/suite_lab3.log 2>&1 || { cat gpurun_out/suite_lab3.log; exit 2; }
grep -v amdgpu.ids gpurun_out/suite_lab3.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lab3prof/trace -o run -- python3 $R/tools/lab3_prof_run.py 32 > $R/gpurun_out/lab3prof/trace.log 2>&1 || { tail -20 $R/gpurun_out/lab3prof/trace.log; exit 3; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/lab3prof/pmc$i -o run -- python3 $R/tools/lab3_prof_run.py 32 > $R/gpurun_out/lab3prof/pmc$i.log 2>&1 || { echo "pmc group $i failed"; tail -5 $R/gpurun_out/lab3prof/pmc$i.log; exit 4; }
done
echo done
