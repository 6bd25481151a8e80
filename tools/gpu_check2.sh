#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pmc
timeout -k 10 300 python tools/kcheck.py > gpurun_out/kcheck.log 2>&1; rc=$?
cat gpurun_out/kcheck.log
[ $rc -ne 0 ] && exit $rc
cat > /tmp/pmc_run.py <<'PY'
import sys, torch
sys.path.insert(0, '.')
from cuda_mpi_openmp_amd import ops
dev = torch.device('cuda:0')
img = torch.randint(0, 256, (4096, 4096, 4), dtype=torch.uint8, device=dev)
out = torch.empty_like(img)
for _ in range(3):
    ops.conv(img, 'sobel5', out); ops.conv(img, 'roberts', out); out.copy_(img)
torch.cuda.synchronize()
PY
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum" "TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/g$i -o run -- python3 /tmp/pmc_run.py > gpurun_out/pmc/g$i.log 2>&1 || { echo "pmc group $i failed"; tail -5 gpurun_out/pmc/g$i.log; }
done
ls -R gpurun_out/pmc | head -30
