#!/bin/bash
# PMC counters of the band kernel vs the wave kernel and the copy floors,
# rotated (tools/conv_floor_prof.py), one counter group per pass.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r2/band_pmc
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/conv_floor_prof.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- python3 $R/tools/conv_floor_prof.py > $O/pmc$i.log 2>&1 || { echo "pmc group $i failed"; tail -5 $O/pmc$i.log; exit 2; }
  echo "pmc group $i ok"
done
