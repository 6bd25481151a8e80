#!/bin/bash
# Cold first-launch check: one process per launch (MPX_TIMING=cold), tuned vs
# reference geometry, on a reference lab2 image and a lab1 n=1e6 vector pair;
# HIP_ENABLE_DEFERRED_LOADING=0 from the environment as the control.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/cold_ab; mkdir -p $O
IMG=labs/lab2/metric_calc/small/02.data
python3 -c "
import numpy as np
r=np.random.default_rng(0); n=1000000
a=r.uniform(-1e3,1e3,n); b=r.uniform(-1e3,1e3,n)
open('$O/v1e6.txt','w').write(str(n)+'\n'+' '.join('%.10e'%x for x in a)+'\n'+' '.join('%.10e'%x for x in b)+'\n')"
lab2() { printf "%s\n%s\n%s\n" "$1" "$IMG" "$O/out.data" | timeout -k 5 60 env "${@:2}" labs/lab2/src/to_plot_hip_exe | head -1; }
lab1() { { printf "%s\n" "$1"; cat $O/v1e6.txt; } | timeout -k 5 60 env "${@:2}" labs/lab1/src/to_plot_hip_exe | head -1; }
{
for i in 1 2 3 4 5; do echo "lab2 tuned    $(lab2 '0 0 0 0' MPX_TIMING=cold)"; done
for i in 1 2 3 4 5; do echo "lab2 32x32/16 $(lab2 '32 32 16 16' MPX_TIMING=cold)"; done
for i in 1 2 3; do echo "lab2 32x32/16 DEFERRED=0 $(lab2 '32 32 16 16' MPX_TIMING=cold HIP_ENABLE_DEFERRED_LOADING=0)"; done
for i in 1 2 3 4 5; do echo "lab1 n=1e6 [512,512] $(lab1 '512 512' MPX_TIMING=cold)"; done
for i in 1 2 3 4 5; do echo "lab1 n=1e6 tuned     $(lab1 '0 0' MPX_TIMING=cold)"; done
for i in 1 2 3; do echo "lab1 n=1e6 [512,512] warm $(lab1 '512 512' MPX_TIMING=warm)"; done
} | tee $O/cold_ab.txt
rm -f $O/v1e6.txt $O/out.data
