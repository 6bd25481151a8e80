set -o pipefail
O=gpurun_out/r3/g8; mkdir -p $O
for args in "--gpus 2 --size 1024" "--gpus 2 --size 4096" "--gpus 2"; do
  timeout -k 10 120 bin/mpx_mgpu jacobi --halo peer --shared $args --iters 100 --warmup 10 > $O/m.json 2>$O/m.err; rc=$?
  echo "native $args rc=$rc $(grep -o '"verified": [a-z]*\|"one_device_equal": [a-z]*' $O/m.json | tr '\n' ' ') $(head -c 600 $O/m.err)"
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
done
