#!/bin/bash
# round 4: walker block size (dwords per thread per block) variants: parity, then C3 cost
set -o pipefail
mkdir -p gpurun_out/r4z
for v in w8 w4; do
  export ADFL_LIB_VARIANT=tools/_variants/libadfl_slq_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "not abi" > gpurun_out/r4z/pytest_$v.txt 2>&1
  rc=$?
  echo "$v $(tail -1 gpurun_out/r4z/pytest_$v.txt)"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u tools/torch_norm_bench.py --reps 9 --no-seq > gpurun_out/r4z/$v.txt 2>&1 || exit $?
  grep "^C3" gpurun_out/r4z/$v.txt | cut -c1-160
done
