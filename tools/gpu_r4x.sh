#!/bin/bash
# round 4: tile-size variants of the look-back norm (threads x dwords per lane): parity, then C2 / C3 cost
set -o pipefail
mkdir -p gpurun_out/r4x
for v in t256r32 t512r32 t1024r16 t512r64; do
  export ADFL_LIB_VARIANT=tools/_variants/libadfl_slq_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "not abi" > gpurun_out/r4x/pytest_$v.txt 2>&1
  rc=$?
  echo "$v $(tail -1 gpurun_out/r4x/pytest_$v.txt)"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u tools/torch_norm_bench.py --reps 5 --no-seq > gpurun_out/r4x/$v.txt 2>&1 || exit $?
  grep "^C" gpurun_out/r4x/$v.txt | cut -c1-200
done
