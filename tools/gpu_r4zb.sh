#!/bin/bash
# round 4: walker prefetch depth A/B: db = one block ahead (HEAD), tb = two blocks ahead, tb4 = two ahead, 1024-element blocks
set -o pipefail
mkdir -p gpurun_out/r4zb
for v in rg rg4 tb; do
  export ADFL_LIB_VARIANT=tools/_variants/libadfl_slq_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "not abi" > gpurun_out/r4zb/pytest_$v.txt 2>&1
  rc=$?
  echo "$v $(tail -1 gpurun_out/r4zb/pytest_$v.txt)"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u tools/torch_norm_bench.py --reps 9 --no-seq > gpurun_out/r4zb/$v.txt 2>&1 || exit $?
  grep "^C3" gpurun_out/r4zb/$v.txt | cut -c1-160
done
