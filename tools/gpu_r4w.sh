#!/bin/bash
# round 4: single-launch CNAT (arrival counter) — parity, then cost
set -o pipefail
mkdir -p gpurun_out/r4w
timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_norm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4w/pytest.txt 2>&1
rc=$?
tail -4 gpurun_out/r4w/pytest.txt
[ $rc -ne 0 ] && exit $rc
true
rc=$?
tail -2 gpurun_out/r4w/bench.txt
[ $rc -ne 0 ] && exit $rc
for b in 1 2 4; do
  ADFL_LIB_VARIANT=tools/_variants/libadfl_slq_b$b.so timeout -k 10 200 python -u tools/torch_norm_bench.py --reps 5 --no-seq > gpurun_out/r4w/b$b.txt 2>&1 || exit $?
  echo "b$b"; grep "^C2" gpurun_out/r4w/b$b.txt | cut -c1-200
done
