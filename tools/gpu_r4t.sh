#!/bin/bash
# round 4: look-back torch-order norm — parity tests, then cost against the default norm
set -o pipefail
mkdir -p gpurun_out/r4t
timeout -k 10 400 python -u -m pytest tests/test_gpu_torch_norm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4t/pytest.txt 2>&1
rc=$?
tail -5 gpurun_out/r4t/pytest.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/torch_norm_bench.py --reps 15 > gpurun_out/r4t/bench.txt 2>&1
rc=$?
cat gpurun_out/r4t/bench.txt | tail -4
exit $rc
