#!/bin/bash
# round 4: the default build (512 x 32 tiles): torch-norm parity + the stochastic GPU suites, then cost
set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_norm.py tests/test_gpu_stoch.py tests/test_gpu_stoch_dt.py tests/test_gpu_stoch_resident.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4y/pytest.txt 2>&1
rc=$?
tail -2 gpurun_out/r4y/pytest.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/torch_norm_bench.py --reps 9 > gpurun_out/r4y/bench.txt 2>&1
rc=$?
tail -1 gpurun_out/r4y/bench.txt
exit $rc
