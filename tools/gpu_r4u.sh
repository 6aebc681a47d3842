#!/bin/bash
# round 4: look-back torch-order norm — cost only (after a green tools/gpu_r4t.sh)
set -o pipefail
mkdir -p gpurun_out/r4u
timeout -k 10 300 python -u tools/torch_norm_bench.py --reps 9 > gpurun_out/r4u/bench.txt 2>&1
rc=$?
tail -3 gpurun_out/r4u/bench.txt
exit $rc
