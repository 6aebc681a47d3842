#!/bin/bash
# round 4: look-back round size sweep (kBatch windows of 8 predecessors per round trip)
set -o pipefail
mkdir -p gpurun_out/r4v
for b in 1 2 4; do
  ADFL_LIB_VARIANT=tools/_variants/libadfl_slq_b$b.so timeout -k 10 200 python -u tools/torch_norm_bench.py --reps 5 --no-seq > gpurun_out/r4v/b$b.txt 2>&1 || exit $?
  echo "b$b"; grep "^C2" gpurun_out/r4v/b$b.txt | cut -c1-300
done
