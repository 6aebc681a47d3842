#!/bin/bash
# round 4: walker cost split: diag1 = no chain walk (streaming skeleton), diag2 = the FMA chain without LDS reads
set -o pipefail
mkdir -p gpurun_out/r4zc
for v in diag1 diag2 tb; do
  export ADFL_LIB_VARIANT=tools/_variants/libadfl_slq_$v.so
  timeout -k 10 200 python -u tools/torch_norm_bench.py --reps 9 --no-seq > gpurun_out/r4zc/$v.txt 2>&1 || exit $?
  echo $v; grep "^C3" gpurun_out/r4zc/$v.txt | cut -c1-200
done
