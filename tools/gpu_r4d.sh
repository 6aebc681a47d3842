# Round 4 (d): int4 unpack+dequantize variants vs the int8 decode on one input (2^30 and 2^28).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4d
mkdir -p $O
timeout -k 10 150 $R/tools/microbench_d4var 30 11 > $O/d4var_30.txt 2>&1 && cat $O/d4var_30.txt &&
timeout -k 10 120 $R/tools/microbench_d4var 28 21 > $O/d4var_28.txt 2>&1 && cat $O/d4var_28.txt
