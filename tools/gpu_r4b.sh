# Round 4 (b): the 8-rank bench rehearsal on one GPU; int8 vs int4 flat kernels on one input (microbench);
# the box's counter list for the PMC passes that follow.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -x -s --timeout 250 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_bench_contract.py::test_bench_eight_ranks_share_one_gpu" "tests/test_gpu_bench_contract.py::test_bench_extras_c3_c5_pcie" > $O/pytest8.txt 2>&1
rc=$?; tail -5 $O/pytest8.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 $R/tools/microbench_q8q4 30 15 > $O/q8q4.txt 2>&1 && cat $O/q8q4.txt &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1; echo "list rc $?"; grep -c . $O/counters_list.txt
