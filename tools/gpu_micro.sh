set -o pipefail
mkdir -p gpurun_out
echo "== microbench"; timeout -k 10 300 ./tools/microbench 28 > gpurun_out/microbench.txt 2>&1; rc=$?; cat gpurun_out/microbench.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
echo "== rocprof bench"; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1; rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log; exit $rc
