# Cooperative one-launch bucketed encode (opt-in): parity tests, the C3 config bench with the coop A/B,
# and a rocprofv3 kernel trace of the default C3 bench (product encodes only).
set -o pipefail
mkdir -p gpurun_out
echo "== tests"; timeout -k 10 300 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_coop.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_coop.log; [ $rc -eq 0 ] || exit $rc
echo "== c3 + coop A/B"; timeout -k 10 300 python tools/bench_configs.py --mode c3 --coop-ab > gpurun_out/c3_coop.json 2> gpurun_out/c3_coop.err || exit $?; cat gpurun_out/c3_coop.json
echo "== rocprof"; cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3 -o c3 -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --mode c3 > $GRAFT_REPO_ROOT/gpurun_out/c3_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/c3_prof.err; echo rc=$?
