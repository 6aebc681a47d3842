# round 6: direct native per-range QSGD / CNAT encode in the host pipeline — stochastic parity, then the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06r}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_stoch.py tests/test_gpu_stoch_dt.py tests/test_gpu_host_error_path.py tests/test_gpu_stoch_resident.py tests/test_gpu_channel.py > $O/tests.txt 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/bench_line.json 2> $O/bench.err
echo rc=$?
