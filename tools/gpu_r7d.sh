# round 6: CNAT encode with the reference's norm on a side stream beside it — stochastic parity, then timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07d}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stoch.py tests/test_gpu_stoch_resident.py tests/test_gpu_channel.py tests/test_gpu_stoch_dt.py tests/test_gpu_custom_ops.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes f32 --reps 21 > $O/bench.txt 2>&1
echo rc=$?
