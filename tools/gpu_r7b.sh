# round 6: phase C keeps the bucket's last 192 MiB in the Infinity Cache for the reverse-order QSGD quantize —
# norm + stochastic parity, then C2 / C3 fp32 timing (QSGD encode with the reference's norm)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py tests/test_gpu_stoch.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes f32 --reps 21 > $O/bench.txt 2>&1
echo rc=$?
