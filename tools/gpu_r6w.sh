# round 6: fp16 short tensors by k_tn_short_f16 — norm parity (every dtype), then C3 / C2 timing per dtype
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06w}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm_dt.py tests/test_gpu_stoch_dt.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes f16,bf16 --reps 11 > $O/bench.txt 2>&1
echo rc=$?
