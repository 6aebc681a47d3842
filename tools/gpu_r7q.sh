# round 6: k_tn_short_bf16 with split loads — bf16 / fp16 norm parity, C3 timing per dtype
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm_dt.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes bf16,f16 --reps 21 --cfgs C3 > $O/bench.txt 2>&1
echo rc=$?
