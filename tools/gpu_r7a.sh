# round 6: bf16 short tensors by k_tn_short_bf16 — norm parity (every dtype), timing per dtype, counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm_dt.py tests/test_gpu_torch_norm.py tests/test_gpu_stoch_dt.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes f32,f16,bf16 --reps 11 --cfgs C3 > $O/bench.txt 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3 --dtype bf16 --reps 2 > $O/stats.txt 2>&1
echo rc=$?
