# round 6: phase D window records decoded once per window — parity, timing, trace, counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07c}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py tests/test_gpu_qerror.py tests/test_gpu_stoch.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes f32 --reps 11 > $O/bench.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/ref_norm_prof.py --cfg c2,c3,c3lu_raw --reps 5 > $O/prof.log 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c2 --reps 1 > $O/stats.txt 2>&1
echo rc=$?
