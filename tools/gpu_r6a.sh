# round 6: the short-tensor norm kernel (k_tn_short) — parity, then timing against the walker, then the phase stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py tests/test_gpu_host_error_path.py > $O/tests.txt 2>&1 &&
timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --cfgs C3 --reps 21 > $O/bench_new.txt 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_walker.so timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --cfgs C3 --reps 21 > $O/bench_walker.txt 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3lu,c3lu_raw --reps 1 > $O/stats.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu,c3lu_raw --reps 5 > $O/prof.log 2>&1
echo rc=$?
