# round 6: k_tn_short (double-buffered, screened tie check) — parity, timing, counters, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06f}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py tests/test_gpu_qerror.py tests/test_gpu_hostcopy_event.py tests/test_gpu_host_error_path.py > $O/tests.txt 2>&1 &&
timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --cfgs C3 --reps 21 > $O/bench.txt 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3,c3lu --reps 1 > $O/stats.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/ref_norm_prof.py --cfg c3 --reps 5 > $O/prof.log 2>&1
echo rc=$?
if [ -n "$2" ]; then
  ADFL_LIB_VARIANT=tools/_variants/libadfl_$2.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$2 -o run -- python tools/ref_norm_prof.py --cfg c3 --reps 5 > $O/prof_$2.log 2>&1
fi
