# round 6: k_tn_short with every wave's first-segment loads queued first — parity, C3 timing, trace, timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06t}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes f32 --reps 21 --cfgs C3 > $O/bench.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu --reps 10 > $O/prof.log 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3 --reps 2 > $O/stats.txt 2>&1
echo rc=$?
