# round 6: k_tn_short A/B — each segment's loads issued before the walk (product) or after the previous stage
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07e}
mkdir -p $O
ADFL_LIB_VARIANT=tools/_variants/libadfl_lateload.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py -k "f32 or not dt" > $O/tests.txt 2>&1 &&
timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --reps 21 --cfgs C3 > $O/bench_product.txt 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_lateload.so timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --reps 21 --cfgs C3 > $O/bench_lateload.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_p -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu --reps 10 > $O/prof_p.log 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_lateload.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_l -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu --reps 10 > $O/prof_l.log 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_lateloadstats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3 --reps 2 > $O/stats_l.txt 2>&1
echo rc=$?
