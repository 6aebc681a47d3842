# round 6: sampled phase A with a reduce-scatter and two chunks per wave — norm parity, C2 per dtype, phase D counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07o}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes f32,bf16,f16 --reps 11 --cfgs C2 > $O/bench.txt 2>&1 &&
for d in f32 bf16 f16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$d -o run -- python tools/ref_norm_prof.py --cfg c2 --dtype $d --reps 3 > $O/prof_$d.log 2>&1 || exit $?
done &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c2 --reps 1 > $O/stats.txt 2>&1
echo rc=$?
