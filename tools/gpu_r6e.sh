# round 6: k_tn_short A/B (prefetch depth 2 / 3) with per-wave counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
for v in stats d3stats; do
  ADFL_LIB_VARIANT=tools/_variants/libadfl_$v.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3,c3lu --reps 1 > $O/stats_$v.txt 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --cfgs "C3 equal" --reps 21 > $O/bench_d2.txt 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_d3.so timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --cfgs "C3 equal" --reps 21 > $O/bench_d3.txt 2>&1
echo rc=$?
