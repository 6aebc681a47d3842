# round 6: k_tn_short on the log-uniform C3 layouts (kernel trace), product (16 steps per lane) and a variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06l}
mkdir -p $O
timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --cfgs C3 --reps 21 > $O/bench.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu,c3lu_raw --reps 5 > $O/prof.log 2>&1 &&
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3lu --reps 1 > $O/stats.txt 2>&1
echo rc=$?
if [ -n "$2" ]; then
  ADFL_LIB_VARIANT=tools/_variants/libadfl_$2.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$2 -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu --reps 5 > $O/prof_$2.log 2>&1
fi
