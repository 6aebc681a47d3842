# round 6: k_tn_short_f16 counters on C3 equal fp16 (stats build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06y}
mkdir -p $O
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3 --dtype f16 --reps 2 > $O/stats.txt 2>&1
echo rc=$?
