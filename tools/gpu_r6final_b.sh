# round 6 final, part B: rocprofv3 kernel trace + FETCH / WRITE passes of the bench's timed loop and of the
# reference-order norm (C2, C3 equal, C3 log-uniform), and the norm's timing per dtype
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06final}
mkdir -p $O
bash tools/gpu_prof.sh r06bench --secs 400 -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --pmc off --extras off > $O/prof_bench.log 2>&1 &&
bash tools/gpu_prof.sh r06norm --secs 300 -- python3 tools/ref_norm_prof.py --cfg c2,c3,c3lu --reps 3 > $O/prof_norm.log 2>&1 &&
timeout -k 10 400 python -u tools/ref_norm_bench.py --reps 11 > $O/norm_bench.txt 2>&1
echo rc=$?
