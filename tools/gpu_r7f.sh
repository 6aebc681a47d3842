# round 6: maps_exact composes exact-square (bf16 / fp16) lane maps in fp32 by DPP — norm parity, timing, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07f}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_torch_norm_dt.py tests/test_gpu_stoch_dt.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ref_norm_bench.py --dtypes bf16,f16 --reps 11 > $O/bench.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bf16 -o run -- python tools/ref_norm_prof.py --cfg c2 --dtype bf16 --reps 3 > $O/prof_bf16.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f16 -o run -- python tools/ref_norm_prof.py --cfg c2 --dtype f16 --reps 3 > $O/prof_f16.log 2>&1
echo rc=$?
