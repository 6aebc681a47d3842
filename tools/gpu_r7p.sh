# round 6: k_tn_short A/B — a segment's loads split around the walk and stage (ADFL_TN_SPLIT_LOAD)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07p}
mkdir -p $O
ADFL_LIB_VARIANT=tools/_variants/libadfl_splitload.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torch_norm.py tests/test_gpu_torch_norm_dt.py -k "f32 or not dt" > $O/tests.txt 2>&1 &&
for v in product splitload; do
  if [ $v = product ]; then L=; else L=tools/_variants/libadfl_$v.so; fi
  ADFL_LIB_VARIANT=$L timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --reps 21 --cfgs C3 > $O/bench_$v.txt 2>&1 || exit $?
  ADFL_LIB_VARIANT=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu --reps 10 > $O/prof_$v.log 2>&1 || exit $?
done
echo rc=0
