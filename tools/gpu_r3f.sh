# Round 3 (f): C3 bucketed exchange order check (first-run effect?).
set -o pipefail
for L in c3_loguniform c3_equal c3_equal c3_loguniform; do
  for P in "--packed" ""; do
    echo "== exchange $L $P"; timeout -k 10 200 python tools/bench_configs.py --mode exchange --layout $L $P --steps 50 --warmup 10 2> gpurun_out/ex_err.txt | grep "^{" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['bytes_per_rank_on_wire'])" || exit 1
  done
done
exit 0
