# Round 3 (g): exchange eager vs HIP graph replay at world 1 (C3 layouts, C4/C5 flat shapes).
set -o pipefail
run() { timeout -k 10 200 python tools/bench_configs.py --mode exchange "$@" --steps 50 --warmup 10 2> gpurun_out/ex_err.txt | grep "^{" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['metric'].split(', ',1)[1], d['ms_per_step'])"; }
for G in "" "--graph"; do
  run --layout c3_equal $G || exit 1
  run --layout c3_equal --packed $G || exit 1
  run --layout c3_loguniform $G || exit 1
  run --elems 268435456 $G || exit 1
  run --elems 1073741824 --packed --chunks 8 $G || exit 1
done
exit 0
