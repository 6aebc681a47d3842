# Round 4 (p): host channel with the process bound to the GPU's NUMA node vs the other node (taskset), pool 8.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4p
mkdir -p $O
N0=$(cat /sys/devices/system/node/node0/cpulist); N1=$(cat /sys/devices/system/node/node1/cpulist)
echo "node0 $N0 node1 $N1"
for rep in 1 2; do
  timeout -k 10 200 taskset -c $N0 python -u $R/tools/channel_timeline.py --calls 60 > $O/n0_$rep.json 2> $O/n0_$rep.err || exit 1
  timeout -k 10 200 taskset -c $N1 python -u $R/tools/channel_timeline.py --calls 60 > $O/n1_$rep.json 2> $O/n1_$rep.err || exit 1
  timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/any_$rep.json 2> $O/any_$rep.err || exit 1
done
python - <<'PY'
import json
for rep in (1, 2):
    for v in ("n0", "n1", "any"):
        d = json.load(open(f"gpurun_out/r4p/{v}_{rep}.json"))
        print(v, rep, {w: d["spread"][w]["p10_p50_p90_ms"] for w in ("encode", "decode")})
PY
