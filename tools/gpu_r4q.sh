# Round 4 (q): host channel with the copy pool bound to the GPU's NUMA node (and pinned staging allocated
# there) vs not, main thread unbound; alternating processes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4q
mkdir -p $O
for rep in 1 2 3; do
  ADFL_HOST_BIND=1 timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/bind_$rep.json 2> $O/bind_$rep.err || exit 1
  ADFL_HOST_BIND=0 timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/nobind_$rep.json 2> $O/nobind_$rep.err || exit 1
done
python - <<'PY'
import json
for rep in (1, 2, 3):
    for v in ("bind", "nobind"):
        d = json.load(open(f"gpurun_out/r4q/{v}_{rep}.json"))
        print(v, rep, {w: d["spread"][w]["p10_p50_p90_ms"] for w in ("encode", "decode")})
PY
