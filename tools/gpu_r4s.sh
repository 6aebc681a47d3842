# Round 4 (s): host channel, caller thread on the GPU's node during the call (ADFL_HOST_BIND_CALLER) vs not.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s
mkdir -p $O
for rep in 1 2 3; do
  ADFL_HOST_BIND_CALLER=1 timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/caller_$rep.json 2> $O/caller_$rep.err || exit 1
  ADFL_HOST_BIND_CALLER=0 timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/pool_$rep.json 2> $O/pool_$rep.err || exit 1
done
python - <<'PY'
import json
for rep in (1, 2, 3):
    for v in ("caller", "pool"):
        d = json.load(open(f"gpurun_out/r4s/{v}_{rep}.json"))
        print(v, rep, {w: d["spread"][w]["p10_p50_p90_ms"] for w in ("encode", "decode")})
PY
