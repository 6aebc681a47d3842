# Round 4 (l): host channel A/B — glibc keeps freed heap (hostcopy.keep_host_heap) vs not, alternating
# processes on one box; spread per variant.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4l
mkdir -p $O
for rep in 1 2 3; do
  ADFL_KEEP_HOST_HEAP=1 timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/keep_$rep.json 2> $O/keep_$rep.err || exit 1
  ADFL_KEEP_HOST_HEAP=0 timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/nokeep_$rep.json 2> $O/nokeep_$rep.err || exit 1
done
python - <<'PY'
import json
for rep in (1, 2, 3):
    for v in ("keep", "nokeep"):
        d = json.load(open(f"gpurun_out/r4l/{v}_{rep}.json"))
        print(v, rep, {w: (d["spread"][w]["p10_p50_p90_ms"], d[w]["free_previous_result_ms_median"]) for w in ("encode", "decode")})
PY
