# Round 4 (m): encode timeline with the native job waits and per-range stamps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4m
mkdir -p $O
timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/t.json 2> $O/t.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4m/t.json"))
for w in ("encode", "decode"):
    sp = d["spread"][w]
    print(w, sp["p10_p50_p90_ms"])
    for k, v in sp["fastest_quarter_phases"].items():
        print("   ", k, v)
PY
