# Round 4 (k): host channel call-to-call spread: fastest vs slowest quarter phases.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4k
mkdir -p $O
timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 80 > $O/pipe.json 2> $O/pipe.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4k/pipe.json"))
for w in ("encode", "decode"):
    sp = d["spread"][w]
    print(w, sp["p10_p50_p90_ms"])
    for tag in ("fastest_quarter_phases", "slowest_quarter_phases"):
        print("  ", tag, {k.split(" (")[0]: v for k, v in sp[tag].items()})
PY
