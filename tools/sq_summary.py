"""Summarise a rocprofv3 --pmc pass of SQ counters per kernel (and grid size): per-dispatch averages and the
derived issue figures used in DESIGN.md. SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_INSTS_VMEM_* count wave-level
instructions; SQ_WAVE_CYCLES = SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY (MI355X_MICROARCH.md).

    python tools/sq_summary.py gpurun_out/prof_sq/sq_counter_collection.csv [elements_by_grid.json] > out.txt
"""
import collections
import csv
import json
import sys


def main(path, elems_json=None):
    elems = json.load(open(elems_json)) if elems_json else {}
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        key = (name, int(r["Grid_Size"]))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, grid), cs in sorted(acc.items(), key=lambda kv: kv[0]):
        if name.startswith("at::") or "k_flush" in name or "k_fill" in name:
            continue
        avg = {k: sum(v) / len(v) for k, v in cs.items()}
        line = {"kernel": name, "grid": grid, "dispatches": max(len(v) for v in cs.values())}
        line.update({k: round(v) for k, v in sorted(avg.items())})
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if k in avg:
                    line[k.replace("SQ_", "frac_")] = round(avg[k] / wc, 3)
        n = elems.get(str(grid))
        if n and "SQ_INSTS_VALU" in avg:
            line["valu_lane_insts_per_elem"] = round(avg["SQ_INSTS_VALU"] * 64 / n, 2)
        print(json.dumps(line))


if __name__ == "__main__":
    main(*sys.argv[1:3])
