"""Summarise the rocprofv3 --pmc passes over tools/microbench_q8q4 (tools/gpu_r4c.sh): per kernel and size,
the mean of every counter over its launches, with the memory-side counters normalised per element.
    python tools/pmc_q8q4_summary.py gpurun_out/r4c > profiles/r04/pmc_q8q4.txt"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
KERNELS = ("k_quantize_flat", "k_quantize_int4_flat", "k_dequantize_flat", "k_dequantize_int4_flat")
passes = {}
with open(os.path.join(root, "pmc_index.txt")) as f:
    for ln in f:
        m = re.match(r"pass (\d+) \(2\^(\d+)\): (.*)", ln.strip())
        passes[int(m.group(1))] = (int(m.group(2)), m.group(3).split())
vals = defaultdict(lambda: defaultdict(list))   # (lg, kernel) -> counter -> values
for p, (lg, _) in passes.items():
    for path in glob.glob(os.path.join(root, f"pmc_{p}", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                k = next((k for k in KERNELS if name.startswith(k + "(") or f" {k}" in name or name.startswith(k + "<")
                          or f"::{k}" in name or re.search(rf"\b{k}\b", name)), None)
                if k is None:
                    continue
                vals[(lg, k)][row["Counter_Name"]].append(float(row["Counter_Value"]))
counters = sorted({c for d in vals.values() for c in d})
print("rocprofv3 --pmc over tools/microbench_q8q4 (3 rounds per pass; one pass per counter set, tools/gpu_r4c.sh).")
print("Per launch means. EA0 requests: RDREQ counts 64 B units of the 128 B reads (MI355X_MICROARCH §HBM);")
print("per element = counter / n. TA/TD/GRBM/SQ as reported (SQ cycles are summed over waves).")
for lg in sorted({lg for lg, _ in vals}):
    n = 1 << lg
    print(f"\n== n = 2^{lg}")
    print(f"{'counter':38s}" + "".join(f"{k:>24s}" for k in KERNELS))
    for c in counters:
        row = []
        for k in KERNELS:
            v = vals[(lg, k)].get(c)
            row.append(sum(v) / len(v) if v else float("nan"))
        print(f"{c:38s}" + "".join(f"{x:24.4g}" for x in row))
    for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"):
        row = []
        for k in KERNELS:
            v = vals[(lg, k)].get(c)
            row.append(sum(v) / len(v) / n if v else float("nan"))
        print(f"{c + ' / elem':38s}" + "".join(f"{x:24.4f}" for x in row))
