"""Inter-kernel gaps of the C3 bucketed round trip from a rocprofv3 kernel trace of
`tools/bench_configs.py --mode c3` (equal layout, int8): for every encode -> decode pair the encode and
decode durations and the idle gap between them (the launch boundary the one-launch encode removed one of).

    python tools/trace_gaps.py gpurun_out/prof_r02/trace_c3/c3_kernel_trace.csv > profiles/r02/c3_trace_gaps.json
"""
import csv
import json
import statistics
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    enc_name, dec_name = "k_encode_resident(", "k_dequantize_batched("
    pairs = []
    for a, b in zip(rows, rows[1:]):
        if enc_name in a["Kernel_Name"] and dec_name in b["Kernel_Name"] and "int4" not in b["Kernel_Name"]:
            a0, a1, b0, b1 = (int(a["Start_Timestamp"]), int(a["End_Timestamp"]), int(b["Start_Timestamp"]),
                              int(b["End_Timestamp"]))
            pairs.append({"encode_us": (a1 - a0) / 1e3, "gap_us": (b0 - a1) / 1e3, "decode_us": (b1 - b0) / 1e3,
                          "span_us": (b1 - a0) / 1e3})
    med = {k: round(statistics.median(p[k] for p in pairs), 2) for k in ("encode_us", "gap_us", "decode_us", "span_us")}
    print(json.dumps({"source": path, "pairs": len(pairs), "median": med,
                      "note": "encode = k_encode_resident (one launch, x read once), decode = k_dequantize_batched; "
                              "gap = idle time between the two launches on the stream"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
