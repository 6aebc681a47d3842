"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd .db): count, average / min / max
duration (us), grid, VGPRs, LDS. Optional --order prints each dispatch in order (name, us).

    python tools/kt_db.py gpurun_out/prof/run_results.db [--filter tn_] [--order]
"""
import argparse
import glob
import re
import sqlite3
import statistics


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name[-90:]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--filter", default="")
    p.add_argument("--order", action="store_true")
    a = p.parse_args()
    path = a.db if a.db.endswith(".db") else glob.glob(a.db + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration, grid_x, grid_y, workgroup_x, vgpr_count, lds_size from kernels "
                     "order by start").fetchall()
    rows = [r for r in rows if a.filter in r[0]]
    if a.order:
        for r in rows:
            print(f"{r[1] / 1e3:10.2f}  {short(r[0])}")
        return
    by = {}
    for r in rows:
        by.setdefault(short(r[0]), []).append(r)
    for k, rs in sorted(by.items(), key=lambda kv: -sum(r[1] for r in kv[1])):
        d = [r[1] / 1e3 for r in rs]
        print(f"{len(d):5d} avg {statistics.mean(d):10.2f} min {min(d):10.2f} max {max(d):10.2f} us  "
              f"grid {rs[0][2]}x{rs[0][3]} wg {rs[0][4]} vgpr {rs[0][5]} lds {rs[0][6]}  {k}")


if __name__ == "__main__":
    main()
