"""Summarise rocprofv3 PMC passes of bench.py (tools/profile_box.sh output) for
one kernel into the per-launch JSON that bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py gpurun_out/<tag> profiles/r2/k_djn_pow_pmc.json --win 23 --n 1000000 [--kernel k_djn_pow]

Units and corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE
and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-B
per-lane reads, so fetched bytes = 2 x FETCH_SIZE x 1024. Only the largest
dispatches (the bench's full-size launches) are averaged.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def per_dispatch(d, kernel):
    rows = list(csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))))
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    grid = {}
    for r in rows:
        m = re.search(r"(\w+)\s*(?:<|\()", r["Kernel_Name"])  # the kernel's own name (k_djn_pmd, not k_djn_pmdx)
        if not m or m.group(1) != kernel:
            continue
        out[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
        if "Start_Timestamp" in r:
            out[r["Dispatch_Id"]]["_duration_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return out, grid


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_djn_pow"
    vals = collections.defaultdict(list)
    grid_max = 0
    for d in sorted(glob.glob(os.path.join(src, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        per, grid = per_dispatch(d, kernel)
        if not grid:
            continue
        gmax = max(grid.values())
        grid_max = max(grid_max, gmax)
        for k, counters in per.items():
            if grid[k] == gmax:
                for c, v in counters.items():
                    vals[c].append(v)
    avg = {c: sum(v) / len(v) for c, v in vals.items()}
    rec = {"kernel": kernel, "grid_size": grid_max, "counters_per_launch": avg}
    if "--win" in sys.argv:  # window spec as bench.py --win takes it: "23" or "23s" (split)
        rec["win"] = sys.argv[sys.argv.index("--win") + 1]
    if "--n" in sys.argv:
        rec["n"] = int(sys.argv[sys.argv.index("--n") + 1])
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = 2 * avg["FETCH_SIZE"] * 1024
        write = avg["WRITE_SIZE"] * 1024
        rec.update({"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                    "correction": "fetch = 2 x FETCH_SIZE KiB (gfx950 16-B/lane reads), write = WRITE_SIZE KiB"})
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        rec["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
    # clock from SQ_BUSY_CYCLES (32 SQs: 8 XCDs x 4 SEs), then the VALU issue
    # fraction: a wave64 VALU instruction takes 4 cycles of its SIMD, 1024 SIMDs
    dur = avg.get("_duration_ns")
    if dur and "SQ_BUSY_CYCLES" in avg:
        clk = avg["SQ_BUSY_CYCLES"] / (dur * 1e-9) / 32
        rec["duration_ms"] = dur * 1e-6
        rec["clock_ghz"] = clk / 1e9
        quad_cycles = dur * 1e-9 * clk / 4 * 1024
        if "SQ_ACTIVE_INST_VALU" in avg:
            rec["valu_busy_frac"] = avg["SQ_ACTIVE_INST_VALU"] / quad_cycles
    if dur and "SQ_INSTS_VALU" in avg and rec.get("clock_ghz"):
        rec["valu_issue_frac"] = avg["SQ_INSTS_VALU"] / (dur * 1e-9 * rec["clock_ghz"] * 1e9 / 4 * 1024)
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
