"""Summarise rocprofv3 PMC passes (scripts/pmc_passes.sh) and --stats kernel summaries into a
small JSON for profiles/.

    python scripts/pmc_summary.py <pmc_dir> <out.json> [--kernel render_philox] [--note TEXT]

For every pass directory under <pmc_dir>, reads p_counter_collection.csv, keeps the dispatches of
the kernel whose name contains --kernel, and averages each counter per dispatch. Derived values
follow MI355X_MICROARCH.md "HBM [CDNA4]": on gfx950 FETCH_SIZE (KiB) reports half the bytes of a
wide streaming read, so hbm_read_bytes = 2 * FETCH_SIZE * 1024 (the render kernel's 8-64 B
gathers are uncalibrated: the doubling is the guide's correction, kept for comparability);
WRITE_SIZE (KiB) is taken as is.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="render_philox")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    vals = defaultdict(list)
    durs = []
    names = set()
    for f in sorted(glob.glob(os.path.join(a.pmc_dir, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        seen = set()
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if a.kernel not in row["Kernel_Name"]:
                    continue
                names.add(row["Kernel_Name"])
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                key = (f, row["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    if not vals:
        raise SystemExit(f"no dispatch of a kernel matching {a.kernel!r} under {a.pmc_dir}")
    avg = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    dur = sum(durs) / len(durs)
    out = {"kernels": sorted(names), "dispatches": len(durs), "avg_duration_s": dur,
           "counters_per_dispatch": avg, "note": a.note}
    d = {}
    if "FETCH_SIZE" in avg:
        d["hbm_read_bytes"] = 2 * avg["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in avg:
        d["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
        d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        d["hbm_gbs"] = d["hbm_bytes"] / dur / 1e9
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        d["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        d["valu_lane_utilisation"] = avg["SQ_THREAD_CYCLES_VALU"] / max(1.0, 64 * avg["SQ_ACTIVE_INST_VALU"])
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        pass
    if "SQ_WAIT_ANY" in avg and "SQ_ACTIVE_INST_ANY" in avg and "SQ_WAIT_INST_ANY" in avg:
        tot = avg["SQ_WAIT_ANY"] + avg["SQ_ACTIVE_INST_ANY"] + avg["SQ_WAIT_INST_ANY"]
        d["wave_cycles_split"] = {"wait_any": avg["SQ_WAIT_ANY"] / tot, "wait_inst_any": avg["SQ_WAIT_INST_ANY"] / tot,
                                  "active_inst_any": avg["SQ_ACTIVE_INST_ANY"] / tot}
    out["derived"] = d
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
