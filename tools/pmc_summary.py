"""Summarise rocprofv3 --pmc passes (tools/pmc_profile.sh output) per kernel.

    python tools/pmc_summary.py gpurun_out/pmc1 [--match synth] [--json out.json]

Per kernel: mean counter value per dispatch, mean dispatch duration, and derived figures:
  valu_busy  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (share of wave time issuing VALU)
  wait_frac  = SQ_WAIT_ANY / SQ_WAVE_CYCLES            (s_waitcnt / barrier parked)
  clock_GHz  = GRBM_GUI_ACTIVE / 8 XCDs / duration     (MI355X_MICROARCH.md 'DVFS give-back')
  hbm_read_B = 2 * FETCH_SIZE * 1024 (gfx950 FETCH_SIZE counts half of wide streaming reads)
  hbm_write_B= WRITE_SIZE * 1024
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d):
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "pass*", "*counter_collection.csv"))):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in load(args.dir):
        name = r["Kernel_Name"]
        if args.match and args.match not in name:
            continue
        short = name.split("(")[0].replace("void ", "")
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[(short, r["Counter_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for k, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        ns = [x for (kk, c), xs in dur.items() if kk == k for x in xs]
        d["duration_ns"] = sum(ns) / len(ns)
        d["dispatches"] = max(len(v) for v in cs.values())
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            for c, lab in (("SQ_ACTIVE_INST_VALU", "valu_busy"), ("SQ_WAIT_ANY", "wait_frac"),
                           ("SQ_WAIT_INST_ANY", "wait_inst_frac"), ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if c in d:
                    d[lab] = d[c] / wc
        if "GRBM_GUI_ACTIVE" in d:
            d["clock_GHz"] = d["GRBM_GUI_ACTIVE"] / 8 / d["duration_ns"]
        if "FETCH_SIZE" in d:
            d["hbm_read_B"] = 2 * d["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in d:
            d["hbm_write_B"] = d["WRITE_SIZE"] * 1024
        out[k] = d
        print(f"== {k}  ({d['dispatches']} dispatches, {d['duration_ns'] / 1e6:.3f} ms)")
        for c in sorted(d):
            if c not in ("duration_ns", "dispatches"):
                print(f"   {c:28s} {d[c]:.6g}")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
