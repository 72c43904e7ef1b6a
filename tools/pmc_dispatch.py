"""Per-kernel-shape summary of rocprofv3 --pmc passes (tools/pmc_passes.sh output): dispatches of one kernel with
different grid sizes (e.g. the DM and the RN+GW k_grid_dft_gen of a C2 step) are kept apart.

    python tools/pmc_dispatch.py gpurun_out/r03c_c2 [--match dft,interp]

mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs): the share of the matrix pipes' cycles
(64 busy cycles per v_mfma_f64_16x16x4_f64: busy cycles = 64 x SQ_INSTS_VALU_MFMA_F64); hbm bytes as in pmc_summary.
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="dft,interp,fused,gen_mix,epoch,part,mix")
    args = ap.parse_args()
    keys = [k for k in args.match.split(",") if k]
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(args.dir, "pass*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fpta::", "")
            if keys and not any(k in n for k in keys):
                continue
            key = (n, r.get("Grid_Size", r.get("Grid_Size_X", "")))
            d[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            d[key]["dur"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for (name, grid), cs in d.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        dur = m["dur"]
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
        hit, miss = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
        print(f"{name} (grid {grid}, {len(cs['dur'])} dispatch records)")
        print(f"   duration_us      {dur / 1e3:.1f}")
        print(f"   clock_GHz        {cyc / dur:.2f}")
        print(f"   mfma_busy        {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(1.0, cyc * 1024):.3f}")
        for c, lab in (("SQ_WAIT_INST_ANY", "wait_inst_frac"), ("SQ_ACTIVE_INST_VALU", "valu_active_frac"),
                       ("SQ_ACTIVE_INST_ANY", "active_frac")):
            print(f"   {lab:16s} {m.get(c, 0) / wc:.3f}")
        for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
                  "SQ_INSTS_VALU_MFMA_F64", "SQ_LDS_BANK_CONFLICT", "TCP_PENDING_STALL_CYCLES_sum", "TA_TA_BUSY_sum",
                  "TD_TD_BUSY_sum"):
            if c in m:
                print(f"   {c:28s} {m[c]:.4g}")
        if hit + miss:
            print(f"   L2_hit_frac      {hit / (hit + miss):.3f}")
        if "FETCH_SIZE" in m:
            print(f"   hbm_read_B       {2 * m['FETCH_SIZE'] * 1024:.4g}")
        if "WRITE_SIZE" in m:
            print(f"   hbm_write_B      {m['WRITE_SIZE'] * 1024:.4g}")


if __name__ == "__main__":
    main()
