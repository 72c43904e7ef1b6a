"""Per-step kernel timeline of a rocprofv3 kernel trace (container-side analysis of gpurun_out/ traces).

    python tools/trace_steps.py <run_kernel_trace.csv> [--marker k_grid_interp] [--last N]

Takes the launches of the last N steps (a step ends with a launch whose name contains --marker), and prints per
kernel: launches per step, mean duration, and the step's wall span / busy union of all kernels."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_grid_interp")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--timeline", type=int, default=0,
                    help="also list every launch (copies included) of the last N steps: start/end/duration us "
                         "relative to the end of the step before them, stream, name")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", ""),
                  r.get("VGPR_Count", ""), r.get("Accum_VGPR_Count", ""), r.get("LDS_Block_Size", ""),
                  r.get("Grid_Size_X", ""))
                 for r in rows), key=lambda e: e[0])
    ends = [i for i, e in enumerate(ev) if a.marker in e[2]]
    if len(ends) < a.last + 1:
        raise SystemExit("not enough steps in the trace")
    lo = ends[-a.last - 1] + 1
    sel = [e for e in ev[lo:ends[-1] + 1] if "rocclr" not in e[2]]
    t0, t1 = ev[ends[-a.last - 1]][1], ev[ends[-1]][1]
    by = collections.defaultdict(list)
    for e in sel:
        by[e[2].split("(")[0]].append(e)
    print(f"steps {a.last}: wall {(t1 - t0) / a.last / 1e6:.4f} ms/step (end of one {a.marker} to the next)")
    for k, es in sorted(by.items(), key=lambda kv: -sum(e[1] - e[0] for e in kv[1])):
        d = [(e[1] - e[0]) / 1e6 for e in es]
        print(f"  {k[:70]:70s} {len(es) / a.last:5.2f}/step  mean {sum(d) / len(d):.4f} ms  "
              f"sum/step {sum(d) / a.last:.4f} ms  vgpr {es[0][4]}+{es[0][5]} lds {es[0][6]} grid {es[0][7]} "
              f"stream {es[0][3]}")
    if a.timeline:
        z = ev[ends[-a.timeline - 1]][1]
        print(f"timeline of the last {a.timeline} steps (us from the end of the {a.marker} before them)")
        for e in ev[ends[-a.timeline - 1] + 1:ends[-1] + 1]:
            print(f"  {(e[0] - z) / 1e3:9.1f} {(e[1] - z) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f} s{e[3]} "
                  f"{e[2].split('(')[0][:60]}")


if __name__ == "__main__":
    main()
