"""Summary of profiles/r06/share_pmc.sh: per spec, k_render_cor's (and k_group_list's) mean duration and counters in
the PMC passes (kernels serialised), FETCH in bytes with the gfx950 correction (x2, MI355X_MICROARCH.md "HBM"), the
L2 hit rate, and the wave timeline's head lines.
  python profiles/r06/share_pmc_summary.py <tag> <spec>..."""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
tag, specs = sys.argv[1], sys.argv[2:]
O = os.path.join(ROOT, "gpurun_out", tag)


def means(d, kname):
    """per-dispatch counters of kname, averaged over the dispatches of the share's own grid (the most common grid
    size: a share's bench first renders three whole frames for the balancing profile)"""
    disp = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kname not in row["Kernel_Name"]:
                continue
            e = disp[(f, row["Dispatch_Id"])]
            e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            e["_dur"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            e["_grid"] = int(row.get("Grid_Size", row.get("Grid_Size_X", 0)) or 0)
    if not disp:
        return {}, 0.0, 0
    grids = defaultdict(int)
    for e in disp.values():
        grids[e["_grid"]] += 1
    g = max(grids, key=grids.get)
    sel = [e for e in disp.values() if e["_grid"] == g]
    keys = set().union(*[e.keys() for e in sel])
    m = {k: sum(e.get(k, 0.0) for e in sel) / len(sel) for k in keys}
    return m, m["_dur"] / 1e3, len(sel)


for spec in specs:
    t = spec.replace(":", "_")
    print(f"== {spec}")
    for kname in ("k_render_cor", "k_group_list"):
        sq, dur, nd = means(os.path.join(O, f"sq_{t}"), kname)
        tcc, _, _ = means(os.path.join(O, f"tcc_{t}"), kname)
        fe, _, _ = means(os.path.join(O, f"fetch_{t}"), kname)
        if not sq:
            continue
        waves = sq.get("SQ_WAVES", 1.0)
        hit, miss = tcc.get("TCC_HIT_sum", 0.0), tcc.get("TCC_MISS_sum", 0.0)
        print(f"  {kname}: {dur:.1f} us alone ({nd} dispatches), {waves:.0f} waves, "
              f"VALU/wave {sq.get('SQ_INSTS_VALU', 0) / waves:.0f}, LDS/wave {sq.get('SQ_INSTS_LDS', 0) / waves:.0f}, "
              f"wave-cycles/wave {sq.get('SQ_WAVE_CYCLES', 0) / waves:.0f}, busy cycles {sq.get('SQ_BUSY_CYCLES', 0):.3g}, "
              f"GRBM active {sq.get('GRBM_GUI_ACTIVE', 0):.3g}, L2 hit {hit / max(hit + miss, 1):.3f}, "
              f"FETCH x2 {2 * fe.get('FETCH_SIZE', 0) / 1e3:.1f} MB")
    wt = os.path.join(O, f"wt_{t}.txt")
    if os.path.exists(wt):
        for line in open(wt):
            print("  | " + line.rstrip())
