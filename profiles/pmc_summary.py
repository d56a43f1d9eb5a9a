"""Per-kernel mean of every PMC counter in gpurun_out/pmc_<tag>/<lib>/{sq,sq2,sq3} (profiles/pmc_ab.sh, profiles/pmc_env_ab.sh):
  python profiles/pmc_summary.py <tag> [kernel-substring]"""
import csv, glob, os, sys
from collections import defaultdict
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]; ks = sys.argv[2] if len(sys.argv) > 2 else "k_render_cor"
for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmc_" + tag, "*"))):
    vals = defaultdict(list); dur = {}
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if ks not in row["Kernel_Name"]:
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
            dur[(f, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    waves = m.get("SQ_WAVES", 1)
    print(os.path.basename(d), "dur_us %.1f" % (sum(dur.values()) / max(len(dur), 1) / 1e3))
    for k in sorted(m):
        print("   %-22s %14.4g  per-wave %10.1f" % (k, m[k], m[k] / waves))
