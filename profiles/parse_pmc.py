"""Summarise a profiles/collect.sh run (gpurun_out/prof_<tag>/) into committed files under profiles/.

  python profiles/parse_pmc.py <tag> <config>

writes
  profiles/<tag>_<config>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (per-kernel durations)
  profiles/<tag>_<config>_pmc.json           per-kernel mean of every PMC counter over its dispatches
  profiles/pmc_traffic.json                  HBM bytes per launch of the timed kernel, read by bench.py

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE are in KiB, and on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so traffic = 2 * FETCH + WRITE.
The render kernels read records and SH rows with 16 B/lane loads, the case the x2 correction is
calibrated for.
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def base_name(full):
    m = re.search(r"(k_\w+)", full)
    return m.group(1) if m else full


def read_counters(path):
    per = defaultdict(lambda: defaultdict(list))  # kernel full name -> counter -> values per dispatch
    with open(path) as f:
        for row in csv.DictReader(f):
            per[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copyfile(stats, os.path.join(HERE, f"{tag}_{cfg}_kernel_stats.csv"))
    summary = {}
    for sub in ("fetch", "write", "sq", "sq2", "sq3"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for kname, ctrs in read_counters(p).items():
            if "gsrt::" not in kname:
                continue
            d = summary.setdefault(kname, {})
            for c, vals in ctrs.items():
                # counters are summed over XCD/SE instances per dispatch by rocprofv3: one value per dispatch
                d[c] = sum(vals) / len(vals)
                d.setdefault("dispatches", {})[sub] = len(vals)
    for kname, d in summary.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = 2.0 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
        if "SQ_ACTIVE_INST_VALU" in d and "SQ_BUSY_CYCLES" in d and "SQ_WAVE_CYCLES" in d:
            d["valu_active_per_wave_cycle"] = d["SQ_ACTIVE_INST_VALU"] / max(d["SQ_WAVE_CYCLES"], 1.0)
    with open(os.path.join(HERE, f"{tag}_{cfg}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    timed = [k for k in summary if base_name(k) in ("k_render_cor", "k_render_ref") and "hbm_bytes_per_launch" in summary[k]]
    if timed:
        k = max(timed, key=lambda k: summary[k]["hbm_bytes_per_launch"])
        out = {"config": cfg, "tag": tag, "kernel": k, "fetch_kib": summary[k]["FETCH_SIZE"],
               "write_kib": summary[k]["WRITE_SIZE"], "hbm_bytes_per_launch": summary[k]["hbm_bytes_per_launch"],
               "method": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving), mean over dispatches"}
        with open(os.path.join(HERE, "pmc_traffic.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))
    for k, d in sorted(summary.items()):
        print(base_name(k), {c: round(v, 3) for c, v in d.items() if isinstance(v, float)})


if __name__ == "__main__":
    main()
