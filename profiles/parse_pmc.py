"""Summarise a profiles/collect.sh run (gpurun_out/prof_<tag>/) into committed files under profiles/.

  python profiles/parse_pmc.py <tag> <config>

writes
  profiles/<tag>/<config>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (per-kernel durations)
  profiles/<tag>/<config>_pmc.json           per-kernel mean of every PMC counter over its dispatches
  profiles/pmc_traffic.json                  per config: HBM bytes per launch of the timed kernel, its VALU issue and
                                             LDS-array time, read by bench.py (only while bench.src_hash() matches)

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE are in KiB, and on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so traffic = 2 * FETCH + WRITE.
The render kernels read records and SH rows with 16 B/lane loads, the case the x2 correction is
calibrated for.

VALU issue time: SQ_INSTS_VALU wave-instructions x 2 cycles (64 lanes on a SIMD-32) / 1024 SIMDs / clock, the
clock being GRBM_GUI_ACTIVE / 8 XCDs / kernel duration ("DVFS give-back" in MI355X_MICROARCH.md), all from the
same pass. PMC passes serialise the dispatches, so the kernel runs there without the prep kernels beside it.
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CUS, SIMDS, src_hash  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def base_name(full):
    m = re.search(r"(k_\w+)", full)
    return m.group(1) if m else full


def read_counters(path):
    # kernel full name -> counter -> values per dispatch; "_dur_ns" -> dispatch durations
    per = defaultdict(lambda: defaultdict(list))
    seen = defaultdict(dict)
    with open(path) as f:
        for row in csv.DictReader(f):
            per[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
            seen[row["Kernel_Name"]][row["Dispatch_Id"]] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    for k, d in seen.items():
        per[k]["_dur_ns"] = [float(v) for v in d.values()]
    return per


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    out_dir = os.path.join(HERE, tag)
    os.makedirs(out_dir, exist_ok=True)
    shutil.copyfile(stats, os.path.join(out_dir, f"{cfg}_kernel_stats.csv"))
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
                d[c if c != "_dur_ns" else "dur_ns_" + sub] = sum(vals) / len(vals)
                d.setdefault("dispatches", {})[sub] = len(vals)
    for kname, d in summary.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = 2.0 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
        if "SQ_ACTIVE_INST_VALU" in d and "SQ_BUSY_CYCLES" in d and "SQ_WAVE_CYCLES" in d:
            d["valu_active_per_wave_cycle"] = d["SQ_ACTIVE_INST_VALU"] / max(d["SQ_WAVE_CYCLES"], 1.0)
        if "SQ_INSTS_VALU" in d and "GRBM_GUI_ACTIVE" in d and d.get("dur_ns_sq"):
            clk = d["GRBM_GUI_ACTIVE"] / 8.0 / (d["dur_ns_sq"] * 1e-9)  # Hz
            d["clock_ghz"] = clk / 1e9
            d["valu_issue_ms"] = d["SQ_INSTS_VALU"] * 2.0 / SIMDS / clk * 1e3
            d["valu_issue_frac_alone"] = d["valu_issue_ms"] / (d["dur_ns_sq"] * 1e-6)
            if "SQ_LDS_IDX_ACTIVE" in d:
                # LDS-array cycles summed over the CUs (MI355X_MICROARCH.md "LDS"): busy time of one CU's array
                d["lds_array_ms"] = d["SQ_LDS_IDX_ACTIVE"] / CUS / clk * 1e3
                d["lds_array_frac_alone"] = d["lds_array_ms"] / (d.get("dur_ns_sq2", d["dur_ns_sq"]) * 1e-6)
    with open(os.path.join(out_dir, f"{cfg}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    timed = [k for k in summary if base_name(k) in ("k_render_cor", "k_render_ref") and "hbm_bytes_per_launch" in summary[k]]
    if timed:
        k = max(timed, key=lambda k: summary[k]["hbm_bytes_per_launch"])
        d = summary[k]
        out = {"config": cfg, "tag": tag, "src_hash": src_hash(), "kernel": k, "fetch_kib": d["FETCH_SIZE"],
               "write_kib": d["WRITE_SIZE"], "hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
               "method": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving), mean over dispatches",
               "valu_issue_ms": d.get("valu_issue_ms"), "clock_ghz": d.get("clock_ghz"),
               "valu_issue_frac_alone": d.get("valu_issue_frac_alone"),
               "valu_method": "SQ_INSTS_VALU x 2 cycles / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 / duration)",
               "lds_array_ms": d.get("lds_array_ms"), "lds_array_frac_alone": d.get("lds_array_frac_alone"),
               "lds_method": "SQ_LDS_IDX_ACTIVE / 256 CUs / clock (pass sq2, clock from pass sq)"}
        # one entry per config, keyed by its name (the other configs' entries are kept)
        path = os.path.join(HERE, "pmc_traffic.json")
        try:
            with open(path) as f:
                allc = json.load(f)
        except (OSError, ValueError):
            allc = {}
        if "config" in allc:  # the one-config layout of rounds 2-4
            allc = {allc["config"]: allc}
        allc[cfg] = out
        with open(path, "w") as f:
            json.dump(allc, f, indent=1, sort_keys=True)
        print(json.dumps(out))
    for k, d in sorted(summary.items()):
        print(base_name(k), {c: round(v, 3) for c, v in d.items() if isinstance(v, float)})


if __name__ == "__main__":
    main()
