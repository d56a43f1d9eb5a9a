"""The render kernel's mean duration from a rocprofv3 --kernel-trace CSV of a bench.py run, the way bench.py's
roofline takes it: over the timed frames, and over the serialised frames bench.py renders after the timed region
when frames overlapped (slot streams; `kernel_ms_from` in the line). Reproduces `roofline.kernel_ms`.

  python profiles/kernel_ms_from_trace.py <run_kernel_trace.csv> <steps> [serialised_frames=12]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_render_cor<" in r["Kernel_Name"] or "k_render_ref<" in r["Kernel_Name"]]
rows = [r for r in rows if not r["Kernel_Name"].rstrip().endswith("true>(gsrt::KArgs)")]  # the counting pass
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2])
ser = int(sys.argv[3]) if len(sys.argv) > 3 else 12
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print(f"{len(d)} dispatches; mean of all {sum(d) / len(d):.4f} ms")
print(f"last {ser} (serialised pass): {sum(d[-ser:]) / ser:.4f} ms")
timed = d[-ser - steps:-ser]
print(f"the {steps} before them (timed frames, if a serialised pass ran): {sum(timed) / len(timed):.4f} ms")
timed2 = d[-steps:]
print(f"the last {steps} (timed frames, if none ran): {sum(timed2) / len(timed2):.4f} ms")
