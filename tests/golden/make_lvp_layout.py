"""Generates tests/golden/lvp_layout.json: byte offsets / sizes of the lavapipe and Vulkan structures the driver-side
drop-in (tests/integration/vksim_shim.cpp) reads, measured on the REFERENCE's own headers by
oracle/ref/lvp_layout_probe.c (built by `make -C oracle lvp-layout` from /root/reference/mesa-vulkan-sim: its
vulkan_core.h, p_state.h, vk_object.h, vk_descriptor_set_layout.h, vk_image.h and the struct line ranges of
lavapipe/lvp_private.h). Run in the container that holds /root/reference:

  python tests/golden/make_lvp_layout.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "lvp_layout.json")

subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "lvp-layout"], check=True)
out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "lvp_layout_probe")], check=True, capture_output=True,
                     text=True).stdout
layout = json.loads(out)
with open(OUT, "w") as f:
    json.dump(layout, f, indent=1, sort_keys=True)
    f.write("\n")
print(OUT, len(layout), "entries")
