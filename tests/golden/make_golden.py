"""Regenerate the golden fixtures in tests/golden/ with the CPU oracle (oracle/gsrt_oracle.c).

The reference itself cannot be built or run, so the only reference-derived known
answer is KAT-1 (scene 33 at 16x16), whose values are hand-derived from the reference shaders and
asserted independently in tests/test_oracle.py. The other fixtures pin the oracle (and, through the
GPU tests, the HIP path) to fixed bytes across builds and machines.

Usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402

# contents of two RayTracingInVulkan/Scenes/*.camera files (eye xyz, centre xyz), kept as data
CAMERA_FILES = {
    "Bathroom/Camera.camera": "3.281494617462158 20.03567123413086 40.006858825683594\n"
                              "3.056297540664673 19.762132227420807 39.07173180580139\n",
    "Blender_2.78/camera.camera": "-0.35024330019950867 1.1617968082427979 1.0811127424240112\n"
                                  "-0.06039896607398987 1.5020394325256348 0.18655967712402344\n",
}


def synth_inputs(kind, n, seed, sh=False):
    c, r, s, o, shc = O.synth_cloud(kind, n, seed, sh)
    return c, r, s, o, shc


def main():
    # ExpLUT (ExpLUT.hpp:10-24)
    np.savez(os.path.join(HERE, "exp_lut.npz"), lut=O.exp_lut())

    # KAT-1: scene 33, 16x16, S=1, B=16, REF
    p, a = O.scene33()
    ubo = O.make_ubo(O.translate(0, 0, -2), 90.0, 16, 16, 2.0, 1, 16)
    out = O.render(p, a, ubo, O.MODE_REF, want_raystate=True, want_stats=True)
    np.savez(os.path.join(HERE, "kat1_scene33.npz"), params=p, aabbs=a, ubo=ubo.view(np.uint8),
             raystate=out["raystate"].view(np.uint8), rgba=out["rgba"], stats=out["stats"])

    # GF-REF needles: REF-active synthetic scene (multi-round K-buffer)
    mv = O.lookat((0, 0, 0), (0, 0, -1))
    c, r, s, o, _ = synth_inputs(O.SYNTH_NEEDLE, 300, 42)
    p, a = O.gauss_from_model(c, r, s, o)
    ubo = O.make_ubo(mv, 60.0, 64, 48, 1.0, 1, 16)
    out = O.render(p, a, ubo, O.MODE_REF, want_raystate=True, want_stats=True)
    np.savez(os.path.join(HERE, "ref_needles_300.npz"), center=c, rot=r, scale=s, opacity=o, ubo=ubo.view(np.uint8),
             raystate=out["raystate"].view(np.uint8), stats=out["stats"])

    # GF-COR-10k: front-facing cloud, 64x48, 1 spp
    c, r, s, o, _ = synth_inputs(O.SYNTH_COR, 10000, 42)
    p, a = O.gauss_from_model(c, r, s, o)
    ubo = O.make_ubo(mv, 60.0, 64, 48, 1.0, 1, 16)
    out = O.render(p, a, ubo, O.MODE_COR, bvh=O.Bvh(a), want_stats=True)
    np.savez(os.path.join(HERE, "cor_10k.npz"), center=c, rot=r, scale=s, opacity=o, ubo=ubo.view(np.uint8),
             rgba=out["rgba"], stats=out["stats"])

    # GF-COR-SH: 1k Gaussians with SH-3, 48x32, 4 spp
    c, r, s, o, sh = synth_inputs(O.SYNTH_COR, 1000, 5, sh=True)
    p, a = O.gauss_from_model(c, r, s, o)
    ubo = O.make_ubo(mv, 60.0, 48, 32, 1.0, 4, 16)
    out = O.render(p, a, ubo, O.MODE_COR, sh=sh, bvh=O.Bvh(a), want_stats=True)
    np.savez(os.path.join(HERE, "cor_sh3_1k.npz"), center=c, rot=r, scale=s, opacity=o, sh=sh,
             ubo=ubo.view(np.uint8), rgba=out["rgba"], stats=out["stats"])

    # cameras: .camera file -> UBO bytes (lookAt + ModelViewController + perspective)
    cams = {}
    for name, text in CAMERA_FILES.items():
        v = [float(x) for x in text.split()]
        mv = O.lookat(v[:3], v[3:])
        ubo = O.make_ubo(mv, 60.0, 1280, 720, 1.0, 8, 16)
        cams[name] = {"text": text, "ubo_hex": ubo.tobytes().hex()}
    with open(os.path.join(HERE, "cameras.json"), "w") as f:
        json.dump(cams, f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
