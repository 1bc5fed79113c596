#!/usr/bin/env python3
"""Generate the committed golden vectors (tests/golden/*.npz) from the CPU oracle.

The reference repository holds no fixtures or golden outputs for this path
(SURVEY.md 4, 8c), so these vectors are the oracle's own outputs on small,
fully specified inputs.  They pin the oracle against regressions (CPU tests)
and give the GPU tests a target that does not need the oracle at run time.
The oracle itself is pinned by the closed-form KATs and the independent
restatement in tests/test_oracle_kat.py.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]

from oracle import oracle as O          # noqa: E402
from vct import scenes                  # noqa: E402
from vct.camera import Camera           # noqa: E402

CASES = {
    # name: (scene, n, gbuffer, w, h, aniso, n_diffuse, specular)
    "cornell16_scene": ("cornell", 16, "scene", 32, 24, True, 9, True),
    "atrium16_rand": ("atrium", 16, "rand", 24, 16, True, 9, True),
    "atrium16_iso_c16": ("atrium", 16, "scene", 24, 16, False, 16, True),
    "random16_c1": ("random", 16, "rand", 16, 16, True, 1, False),
}


def build_case(scene, n, gbuf, w, h, aniso, nd, spec):
    s = scenes.random_triangles(80, seed=5) if scene == "random" else scenes.SCENES[scene]()
    v, i, m, k = s.arrays()
    g0, E = scenes.grid_for_unit_box(n)
    st = O.pipeline(n, g0, E, v, i, m, k, scenes.LIGHT_DIR, aniso=aniso)
    cam = Camera()
    if gbuf == "scene":
        pos, nrm, alb = scenes.raycast_numpy(s, cam, w, h)
    else:
        pos, nrm, alb = scenes.gbuffer_rand(st["albedo_occ"], st["normal"], g0, E, w, h, seed=42)
    res = O.trace(n, g0, E, st["r0"], st["pyr"], pos, nrm, alb, cam.position, aniso=aniso, n_diffuse=nd,
                  specular=spec)
    occ = st["counts"] > 0
    return dict(
        cfg=np.array([n, w, h, int(aniso), nd, int(spec)], np.int64),
        aabb=np.array(list(g0) + [E], np.float32),
        eye=np.asarray(cam.position, np.float32),
        counts=st["counts"], sums_occ=st["sums"][occ], r0=st["r0"], pyr=st["pyr"],
        pos=pos, nrm=nrm, alb=alb, diffuse=res["diffuse"], spec=res["spec"], steps_px=res["steps_px"],
    )


def main():
    O.build()
    for name, c in CASES.items():
        d = build_case(*c)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print(name, os.path.getsize(os.path.join(HERE, name + ".npz")), "bytes")


if __name__ == "__main__":
    main()
