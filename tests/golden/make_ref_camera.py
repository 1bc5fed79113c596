#!/usr/bin/env python3
"""Writes tests/golden/ref_camera.json from the reference's own code.

Runs oracle/_ref/ref_probe (oracle/ref_probe.cpp compiled against
/root/reference/include and the reference's scene/camera.cpp by
`make -C oracle ref`; container only, the reference never travels).  The
fixture holds hex floats: the reference Vertex layout (stdafx.h:36-42), the
model matrix of VoxelizationRenderer::Render (r_voxelization.cpp:26-29) and, per
camera, GLM's Position/Front/Right/Up/Zoom, view matrix and
perspective(radians(Zoom), w/h, 0.1, 100) (camera.cpp:24-83,
r_voxelization.cpp:16-18).
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main():
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    out = subprocess.run([os.path.join(REPO, "oracle", "_ref", "ref_probe")], capture_output=True, text=True,
                         check=True).stdout
    data = json.loads(out)
    data["generator"] = "oracle/ref_probe.cpp (GLM + camera.cpp of the reference) via tests/golden/make_ref_camera.py"
    with open(os.path.join(HERE, "ref_camera.json"), "w") as f:
        json.dump(data, f, indent=1)
    print(f"wrote ref_camera.json: {len(data['cameras'])} cameras")


if __name__ == "__main__":
    main()
