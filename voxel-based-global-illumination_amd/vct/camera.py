"""FPS camera with the reference's conventions.

Mirrors assets/code/scene/camera.{h,cpp}: defaults YAW = -90, PITCH = 0,
ZOOM = 45 (camera.h:14-18); Front from yaw/pitch and Right/Up by cross
products (camera.cpp:73-83); view = lookAt(Position, Position + Front, Up)
(camera.cpp:24-27); projection = perspective(radians(Zoom), w/h, 0.1, 100)
(r_voxelization.cpp:18).  The VCT path consumes it as a vct_camera (include/vct.h).
"""
from __future__ import annotations

import math

import numpy as np

from ._lib import VctCamera

YAW, PITCH, SPEED, SENSITIVITY, ZOOM = -90.0, 0.0, 2.5, 0.1, 45.0


def _normalize(v):
    v = np.asarray(v, np.float64)
    return v / np.linalg.norm(v)


class Camera:
    def __init__(self, position=(0.0, 0.0, 3.0), up=(0.0, 1.0, 0.0), yaw=YAW, pitch=PITCH):
        self.position = np.asarray(position, np.float64)
        self.world_up = np.asarray(up, np.float64)
        self.yaw, self.pitch, self.zoom = float(yaw), float(pitch), ZOOM
        self.near, self.far = 0.1, 100.0
        self._update()

    def _update(self):  # camera.cpp:73-83
        y, p = math.radians(self.yaw), math.radians(self.pitch)
        self.front = _normalize([math.cos(y) * math.cos(p), math.sin(p), math.sin(y) * math.cos(p)])
        self.right = _normalize(np.cross(self.front, self.world_up))
        self.up = _normalize(np.cross(self.right, self.front))

    def process_mouse(self, dx: float, dy: float, constrain_pitch: bool = True):  # camera.cpp:42-61
        self.yaw += dx * SENSITIVITY
        self.pitch += dy * SENSITIVITY
        if constrain_pitch:
            self.pitch = max(-89.0, min(89.0, self.pitch))
        self._update()

    def process_scroll(self, dy: float):  # camera.cpp:63-71
        if 1.0 <= self.zoom <= 45.0:
            self.zoom -= dy
        self.zoom = min(45.0, max(1.0, self.zoom))

    def process_keyboard(self, direction: str, dt: float):  # camera.cpp:29-40
        v = SPEED * dt
        step = {"FORWARD": self.front, "BACKWARD": -self.front, "LEFT": -self.right, "RIGHT": self.right}[direction]
        self.position = self.position + step * v

    def view_matrix(self) -> np.ndarray:
        """glm::lookAtRH(Position, Position + Front, Up) (camera.cpp:26)."""
        f, s, u = self.front, self.right, np.cross(self.right, self.front)
        m = np.eye(4)
        m[0, :3], m[1, :3], m[2, :3] = s, u, -f
        m[0, 3], m[1, 3], m[2, 3] = -s @ self.position, -u @ self.position, f @ self.position
        return m

    def projection_matrix(self, aspect: float) -> np.ndarray:
        """glm::perspectiveRH_NO(radians(Zoom), aspect, 0.1, 100) (r_voxelization.cpp:18)."""
        t = math.tan(math.radians(self.zoom) / 2)
        n, f = self.near, self.far
        m = np.zeros((4, 4))
        m[0, 0], m[1, 1] = 1 / (aspect * t), 1 / t
        m[2, 2], m[2, 3], m[3, 2] = -(f + n) / (f - n), -2 * f * n / (f - n), -1.0
        return m

    def to_ctypes(self) -> VctCamera:
        c = VctCamera()
        c.position[:] = [float(x) for x in self.position]
        c.front[:] = [float(x) for x in self.front]
        c.up[:] = [float(x) for x in self.up]
        c.right[:] = [float(x) for x in self.right]
        c.zoom_deg, c.near_plane, c.far_plane = self.zoom, self.near, self.far
        return c


def reference_model_matrix() -> np.ndarray:
    """The model matrix of VoxelizationRenderer::Render, column-major float32:
    glm::scale(glm::translate(mat4(1), (0, -1.75, 0)), (0.2, 0.2, 0.2))
    (r_voxelization.cpp:26-29), in GLM's float operation order."""
    m = np.eye(4, dtype=np.float32).T.reshape(-1).copy()        # column-major identity
    t = np.array([0.0, -1.75, 0.0], np.float32)
    for row in range(4):                                         # translate: col3 = c0 tx + c1 ty + c2 tz + c3
        m[12 + row] = ((m[row] * t[0] + m[4 + row] * t[1]) + m[8 + row] * t[2]) + m[12 + row]
    m[:12] = m[:12] * np.float32(0.2)                            # scale: columns 0..2
    return m

