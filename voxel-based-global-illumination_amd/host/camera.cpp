// camera.cpp — see camera.h.
#include "camera.h"

#include <cmath>

namespace vcthost {

// The float operation sequence of GLM as the reference calls it (bit-identical;
// tests/test_ref_conventions.py checks every vector against the reference's own
// camera.cpp + GLM, tests/golden/ref_camera.json):
//  * glm::radians(d) = d * float(0.01745329251994329576923690768489)
//    (glm/detail/func_trigonometric.inl:9-14);
//  * glm::normalize(v) = v * (1 / sqrt(dot(v, v))), dot = (x x + y y) + z z
//    (func_geometric.inl:48-55,82-90; func_exponential.inl:136-139).
namespace {
constexpr float kDeg = (float)0.01745329251994329576923690768489;
void normalize(float v[3]) {
    const float inv = 1.0f / std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
}
void cross(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
}  // namespace

Camera::Camera(float px, float py, float pz, float yaw, float pitch)
    : Position{px, py, pz}, Front{0, 0, -1}, Up{0, 1, 0}, Right{1, 0, 0}, WorldUp{0, 1, 0},
      Yaw(yaw), Pitch(pitch), MovementSpeed(kSpeed), MouseSensitivity(kSensitivity), Zoom(kZoom) {
    updateCameraVectors();
}

void Camera::ProcessKeyboard(CameraMovement d, float dt) {
    const float v = MovementSpeed * dt;
    for (int k = 0; k < 3; ++k) {
        if (d == FORWARD) Position[k] += Front[k] * v;
        if (d == BACKWARD) Position[k] -= Front[k] * v;
        if (d == LEFT) Position[k] -= Right[k] * v;
        if (d == RIGHT) Position[k] += Right[k] * v;
    }
}

void Camera::ProcessMouseMovement(float dx, float dy, bool constrain) {
    Yaw += dx * MouseSensitivity;
    Pitch += dy * MouseSensitivity;
    if (constrain) {
        if (Pitch > 89.0f) Pitch = 89.0f;
        if (Pitch < -89.0f) Pitch = -89.0f;
    }
    updateCameraVectors();
}

void Camera::ProcessMouseScroll(float dy) {
    if (Zoom >= 1.0f && Zoom <= 45.0f) Zoom -= dy;
    if (Zoom <= 1.0f) Zoom = 1.0f;
    if (Zoom >= 45.0f) Zoom = 45.0f;
}

void Camera::updateCameraVectors() {
    Front[0] = std::cos(Yaw * kDeg) * std::cos(Pitch * kDeg);
    Front[1] = std::sin(Pitch * kDeg);
    Front[2] = std::sin(Yaw * kDeg) * std::cos(Pitch * kDeg);
    normalize(Front);
    cross(Front, WorldUp, Right);
    normalize(Right);
    cross(Right, Front, Up);
    normalize(Up);
}

vct_camera Camera::ToVct() const {
    vct_camera c{};
    for (int k = 0; k < 3; ++k) {
        c.position[k] = Position[k];
        c.front[k] = Front[k];
        c.up[k] = Up[k];
        c.right[k] = Right[k];
    }
    c.zoom_deg = Zoom;
    c.near_plane = 0.1f;
    c.far_plane = 100.0f;
    return c;
}

}  // namespace vcthost
