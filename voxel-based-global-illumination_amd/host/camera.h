// camera.h — FPS camera with the reference's conventions (scene/camera.h:6-54).
#pragma once
#include "vct.h"

namespace vcthost {

constexpr float kYaw = -90.0f, kPitch = 0.0f, kSpeed = 2.5f, kSensitivity = 0.1f, kZoom = 45.0f;

enum CameraMovement { FORWARD, BACKWARD, LEFT, RIGHT };   // camera.h:6-11

class Camera {
public:
    float Position[3], Front[3], Up[3], Right[3], WorldUp[3];
    float Yaw, Pitch, MovementSpeed, MouseSensitivity, Zoom;

    explicit Camera(float px = 0, float py = 0, float pz = 3, float yaw = kYaw, float pitch = kPitch);

    void ProcessKeyboard(CameraMovement d, float dt);                 // camera.cpp:29-40
    void ProcessMouseMovement(float dx, float dy, bool constrain = true);  // camera.cpp:42-61
    void ProcessMouseScroll(float dy);                                 // camera.cpp:63-71

    // the vct_camera the cone-trace path consumes (perspective 0.1..100, r_voxelization.cpp:18)
    vct_camera ToVct() const;

private:
    void updateCameraVectors();                                        // camera.cpp:73-83
};

}  // namespace vcthost
