// ref_probe.cpp — input-side conventions of the reference, measured from the
// reference's own code (TEST INFRASTRUCTURE: builds only where /root/reference
// exists; output -> tests/golden/ref_camera.json via tests/golden/make_ref_camera.py).
//
// Compiled against /root/reference/include (GLM + stdafx.h, unmodified) together
// with the reference's scene/camera.cpp where it lies (oracle/Makefile target
// `ref`, binary in oracle/_ref/).  It prints, as JSON with hex floats:
//  * sizeof / offsetof of the reference `Vertex` (include/stdafx.h:36-42);
//  * the model matrix of VoxelizationRenderer::Render,
//    translate(T(0,-1.75,0)) then scale(0.2) (assets/code/renderer/r_voxelization.cpp:26-29);
//  * for a set of cameras driven through the reference Camera API
//    (scene/camera.cpp: constructor :4-12, GetViewMatrix :24-27, ProcessKeyboard
//    :29-40, ProcessMouseMovement :42-61, ProcessMouseScroll :63-71,
//    updateCameraVectors :73-83): Position / Front / Right / Up / Zoom, the view
//    matrix, and glm::perspective(radians(Zoom), w / h, 0.1f, 100.0f) for several
//    window sizes (r_voxelization.cpp:16-18).
#include "stdafx.h"
#include "camera.h"

#include <cstddef>
#include <cstdio>

static void hexf(float v, bool comma = true) { std::printf("\"%a\"%s", (double)v, comma ? ", " : ""); }
static void vec3(const char* name, const glm::vec3& v) {
    std::printf("\"%s\": [", name);
    hexf(v.x); hexf(v.y); hexf(v.z, false);
    std::printf("], ");
}
static void mat4(const char* name, const glm::mat4& m, bool comma = true) {   // column-major, m[col][row]
    std::printf("\"%s\": [", name);
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) hexf(m[c][r], !(c == 3 && r == 3));
    std::printf("]%s", comma ? ", " : "");
}

struct Op { char kind; float a, b; };   // m: mouse (dx, dy); s: scroll (dy); f/b/l/r: keyboard (dt)

int main() {
    std::printf("{\"vertex\": {\"sizeof\": %zu, \"Position\": %zu, \"Normal\": %zu, \"TexCoords\": %zu, "
                "\"Tangent\": %zu, \"Bitangent\": %zu}, ",
                sizeof(Vertex), offsetof(Vertex, Position), offsetof(Vertex, Normal), offsetof(Vertex, TexCoords),
                offsetof(Vertex, Tangent), offsetof(Vertex, Bitangent));
    glm::mat4 modelM = glm::mat4(1.0f);                      // r_voxelization.cpp:26-29
    modelM = glm::translate(modelM, glm::vec3(0.0f, -1.75f, 0.0f));
    modelM = glm::scale(modelM, glm::vec3(0.2f, 0.2f, 0.2f));
    mat4("model", modelM);
    const int sizes[][2] = {{800, 600}, {1280, 720}, {1920, 1080}, {3840, 2160}, {160, 120}, {200, 130}, {64, 48}};
    struct Case { float px, py, pz, yaw, pitch; std::vector<Op> ops; };
    const Case cases[] = {
        {0.0f, 0.0f, 3.0f, -90.0f, 0.0f, {}},                                   // assets.cpp:25 default
        {0.0f, 0.0f, 3.0f, -90.0f, 0.0f, {{'m', 120.0f, -45.0f}}},
        {0.3f, -0.2f, 2.5f, -90.0f, 0.0f, {{'m', -200.0f, 130.0f}, {'s', 10.0f, 0}}},
        {0.0f, 0.5f, 0.9f, -90.0f, 0.0f, {{'m', 330.0f, -520.0f}, {'f', 0.25f, 0}, {'s', -3.0f, 0}}},
        {-0.4f, 0.1f, 2.0f, -60.0f, 10.0f, {{'m', 0.0f, 2000.0f}, {'l', 0.1f, 0}, {'s', 50.0f, 0}}},   // pitch clamp, zoom clamp
        {0.2f, 0.0f, 1.5f, -120.0f, -20.0f, {{'r', 0.05f, 0}, {'b', 0.1f, 0}, {'m', 37.5f, 12.25f}}},
    };
    std::printf("\"cameras\": [");
    bool first = true;
    for (const Case& cs : cases) {
        Camera cam(glm::vec3(cs.px, cs.py, cs.pz), glm::vec3(0.0f, 1.0f, 0.0f), cs.yaw, cs.pitch);
        for (const Op& o : cs.ops) {
            switch (o.kind) {
                case 'm': cam.ProcessMouseMovement(o.a, o.b); break;
                case 's': cam.ProcessMouseScroll(o.a); break;
                case 'f': cam.ProcessKeyboard(FORWARD, o.a); break;
                case 'b': cam.ProcessKeyboard(BACKWARD, o.a); break;
                case 'l': cam.ProcessKeyboard(LEFT, o.a); break;
                case 'r': cam.ProcessKeyboard(RIGHT, o.a); break;
            }
        }
        std::printf("%s{\"init\": [", first ? "" : ", ");
        first = false;
        hexf(cs.px); hexf(cs.py); hexf(cs.pz); hexf(cs.yaw); hexf(cs.pitch, false);
        std::printf("], \"ops\": [");
        for (size_t i = 0; i < cs.ops.size(); ++i) {
            std::printf("%s[\"%c\", ", i ? ", " : "", cs.ops[i].kind);
            hexf(cs.ops[i].a); hexf(cs.ops[i].b, false);
            std::printf("]");
        }
        std::printf("], ");
        vec3("position", cam.Position);
        vec3("front", cam.Front);
        vec3("right", cam.Right);
        vec3("up", cam.Up);
        std::printf("\"yaw\": "); hexf(cam.Yaw);
        std::printf("\"pitch\": "); hexf(cam.Pitch);
        std::printf("\"zoom\": "); hexf(cam.Zoom);
        mat4("view", cam.GetViewMatrix());
        std::printf("\"proj\": {");
        for (size_t i = 0; i < sizeof sizes / sizeof sizes[0]; ++i) {
            const int w = sizes[i][0], h = sizes[i][1];
            const glm::mat4 P = glm::perspective(glm::radians(cam.Zoom), (float)w / (float)h, 0.1f, 100.0f);
            char key[32];
            std::snprintf(key, sizeof key, "%dx%d", w, h);
            mat4(key, P, i + 1 < sizeof sizes / sizeof sizes[0]);
        }
        std::printf("}}");
    }
    std::printf("]}\n");
    return 0;
}
