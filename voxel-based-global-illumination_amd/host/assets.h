// assets.h — name-keyed plug-in registry, shaped like assets/code/core/assets.h:10-32
// (lazy singleton, not thread-safe, maps of cameras / models / renderers).
#pragma once
#include <map>
#include <memory>
#include <string>

#include "camera.h"
#include "renderer.h"
#include "scene.h"

namespace vcthost {

class AssetsManager {
public:
    static AssetsManager& Instance() {
        static AssetsManager inst;
        return inst;
    }
    std::map<std::string, std::shared_ptr<Camera>> cameras;
    std::map<std::string, std::shared_ptr<Model>> models;
    std::map<std::string, std::shared_ptr<Renderer>> renderers;
    std::string active_camera = "FPS";

    std::shared_ptr<Camera> ActiveCamera() { return cameras[active_camera]; }

    AssetsManager(const AssetsManager&) = delete;
    AssetsManager& operator=(const AssetsManager&) = delete;

private:
    AssetsManager() = default;
};

}  // namespace vcthost
