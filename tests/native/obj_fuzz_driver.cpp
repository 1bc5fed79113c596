// obj_fuzz_driver.cpp — runs the host OBJ/MTL loader (host/scene.cpp through
// include/vct_host.h) and the placement helpers over every file named on the
// command line.  Built with -fsanitize=address,undefined -fno-sanitize-recover=all
// (tests/native/Makefile): any out-of-bounds access, use-after-free, leak or UB
// aborts the process.  TEST INFRASTRUCTURE (tests/test_sanitizers.py).
#include <cstdio>
#include <cstring>

#include "vct_host.h"

int main(int argc, char** argv) {
    int loaded = 0, rejected = 0;
    for (int a = 1; a < argc; ++a) {
        vcth_model* m = nullptr;
        char err[256];
        if (vcth_load_obj(argv[a], &m, err, (int)sizeof err) != 0) {
            ++rejected;
            continue;
        }
        ++loaded;
        float M[16];
        vcth_reference_model_matrix(M);
        vcth_transform(m, M);
        float lo[3], hi[3], g0[3], e = 0.0f;
        if (vcth_bounds(m, lo, hi) == 0) vcth_grid_for_bounds(lo, hi, 64, g0, &e);
        double acc = 0.0;   // touch every byte the accessors hand out
        for (uint32_t i = 0; i < vcth_num_meshes(m); ++i) {
            const void* v = nullptr;
            const uint32_t* idx = nullptr;
            uint32_t nv = 0, ni = 0, mat = 0;
            if (vcth_mesh(m, i, &v, &nv, &idx, &ni, &mat) != 0) return 3;
            const float* f = (const float*)v;
            for (uint32_t k = 0; k < nv * 14; ++k) acc += f[k] == f[k] ? 0.0 : 1.0;
            for (uint32_t k = 0; k < ni; ++k)
                if (idx[k] >= nv) return 4;                      // a mesh's indices address its own vertices
            if (mat >= vcth_num_materials(m)) return 5;
        }
        for (uint32_t i = 0; i < vcth_num_materials(m); ++i) {
            const char* name = nullptr;
            float ka[4], kd[4], ks[4];
            if (vcth_material(m, i, &name, ka, kd, ks) != 0 || !name) return 6;
            acc += std::strlen(name);
        }
        vcth_free(m);
        if (acc < 0) return 7;
    }
    std::printf("loaded %d rejected %d\n", loaded, rejected);
    return 0;
}
