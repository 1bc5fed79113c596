// obj_fuzz_driver.cpp — runs the host OBJ/MTL loader (host/scene.cpp through
// include/vct_host.h) and the placement helpers over every file named on the
// command line; with --png first, the PNG decoder (host/png.cpp) instead.  Built with -fsanitize=address,undefined -fno-sanitize-recover=all
// (tests/native/Makefile): any out-of-bounds access, use-after-free, leak or UB
// aborts the process.  TEST INFRASTRUCTURE (tests/test_sanitizers.py).
#include <cstdio>
#include <cstring>

#include "vct_host.h"

#include <vector>

static int decode_pngs(int argc, char** argv) {
    int ok = 0, rejected = 0;
    for (int a = 2; a < argc; ++a) {
        FILE* f = std::fopen(argv[a], "rb");
        if (!f) return 8;
        std::vector<uint8_t> buf;
        uint8_t chunk[4096];
        size_t n;
        while ((n = std::fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + n);
        std::fclose(f);
        uint8_t* data = nullptr;
        uint32_t w = 0, h = 0;
        int comp = 0;
        char err[128];
        if (vcth_decode_png(buf.data(), buf.size(), &data, &w, &h, &comp, err, (int)sizeof err) != 0) {
            ++rejected;
            continue;
        }
        unsigned acc = 0;   // touch every byte handed out
        for (size_t i = 0; i < (size_t)w * h * comp; ++i) acc += data[i];
        vcth_free_image(data);
        ok += 1 + (int)(acc & 0);
    }
    std::printf("decoded %d rejected %d\n", ok, rejected);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "--png") == 0) return decode_pngs(argc, argv);
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
            const char* path = nullptr;
            int32_t tex = -2;
            if (vcth_material_diffuse_map(m, i, &path, &tex) != 0 || !path || tex < -1 ||
                tex >= (int32_t)vcth_num_textures(m))
                return 9;
        }
        for (uint32_t i = 0; i < vcth_num_textures(m); ++i) {
            const uint8_t* px = nullptr;
            uint32_t w = 0, h = 0;
            if (vcth_texture(m, i, &px, &w, &h, nullptr) != 0) return 10;
            for (size_t k = 0; k < (size_t)w * h * 4; ++k) acc += px[k];
        }
        vcth_free(m);
        if (acc < 0) return 7;
    }
    std::printf("loaded %d rejected %d\n", loaded, rejected);
    return 0;
}
