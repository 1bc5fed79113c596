// ref_stb_probe.cpp — runs the REFERENCE's own image decoder (TEST INFRASTRUCTURE).
//
// The reference decodes its diffuse maps with the stb_image it vendors
// (assets/code/support/stb_image.cpp, the STB_IMAGE_IMPLEMENTATION unit) through
// `stbi_load(filename, &width, &height, &nrComponents, 0)` (assets/code/scene/
// model.cpp:197).  oracle/Makefile (`make -C oracle ref`) compiles that unit where
// it lies under /root/reference together with this driver into oracle/_ref/ (never
// copied, never shipped; only in the build container).  tests/golden/
// make_tex_golden.py runs it to pin the host PNG decoder (host/png.cpp) and the
// texture fixtures of the diffuse-map parity tests.
//
// usage: ref_stb_probe IN.png OUT.raw [IN2.png OUT2.raw ...]
// prints one line per image: "<w> <h> <comp>" (or "fail <reason>"); OUT.raw gets
// the h x w x comp bytes exactly as stbi_load returned them.
#include <cstdio>

#include "stb_image.h"

int main(int argc, char** argv) {
    if (argc < 3 || argc % 2 == 0) {
        std::fprintf(stderr, "usage: %s IN.png OUT.raw [...]\n", argv[0]);
        return 2;
    }
    for (int i = 1; i + 1 < argc; i += 2) {
        int w = 0, h = 0, comp = 0;
        unsigned char* data = stbi_load(argv[i], &w, &h, &comp, 0);   // model.cpp:197
        if (!data) {
            std::printf("fail %s\n", stbi_failure_reason());
            continue;
        }
        FILE* f = std::fopen(argv[i + 1], "wb");
        if (!f) return 1;
        std::fwrite(data, 1, (size_t)w * h * comp, f);
        std::fclose(f);
        std::printf("%d %d %d\n", w, h, comp);
        stbi_image_free(data);
    }
    return 0;
}
