/*
 * vct_dumpio.c — the "vct-dump/2" grid dump format (see vct_dumpio.h): header JSON,
 * sectioned payload, SHA-256 over the payload.  Plain C; also compiled as HIP C++.
 */
#include "vct_dumpio.h"

#include <errno.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>

#define VDUMP_FORMAT "vct-dump/2"

static int verr(char* err, size_t errlen, const char* fmt, ...) {
    if (err && errlen) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(err, errlen, fmt, ap);
        va_end(ap);
    }
    return 1;
}

/* ---- SHA-256 (FIPS 180-4) ------------------------------------------------------- */
static const uint32_t kSha[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static uint32_t rotr(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

static void sha_block(uint32_t* h, const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 64; ++i) {
        const uint32_t t1 = k + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kSha[i] + w[i];
        const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

void vdump_sha256_init(vdump_sha256* s) {
    static const uint32_t h0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    memcpy(s->h, h0, sizeof h0);
    s->len = 0;
    s->fill = 0;
}

void vdump_sha256_update(vdump_sha256* s, const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    s->len += n;
    if (s->fill) {
        const size_t k = n < 64 - s->fill ? n : 64 - s->fill;
        memcpy(s->buf + s->fill, p, k);
        s->fill += (uint32_t)k;
        p += k;
        n -= k;
        if (s->fill < 64) return;
        sha_block(s->h, s->buf);
        s->fill = 0;
    }
    for (; n >= 64; p += 64, n -= 64) sha_block(s->h, p);
    memcpy(s->buf, p, n);
    s->fill = (uint32_t)n;
}

void vdump_sha256_hex(vdump_sha256* s, char out[65]) {
    const uint64_t bits = s->len * 8u;
    uint8_t pad[72];
    size_t np = (s->fill < 56 ? 56 : 120) - s->fill;
    memset(pad, 0, sizeof pad);
    pad[0] = 0x80;
    for (int i = 0; i < 8; ++i) pad[np + i] = (uint8_t)(bits >> (56 - 8 * i));
    const uint64_t keep = s->len;
    vdump_sha256_update(s, pad, np + 8);
    s->len = keep;
    for (int i = 0; i < 8; ++i) snprintf(out + 8 * i, 9, "%08x", s->h[i]);
}

/* ---- sizes ------------------------------------------------------------------------ */
uint32_t vdump_levels(const vct_config* cfg) {
    uint32_t L = 0;
    while ((1u << (L + 1)) <= cfg->n) ++L;
    return L + 1;
}

uint32_t vdump_faces(const vct_config* cfg, uint32_t level) { return level > 0 && cfg->aniso ? 6u : 1u; }

uint64_t vdump_voxels_bytes(const vdump_header* h) {
    return (h->what & VCT_DUMP_VOXELS) ? h->occupied * (4u + 48u + 4u) : 0u;
}

uint64_t vdump_level0_bytes(const vdump_header* h) {
    const uint64_t n = h->cfg.n;
    return (h->what & VCT_DUMP_LEVEL0) ? n * n * n * 16u : 0u;
}

uint64_t vdump_pyramid_bytes(const vdump_header* h) {
    if (!(h->what & VCT_DUMP_PYRAMID)) return 0u;
    uint64_t b = 0;
    const uint32_t nl = vdump_levels(&h->cfg);
    for (uint32_t l = 1; l < nl; ++l) {
        const uint64_t m = h->cfg.n >> l;
        b += (uint64_t)vdump_faces(&h->cfg, l) * m * m * m * 16u;
    }
    return b;
}

uint64_t vdump_payload_bytes(const vdump_header* h) {
    return vdump_voxels_bytes(h) + vdump_level0_bytes(h) + vdump_pyramid_bytes(h);
}

/* ---- paths and the header --------------------------------------------------------- */
static int stem_paths(const char* stem, vdump_file* f, char* err, size_t errlen) {
    if (!stem || !*stem) return verr(err, errlen, "empty dump path");
    size_t n = strlen(stem);
    if (n >= 5 && strcmp(stem + n - 5, ".json") == 0) n -= 5;
    else if (n >= 4 && strcmp(stem + n - 4, ".bin") == 0) n -= 4;
    if (n + 6 > sizeof f->json) return verr(err, errlen, "dump path too long");
    memcpy(f->json, stem, n);
    memcpy(f->bin, stem, n);
    strcpy(f->json + n, ".json");
    strcpy(f->bin + n, ".bin");
    return 0;
}

static const char* base_name(const char* p) {
    const char* s = strrchr(p, '/');
    return s ? s + 1 : p;
}

int vdump_open_write(vdump_file* w, const char* stem, const vdump_header* h, char* err, size_t errlen) {
    memset(w, 0, sizeof *w);
    if (stem_paths(stem, w, err, errlen)) return 1;
    w->h = *h;
    w->f = fopen(w->bin, "wb");
    if (!w->f) return verr(err, errlen, "%s: %s", w->bin, strerror(errno));
    vdump_sha256_init(&w->sha);
    return 0;
}

int vdump_write(vdump_file* w, const void* data, size_t n, char* err, size_t errlen) {
    if (n && fwrite(data, 1, n, w->f) != n) return verr(err, errlen, "%s: write failed", w->bin);
    vdump_sha256_update(&w->sha, data, n);
    w->bytes += n;
    return 0;
}

int vdump_close_write(vdump_file* w, char* err, size_t errlen) {
    const int bad = fclose(w->f) != 0;
    w->f = NULL;
    if (bad) return verr(err, errlen, "%s: close failed", w->bin);
    if (w->bytes != vdump_payload_bytes(&w->h))
        return verr(err, errlen, "payload is %llu bytes, the header's sections %llu", (unsigned long long)w->bytes,
                    (unsigned long long)vdump_payload_bytes(&w->h));
    char hex[65];
    vdump_sha256_hex(&w->sha, hex);
    FILE* j = fopen(w->json, "w");
    if (!j) return verr(err, errlen, "%s: %s", w->json, strerror(errno));
    const vct_config* c = &w->h.cfg;
    const uint32_t what = w->h.what;
    fprintf(j,
            "{\n \"format\": \"" VDUMP_FORMAT "\",\n \"kind\": \"grid\",\n \"n\": %u,\n"
            " \"aabb_min\": [%.9g, %.9g, %.9g],\n \"extent\": %.9g,\n \"aniso\": %s,\n \"n_diffuse\": %u,\n"
            " \"specular\": %s,\n \"what\": %u,\n \"sections\": [%s%s%s%s%s],\n \"occupied\": %llu,\n"
            " \"payload\": \"%s\",\n \"payload_bytes\": %llu,\n \"sha256\": \"%s\"\n}\n",
            c->n, (double)c->aabb_min[0], (double)c->aabb_min[1], (double)c->aabb_min[2], (double)c->extent,
            c->aniso ? "true" : "false", c->n_diffuse, c->specular ? "true" : "false", what,
            (what & VCT_DUMP_VOXELS) ? "\"voxels\"" : "", (what & VCT_DUMP_VOXELS) && (what & 6u) ? ", " : "",
            (what & VCT_DUMP_LEVEL0) ? "\"level0\"" : "", (what & VCT_DUMP_LEVEL0) && (what & 4u) ? ", " : "",
            (what & VCT_DUMP_PYRAMID) ? "\"pyramid\"" : "", (unsigned long long)w->h.occupied, base_name(w->bin),
            (unsigned long long)w->bytes, hex);
    if (fclose(j) != 0) return verr(err, errlen, "%s: write failed", w->json);
    return 0;
}

/* the value after "key": in the header text (our own writer's flat layout) */
static const char* json_value(const char* txt, const char* key) {
    char pat[64];
    snprintf(pat, sizeof pat, "\"%s\"", key);
    for (const char* p = strstr(txt, pat); p; p = strstr(p + 1, pat)) {
        const char* q = p + strlen(pat);
        while (*q == ' ' || *q == '\t' || *q == '\n' || *q == '\r') ++q;
        if (*q != ':') continue;
        ++q;
        while (*q == ' ' || *q == '\t' || *q == '\n' || *q == '\r') ++q;
        return q;
    }
    return NULL;
}

static int json_u64(const char* txt, const char* key, uint64_t* out) {
    const char* v = json_value(txt, key);
    if (!v) return 1;
    char* end = NULL;
    errno = 0;
    const unsigned long long x = strtoull(v, &end, 10);
    if (end == v || errno) return 1;
    *out = x;
    return 0;
}

static int json_f32(const char** p, float* out) {
    char* end = NULL;
    *out = strtof(*p, &end);
    if (end == *p) return 1;
    *p = end;
    return 0;
}

static int json_bool(const char* txt, const char* key, uint32_t* out) {
    const char* v = json_value(txt, key);
    if (!v) return 1;
    if (strncmp(v, "true", 4) == 0) *out = 1;
    else if (strncmp(v, "false", 5) == 0) *out = 0;
    else return 1;
    return 0;
}

static int json_str(const char* txt, const char* key, char* out, size_t len) {
    const char* v = json_value(txt, key);
    if (!v || *v != '"') return 1;
    const char* e = strchr(v + 1, '"');
    if (!e || (size_t)(e - v - 1) >= len) return 1;
    memcpy(out, v + 1, (size_t)(e - v - 1));
    out[e - v - 1] = 0;
    return 0;
}

static int parse_header(const char* txt, vdump_header* h, char* sha, uint64_t* bytes, char* err, size_t errlen) {
    char fmt[32], kind[32];
    if (json_str(txt, "format", fmt, sizeof fmt) || strcmp(fmt, VDUMP_FORMAT) != 0 ||
        json_str(txt, "kind", kind, sizeof kind) || strcmp(kind, "grid") != 0)
        return verr(err, errlen, "not a " VDUMP_FORMAT " grid dump");
    memset(h, 0, sizeof *h);
    uint64_t n = 0, nd = 0, what = 0, occ = 0;
    uint32_t aniso = 0, spec = 0;
    float e = 0.0f;
    const char* a = json_value(txt, "aabb_min");
    const char* ev = json_value(txt, "extent");
    int bad = json_u64(txt, "n", &n) || json_u64(txt, "n_diffuse", &nd) || json_u64(txt, "what", &what) ||
              json_u64(txt, "occupied", &occ) || json_u64(txt, "payload_bytes", bytes) ||
              json_bool(txt, "aniso", &aniso) || json_bool(txt, "specular", &spec) || !a || *a != '[' || !ev ||
              json_f32(&ev, &e) || json_str(txt, "sha256", sha, 65) || strlen(sha) != 64;
    if (!bad) {
        ++a;
        for (int i = 0; i < 3 && !bad; ++i) {
            while (*a == ' ' || *a == ',') ++a;
            bad = json_f32(&a, &h->cfg.aabb_min[i]);
        }
    }
    if (bad || n < 4 || n > 1024 || (n & (n - 1)) || (what & ~7ull) || !what)
        return verr(err, errlen, "malformed dump header");
    h->cfg.n = (uint32_t)n;
    h->cfg.extent = e;
    h->cfg.aniso = aniso;
    h->cfg.n_diffuse = (uint32_t)nd;
    h->cfg.specular = spec;
    h->cfg.device = -1;
    h->what = (uint32_t)what;
    h->occupied = occ;
    if (occ > (uint64_t)n * n * n) return verr(err, errlen, "malformed dump header (occupied > n^3)");
    if (*bytes != vdump_payload_bytes(h)) return verr(err, errlen, "dump header: payload_bytes disagrees with its sections");
    return 0;
}

static int read_text(const char* path, char* buf, size_t len, char* err, size_t errlen) {
    FILE* f = fopen(path, "rb");
    if (!f) return verr(err, errlen, "%s: %s", path, strerror(errno));
    const size_t got = fread(buf, 1, len - 1, f);
    const int more = fgetc(f) != EOF;
    fclose(f);
    if (more) return verr(err, errlen, "%s: header too large", path);
    buf[got] = 0;
    return 0;
}

int vdump_read_header(const char* stem, vdump_header* h, char* err, size_t errlen) {
    vdump_file f;
    memset(&f, 0, sizeof f);
    if (stem_paths(stem, &f, err, errlen)) return 1;
    char txt[4096], sha[65];
    uint64_t bytes = 0;
    if (read_text(f.json, txt, sizeof txt, err, errlen)) return 1;
    return parse_header(txt, h, sha, &bytes, err, errlen);
}

int vdump_open_read(vdump_file* r, const char* stem, char* err, size_t errlen) {
    memset(r, 0, sizeof *r);
    if (stem_paths(stem, r, err, errlen)) return 1;
    char txt[4096], sha[65];
    uint64_t bytes = 0;
    if (read_text(r->json, txt, sizeof txt, err, errlen)) return 1;
    if (parse_header(txt, &r->h, sha, &bytes, err, errlen)) return 1;
    r->f = fopen(r->bin, "rb");
    if (!r->f) return verr(err, errlen, "%s: %s", r->bin, strerror(errno));
    /* one pass over the payload: length and sha256 before anything is used */
    vdump_sha256 s;
    vdump_sha256_init(&s);
    uint64_t total = 0;
    size_t cap = 1u << 22;
    uint8_t* buf = (uint8_t*)malloc(cap);
    if (!buf) { vdump_close(r); return verr(err, errlen, "out of host memory"); }
    for (;;) {
        const size_t got = fread(buf, 1, cap, r->f);
        if (!got) break;
        vdump_sha256_update(&s, buf, got);
        total += got;
    }
    free(buf);
    char hex[65];
    vdump_sha256_hex(&s, hex);
    if (total != bytes || strcmp(hex, sha) != 0) {
        vdump_close(r);
        return verr(err, errlen, "%s: payload does not match its header (%s)", r->bin,
                    total != bytes ? "length" : "sha256");
    }
    rewind(r->f);
    r->bytes = bytes;
    return 0;
}

int vdump_read(vdump_file* r, void* data, size_t n, char* err, size_t errlen) {
    if (n && fread(data, 1, n, r->f) != n) return verr(err, errlen, "%s: short read", r->bin);
    return 0;
}

void vdump_close(vdump_file* f) {
    if (f->f) fclose(f->f);
    f->f = NULL;
}

int vdump_check_config(const vdump_header* h, const vct_config* cfg, char* err, size_t errlen) {
    const vct_config* d = &h->cfg;
    if (d->n != cfg->n || (d->aniso != 0) != (cfg->aniso != 0) || memcmp(d->aabb_min, cfg->aabb_min, 12) != 0 ||
        memcmp(&d->extent, &cfg->extent, 4) != 0)
        return verr(err, errlen,
                    "dump grid n=%u aniso=%u aabb_min=(%.9g, %.9g, %.9g) extent=%.9g, context n=%u aniso=%u "
                    "aabb_min=(%.9g, %.9g, %.9g) extent=%.9g",
                    d->n, d->aniso, (double)d->aabb_min[0], (double)d->aabb_min[1], (double)d->aabb_min[2],
                    (double)d->extent, cfg->n, cfg->aniso ? 1u : 0u, (double)cfg->aabb_min[0],
                    (double)cfg->aabb_min[1], (double)cfg->aabb_min[2], (double)cfg->extent);
    return 0;
}
