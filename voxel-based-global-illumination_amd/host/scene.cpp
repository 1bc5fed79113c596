// scene.cpp — Wavefront OBJ/MTL loader reproducing what the reference's
// Model::loadModel gets from assimp (scene/model.cpp:21-148):
//   Assimp::Importer::ReadFile(path, aiProcess_Triangulate | aiProcess_FlipUVs |
//                                    aiProcess_CalcTangentSpace)   (model.cpp:24)
// then loadMaterials() (Ka/Kd/Ks as vec4(rgb, 1), model.cpp:38-65) and
// loadMeshes() (one 56-B Vertex per aiMesh vertex, indices face by face,
// model.cpp:67-148).
//
// The rules below are those of assimp 3.3's OBJ importer and post-process
// steps, restated from their observable behaviour and pinned against the
// library itself (tests/golden/make_obj_golden.py, tests/test_scene_loader.py):
//  * materials: "DefaultMaterial" (Kd 0.6) first, then the .mtl entries in
//    newmtl order;
//  * meshes: an object ("o" with a new name, "g" with a name different from the
//    active group, or "defaultobject" for faces before either) opens a mesh;
//    "usemtl" opens a new mesh in the current object when the current mesh
//    has faces and a different material; "o" naming an existing object only
//    re-selects the object (faces keep going to the current mesh); meshes
//    without faces are dropped; output order = objects, then their meshes; a
//    mesh no "usemtl" reached gets the last material of the list;
//  * vertices are per face corner (no sharing), FlipUVs is v' = 1 - v;
//  * Triangulate: triangles copied; quads fanned from the concave corner (or
//    corner 0); larger polygons ear-cut in the plane of their Newell normal,
//    zero-area (< 1e-5) triangles dropped;
//  * CalcTangentSpace: per-face tangent/bitangent from the first three corners,
//    projected per vertex into the normal's plane, then smoothed over vertices
//    at the same position (1e-4 x AABB diagonal) whose normals agree to 0.9999
//    and tangents/bitangents to cos 45 deg.
#include "scene.h"

#include "png.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>

namespace vcthost {

namespace {

struct V3 {
    float x = 0, y = 0, z = 0;
};
V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float length(V3 a) { return std::sqrt(dot(a, a)); }
V3 normalized(V3 a) {                      // x / |a| per component (0/0 -> NaN, as assimp)
    const float l = length(a);
    return {a.x / l, a.y / l, a.z / l};
}
bool special(V3 a) { return !std::isfinite(a.x) || !std::isfinite(a.y) || !std::isfinite(a.z); }

struct Corner {
    int v = -1, t = -1, n = -1;
};

struct ObjMesh {
    std::vector<std::vector<Corner>> faces;
    int material = -1;                     // -1 = no material assigned (-> DefaultMaterial)
};

struct ObjObject {
    std::string name;
    std::vector<int> meshes;
};

// assimp's fast_atoreal_move<float> (fast_atof.h), which the OBJ and MTL
// parsers use for every number: integer part as uint64 -> float, up to 15
// fraction digits as uint64 * 10^-k in double, rounded to float and ADDED in
// float (two roundings: "1.20905" reads as 1.2090499, not 1.20905), then an
// optional exponent applied with powf.
float ai_atof(const std::string& tok) {
    const char* c = tok.c_str();
    const bool inv = *c == '-';
    if (inv || *c == '+') ++c;
    auto digits = [](const char*& p, unsigned max, unsigned* count) {
        uint64_t v = 0;
        unsigned n = 0;
        while (*p >= '0' && *p <= '9') {
            if (n < max) { v = v * 10 + (uint64_t)(*p - '0'); ++n; }
            ++p;
        }
        if (count) *count = n;
        return v;
    };
    float f = 0;
    if (*c != '.') f = (float)digits(c, 64, nullptr);
    if (*c == '.' && c[1] >= '0' && c[1] <= '9') {
        ++c;
        static const double table[16] = {0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001,
                                         0.00000001, 0.000000001, 0.0000000001, 0.00000000001,
                                         0.000000000001, 0.0000000000001, 0.00000000000001, 0.000000000000001};
        unsigned k = 0;
        double pl = (double)digits(c, 15, &k);
        pl *= table[k];
        f += (float)pl;
    } else if (*c == '.') {
        ++c;
    }
    if (*c == 'e' || *c == 'E') {
        ++c;
        const bool einv = *c == '-';
        if (einv || *c == '+') ++c;
        float e = (float)digits(c, 64, nullptr);
        if (einv) e = -e;
        f *= std::pow(10.0f, e);
    }
    return inv ? -f : f;
}

// up to n numbers from the rest of a line
void read_floats(std::istringstream& ss, float* out, int n) {
    std::string tok;
    for (int i = 0; i < n && (ss >> tok); ++i) out[i] = ai_atof(tok);
}

std::string dir_of(const std::string& p) {
    size_t s = p.find_last_of("/\\");
    return s == std::string::npos ? std::string() : p.substr(0, s + 1);
}

std::string rest_of_line(std::istringstream& ss) {
    std::string r;
    std::getline(ss, r);
    const size_t a = r.find_first_not_of(" \t\r"), b = r.find_last_not_of(" \t\r");
    return a == std::string::npos ? std::string() : r.substr(a, b - a + 1);
}

std::string texture_name(const std::string& rest);

void load_mtl(const std::string& path, std::vector<Material>& mats) {
    std::ifstream f(path);
    if (!f) return;                        // assimp logs and continues without the library
    std::string line;
    Material* cur = nullptr;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag;
        if (tag == "newmtl") {
            Material m;
            m.name = rest_of_line(ss);
            m.Kd = {0.6f, 0.6f, 0.6f, 1.0f};   // assimp ObjFile::Material defaults
            mats.push_back(m);
            cur = &mats.back();
        } else if (cur && (tag == "Kd" || tag == "Ka" || tag == "Ks")) {
            std::array<float, 4>& k = tag == "Kd" ? cur->Kd : (tag == "Ka" ? cur->Ka : cur->Ks);
            read_floats(ss, k.data(), 3);
        } else if (cur && tag == "map_Kd") {
            // the diffuse map (one per material: a later map_Kd replaces it); leading
            // texture options (-clamp on, -o u v w, ...) are skipped, the rest of the line
            // is the file name
            cur->diffuse_map = texture_name(rest_of_line(ss));
        }
    }
}

// the file name of a map_* statement, as assimp 3.3's MTL reader takes it: while the
// next token starts with '-', an option is skipped with a fixed token count (matched
// as a case-insensitive prefix, in this order): -clamp 2; -blendu -blendv -boost
// -texres -bm -imfchan -type 2; -mm 3; -o -s -t 4 (option + 3 values); any other 1.
// The rest of the line (spaces kept) is the name.  Pinned by tests/golden/obj_maps.npz.
std::string texture_name(const std::string& rest) {
    static const std::pair<const char*, int> opts[] = {
        {"-clamp", 2}, {"-blendu", 2}, {"-blendv", 2}, {"-boost", 2}, {"-texres", 2}, {"-bm", 2},
        {"-imfchan", 2}, {"-type", 2}, {"-mm", 3}, {"-o", 4}, {"-s", 4}, {"-t", 4}};
    auto skip_ws = [&](size_t p) {
        while (p < rest.size() && std::isspace((unsigned char)rest[p])) ++p;
        return p;
    };
    auto prefix = [&](size_t p, const char* o) {
        for (size_t i = 0; o[i]; ++i)
            if (p + i >= rest.size() || std::tolower((unsigned char)rest[p + i]) != o[i]) return false;
        return true;
    };
    size_t p = skip_ws(0);
    while (p < rest.size() && rest[p] == '-') {
        int skip = 1;
        for (const auto& o : opts)
            if (prefix(p, o.first)) { skip = o.second; break; }
        for (int i = 0; i < skip; ++i) {   // past this token and the whitespace after it
            while (p < rest.size() && !std::isspace((unsigned char)rest[p])) ++p;
            p = skip_ws(p);
        }
    }
    const size_t e = rest.find_last_not_of(" \t\r");
    return p >= rest.size() || e == std::string::npos || e < p ? std::string() : rest.substr(p, e - p + 1);
}

// "v", "v/vt", "v//vn", "v/vt/vn"; 1-based or negative (relative) indices
Corner parse_corner(const std::string& tok, int nv, int nt, int nn) {
    int vals[3] = {0, 0, 0};
    bool have[3] = {false, false, false};
    size_t start = 0;
    for (int k = 0; k < 3 && start <= tok.size(); ++k) {
        size_t slash = tok.find('/', start);
        std::string part = tok.substr(start, slash == std::string::npos ? std::string::npos : slash - start);
        if (!part.empty()) { vals[k] = std::atoi(part.c_str()); have[k] = true; }
        if (slash == std::string::npos) break;
        start = slash + 1;
    }
    auto fix = [](int v, int n) { return v > 0 ? v - 1 : n + v; };
    Corner c;
    if (have[0]) c.v = fix(vals[0], nv);
    if (have[1]) c.t = fix(vals[1], nt);
    if (have[2]) c.n = fix(vals[2], nn);
    return c;
}

// --- aiProcess_Triangulate ---------------------------------------------------
double area2d(const float* a, const float* b, const float* c) {   // GetArea2D(v1, v2, v3), in double
    return 0.5 * (a[0] * ((double)c[1] - b[1]) + b[0] * ((double)a[1] - c[1]) + c[0] * ((double)b[1] - a[1]));
}
// OnLeftSideOfLine2D(p0, p1, p2): p2 left of the line p0 -> p1
bool on_left(const float* p0, const float* p1, const float* p2) { return area2d(p0, p2, p1) > 0; }
bool in_triangle(const float* p0, const float* p1, const float* p2, const float* pp) {
    const float v0[2] = {p1[0] - p0[0], p1[1] - p0[1]}, v1[2] = {p2[0] - p0[0], p2[1] - p0[1]};
    const float v2[2] = {pp[0] - p0[0], pp[1] - p0[1]};
    double d00 = v0[0] * v0[0] + v0[1] * v0[1], d01 = v0[0] * v1[0] + v0[1] * v1[1];
    const double d02 = v0[0] * v2[0] + v0[1] * v2[1];
    double d11 = v1[0] * v1[0] + v1[1] * v1[1];
    const double d12 = v1[0] * v2[0] + v1[1] * v2[1];
    const double inv = 1 / (d00 * d11 - d01 * d01);
    d11 = (d11 * d02 - d01 * d12) * inv;
    d00 = (d00 * d12 - d01 * d02) * inv;
    return d11 > 0 && d00 > 0 && d11 + d00 < 1;
}

// one face (local corner indices 0..n-1 of the mesh vertices in `idx`) -> triangles
void triangulate(const std::vector<V3>& P, const std::vector<unsigned>& idx, std::vector<unsigned>& out) {
    const int n = (int)idx.size();
    if (n <= 3) {
        if (n == 3) out.insert(out.end(), idx.begin(), idx.end());
        return;
    }
    if (n == 4) {   // at most one concave corner: fan from it
        int start = 0;
        for (int i = 0; i < 4; ++i) {
            const V3 v = P[idx[i]];
            V3 left = P[idx[(i + 3) % 4]] - v, diag = P[idx[(i + 2) % 4]] - v, right = P[idx[(i + 1) % 4]] - v;
            left = normalized(left); diag = normalized(diag); right = normalized(right);
            const float angle = std::acos(dot(left, diag)) + std::acos(dot(right, diag));
            if (angle > 3.1415926538f) { start = i; break; }
        }
        const unsigned t[4] = {idx[0], idx[1], idx[2], idx[3]};
        const unsigned tri[6] = {t[start], t[(start + 1) % 4], t[(start + 2) % 4],
                                 t[start], t[(start + 2) % 4], t[(start + 3) % 4]};
        out.insert(out.end(), tri, tri + 6);
        return;
    }
    // Newell normal -> projection plane
    float sxy = 0, syz = 0, szx = 0;
    for (int k = 0; k < n; ++k) {
        const V3 c = P[idx[(k + 1) % n]], lo = P[idx[k]], hi = P[idx[(k + 2) % n]];
        sxy += c.x * (hi.y - lo.y);
        syz += c.y * (hi.z - lo.z);
        szx += c.z * (hi.x - lo.x);
    }
    const V3 nrm{syz, szx, sxy};
    const float ax = std::fabs(nrm.x), ay = std::fabs(nrm.y), az = std::fabs(nrm.z);
    int ac = 0, bc = 1;
    float inv = nrm.z;
    if (ax > ay) {
        if (ax > az) { ac = 1; bc = 2; inv = nrm.x; }
    } else if (ay > az) {
        ac = 2; bc = 0; inv = nrm.y;
    }
    if (inv < 0.f) std::swap(ac, bc);
    std::vector<std::array<float, 2>> q(n);
    std::vector<char> done(n, 0);
    for (int k = 0; k < n; ++k) {
        const float c[3] = {P[idx[k]].x, P[idx[k]].y, P[idx[k]].z};
        q[k] = {c[ac], c[bc]};
    }
    std::vector<std::array<int, 3>> tris;
    int num = n, ear = 0, prev = n - 1, next = 0;
    bool fail = false;
    while (num > 3) {
        int num_found = 0;
        for (ear = next;; prev = ear, ear = next) {
            for (next = ear + 1; done[(next >= n ? next = 0 : next)]; ++next) {}
            if (next < ear && ++num_found == 2) break;
            const float *p1 = q[ear].data(), *p0 = q[prev].data(), *p2 = q[next].data();
            if (on_left(p0, p2, p1)) continue;
            int tmp = 0;
            for (; tmp < n; ++tmp) {
                const float* v = q[tmp].data();
                auto same = [](const float* a, const float* b) { return a[0] == b[0] && a[1] == b[1]; };
                if (!same(v, p1) && !same(v, p2) && !same(v, p0) && in_triangle(p0, p1, p2, v)) break;
            }
            if (tmp != n) continue;
            break;
        }
        if (num_found == 2) { fail = true; break; }   // not a simple polygon: assimp drops the rest
        tris.push_back({prev, ear, next});
        done[ear] = 1;
        --num;
    }
    if (!fail && num > 0) {
        int tmp = 0;
        std::array<int, 3> t{};
        for (int k = 0; k < 3; ++k) {
            while (done[tmp]) ++tmp;
            t[k] = tmp++;
        }
        tris.push_back(t);
    }
    for (const auto& t : tris) {
        if (std::fabs(area2d(q[t[0]].data(), q[t[1]].data(), q[t[2]].data())) < 1e-5f) continue;   // 0-area
        out.push_back(idx[t[0]]);
        out.push_back(idx[t[1]]);
        out.push_back(idx[t[2]]);
    }
}

// --- aiProcess_CalcTangentSpace ------------------------------------------------
void calc_tangents(std::vector<Vertex>& vx, const std::vector<unsigned>& tri) {
    const size_t nv = vx.size();
    auto P = [&](size_t i) { return V3{vx[i].Position[0], vx[i].Position[1], vx[i].Position[2]}; };
    auto N = [&](size_t i) { return V3{vx[i].Normal[0], vx[i].Normal[1], vx[i].Normal[2]}; };
    std::vector<V3> T(nv), B(nv);
    std::vector<char> done(nv, 0);
    for (size_t f = 0; f + 2 < tri.size(); f += 3) {
        const unsigned p0 = tri[f], p1 = tri[f + 1], p2 = tri[f + 2];
        const V3 v = P(p1) - P(p0), w = P(p2) - P(p0);
        float sx = vx[p1].TexCoords[0] - vx[p0].TexCoords[0], sy = vx[p1].TexCoords[1] - vx[p0].TexCoords[1];
        float tx = vx[p2].TexCoords[0] - vx[p0].TexCoords[0], ty = vx[p2].TexCoords[1] - vx[p0].TexCoords[1];
        const float dir = (tx * sy - ty * sx) < 0.0f ? -1.0f : 1.0f;
        if (sx == 0 && sy == 0 && tx == 0 && ty == 0) { sx = 0.0f; sy = 1.0f; tx = 1.0f; ty = 0.0f; }
        const V3 tan{(w.x * sy - v.x * ty) * dir, (w.y * sy - v.y * ty) * dir, (w.z * sy - v.z * ty) * dir};
        const V3 bit{(w.x * sx - v.x * tx) * dir, (w.y * sx - v.y * tx) * dir, (w.z * sx - v.z * tx) * dir};
        for (int b = 0; b < 3; ++b) {
            const unsigned p = tri[f + b];
            const V3 n = N(p);
            V3 lt = normalized(tan - n * dot(tan, n)), lb = normalized(bit - n * dot(bit, n));
            const bool it = special(lt), ib = special(lb);
            if (it != ib) {
                if (it) lt = normalized(cross(n, lb));
                else lb = normalized(cross(lt, n));
            }
            T[p] = lt;
            B[p] = lb;
        }
    }
    // smoothing over vertices at one position (SpatialSort along a fixed plane normal)
    V3 lo = P(0), hi = P(0);
    for (size_t i = 1; i < nv; ++i) {
        const V3 p = P(i);
        lo = {std::min(lo.x, p.x), std::min(lo.y, p.y), std::min(lo.z, p.z)};
        hi = {std::max(hi.x, p.x), std::max(hi.y, p.y), std::max(hi.z, p.z)};
    }
    const float eps = length(hi - lo) * 1e-4f;
    const V3 pn = normalized(V3{0.8523f, 0.34321f, 0.5736f});
    std::vector<std::pair<float, unsigned>> sorted(nv);
    for (size_t i = 0; i < nv; ++i) sorted[i] = {dot(P(i), pn), (unsigned)i};
    std::sort(sorted.begin(), sorted.end(),
              [](const std::pair<float, unsigned>& a, const std::pair<float, unsigned>& b) { return a.first < b.first; });
    const float limit = std::cos(0.785398163f);   // configMaxAngle 45 deg
    std::vector<unsigned> close;
    for (size_t a = 0; a < nv; ++a) {
        if (done[a]) continue;
        const V3 op = P(a), on = N(a), ot = T[a], ob = B[a];
        close.assign(1, (unsigned)a);
        const float d = dot(op, pn);
        auto it = std::lower_bound(sorted.begin(), sorted.end(), d - eps,
                                   [](const std::pair<float, unsigned>& e, float v) { return e.first < v; });
        for (; it != sorted.end() && it->first < d + eps; ++it) {
            const unsigned i = it->second;
            const V3 dp = P(i) - op;
            if (!(dot(dp, dp) < eps * eps) || done[i]) continue;
            if (dot(N(i), on) < 0.9999f || dot(T[i], ot) < limit || dot(B[i], ob) < limit) continue;
            close.push_back(i);
            done[i] = 1;
        }
        V3 st, sb;
        for (unsigned i : close) { st = st + T[i]; sb = sb + B[i]; }
        st = normalized(st);
        sb = normalized(sb);
        for (unsigned i : close) { T[i] = st; B[i] = sb; }
    }
    for (size_t i = 0; i < nv; ++i) {
        vx[i].Tangent[0] = T[i].x; vx[i].Tangent[1] = T[i].y; vx[i].Tangent[2] = T[i].z;
        vx[i].Bitangent[0] = B[i].x; vx[i].Bitangent[1] = B[i].y; vx[i].Bitangent[2] = B[i].z;
    }
}

}  // namespace

bool Model::LoadObj(const std::string& path, std::string* err, bool load_textures) {
    std::ifstream f(path);
    if (!f) {
        if (err) *err = "cannot open " + path;   // model.cpp:25-29 prints and returns
        return false;
    }
    {   // model.cpp:30: directory = path.substr(0, path.find_last_of('/'))
        const size_t s = path.find_last_of('/');
        directory = s == std::string::npos ? std::string(".") : path.substr(0, s);
    }
    textures.clear();
    texture_errors.clear();
    std::vector<V3> P, N;
    std::vector<std::array<float, 2>> T;
    materials.clear();
    meshes.clear();
    Material def;
    def.name = "DefaultMaterial";
    def.Kd = {0.6f, 0.6f, 0.6f, 1.0f};
    materials.push_back(def);
    auto mat_index = [&](const std::string& name) {
        for (size_t i = 0; i < materials.size(); ++i)
            if (materials[i].name == name) return (int)i;
        return -1;
    };
    std::vector<ObjObject> objects;
    std::vector<ObjMesh> omesh;
    int cur_obj = -1, cur_mesh = -1, cur_mat = -1;   // cur_mat: material the parser has selected
    std::string active_group;
    bool have_group = false;
    auto create_mesh = [&]() {
        omesh.push_back(ObjMesh{});
        cur_mesh = (int)omesh.size() - 1;
        if (cur_obj >= 0) objects[cur_obj].meshes.push_back(cur_mesh);
    };
    auto create_object = [&](const std::string& name) {
        objects.push_back(ObjObject{name, {}});
        cur_obj = (int)objects.size() - 1;
        create_mesh();
        if (cur_mat >= 0) omesh[cur_mesh].material = cur_mat;
    };
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag;
        if (tag == "v" || tag == "vn") {
            float x[3] = {0, 0, 0};
            read_floats(ss, x, 3);
            (tag == "v" ? P : N).push_back(V3{x[0], x[1], x[2]});
        } else if (tag == "vt") {
            std::array<float, 2> t{};
            read_floats(ss, t.data(), 2);
            T.push_back(t);
        } else if (tag == "mtllib") {
            load_mtl(dir_of(path) + rest_of_line(ss), materials);
        } else if (tag == "usemtl") {
            const std::string name = rest_of_line(ss);
            if (name.empty() || (cur_mat >= 0 && materials[cur_mat].name == name)) continue;   // ignored
            int mi = mat_index(name);
            if (mi < 0) mi = 0;                                  // unknown -> DefaultMaterial
            cur_mat = mi;
            const bool need_new = cur_mesh < 0 || (omesh[cur_mesh].material >= 0 &&
                                                   omesh[cur_mesh].material != mi && !omesh[cur_mesh].faces.empty());
            if (need_new) create_mesh();
            omesh[cur_mesh].material = mi;
        } else if (tag == "o") {
            const std::string name = rest_of_line(ss);
            if (name.empty()) continue;
            int found = -1;
            for (size_t i = 0; i < objects.size(); ++i)
                if (objects[i].name == name) { found = (int)i; break; }
            if (found >= 0) cur_obj = found;             // re-selects the object only
            else create_object(name);
        } else if (tag == "g") {
            const std::string name = rest_of_line(ss);
            if (!have_group || name != active_group) {
                create_object(name);
                active_group = name;
                have_group = true;
            }
        } else if (tag == "f") {
            if (cur_obj < 0) create_object("defaultobject");   // (the face's own material is not the parser's)
            std::vector<Corner> face;
            std::string tok;
            while (ss >> tok) {
                const Corner c = parse_corner(tok, (int)P.size(), (int)T.size(), (int)N.size());
                if (c.v < 0 || c.v >= (int)P.size()) {
                    if (err) *err = "face index out of range in " + path;
                    return false;
                }
                face.push_back(c);
            }
            if (cur_mesh < 0) create_mesh();
            omesh[cur_mesh].faces.push_back(face);
        }
    }
    for (const ObjObject& o : objects) {
        for (int mi : o.meshes) {
            const ObjMesh& om = omesh[mi];
            if (om.faces.empty()) continue;
            Mesh m;
            // a mesh no usemtl reached gets the LAST material (assimp 3.3's NoMaterial outcome)
            m.material = om.material >= 0 ? om.material : (int)materials.size() - 1;
            bool has_n = false, has_t = false;
            for (const auto& fc : om.faces)
                for (const Corner& c : fc) {
                    has_n |= c.n >= 0 && c.n < (int)N.size();
                    has_t |= c.t >= 0 && c.t < (int)T.size();
                }
            std::vector<V3> pos;
            for (const auto& fc : om.faces) {
                std::vector<unsigned> local;
                for (const Corner& c : fc) {
                    Vertex v{};
                    v.Position[0] = P[c.v].x; v.Position[1] = P[c.v].y; v.Position[2] = P[c.v].z;
                    if (c.n >= 0 && c.n < (int)N.size()) {
                        v.Normal[0] = N[c.n].x; v.Normal[1] = N[c.n].y; v.Normal[2] = N[c.n].z;
                    }
                    if (has_t) {
                        const float tv = (c.t >= 0 && c.t < (int)T.size()) ? T[c.t][1] : 0.0f;
                        v.TexCoords[0] = (c.t >= 0 && c.t < (int)T.size()) ? T[c.t][0] : 0.0f;
                        v.TexCoords[1] = 1.0f - tv;                        // aiProcess_FlipUVs
                    }
                    local.push_back((unsigned)m.vertices.size());
                    m.vertices.push_back(v);
                    pos.push_back(P[c.v]);
                }
                triangulate(pos, local, m.indices);                       // aiProcess_Triangulate
            }
            if (has_n && has_t) calc_tangents(m.vertices, m.indices);     // aiProcess_CalcTangentSpace
            meshes.push_back(std::move(m));
        }
    }
    if (load_textures) LoadTextures();
    return true;
}

void Model::LoadTextures() {
    for (Material& mt : materials) {
        mt.diffuseMaps.clear();
        if (mt.diffuse_map.empty()) continue;
        int found = -1;
        for (size_t j = 0; j < textures.size(); ++j)
            if (textures[j].path == mt.diffuse_map) { found = (int)j; break; }   // model.cpp:160-166
        if (found < 0) {
            // TextureFromFile (model.cpp:188-226): directory + '/' + path, stbi_load(.., 0)
            PngImage img;
            Texture t;
            std::string e;
            if (!LoadPng(directory + '/' + mt.diffuse_map, &img, &e) || !ExpandToRgba(img, &t.rgba, &e)) {
                texture_errors.push_back(mt.diffuse_map + ": " + e);
                continue;
            }
            t.type = "texture_diffuse";
            t.path = mt.diffuse_map;
            t.width = img.width;
            t.height = img.height;
            textures.push_back(std::move(t));
            found = (int)textures.size() - 1;
        }
        mt.diffuseMaps.push_back(found);
    }
}

std::vector<int32_t> Model::MaterialMap() const {
    std::vector<int32_t> m;
    for (const Material& mt : materials) m.push_back(mt.diffuseMaps.empty() ? -1 : mt.diffuseMaps[0]);
    return m;
}

void Model::Transform(const float m[16]) {
    for (Mesh& me : meshes)
        for (Vertex& v : me.vertices) {
            const float x = v.Position[0], y = v.Position[1], z = v.Position[2];
            v.Position[0] = m[0] * x + m[4] * y + m[8] * z + m[12];
            v.Position[1] = m[1] * x + m[5] * y + m[9] * z + m[13];
            v.Position[2] = m[2] * x + m[6] * y + m[10] * z + m[14];
        }
}

bool Model::Bounds(float lo[3], float hi[3]) const {
    bool any = false;
    for (const Mesh& me : meshes)
        for (const Vertex& v : me.vertices) {
            for (int k = 0; k < 3; ++k) {
                lo[k] = any ? std::min(lo[k], v.Position[k]) : v.Position[k];
                hi[k] = any ? std::max(hi[k], v.Position[k]) : v.Position[k];
            }
            any = true;
        }
    return any;
}

void ReferenceModelMatrix(float m[16]) {
    // glm::translate(mat4(1), t): column 3 = c0 t.x + c1 t.y + c2 t.z + c3 (matrix_transform.inl),
    // then glm::scale(., s): columns 0..2 scaled
    const float t[3] = {0.0f, -1.75f, 0.0f}, sc = 0.2f;
    float r[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    for (int row = 0; row < 4; ++row)
        r[12 + row] = ((r[row] * t[0] + r[4 + row] * t[1]) + r[8 + row] * t[2]) + r[12 + row];
    for (int c = 0; c < 3; ++c)
        for (int row = 0; row < 4; ++row) r[4 * c + row] = r[4 * c + row] * sc;
    for (int i = 0; i < 16; ++i) m[i] = r[i];
}

void GridForBounds(const float lo[3], const float hi[3], uint32_t n, float aabb_min[3], float* extent) {
    float e = 0.0f;
    for (int k = 0; k < 3; ++k) e = std::max(e, hi[k] - lo[k]);
    if (!(e > 0.0f)) e = 1.0f;
    const float E = e * (float)n / (float)(n - 2);
    for (int k = 0; k < 3; ++k) aabb_min[k] = 0.5f * (lo[k] + hi[k]) - 0.5f * E;
    *extent = E;
}

void Model::Flatten(std::vector<Vertex>& v, std::vector<unsigned>& idx, std::vector<unsigned>& tri_mat,
                    std::vector<float>& kd4) const {
    v.clear(); idx.clear(); tri_mat.clear(); kd4.clear();
    for (const Mesh& me : meshes) {
        const unsigned base = (unsigned)v.size();
        v.insert(v.end(), me.vertices.begin(), me.vertices.end());
        for (unsigned i : me.indices) idx.push_back(base + i);
        for (size_t t = 0; t < me.indices.size() / 3; ++t) tri_mat.push_back((unsigned)me.material);
    }
    for (const Material& m : materials) kd4.insert(kd4.end(), m.Kd.begin(), m.Kd.end());
}

}  // namespace vcthost
