// scene.cpp — minimal OBJ/MTL reader + flattening into the vct_voxelize arrays.
#include "scene.h"

#include <cmath>
#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>

namespace vcthost {

namespace {

std::string dir_of(const std::string& p) {
    size_t s = p.find_last_of("/\\");
    return s == std::string::npos ? std::string() : p.substr(0, s + 1);
}

void load_mtl(const std::string& path, std::vector<Material>& mats, std::map<std::string, int>& by_name) {
    std::ifstream f(path);
    if (!f) return;
    std::string line;
    Material* cur = nullptr;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag;
        if (tag == "newmtl") {
            Material m;
            ss >> m.name;
            mats.push_back(m);
            by_name[mats.back().name] = (int)mats.size() - 1;
            cur = &mats.back();
        } else if (cur && (tag == "Kd" || tag == "Ka" || tag == "Ks")) {
            std::array<float, 4>& k = tag == "Kd" ? cur->Kd : (tag == "Ka" ? cur->Ka : cur->Ks);
            ss >> k[0] >> k[1] >> k[2];
        }
    }
}

// "v", "v/vt", "v//vn", "v/vt/vn" with 1-based or negative indices
void parse_corner(const std::string& tok, int nv, int nt, int nn, int& vi, int& ti, int& ni) {
    vi = ti = ni = -1;
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
    if (have[0]) vi = fix(vals[0], nv);
    if (have[1]) ti = fix(vals[1], nt);
    if (have[2]) ni = fix(vals[2], nn);
}

}  // namespace

bool Model::LoadObj(const std::string& path, std::string* err) {
    std::ifstream f(path);
    if (!f) {
        if (err) *err = "cannot open " + path;   // model.cpp:25-29 prints and returns
        return false;
    }
    std::vector<std::array<float, 3>> P, N;
    std::vector<std::array<float, 2>> T;
    std::map<std::string, int> by_name;
    materials.clear();
    meshes.clear();
    materials.push_back(Material{"default"});
    int cur_mat = 0;
    Mesh* mesh = nullptr;
    auto open_mesh = [&](int mat) {
        meshes.push_back(Mesh{});
        meshes.back().material = mat;
        mesh = &meshes.back();
    };
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag;
        if (tag == "v") {
            std::array<float, 3> p{};
            ss >> p[0] >> p[1] >> p[2];
            P.push_back(p);
        } else if (tag == "vn") {
            std::array<float, 3> n{};
            ss >> n[0] >> n[1] >> n[2];
            N.push_back(n);
        } else if (tag == "vt") {
            std::array<float, 2> t{};
            ss >> t[0] >> t[1];
            T.push_back(t);
        } else if (tag == "mtllib") {
            std::string name;
            ss >> name;
            load_mtl(dir_of(path) + name, materials, by_name);
        } else if (tag == "usemtl") {
            std::string name;
            ss >> name;
            auto it = by_name.find(name);
            cur_mat = it == by_name.end() ? 0 : it->second;
            open_mesh(cur_mat);
        } else if (tag == "f") {
            if (!mesh) open_mesh(cur_mat);
            std::vector<unsigned> poly;
            std::string tok;
            while (ss >> tok) {
                int vi, ti, ni;
                parse_corner(tok, (int)P.size(), (int)T.size(), (int)N.size(), vi, ti, ni);
                if (vi < 0 || vi >= (int)P.size()) {
                    if (err) *err = "face index out of range in " + path;
                    return false;
                }
                Vertex v{};
                for (int k = 0; k < 3; ++k) v.Position[k] = P[vi][k];
                if (ni >= 0 && ni < (int)N.size())
                    for (int k = 0; k < 3; ++k) v.Normal[k] = N[ni][k];
                if (ti >= 0 && ti < (int)T.size()) {
                    v.TexCoords[0] = T[ti][0];
                    v.TexCoords[1] = 1.0f - T[ti][1];   // aiProcess_FlipUVs (model.cpp:24)
                }
                poly.push_back((unsigned)mesh->vertices.size());
                mesh->vertices.push_back(v);
            }
            for (size_t k = 1; k + 1 < poly.size(); ++k) {   // aiProcess_Triangulate (fan)
                mesh->indices.push_back(poly[0]);
                mesh->indices.push_back(poly[k]);
                mesh->indices.push_back(poly[k + 1]);
            }
        }
    }
    return true;
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
