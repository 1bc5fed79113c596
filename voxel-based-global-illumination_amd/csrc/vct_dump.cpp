// vct_dump.cpp — vct_save_grid / vct_load_grid / vct_dump_info (include/vct.h) on the HIP
// library: the "vct-dump/2" files of vct_dumpio.h (shared with the CPU backend).
//
// SURVEY.md section 5 "checkpoint / resume" (the reference persists no state).  K1's state
// is dumped as the occupied voxels' integer sums and counts -- the exact accumulator
// values -- so a loaded context resolves the same voxels (k1_resolve is deterministic),
// injects any light and composites as the original one did: it is relightable without
// its triangles.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "vct_dumpio.h"
#include "vct_internal.h"

using namespace vct;

namespace {

vct_status dfail(vct_ctx* c, vct_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

vct_status dhip(vct_ctx* c, hipError_t e, const char* where) {
    return dfail(c, e == hipErrorOutOfMemory ? VCT_ENOMEM : VCT_EDEVICE,
                 std::string(where) + ": " + hipGetErrorName(e));
}

#define VCT_DHIP(call, where)                             \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return dhip(c, e_, where);  \
    } while (0)

struct DevMem {   // per-call device staging
    void* p = nullptr;
    ~DevMem() { if (p) (void)hipFree(p); }
};

struct Closer {
    vdump_file* f;
    ~Closer() { vdump_close(f); }
};

}  // namespace

extern "C" {

vct_status vct_dump_info(const char* stem, vct_config* cfg, uint32_t* what) {
    if (!stem) return VCT_EINVAL;
    vdump_header h;
    char err[512];
    if (vdump_read_header(stem, &h, err, sizeof err)) return VCT_EINVAL;
    if (cfg) *cfg = h.cfg;
    if (what) *what = h.what;
    return VCT_OK;
}

vct_status vct_save_grid(vct_ctx* c, const char* stem, uint32_t what) {
    if (!c || !stem) return VCT_EINVAL;
    if (!what || (what & ~(VCT_DUMP_VOXELS | VCT_DUMP_LEVEL0 | VCT_DUMP_PYRAMID)))
        return dfail(c, VCT_EINVAL, "save_grid: `what` must be a nonzero set of VCT_DUMP_* bits");
    if ((what & VCT_DUMP_PYRAMID) && !(what & VCT_DUMP_LEVEL0))
        return dfail(c, VCT_EINVAL, "save_grid: VCT_DUMP_PYRAMID needs VCT_DUMP_LEVEL0 (the pyramid is checked against "
                                    "the one rebuilt from level 0)");
    const Grid& g = c->grid;
    if ((what & VCT_DUMP_VOXELS) && !g.voxelized) return dfail(c, VCT_ESTATE, "save_grid: no voxelization to dump");
    if ((what & VCT_DUMP_LEVEL0) && !g.injected) return dfail(c, VCT_ESTATE, "save_grid: no level 0 (inject first)");
    if ((what & VCT_DUMP_PYRAMID) && !g.mipped) return dfail(c, VCT_ESTATE, "save_grid: no pyramid (build_mips first)");
    VCT_DHIP(hipSetDevice(c->device), "hipSetDevice");
    const size_t nv = (size_t)g.n * g.n * g.n;
    std::vector<uint32_t> idx;
    std::vector<long long> rec;                 // [occ][7]
    if (what & VCT_DUMP_VOXELS) {
        // the occupied voxels in ascending index order, from the occupancy bits
        std::vector<unsigned long long> bits(nv / 64);
        VCT_DHIP(hipMemcpyAsync(bits.data(), g.occ_bits, bits.size() * 8, hipMemcpyDeviceToHost, c->stream),
                 "download occupancy bits");
        VCT_DHIP(hipStreamSynchronize(c->stream), "sync");
        for (size_t w = 0; w < bits.size(); ++w)
            for (unsigned long long m = bits[w]; m; m &= m - 1) idx.push_back((uint32_t)(w * 64 + __builtin_ctzll(m)));
        rec.resize(idx.size() * 7);
        if (!idx.empty()) {
            DevMem di, dr;
            VCT_DHIP(hipMalloc(&di.p, idx.size() * 4), "hipMalloc");
            VCT_DHIP(hipMalloc(&dr.p, rec.size() * 8), "hipMalloc");
            VCT_DHIP(hipMemcpyAsync(di.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, c->stream), "upload");
            VCT_DHIP(launch_k1_gather(c, (const uint32_t*)di.p, (uint32_t)idx.size(), (long long*)dr.p), "K1 gather");
            VCT_DHIP(hipMemcpyAsync(rec.data(), dr.p, rec.size() * 8, hipMemcpyDeviceToHost, c->stream), "download");
            VCT_DHIP(hipStreamSynchronize(c->stream), "sync");
        }
    }
    vdump_header h{};
    h.cfg = c->cfg;
    h.cfg.device = -1;
    h.what = what;
    h.occupied = idx.size();
    vdump_file w;
    char err[512];
    if (vdump_open_write(&w, stem, &h, err, sizeof err)) return dfail(c, VCT_EINVAL, std::string("save_grid: ") + err);
    Closer cl{&w};
    if (what & VCT_DUMP_VOXELS) {
        std::vector<long long> sums(idx.size() * 6);
        std::vector<uint32_t> counts(idx.size());
        for (size_t i = 0; i < idx.size(); ++i) {
            for (int j = 0; j < 6; ++j) sums[6 * i + j] = rec[7 * i + j];
            counts[i] = (uint32_t)rec[7 * i + 6];
        }
        if (vdump_write(&w, idx.data(), idx.size() * 4, err, sizeof err) ||
            vdump_write(&w, sums.data(), sums.size() * 8, err, sizeof err) ||
            vdump_write(&w, counts.data(), counts.size() * 4, err, sizeof err))
            return dfail(c, VCT_EINVAL, std::string("save_grid: ") + err);
    }
    if (what & VCT_DUMP_LEVEL0) {
        std::vector<float> buf(nv * 4);
        for (uint32_t l = 0; l <= ((what & VCT_DUMP_PYRAMID) ? g.L : 0u); ++l) {
            const size_t nl = g.n >> l, vl = nl * nl * nl;
            const uint32_t faces = (l == 0 || !g.aniso) ? 1u : (uint32_t)VCT_NUM_FACES;
            for (uint32_t f = 0; f < faces; ++f) {
                vct_status st = vct_download_level(c, l, f, buf.data());
                if (st != VCT_OK) return st;
                if (vdump_write(&w, buf.data(), vl * 16, err, sizeof err))
                    return dfail(c, VCT_EINVAL, std::string("save_grid: ") + err);
            }
        }
    }
    if (vdump_close_write(&w, err, sizeof err)) return dfail(c, VCT_EINVAL, std::string("save_grid: ") + err);
    return VCT_OK;
}

// A load that fails after it began to replace the grid leaves no half-loaded state behind:
// the grid reads as never voxelized (every trace, inject and mips call refuses it with
// VCT_ESTATE until the next voxelization or load).
struct InvalidateOnFail {
    vct_ctx* c;
    bool armed = false;
    ~InvalidateOnFail() {
        if (!armed) return;
        Grid& g = c->grid;
        g.voxelized = g.injected = g.mipped = false;
        g.k2_coarse_ok = g.k3_sparse_ok = g.zm_valid = false;
        ++c->grid_epoch;
    }
};

vct_status vct_load_grid(vct_ctx* c, const char* stem) {
    if (!c || !stem) return VCT_EINVAL;
    InvalidateOnFail guard{c};
    vdump_file r;
    char err[1024];
    if (vdump_open_read(&r, stem, err, sizeof err)) return dfail(c, VCT_EINVAL, std::string("load_grid: ") + err);
    Closer cl{&r};
    const vdump_header& h = r.h;
    if (vdump_check_config(&h, &c->cfg, err, sizeof err)) return dfail(c, VCT_EINVAL, std::string("load_grid: ") + err);
    if ((h.what & VCT_DUMP_PYRAMID) && !(h.what & VCT_DUMP_LEVEL0))
        return dfail(c, VCT_EINVAL, "load_grid: a pyramid section without level 0");
    Grid& g = c->grid;
    const size_t nv = (size_t)g.n * g.n * g.n;
    VCT_DHIP(hipSetDevice(c->device), "hipSetDevice");
    if (h.what & VCT_DUMP_VOXELS) {
        const size_t occ = (size_t)h.occupied;
        std::vector<uint32_t> idx(occ), counts(occ);
        std::vector<long long> sums(occ * 6);
        if (vdump_read(&r, idx.data(), occ * 4, err, sizeof err) || vdump_read(&r, sums.data(), occ * 48, err, sizeof err) ||
            vdump_read(&r, counts.data(), occ * 4, err, sizeof err))
            return dfail(c, VCT_EINVAL, std::string("load_grid: ") + err);
        // a section the writer could not have produced is refused before the grid changes
        for (size_t i = 0; i < occ; ++i)
            if (idx[i] >= nv || (i && idx[i] <= idx[i - 1]) || counts[i] == 0)
                return dfail(c, VCT_EINVAL, "load_grid: voxel section is not ascending in-range occupied voxels");
        std::vector<long long> rec(occ * 7);
        for (size_t i = 0; i < occ; ++i) {
            for (int j = 0; j < 6; ++j) rec[7 * i + j] = sums[6 * i + j];
            rec[7 * i + 6] = counts[i];
        }
        DevMem di, dr;
        if (occ) {
            VCT_DHIP(hipMalloc(&di.p, occ * 4), "hipMalloc");
            VCT_DHIP(hipMalloc(&dr.p, occ * 56), "hipMalloc");
            VCT_DHIP(hipMemcpyAsync(di.p, idx.data(), occ * 4, hipMemcpyHostToDevice, c->stream), "upload");
            VCT_DHIP(hipMemcpyAsync(dr.p, rec.data(), occ * 56, hipMemcpyHostToDevice, c->stream), "upload");
        }
        // what a voxelization invalidates (voxelize_dev), then K1's state written back
        guard.armed = true;
        g.voxelized = g.injected = g.mipped = false;
        g.k2_coarse_ok = g.k3_sparse_ok = g.zm_valid = false;
        g.k3_live_bz = 0;
        ++c->grid_epoch;
        c->mesh.n_tri = 0;                       // the triangles are not part of a dump
        c->mesh.textured = false;
        VCT_DHIP(launch_k1_restore(c, (const uint32_t*)di.p, (uint32_t)occ, (const long long*)dr.p), "K1 restore");
        VCT_DHIP(launch_k3_live(c), "K3 live blocks");
        VCT_DHIP(hipStreamSynchronize(c->stream), "sync");
        g.voxelized = true;
    }
    if (h.what & VCT_DUMP_LEVEL0) {
        std::vector<float> buf(nv * 4), mine(nv * 4);
        if (vdump_read(&r, buf.data(), nv * 16, err, sizeof err)) return dfail(c, VCT_EINVAL, std::string("load_grid: ") + err);
        guard.armed = true;
        vct_status st = vct_upload_level0(c, buf.data());
        if (st == VCT_OK) st = vct_build_mips(c);
        if (st != VCT_OK) return st;
        for (uint32_t l = 1; (h.what & VCT_DUMP_PYRAMID) && l <= g.L; ++l) {
            const size_t nl = g.n >> l, vl = nl * nl * nl;
            const uint32_t faces = g.aniso ? (uint32_t)VCT_NUM_FACES : 1u;
            for (uint32_t f = 0; f < faces; ++f) {
                if (vdump_read(&r, buf.data(), vl * 16, err, sizeof err))
                    return dfail(c, VCT_EINVAL, std::string("load_grid: ") + err);
                if ((st = vct_download_level(c, l, f, mine.data())) != VCT_OK) return st;
                if (std::memcmp(buf.data(), mine.data(), vl * 16) != 0)
                    return dfail(c, VCT_EINVAL, "load_grid: rebuilt level " + std::to_string(l) + " face " +
                                                    std::to_string(f) + " differs from the dump");
            }
        }
    }
    guard.armed = false;
    return VCT_OK;
}

}  // extern "C"
