// vct_capi.cpp — the extern "C" boundary of include/vct.h.
//
// Stands where the reference's `Renderer::Render()` virtual
// (assets/code/renderer/renderer.h:3-10) would call GL.  Every entry point
// validates its arguments, selects the context's device, launches on the
// context stream and turns HIP errors into vct_status + vct_last_error() text.
// No exception crosses the ABI.  There is no CPU fallback: without a HIP device
// vct_create fails with VCT_EDEVICE.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <new>
#include <string>
#include "vct_internal.h"

using namespace vct;

namespace {

vct_status fail(vct_ctx* c, vct_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

vct_status hip_fail(vct_ctx* c, hipError_t e, const char* where) {
    std::string m = std::string(where) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    return fail(c, e == hipErrorOutOfMemory ? VCT_ENOMEM : VCT_EDEVICE, m);
}

#define VCT_HIP(call, where)                            \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return hip_fail(c, e_, where); \
    } while (0)

bool is_pow2(uint32_t n) { return n && !(n & (n - 1)); }

uint32_t ilog2u(uint32_t n) {
    uint32_t l = 0;
    while ((1u << (l + 1)) <= n) ++l;
    return l;
}

vct_status use_device(vct_ctx* c) {
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return hip_fail(c, e, "hipSetDevice");
    return VCT_OK;
}

struct DeviceBuf {  // RAII for per-call uploads
    void* p = nullptr;
    ~DeviceBuf() { if (p) (void)hipFree(p); }
};

}  // namespace

namespace vct {
hipError_t scratch_get(vct_ctx* c, int i, size_t bytes, void** out) {
    Scratch& s = c->scratch[i];
    if (s.bytes < bytes) {
        if (s.p) {
            hipError_t e = hipStreamSynchronize(c->stream);
            if (e != hipSuccess) return e;
            (void)hipFree(s.p);
            s.p = nullptr;
            s.bytes = 0;
        }
        hipError_t e = hipMalloc(&s.p, bytes);
        if (e != hipSuccess) return e;
        s.bytes = bytes;
    }
    *out = s.p;
    return hipSuccess;
}

hipError_t k4_scratch(vct_ctx* c, int i, size_t bytes, void** out, bool* fresh) {
    StreamScratch* set = nullptr;
    for (StreamScratch& e : c->k4s)
        if (e.used && e.s == c->stream) set = &e;
    if (!set)
        for (StreamScratch& e : c->k4s)
            if (!e.used) { set = &e; break; }
    if (!set) {   // a fifth stream: release every set (the device finishes what used them)
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) return e;
        for (StreamScratch& ss : c->k4s) {
            for (Scratch& sc : ss.sc)
                if (sc.p) (void)hipFree(sc.p);
            ss = StreamScratch{};
        }
        set = &c->k4s[0];
    }
    set->used = true;
    set->s = c->stream;
    Scratch& sc = set->sc[i];
    if (fresh) *fresh = false;
    if (sc.bytes < bytes) {
        if (sc.p) {
            hipError_t e = hipStreamSynchronize(c->stream);   // only this stream used the set
            if (e != hipSuccess) return e;
            (void)hipFree(sc.p);
            sc.p = nullptr;
            sc.bytes = 0;
        }
        hipError_t e = hipMalloc(&sc.p, bytes);
        if (e != hipSuccess) return e;
        sc.bytes = bytes;
        if (fresh) *fresh = true;
    }
    *out = sc.p;
    return hipSuccess;
}
hipError_t xchg_enter(vct_ctx* c) {
    if (c->xchg_done && c->xchg_stream != c->stream) return hipStreamWaitEvent(c->stream, c->xchg_done, 0);
    return hipSuccess;
}

hipError_t xchg_leave(vct_ctx* c) {
    if (!c->xchg_done) {
        hipError_t e = hipEventCreateWithFlags(&c->xchg_done, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    c->xchg_stream = c->stream;
    return hipEventRecord(c->xchg_done, c->stream);
}

void xchg_fail(vct_ctx* c) {
    // the end event of an exchange that failed part way must still cover what it queued:
    // on the ctx stream and, for a multi-device context, on every peer stream (a fresh
    // event per peer; if even that fails, the peer stream is drained)
    for (vct_ctx* p : c->peers) {
        if (hipSetDevice(p->device) != hipSuccess || hipEventRecord(p->ev, p->stream) != hipSuccess ||
            hipSetDevice(c->device) != hipSuccess || hipStreamWaitEvent(c->stream, p->ev, 0) != hipSuccess) {
            (void)hipSetDevice(p->device);
            (void)hipStreamSynchronize(p->stream);
        }
    }
    (void)hipSetDevice(c->device);
    (void)xchg_leave(c);
}
}  // namespace vct

extern "C" {

uint32_t vct_abi_version(void) { return VCT_ABI_VERSION; }

const char* vct_status_string(vct_status s) {
    switch (s) {
        case VCT_OK: return "VCT_OK";
        case VCT_EINVAL: return "VCT_EINVAL";
        case VCT_ENOMEM: return "VCT_ENOMEM";
        case VCT_EDEVICE: return "VCT_EDEVICE";
        case VCT_ECOMM: return "VCT_ECOMM";
        case VCT_ESTATE: return "VCT_ESTATE";
    }
    return "VCT_UNKNOWN";
}

const char* vct_last_error(const vct_ctx* c) { return c ? c->err.c_str() : "null context"; }

vct_status vct_create(const vct_config* cfg, vct_ctx** out) {
    if (!cfg || !out) return VCT_EINVAL;
    *out = nullptr;
    if (!is_pow2(cfg->n) || cfg->n < 4 || cfg->n > 1024) return VCT_EINVAL;
    if (!(cfg->extent > 0.0f) || !std::isfinite(cfg->extent)) return VCT_EINVAL;
    if (cfg->n_diffuse != 0 && cfg->n_diffuse != 1 && cfg->n_diffuse != 9 && cfg->n_diffuse != 16)
        return VCT_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VCT_EDEVICE;
    int dev = cfg->device;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) return VCT_EDEVICE;
    }
    if (dev >= ndev) return VCT_EINVAL;
    vct_ctx* c = new (std::nothrow) vct_ctx();
    if (!c) return VCT_ENOMEM;
    c->cfg = *cfg;
    c->device = dev;
    c->cfg.device = dev;
    if (hipSetDevice(dev) != hipSuccess) { delete c; return VCT_EDEVICE; }
    Grid& g = c->grid;
    g.n = cfg->n;
    g.L = ilog2u(cfg->n);
    g.aniso = cfg->aniso ? 1 : 0;
    for (int i = 0; i < 3; ++i) g.g0[i] = cfg->aabb_min[i];
    g.extent = cfg->extent;
    g.inv_h = (float)cfg->n / cfg->extent;
    const uint64_t faces = g.aniso ? VCT_NUM_FACES : 1;
    uint64_t off = 0;
    for (uint32_t l = 0; l <= g.L; ++l) {
        g.lvl_off[l] = off;
        const uint64_t nl = g.n >> l;
        off += (l == 0 ? 1 : faces) * nl * nl * nl;
    }
    for (uint32_t l = g.L + 1; l <= (uint32_t)kMaxLevels; ++l) g.lvl_off[l] = off;
    g.pyr_texels = off;
    const size_t nv = (size_t)g.n * g.n * g.n;
    // +1 texel: a permanent zero texel after the pyramid (zero border of the LDS-DMA staging)
    hipError_t e = hipMalloc(&g.pyr, (off + 1) * sizeof(float4));
    if (e == hipSuccess) e = hipMemset(g.pyr, 0, (off + 1) * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&g.albedo_occ, nv * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&g.normal, nv * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&g.occ_bits, (nv / 64) * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&g.accum, nv * 64);
    // K1's sparse-reset invariant: accumulators, voxels and bits start at zero
    if (e == hipSuccess) e = hipMemset(g.accum, 0, nv * 64);
    if (e == hipSuccess) e = hipMemset(g.albedo_occ, 0, nv * sizeof(float4));
    if (e == hipSuccess) e = hipMemset(g.normal, 0, nv * sizeof(float4));
    if (e == hipSuccess) e = hipMemset(g.occ_bits, 0, (nv / 64) * 8);
    if (e == hipSuccess && g.n >= 16) {
        // K4 empty-space maps (Grid::zmap): level-0 bits, occupancy bytes of levels 2.., bit maps
        // every map level keeps >= 4 texels per axis (its rows are read as dwords)
        g.zm_levels = (int)(g.L - 2 < (uint32_t)Grid::kZLevels ? g.L - 2 : (uint32_t)Grid::kZLevels);
        uint64_t ob = 0;
        uint32_t zw = 0;
        for (int m = 1; m <= g.zm_levels; ++m) {
            const uint64_t nm = g.n >> m;
            if (m >= 2) { g.occ_off[m] = ob; ob += nm * nm * nm; }
            g.zm_dim[m] = (uint32_t)nm + 1u;
            g.zm_rw[m] = (g.zm_dim[m] + 31u) / 32u;
            g.zm_off[m] = zw;
            zw += g.zm_dim[m] * g.zm_dim[m] * g.zm_rw[m];
        }
        e = hipMalloc((void**)&g.b0, nv / 8);
        if (e == hipSuccess) e = hipMalloc((void**)&g.occ, ob ? ob : 1);
        if (e == hipSuccess) e = hipMalloc((void**)&g.zmap, (size_t)zw * 4);
    }
    if (e == hipSuccess) e = hipMalloc((void**)&g.k3_live, nv / 256 > 0 ? nv / 256 : 1);
    if (e == hipSuccess) e = hipMalloc((void**)&g.k3_live_list, (nv / 1024 + 64) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&g.k2_coarse, 2 * 64 * 64 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&g.occ_list, nv * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&g.occ_count, 256);
    if (e == hipSuccess) e = hipMemset(g.occ_count, 0, 256);
    if (e == hipSuccess) {
        StepRow rows[kMaxStepRows];
        const float tau_d = cfg->n_diffuse == 16 ? VCT_TAN20 : VCT_TAN30;
        if (build_step_table(tau_d, g.n, g.L, rows) < 0) e = hipErrorInvalidValue;
        if (e == hipSuccess) e = hipMalloc((void**)&c->step_tab, sizeof rows);
        if (e == hipSuccess) e = hipMemcpy(c->step_tab, rows, sizeof rows, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipMalloc((void**)&c->spec_keys, 2 * kSpecSlots * sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(c->spec_keys, 0xff, kSpecSlots * sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(c->spec_keys + kSpecSlots, 0, kSpecSlots * sizeof(unsigned));
    if (e == hipSuccess) e = hipMalloc((void**)&c->spec_rows, kSpecSlots * 64 * sizeof(StepRow));
    if (e != hipSuccess) {
        vct_destroy(c);
        return e == hipErrorOutOfMemory ? VCT_ENOMEM : VCT_EDEVICE;
    }
    *out = c;
    return VCT_OK;
}

vct_status vct_create_multi(const vct_config* cfg, uint32_t n_devices, vct_ctx** out) {
    if (!cfg || !out || n_devices < 1 || n_devices > 64) return VCT_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VCT_EDEVICE;
    int d0 = cfg->device;
    if (d0 < 0 && hipGetDevice(&d0) != hipSuccess) return VCT_EDEVICE;
    if (d0 >= ndev) return VCT_EINVAL;
    vct_config c0 = *cfg;
    c0.device = d0;
    vct_ctx* c = nullptr;
    vct_status st = vct_create(&c0, &c);
    if (st != VCT_OK) return st;
    auto bail = [&](vct_status s) { vct_destroy(c); return s; };
    if (hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess) return bail(VCT_EDEVICE);
    for (uint32_t r = 1; r < n_devices; ++r) {
        vct_config ci = *cfg;
        ci.device = (int)((d0 + r) % (uint32_t)ndev);   // more ranks than devices: ranks share devices
        vct_ctx* p = nullptr;
        if ((st = vct_create(&ci, &p)) != VCT_OK) return bail(st);
        c->peers.push_back(p);
        if (hipSetDevice(p->device) != hipSuccess ||
            hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess)
            return bail(VCT_EDEVICE);
        p->own_stream = true;
        if (hipEventCreateWithFlags(&p->ev, hipEventDisableTiming) != hipSuccess) return bail(VCT_EDEVICE);
        if (p->device != d0) {   // device r reads device 0's G-buffer and writes its steps_px pixels
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, p->device, d0) != hipSuccess || !can) return bail(VCT_EDEVICE);
            hipError_t e = hipDeviceEnablePeerAccess(d0, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return bail(VCT_EDEVICE);
            (void)hipGetLastError();
        }
    }
    if (hipSetDevice(d0) != hipSuccess) return bail(VCT_EDEVICE);
    *out = c;
    return VCT_OK;
}

uint32_t vct_num_devices(const vct_ctx* c) { return c ? 1u + (uint32_t)c->peers.size() : 0u; }
int32_t vct_trace_form(const vct_ctx* c) {
    return (c && c->k4tune.cur >= 0) ? c->k4tune.e[c->k4tune.cur].chosen : -1;
}

void vct_destroy(vct_ctx* c) {
    if (!c) return;
    (void)vct_comm_destroy(c);
    for (vct_ctx* p : c->peers) vct_destroy(p);
    c->peers.clear();
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    else (void)hipDeviceSynchronize();
    Grid& g = c->grid;
    if (g.pyr) (void)hipFree(g.pyr);
    if (g.albedo_occ) (void)hipFree(g.albedo_occ);
    if (g.normal) (void)hipFree(g.normal);
    if (g.occ_bits) (void)hipFree(g.occ_bits);
    if (g.occ_list) (void)hipFree(g.occ_list);
    if (g.k3_live) (void)hipFree(g.k3_live);
    if (g.k3_live_list) (void)hipFree(g.k3_live_list);
    if (g.k2_coarse) (void)hipFree(g.k2_coarse);
    if (g.b0) (void)hipFree(g.b0);
    if (g.occ) (void)hipFree(g.occ);
    if (g.zmap) (void)hipFree(g.zmap);
    if (g.occ_count) (void)hipFree(g.occ_count);
    if (g.accum) (void)hipFree(g.accum);
    if (c->k1_err) (void)hipFree(c->k1_err);
    if (c->mesh.tri) (void)hipFree(c->mesh.tri);
    if (c->mesh.uv) (void)hipFree(c->mesh.uv);
    if (c->tex.texels) (void)hipFree(c->tex.texels);
    if (c->tex.desc) (void)hipFree(c->tex.desc);
    if (c->step_tab) (void)hipFree(c->step_tab);
    if (c->spec_keys) (void)hipFree(c->spec_keys);
    if (c->spec_rows) (void)hipFree(c->spec_rows);
    for (auto& s : c->scratch)
        if (s.p) (void)hipFree(s.p);
    for (auto& ss : c->k4s)
        for (auto& s : ss.sc)
            if (s.p) (void)hipFree(s.p);
    if (c->ev) (void)hipEventDestroy(c->ev);
    if (c->xchg_done) (void)hipEventDestroy(c->xchg_done);
    for (auto& en : c->k4tune.e) {
        for (auto& f : en.ev)
            for (auto& sl : f)
                for (hipEvent_t e : sl)
                    if (e) (void)hipEventDestroy(e);
        if (en.hist) (void)hipFree(en.hist);
    }
    for (uint32_t* h : c->k4tune.retired) (void)hipFree(h);
    if (c->k4tune.prev_end) (void)hipEventDestroy(c->k4tune.prev_end);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

vct_status vct_get_config(const vct_ctx* c, vct_config* out) {
    if (!c || !out) return VCT_EINVAL;
    *out = c->cfg;
    return VCT_OK;
}

vct_status vct_set_stream(vct_ctx* c, void* stream) {
    if (!c) return VCT_EINVAL;
    c->stream = (hipStream_t)stream;
    return VCT_OK;
}

vct_status vct_synchronize(vct_ctx* c) {
    if (!c) return VCT_EINVAL;
    for (vct_ctx* p : c->peers) {
        VCT_HIP(hipSetDevice(p->device), "hipSetDevice");
        VCT_HIP(hipStreamSynchronize(p->stream), "hipStreamSynchronize (peer)");
    }
    vct_status s = use_device(c);
    if (s != VCT_OK) return s;
    VCT_HIP(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    return VCT_OK;
}

static vct_status voxelize_args(vct_ctx* c, const void* verts, uint32_t stride, uint32_t n_idx, const uint32_t* idx,
                                const float* kd4, uint32_t n_mat) {
    if (!c) return VCT_EINVAL;
    if (n_idx % 3 != 0) return fail(c, VCT_EINVAL, "n_idx must be a multiple of 3");
    if (n_idx > 0 && (!verts || !idx)) return fail(c, VCT_EINVAL, "null vertex or index array");
    if (stride < 12 || stride % 4 != 0) return fail(c, VCT_EINVAL, "vertex_stride < 12 or not a multiple of 4");
    if (kd4 && n_mat == 0) return fail(c, VCT_EINVAL, "material_kd4 with n_materials == 0");
    return use_device(c);
}

// K1 on device-resident geometry; `derr` (device int) receives the index-range flag.
// dmap (device, may be NULL): each material's diffuse map (vct_voxelize_textured).
static vct_status voxelize_dev(vct_ctx* c, const void* dv, uint32_t stride, uint32_t n_verts, const uint32_t* di,
                               uint32_t n_tri, const uint32_t* dm, const float4* dk, uint32_t n_mat,
                               const int32_t* dmap, uint32_t uv_offset, int* derr) {
    Mesh& m = c->mesh;
    const size_t tri_bytes = (size_t)(n_tri ? n_tri : 1) * 4 * sizeof(float4);
    if (m.cap < tri_bytes) {
        VCT_HIP(hipStreamSynchronize(c->stream), "sync");
        if (m.tri) (void)hipFree(m.tri);
        m.tri = nullptr;
        m.cap = 0;
        VCT_HIP(hipMalloc(&m.tri, tri_bytes), "hipMalloc mesh");
        m.cap = tri_bytes;
    }
    const size_t uv_bytes = (size_t)(n_tri ? n_tri : 1) * 2 * sizeof(float4);
    if (dmap && m.uv_cap < uv_bytes) {
        VCT_HIP(hipStreamSynchronize(c->stream), "sync");
        if (m.uv) (void)hipFree(m.uv);
        m.uv = nullptr;
        m.uv_cap = 0;
        VCT_HIP(hipMalloc(&m.uv, uv_bytes), "hipMalloc mesh uv");
        m.uv_cap = uv_bytes;
    }
    m.n_tri = n_tri;
    m.textured = dmap != nullptr;
    // Everything derived from the previous occupancy is invalid from here on, and stays so
    // if a step below fails part way (K1 has already rewritten the accumulators, the
    // occupied list and level 0 by then): only the success path sets `voxelized` again
    Grid& g = c->grid;
    g.voxelized = g.injected = g.mipped = false;
    g.k2_coarse_ok = g.k3_sparse_ok = g.zm_valid = false;
    g.k3_live_bz = 0;
    ++c->grid_epoch;
    int herr = 0;
    for (bool packed : {true, false}) {
        VCT_HIP(hipMemsetAsync(derr, 0, 4, c->stream), "memset err");
        VCT_HIP(launch_voxelize(c, dv, stride, n_verts, di, n_tri, dm, dk, n_mat, dmap, uv_offset, derr, packed),
                "voxelize");
        // the K3 live list of a packed pass is the repeat's too (same occupancy), but it is
        // queued before the one read-back so that its count arrives with the error word
        if (packed) VCT_HIP(launch_k3_live(c), "K3 live blocks");
        VCT_HIP(hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, c->stream), "download err");
        VCT_HIP(hipStreamSynchronize(c->stream), "voxelize sync");
        // a pass whose packed sums may have overflowed is repeated with the seven-atomic form
        if ((herr & kK1ErrIndex) || !(herr & kK1ErrRedo)) break;
    }
    // a grid from out-of-range indices is partial: inject / mips / trace refuse it (VCT_ESTATE)
    if (herr & kK1ErrIndex) return fail(c, VCT_EINVAL, "vertex, material or diffuse-map index out of range");
    g.voxelized = true;
    return VCT_OK;
}

static vct_status map_args(vct_ctx* c, const int32_t* map, uint32_t n_mat, uint32_t stride, uint32_t uv_offset) {
    if (!map) return VCT_OK;
    if (n_mat == 0) return fail(c, VCT_EINVAL, "material_map with n_materials == 0");
    if (uv_offset % 4 != 0 || (uint64_t)uv_offset + 8 > stride)
        return fail(c, VCT_EINVAL, "uv_offset must be a multiple of 4 with uv_offset + 8 <= vertex_stride");
    return VCT_OK;
}

static vct_status voxelize_host(vct_ctx* c, const void* verts, uint32_t stride, uint32_t n_verts,
                                const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_mat, const float* kd4,
                                const int32_t* map, uint32_t n_mat, uint32_t uv_offset) {
    vct_status st = voxelize_args(c, verts, stride, n_idx, idx, kd4, n_mat);
    if (st != VCT_OK) return st;
    if ((st = map_args(c, map, n_mat, stride, uv_offset)) != VCT_OK) return st;
    if (map)
        for (uint32_t i = 0; i < n_mat; ++i)
            if (map[i] < -1 || (map[i] >= 0 && (uint32_t)map[i] >= c->tex.n))
                return fail(c, VCT_EINVAL, "material_map[" + std::to_string(i) + "] = " + std::to_string(map[i]) +
                                               " is not a texture of vct_set_textures (" + std::to_string(c->tex.n) +
                                               " set) or -1");
    const uint32_t n_tri = n_idx / 3;
    // host -> device staging (the reference keeps CPU copies of vertices / indices
    // next to its GL buffers, mesh.h:17-18; this is the same one-time upload)
    DeviceBuf dv, di, dm, dk, dmap, derr;
    const size_t vbytes = (size_t)stride * n_verts;
    if (vbytes) VCT_HIP(hipMalloc(&dv.p, vbytes), "hipMalloc verts");
    if (n_idx) VCT_HIP(hipMalloc(&di.p, (size_t)n_idx * 4), "hipMalloc idx");
    if (tri_mat && n_tri) VCT_HIP(hipMalloc(&dm.p, (size_t)n_tri * 4), "hipMalloc mat");
    if (kd4) VCT_HIP(hipMalloc(&dk.p, (size_t)n_mat * 16), "hipMalloc kd");
    if (map) VCT_HIP(hipMalloc(&dmap.p, (size_t)n_mat * 4), "hipMalloc map");
    VCT_HIP(hipMalloc(&derr.p, 4), "hipMalloc err");
    if (vbytes) VCT_HIP(hipMemcpyAsync(dv.p, verts, vbytes, hipMemcpyHostToDevice, c->stream), "upload verts");
    if (n_idx) VCT_HIP(hipMemcpyAsync(di.p, idx, (size_t)n_idx * 4, hipMemcpyHostToDevice, c->stream), "upload idx");
    if (dm.p) VCT_HIP(hipMemcpyAsync(dm.p, tri_mat, (size_t)n_tri * 4, hipMemcpyHostToDevice, c->stream), "upload mat");
    if (dk.p) VCT_HIP(hipMemcpyAsync(dk.p, kd4, (size_t)n_mat * 16, hipMemcpyHostToDevice, c->stream), "upload kd");
    if (dmap.p) VCT_HIP(hipMemcpyAsync(dmap.p, map, (size_t)n_mat * 4, hipMemcpyHostToDevice, c->stream), "upload map");
    return voxelize_dev(c, dv.p, stride, n_verts, (const uint32_t*)di.p, n_tri, (const uint32_t*)dm.p,
                        (const float4*)dk.p, n_mat, (const int32_t*)dmap.p, uv_offset, (int*)derr.p);
}

static vct_status voxelize_device(vct_ctx* c, const void* verts, uint32_t stride, uint32_t n_verts,
                                  const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_mat, const float* kd4,
                                  const int32_t* map, uint32_t n_mat, uint32_t uv_offset) {
    vct_status st = voxelize_args(c, verts, stride, n_idx, idx, kd4, n_mat);
    if (st != VCT_OK) return st;
    if ((st = map_args(c, map, n_mat, stride, uv_offset)) != VCT_OK) return st;
    if ((kd4 && ((uintptr_t)kd4 & 15)) || ((uintptr_t)verts & 3) || ((uintptr_t)map & 3))
        return fail(c, VCT_EINVAL, "material_kd4 must be 16-byte, verts and material_map 4-byte aligned");
    if (!c->k1_err) VCT_HIP(hipMalloc((void**)&c->k1_err, 4), "hipMalloc err");
    return voxelize_dev(c, verts, stride, n_verts, idx, n_idx / 3, tri_mat, (const float4*)kd4, n_mat, map, uv_offset,
                        c->k1_err);
}

vct_status vct_voxelize(vct_ctx* c, const void* verts, uint32_t stride, uint32_t n_verts,
                        const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_mat,
                        const float* kd4, uint32_t n_mat) {
    return voxelize_host(c, verts, stride, n_verts, idx, n_idx, tri_mat, kd4, nullptr, n_mat, 0);
}

vct_status vct_voxelize_device(vct_ctx* c, const void* verts, uint32_t stride, uint32_t n_verts,
                               const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_mat,
                               const float* kd4, uint32_t n_mat) {
    return voxelize_device(c, verts, stride, n_verts, idx, n_idx, tri_mat, kd4, nullptr, n_mat, 0);
}

vct_status vct_voxelize_textured(vct_ctx* c, const void* verts, uint32_t stride, uint32_t n_verts,
                                 const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_mat, const float* kd4,
                                 const int32_t* map, uint32_t n_mat, uint32_t uv_offset) {
    return voxelize_host(c, verts, stride, n_verts, idx, n_idx, tri_mat, kd4, map, n_mat, uv_offset);
}

vct_status vct_voxelize_textured_device(vct_ctx* c, const void* verts, uint32_t stride, uint32_t n_verts,
                                        const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_mat,
                                        const float* kd4, const int32_t* map, uint32_t n_mat, uint32_t uv_offset) {
    return voxelize_device(c, verts, stride, n_verts, idx, n_idx, tri_mat, kd4, map, n_mat, uv_offset);
}

vct_status vct_set_textures(vct_ctx* c, const vct_texture* tex, uint32_t n) {
    if (!c || (n && !tex)) return c ? fail(c, VCT_EINVAL, "null texture array") : VCT_EINVAL;
    uint64_t total = 0;
    std::vector<TexDesc> desc(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (!tex[i].rgba8 || tex[i].width == 0 || tex[i].height == 0 || tex[i].width > VCT_TEX_MAX_DIM ||
            tex[i].height > VCT_TEX_MAX_DIM)
            return fail(c, VCT_EINVAL, "texture " + std::to_string(i) + ": null data or size outside 1.." +
                                           std::to_string(VCT_TEX_MAX_DIM));
        desc[i] = TexDesc{(uint32_t)total, tex[i].width, tex[i].height, 0u};
        total += (uint64_t)tex[i].width * tex[i].height;
        if (total > 0xffffffffull) return fail(c, VCT_EINVAL, "textures exceed 2^32 texels");
    }
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    Textures& t = c->tex;
    VCT_HIP(hipStreamSynchronize(c->stream), "sync");   // the previous set may still be read
    if (t.texel_cap < total * 4) {
        if (t.texels) (void)hipFree(t.texels);
        t.texels = nullptr;
        t.texel_cap = 0;
        VCT_HIP(hipMalloc((void**)&t.texels, total * 4), "hipMalloc textures");
        t.texel_cap = total * 4;
    }
    if (t.desc_cap < (size_t)n * sizeof(TexDesc)) {
        if (t.desc) (void)hipFree(t.desc);
        t.desc = nullptr;
        t.desc_cap = 0;
        VCT_HIP(hipMalloc((void**)&t.desc, (size_t)n * sizeof(TexDesc)), "hipMalloc texture table");
        t.desc_cap = (size_t)n * sizeof(TexDesc);
    }
    t.n = 0;
    for (uint32_t i = 0; i < n; ++i)
        VCT_HIP(hipMemcpy(t.texels + desc[i].off, tex[i].rgba8, (size_t)desc[i].w * desc[i].h * 4,
                          hipMemcpyHostToDevice),
                "upload texture");
    if (n) VCT_HIP(hipMemcpy(t.desc, desc.data(), (size_t)n * sizeof(TexDesc), hipMemcpyHostToDevice), "upload table");
    t.n = n;
    return VCT_OK;
}

vct_status vct_inject_directional(vct_ctx* c, const float dir[3], const float color[3]) {
    if (!c || !dir || !color) return VCT_EINVAL;
    if (!c->grid.voxelized) return fail(c, VCT_ESTATE, "inject before voxelize");
    float lx = dir[0], ly = dir[1], lz = dir[2];
    const float len = sqrtf((lx * lx + ly * ly) + lz * lz);
    if (!(len > 0.0f) || !std::isfinite(len)) return fail(c, VCT_EINVAL, "zero or non-finite light direction");
    lx = lx / len; ly = ly / len; lz = lz / len;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(launch_inject(c, lx, ly, lz, color[0], color[1], color[2]), "inject");
    c->grid.injected = true;
    c->grid.mipped = false;
    c->grid.l0_on_peers = false;
    return VCT_OK;
}

vct_status vct_build_mips(vct_ctx* c) {
    if (!c) return VCT_EINVAL;
    if (!c->grid.injected) return fail(c, VCT_ESTATE, "build_mips before inject / upload_level0");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    if (!c->peers.empty() && !c->grid.l0_on_peers) {
        // the replicated grid: level 0 from device 0 to every other device
        // over xGMI, ordered after the work queued on device 0 (K2)
        const size_t bytes = (size_t)c->grid.n * c->grid.n * c->grid.n * sizeof(float4);
        VCT_HIP(hipEventRecord(c->ev, c->stream), "event record");
        for (vct_ctx* p : c->peers) {
            VCT_HIP(hipSetDevice(p->device), "hipSetDevice");
            VCT_HIP(hipStreamWaitEvent(p->stream, c->ev, 0), "stream wait");
            VCT_HIP(hipMemcpyPeerAsync(p->grid.pyr, p->device, c->grid.pyr, c->device, bytes, p->stream),
                    "level-0 peer copy");
            p->grid.injected = true;
            p->grid.l0_dense = true;
        }
        c->grid.l0_on_peers = true;
    }
    for (vct_ctx* p : c->peers) {
        VCT_HIP(hipSetDevice(p->device), "hipSetDevice");
        VCT_HIP(launch_mips(p), "mips (peer)");
        p->grid.mipped = true;
    }
    if (!c->peers.empty() && (st = use_device(c)) != VCT_OK) return st;
    VCT_HIP(launch_mips(c), "mips");
    c->grid.mipped = true;
    return VCT_OK;
}

uint32_t vct_tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t world) {
    return tiles_for_rank(w, h, rank, world);
}

// K4 over the devices of a multi-device context (device-0 pointers in `a`).  Device r
// traces the 64x64 tiles t with t % world == r into rank-compact planes: device 0
// straight into slot 0 of a gather buffer on device 0, the others into their own HBM,
// then one peer copy over xGMI each into their slot; device 0 waits for those copies
// and un-permutes both planes into the caller's frame (vct_untile_planes_device).
// Devices 1.. read the G-buffer and write their pixels of steps_px through peer access;
// their step / texel counters are copied over and folded into the caller's.
static vct_status trace_multi(vct_ctx* c, const vct_trace_args* a) {
    if (a->tile_world > 1 || a->tile_compact)
        return fail(c, VCT_EINVAL, "a multi-device context splits the frame itself (tile_world / tile_compact)");
    const uint32_t world = 1 + (uint32_t)c->peers.size();
    const uint32_t w = a->width, h = a->height;
    const size_t npx = (size_t)tiles_for_rank(w, h, 0, world) * VCT_TILE * VCT_TILE;
    const size_t slice = 2 * npx * sizeof(float4);          // one device's [diffuse | specular]
    const bool counting = a->cone_steps || a->texel_fetches;
    void* gp = nullptr;
    void* cp = nullptr;
    VCT_HIP(xchg_enter(c), "stream wait (previous exchange)");
    XchgScope xs{c};                           // every exit below records the exchange's end
    VCT_HIP(scratch_get(c, 8, world * slice, &gp), "gather buffer");
    if (counting) {
        VCT_HIP(scratch_get(c, 9, world * 16, &cp), "counter buffer");
        VCT_HIP(hipMemsetAsync(cp, 0, world * 16, c->stream), "memset counters");
    }
    // the other devices start after everything queued on device 0 so far (the G-buffer,
    // the previous call's untile of the gather buffer)
    VCT_HIP(hipEventRecord(c->ev, c->stream), "event record");
    for (uint32_t r = 1; r < world; ++r) {
        vct_ctx* p = c->peers[r - 1];
        VCT_HIP(hipSetDevice(p->device), "hipSetDevice");
        VCT_HIP(hipStreamWaitEvent(p->stream, c->ev, 0), "stream wait");
        void* tp = nullptr;
        VCT_HIP(scratch_get(p, 8, slice + 16, &tp), "tile buffer (peer)");
        unsigned long long* pc = (unsigned long long*)((char*)tp + slice);
        if (counting) VCT_HIP(hipMemsetAsync(pc, 0, 16, p->stream), "memset counters (peer)");
        vct_trace_args b = *a;
        b.tile_rank = r;
        b.tile_world = world;
        b.tile_compact = 1;
        b.diffuse4 = (float*)tp;
        b.spec4 = (float*)tp + npx * 4;
        b.cone_steps = a->cone_steps ? pc : nullptr;
        b.texel_fetches = a->texel_fetches ? pc + 1 : nullptr;
        VCT_HIP(launch_trace(p, &b), "trace (peer)");
        VCT_HIP(hipMemcpyPeerAsync((char*)gp + r * slice, c->device, tp, p->device, slice, p->stream),
                "tile peer copy");
        if (counting)
            VCT_HIP(hipMemcpyPeerAsync((char*)cp + 16 * r, c->device, pc, p->device, 16, p->stream),
                    "counter peer copy");
        VCT_HIP(hipEventRecord(p->ev, p->stream), "event record (peer)");
    }
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    vct_trace_args b = *a;
    b.tile_rank = 0;
    b.tile_world = world;
    b.tile_compact = 1;
    b.diffuse4 = (float*)gp;
    b.spec4 = (float*)gp + npx * 4;
    VCT_HIP(launch_trace(c, &b), "trace");
    for (vct_ctx* p : c->peers) VCT_HIP(hipStreamWaitEvent(c->stream, p->ev, 0), "stream wait (peer)");
    if (counting)
        VCT_HIP(launch_add_counters(c, (const unsigned long long*)cp, world, a->cone_steps, a->texel_fetches),
                "fold counters");
    float4* f[2] = {(float4*)a->diffuse4, (float4*)a->spec4};
    VCT_HIP(launch_untile(c, (const float4*)gp, 2, w, h, world, f), "untile");
    VCT_HIP(xchg_leave(c), "event record (exchange end)");
    xs.done = true;
    return VCT_OK;
}

static vct_status trace_any(vct_ctx* c, const vct_trace_args* a) {
    if (!c->peers.empty()) return trace_multi(c, a);
    VCT_HIP(launch_trace(c, a), "trace");
    return VCT_OK;
}

vct_status vct_trace_device(vct_ctx* c, const vct_trace_args* a) {
    if (!c || !a) return VCT_EINVAL;
    if (!c->grid.mipped) return fail(c, VCT_ESTATE, "trace before build_mips");
    if (!a->pos4 || !a->nrm4 || !a->alb4 || !a->diffuse4 || !a->spec4)
        return fail(c, VCT_EINVAL, "null G-buffer or output pointer");
    if (a->width == 0 || a->height == 0 || a->width > 65536 || a->height > 65536 ||
        (uint64_t)a->width * a->height > 0xffffffffull)   // K4 indexes pixels with 32 bits
        return fail(c, VCT_EINVAL, "bad frame size");
    if (a->tile_world > 1 && a->tile_rank >= a->tile_world) return fail(c, VCT_EINVAL, "tile_rank >= tile_world");
    // the counters are 64-bit device atomics: a misaligned target faults the GPU
    if (((uintptr_t)a->cone_steps & 7) || ((uintptr_t)a->texel_fetches & 7))
        return fail(c, VCT_EINVAL, "cone_steps / texel_fetches must be 8-byte aligned");
    if (((uintptr_t)a->pos4 | (uintptr_t)a->nrm4 | (uintptr_t)a->alb4 | (uintptr_t)a->diffuse4 |
         (uintptr_t)a->spec4) & 15)
        return fail(c, VCT_EINVAL, "G-buffer / output pointers must be 16-byte aligned");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    return trace_any(c, a);
}

vct_status vct_trace(vct_ctx* c, const float* pos4, const float* nrm4, const float* alb4, uint32_t w,
                     uint32_t h, const float eye[3], float* diff4, float* spec4, uint32_t* steps_px,
                     uint64_t* cone_steps) {
    if (!c || !pos4 || !nrm4 || !alb4 || !eye || !diff4 || !spec4) return VCT_EINVAL;
    if (!c->grid.mipped) return fail(c, VCT_ESTATE, "trace before build_mips");
    if (w == 0 || h == 0) return fail(c, VCT_EINVAL, "bad frame size");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    // every sub-buffer 256-byte aligned (the u64 step counter is an atomic target)
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t px = (size_t)w * h, fb = al(px * 16), sb = al(px * 4);
    void* sp;
    VCT_HIP(scratch_get(c, 0, fb * 5 + sb + 256, &sp), "scratch");
    char* b = (char*)sp;
    float* dpos = (float*)b;
    float* dnrm = (float*)(b + fb);
    float* dalb = (float*)(b + 2 * fb);
    float* ddif = (float*)(b + 3 * fb);
    float* dspc = (float*)(b + 4 * fb);
    uint32_t* dstp = (uint32_t*)(b + 5 * fb);
    unsigned long long* dtot = (unsigned long long*)(b + 5 * fb + sb);
    VCT_HIP(hipMemcpyAsync(dpos, pos4, px * 16, hipMemcpyHostToDevice, c->stream), "upload pos");
    VCT_HIP(hipMemcpyAsync(dnrm, nrm4, px * 16, hipMemcpyHostToDevice, c->stream), "upload nrm");
    VCT_HIP(hipMemcpyAsync(dalb, alb4, px * 16, hipMemcpyHostToDevice, c->stream), "upload alb");
    VCT_HIP(hipMemsetAsync(dtot, 0, 8, c->stream), "memset");
    vct_trace_args a;
    std::memset(&a, 0, sizeof a);
    a.pos4 = dpos; a.nrm4 = dnrm; a.alb4 = dalb;
    a.width = w; a.height = h;
    a.eye[0] = eye[0]; a.eye[1] = eye[1]; a.eye[2] = eye[2];
    a.diffuse4 = ddif; a.spec4 = dspc;
    a.steps_px = steps_px ? dstp : nullptr;
    a.cone_steps = dtot;
    st = trace_any(c, &a);
    if (st != VCT_OK) return st;
    VCT_HIP(hipMemcpyAsync(diff4, ddif, px * 16, hipMemcpyDeviceToHost, c->stream), "download diffuse");
    VCT_HIP(hipMemcpyAsync(spec4, dspc, px * 16, hipMemcpyDeviceToHost, c->stream), "download spec");
    if (steps_px) VCT_HIP(hipMemcpyAsync(steps_px, dstp, px * 4, hipMemcpyDeviceToHost, c->stream), "download steps");
    unsigned long long tot = 0;
    VCT_HIP(hipMemcpyAsync(&tot, dtot, 8, hipMemcpyDeviceToHost, c->stream), "download total");
    VCT_HIP(hipStreamSynchronize(c->stream), "trace sync");
    if (cone_steps) *cone_steps = tot;
    return VCT_OK;
}

vct_status vct_untile_device(vct_ctx* c, const float* gathered4, uint32_t w, uint32_t h, uint32_t world,
                             float* frame4) {
    if (!c || !gathered4 || !frame4 || w == 0 || h == 0) return VCT_EINVAL;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    float4* f = (float4*)frame4;
    VCT_HIP(launch_untile(c, (const float4*)gathered4, 1, w, h, world, &f), "untile");
    return VCT_OK;
}

vct_status vct_untile_planes_device(vct_ctx* c, const float* gathered4, uint32_t planes, uint32_t w, uint32_t h,
                                    uint32_t world, float* const* frames4) {
    if (!c || !gathered4 || !frames4 || w == 0 || h == 0 || planes == 0 || planes > (uint32_t)kMaxUntilePlanes)
        return VCT_EINVAL;
    float4* f[kMaxUntilePlanes] = {};
    for (uint32_t p = 0; p < planes; ++p) {
        if (!frames4[p]) return VCT_EINVAL;
        f[p] = (float4*)frames4[p];
    }
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(launch_untile(c, (const float4*)gathered4, planes, w, h, world, f), "untile planes");
    return VCT_OK;
}

vct_status vct_untile_planes_packed_device(vct_ctx* c, const float* gathered4, uint32_t planes, uint32_t w,
                                           uint32_t h, uint32_t world, float* const* frames4) {
    if (!c || !gathered4 || !frames4 || w == 0 || h == 0 || planes == 0 || planes > (uint32_t)kMaxUntilePlanes)
        return VCT_EINVAL;
    float4* f[kMaxUntilePlanes] = {};
    for (uint32_t p = 0; p < planes; ++p) {
        if (!frames4[p]) return VCT_EINVAL;
        f[p] = (float4*)frames4[p];
    }
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(launch_untile(c, (const float4*)gathered4, planes, w, h, world, f, true), "untile planes packed");
    return VCT_OK;
}

uint32_t vct_tile_offset(uint32_t w, uint32_t h, uint32_t rank, uint32_t world) {
    if (world == 0) world = 1;
    if (rank >= world) return 0;
    const uint32_t total = ((w + VCT_TILE - 1) / VCT_TILE) * ((h + VCT_TILE - 1) / VCT_TILE);
    const uint32_t q = total / world, rem = total % world;
    return rank * q + (rank < rem ? rank : rem);
}

vct_status vct_gbuffer_raycast_device(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h,
                                      float rough, float* pos4, float* nrm4, float* alb4) {
    if (!c || !cam || !pos4 || !nrm4 || !alb4 || w == 0 || h == 0) return VCT_EINVAL;
    if (!c->mesh.tri) return fail(c, VCT_ESTATE, "raycast before voxelize");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(launch_raycast(c, cam, w, h, rough, (float4*)pos4, (float4*)nrm4, (float4*)alb4), "raycast");
    return VCT_OK;
}

vct_status vct_gbuffer_raster_device(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h, float rough,
                                     float* pos4, float* nrm4, float* alb4) {
    if (!c || !cam || !pos4 || !nrm4 || !alb4 || w == 0 || h == 0) return VCT_EINVAL;
    if ((uint64_t)w * h > 0x7fffffffull || (uint64_t)((w + 15) / 16) * ((h + 15) / 16) > (1u << 20))
        return fail(c, VCT_EINVAL, "raster: frame too large");
    if (!c->mesh.tri) return fail(c, VCT_ESTATE, "raster before voxelize");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(launch_gbuffer_binned(c, cam, w, h, rough, (float4*)pos4, (float4*)nrm4, (float4*)alb4), "raster");
    return VCT_OK;
}

vct_status vct_composite_device(vct_ctx* c, const float* pos4, const float* nrm4, const float* alb4,
                                const float* diffuse4, const float* spec4, uint32_t w, uint32_t h,
                                const float dir_to_light[3], const float color[3], float* out_linear4,
                                uint32_t* out_rgba8) {
    if (!c || !pos4 || !nrm4 || !alb4 || !diffuse4 || !spec4 || !dir_to_light || !color || w == 0 || h == 0)
        return VCT_EINVAL;
    if (!out_linear4 && !out_rgba8) return fail(c, VCT_EINVAL, "composite: no output");
    if ((uint64_t)w * h > 0x7fffffffull) return fail(c, VCT_EINVAL, "composite: frame too large");
    if (!c->grid.voxelized) return fail(c, VCT_ESTATE, "composite before voxelize");
    for (const void* p : {(const void*)pos4, (const void*)nrm4, (const void*)alb4, (const void*)diffuse4,
                          (const void*)spec4, (const void*)out_linear4})
        if (((uintptr_t)p & 15u) != 0) return fail(c, VCT_EINVAL, "composite: float4 buffers must be 16-byte aligned");
    if (((uintptr_t)out_rgba8 & 3u) != 0) return fail(c, VCT_EINVAL, "composite: rgba8 buffer must be 4-byte aligned");
    float l[3] = {dir_to_light[0], dir_to_light[1], dir_to_light[2]};   // normalized as vct_inject_directional
    const float len = sqrtf((l[0] * l[0] + l[1] * l[1]) + l[2] * l[2]);
    if (!(len > 0.0f) || !std::isfinite(len)) return fail(c, VCT_EINVAL, "zero or non-finite light direction");
    l[0] = l[0] / len; l[1] = l[1] / len; l[2] = l[2] / len;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(launch_composite(c, (const float4*)pos4, (const float4*)nrm4, (const float4*)alb4,
                             (const float4*)diffuse4, (const float4*)spec4, w, h, l, color, (float4*)out_linear4,
                             out_rgba8),
            "composite");
    return VCT_OK;
}

vct_status vct_device_alloc(vct_ctx* c, size_t bytes, void** dptr) {
    if (!c || !dptr || bytes == 0) return VCT_EINVAL;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(hipMalloc(dptr, bytes), "hipMalloc");
    return VCT_OK;
}

vct_status vct_device_free(vct_ctx* c, void* dptr) {
    if (!c) return VCT_EINVAL;
    if (!dptr) return VCT_OK;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    VCT_HIP(hipFree(dptr), "hipFree");
    return VCT_OK;
}

vct_status vct_memcpy(vct_ctx* c, void* dst, const void* src, size_t bytes, int kind) {
    if (!c || (!dst && bytes) || (!src && bytes) || kind < 0 || kind > 2) return VCT_EINVAL;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                          : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
    VCT_HIP(hipMemcpyAsync(dst, src, bytes, k, c->stream), "memcpy");
    VCT_HIP(hipStreamSynchronize(c->stream), "memcpy sync");
    return VCT_OK;
}

uint32_t vct_num_levels(const vct_ctx* c) { return c ? c->grid.L + 1 : 0; }

vct_status vct_level_dims(const vct_ctx* c, uint32_t level, uint32_t* n_l, uint32_t* n_faces) {
    if (!c || level > c->grid.L) return VCT_EINVAL;
    if (n_l) *n_l = c->grid.n >> level;
    if (n_faces) *n_faces = (level == 0 || !c->grid.aniso) ? 1 : VCT_NUM_FACES;
    return VCT_OK;
}

vct_status vct_download_level(vct_ctx* c, uint32_t level, uint32_t face, float* host) {
    if (!c || !host || level > c->grid.L) return VCT_EINVAL;
    const uint32_t faces = (level == 0 || !c->grid.aniso) ? 1 : VCT_NUM_FACES;
    if (face >= faces) return fail(c, VCT_EINVAL, "face out of range for level");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    const size_t nl = c->grid.n >> level, vl = nl * nl * nl;
    const float4* src = c->grid.pyr + c->grid.lvl_off[level] + face * vl;
    // the ABI's layout is linear-Z; the pyramid's is vct_device.h's texel layout
    void* tmp;
    VCT_HIP(scratch_get(c, 0, vl * 16, &tmp), "scratch");
    VCT_HIP(launch_relayout(c, src, (float4*)tmp, (uint32_t)nl, true), "relayout");
    VCT_HIP(hipMemcpyAsync(host, tmp, vl * 16, hipMemcpyDeviceToHost, c->stream), "download level");
    VCT_HIP(hipStreamSynchronize(c->stream), "sync");
    return VCT_OK;
}

vct_status vct_upload_level0(vct_ctx* c, const float* host) {
    if (!c || !host) return VCT_EINVAL;
    const size_t nv = (size_t)c->grid.n * c->grid.n * c->grid.n;
    // K4 relies on finite radiance (a terminated lane's fmaf(+0, sample, c) must leave c):
    // refuse Inf / NaN here rather than let them reach other lanes' outputs
    for (size_t i = 0; i < nv * 4; ++i)
        if (!std::isfinite(host[i]))
            return fail(c, VCT_EINVAL, "upload_level0: non-finite value at float " + std::to_string(i));
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    void* tmp;
    VCT_HIP(scratch_get(c, 0, nv * 16, &tmp), "scratch");
    VCT_HIP(hipMemcpyAsync(tmp, host, nv * 16, hipMemcpyHostToDevice, c->stream), "upload level0");
    VCT_HIP(launch_relayout(c, (const float4*)tmp, c->grid.pyr, c->grid.n, false), "relayout");
    VCT_HIP(hipStreamSynchronize(c->stream), "sync");
    c->grid.injected = true;
    c->grid.l0_dense = true;
    c->grid.mipped = false;
    c->grid.l0_on_peers = false;
    return VCT_OK;
}

// the caller may write level 0 through this pointer: the next K2 clears it whole
vct_status vct_level0_device(vct_ctx* c, void** dptr, size_t* bytes) {
    if (!c || !dptr) return VCT_EINVAL;
    *dptr = c->grid.pyr;
    if (bytes) *bytes = (size_t)c->grid.n * c->grid.n * c->grid.n * 16;
    // the caller (e.g. an RCCL broadcast) writes level 0 behind our back
    c->grid.injected = true;
    c->grid.l0_dense = true;
    c->grid.mipped = false;
    c->grid.l0_on_peers = false;
    return VCT_OK;
}

vct_status vct_copy_level0_to_device(vct_ctx* c, void* dst) {
    if (!c || !dst) return VCT_EINVAL;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    const size_t nv = (size_t)c->grid.n * c->grid.n * c->grid.n;
    VCT_HIP(hipMemcpyAsync(dst, c->grid.pyr, nv * 16, hipMemcpyDeviceToDevice, c->stream), "copy level0 out");
    return VCT_OK;
}

vct_status vct_set_level0_from_device(vct_ctx* c, const void* src) {
    if (!c || !src) return VCT_EINVAL;
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    const size_t nv = (size_t)c->grid.n * c->grid.n * c->grid.n;
    VCT_HIP(hipMemcpyAsync(c->grid.pyr, src, nv * 16, hipMemcpyDeviceToDevice, c->stream), "copy level0 in");
    c->grid.injected = true;
    c->grid.l0_dense = true;
    c->grid.mipped = false;
    c->grid.l0_on_peers = false;
    return VCT_OK;
}

vct_status vct_download_voxels(vct_ctx* c, float* albedo_occ4, float* normal4) {
    if (!c) return VCT_EINVAL;
    if (!c->grid.voxelized) return fail(c, VCT_ESTATE, "download_voxels before voxelize");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    const size_t nv = (size_t)c->grid.n * c->grid.n * c->grid.n;
    if (albedo_occ4) VCT_HIP(hipMemcpyAsync(albedo_occ4, c->grid.albedo_occ, nv * 16, hipMemcpyDeviceToHost, c->stream), "download albedo");
    if (normal4) VCT_HIP(hipMemcpyAsync(normal4, c->grid.normal, nv * 16, hipMemcpyDeviceToHost, c->stream), "download normal");
    VCT_HIP(hipStreamSynchronize(c->stream), "sync");
    return VCT_OK;
}

vct_status vct_download_accum(vct_ctx* c, int64_t* sums6, uint32_t* counts) {
    if (!c) return VCT_EINVAL;
    if (!c->grid.voxelized) return fail(c, VCT_ESTATE, "download_accum before voxelize");
    vct_status st = use_device(c);
    if (st != VCT_OK) return st;
    const size_t nv = (size_t)c->grid.n * c->grid.n * c->grid.n;
    // stage the [n^3][8] records through a host buffer, then split
    long long* tmp = new (std::nothrow) long long[nv * 8];
    if (!tmp) return fail(c, VCT_ENOMEM, "host staging");
    hipError_t e = hipMemcpyAsync(tmp, c->grid.accum, nv * 64, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) { delete[] tmp; return hip_fail(c, e, "download accum"); }
    const bool packed = c->grid.accum_packed;
    for (size_t v = 0; v < nv; ++v) {
        const long long* r = tmp + 8 * v;
        if (sums6) {
            if (packed) {   // r + 2^32 g, b + 2^32 nx, ny + 2^32 nz (launch_voxelize)
                for (int k = 0; k < 3; ++k) {
                    const long long lo = (long long)(int32_t)(uint32_t)(unsigned long long)r[k];
                    sums6[6 * v + 2 * k] = lo;
                    sums6[6 * v + 2 * k + 1] = (long long)((unsigned long long)r[k] - (unsigned long long)lo) >> 32;
                }
            } else {
                for (int k = 0; k < 6; ++k) sums6[6 * v + k] = r[k];
            }
        }
        if (counts) counts[v] = (uint32_t)r[packed ? 3 : 6];
    }
    delete[] tmp;
    return VCT_OK;
}

}  // extern "C"
