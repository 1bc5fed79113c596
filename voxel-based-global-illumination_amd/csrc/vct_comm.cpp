// vct_comm.cpp — RCCL exchange of the multi-GPU frame behind include/vct.h
// (SURVEY.md 8e), for a C/C++ host that runs one process per GPU without torch.
//
// The reference engine is one GL thread (engine.cpp:140-157); a host that wants
// the 8-GPU frame starts one process per GPU, creates one vct_ctx in each, and
// joins them with one RCCL communicator:
//   rank 0: vct_comm_get_id(&id)  -> hands `id` to the other processes (file, pipe, MPI, ...)
//   every rank: vct_comm_init(ctx, &id, nranks, rank)
//   light change: rank `root` runs vct_inject_directional, then every rank
//                 vct_comm_broadcast_level0(ctx, root) and vct_build_mips(ctx)
//   per frame:    vct_comm_trace_frame(ctx, &args, root)
// vct_comm_trace_frame traces the rank's interleaved 64x64 tiles (tile t ->
// rank t % nranks) into the rank's slice of a packed tile buffer, then
//  * root >= 0: the other ranks send their slices to `root` (ncclSend / ncclRecv
//    in one group; each rank moves only its own tiles, over its own xGMI link),
//    and `root` un-permutes them into args->diffuse4 / spec4;
//  * root == VCT_ALL_RANKS: one ncclAllGather of the equal-size (padded) rank
//    buffers, and every rank un-permutes the whole frame.
// Everything runs on the ctx stream; the call returns once it is queued.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstring>
#include <string>
#include "vct_internal.h"

using namespace vct;

namespace {

vct_status cfail(vct_ctx* c, vct_status s, const std::string& m) {
    if (c) c->err = m;
    return s;
}

vct_status nccl_fail(vct_ctx* c, ncclResult_t r, const char* where) {
    return cfail(c, VCT_ECOMM, std::string(where) + ": " + ncclGetErrorString(r));
}

#define VCT_NCCL(call, where)                              \
    do {                                                   \
        ncclResult_t r_ = (call);                          \
        if (r_ != ncclSuccess) return nccl_fail(c, r_, where); \
    } while (0)

#define VCT_HIPC(call, where)                                                                          \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return cfail(c, e_ == hipErrorOutOfMemory ? VCT_ENOMEM : VCT_EDEVICE,                      \
                         std::string(where) + ": " + hipGetErrorName(e_));                             \
    } while (0)

ncclComm_t comm_of(const vct_ctx* c) { return (ncclComm_t)c->comm; }

}  // namespace

extern "C" {

vct_status vct_comm_get_id(vct_comm_id* out) {
    if (!out) return VCT_EINVAL;
    static_assert(sizeof(vct_comm_id) == sizeof(ncclUniqueId), "vct_comm_id must hold an ncclUniqueId");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return VCT_ECOMM;
    std::memcpy(out, &id, sizeof id);
    return VCT_OK;
}

vct_status vct_comm_init(vct_ctx* c, const vct_comm_id* id, uint32_t nranks, uint32_t rank) {
    if (!c || !id || nranks == 0 || rank >= nranks) return VCT_EINVAL;
    if (c->comm) return cfail(c, VCT_ESTATE, "comm_init: the context already has a communicator");
    if (!c->peers.empty()) return cfail(c, VCT_EINVAL, "comm_init: a vct_create_multi context exchanges by peer copies");
    VCT_HIPC(hipSetDevice(c->device), "hipSetDevice");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclComm_t comm = nullptr;
    VCT_NCCL(ncclCommInitRank(&comm, (int)nranks, uid, (int)rank), "ncclCommInitRank");
    c->comm = comm;
    c->comm_rank = (int)rank;
    c->comm_size = (int)nranks;
    return VCT_OK;
}

vct_status vct_comm_destroy(vct_ctx* c) {
    if (!c) return VCT_EINVAL;
    if (!c->comm) return VCT_OK;
    VCT_HIPC(hipSetDevice(c->device), "hipSetDevice");
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    const ncclResult_t r = ncclCommDestroy(comm_of(c));
    c->comm = nullptr;
    c->comm_rank = 0;
    c->comm_size = 1;
    if (r != ncclSuccess) return nccl_fail(c, r, "ncclCommDestroy");
    return VCT_OK;
}

vct_status vct_comm_rank(const vct_ctx* c, uint32_t* rank, uint32_t* nranks) {
    if (!c) return VCT_EINVAL;
    if (rank) *rank = (uint32_t)c->comm_rank;
    if (nranks) *nranks = (uint32_t)c->comm_size;
    return VCT_OK;
}

vct_status vct_comm_broadcast_level0(vct_ctx* c, uint32_t root) {
    if (!c) return VCT_EINVAL;
    if (!c->comm) return cfail(c, VCT_ESTATE, "broadcast_level0 before comm_init");
    if ((int)root >= c->comm_size) return cfail(c, VCT_EINVAL, "broadcast_level0: root out of range");
    const bool is_root = (int)root == c->comm_rank;
    if (is_root && !c->grid.injected) return cfail(c, VCT_ESTATE, "broadcast_level0: root has no level 0 (inject first)");
    VCT_HIPC(hipSetDevice(c->device), "hipSetDevice");
    const size_t nv = (size_t)c->grid.n * c->grid.n * c->grid.n;
    // level 0 is the first n^3 float4 of the pyramid: broadcast in place
    VCT_NCCL(ncclBroadcast(c->grid.pyr, c->grid.pyr, nv * 4, ncclFloat32, (int)root, comm_of(c), c->stream),
             "ncclBroadcast level 0");
    if (!is_root) {
        c->grid.injected = true;
        c->grid.l0_dense = true;    // replaced densely: the next K2 clears it whole
    }
    c->grid.mipped = false;
    return VCT_OK;
}

vct_status vct_comm_trace_frame(vct_ctx* c, const vct_trace_args* a, int32_t root) {
    if (!c || !a) return VCT_EINVAL;
    if (!c->comm) return cfail(c, VCT_ESTATE, "trace_frame before comm_init");
    if (root != VCT_ALL_RANKS && (root < 0 || root >= c->comm_size))
        return cfail(c, VCT_EINVAL, "trace_frame: root out of range");
    if (a->tile_world > 1 || a->tile_compact) return cfail(c, VCT_EINVAL, "trace_frame sets the tiling itself");
    if (a->width == 0 || a->height == 0 || a->width > 65536 || a->height > 65536 ||
        (uint64_t)a->width * a->height > 0xffffffffull)   // K4 indexes pixels with 32 bits
        return cfail(c, VCT_EINVAL, "bad frame size");
    const uint32_t R = (uint32_t)c->comm_size, me = (uint32_t)c->comm_rank;
    const bool all = root == VCT_ALL_RANKS;
    const size_t tpx = (size_t)VCT_TILE * VCT_TILE;
    const uint32_t T = vct_tiles_for_rank(a->width, a->height, 0, 1);
    const uint32_t mine = vct_tiles_for_rank(a->width, a->height, me, R);
    const uint32_t maxt = vct_tiles_for_rank(a->width, a->height, 0, R);
    // packed: [2 planes][tiles(r)] per rank at tile offset 2 * prefix(r); all-gather: [R][2][max_tiles]
    const size_t buf_tiles = all ? (size_t)R * 2 * maxt : (size_t)2 * T;
    VCT_HIPC(hipSetDevice(c->device), "hipSetDevice");
    void* gp = nullptr;
    VCT_HIPC(scratch_get(c, 8, buf_tiles * tpx * sizeof(float4) + 256, &gp), "comm gather buffer");
    float4* g = (float4*)gp;
    const size_t off = all ? (size_t)me * 2 * maxt : (size_t)2 * vct_tile_offset(a->width, a->height, me, R);
    const size_t plane = all ? maxt : mine;
    vct_trace_args t = *a;
    t.tile_rank = me;
    t.tile_world = R;
    t.tile_compact = 1;
    t.diffuse4 = (float*)(g + off * tpx);
    t.spec4 = (float*)(g + (off + plane) * tpx);
    vct_status st = VCT_OK;
    if (mine) {
        st = vct_trace_device(c, &t);
        if (st != VCT_OK) return st;
    }
    float* frames[2] = {a->diffuse4, a->spec4};
    if (all) {
        if (R > 1)
            VCT_NCCL(ncclAllGather(g + off * tpx, g, (size_t)2 * maxt * tpx * 4, ncclFloat32, comm_of(c), c->stream),
                     "ncclAllGather tiles");
        return vct_untile_planes_device(c, (const float*)g, 2, a->width, a->height, R, frames);
    }
    if (R > 1) {
        VCT_NCCL(ncclGroupStart(), "ncclGroupStart");
        if ((int)me == root) {
            for (uint32_t r = 0; r < R; ++r) {
                const uint32_t nt = vct_tiles_for_rank(a->width, a->height, r, R);
                if (r == me || nt == 0) continue;
                const size_t o = (size_t)2 * vct_tile_offset(a->width, a->height, r, R);
                VCT_NCCL(ncclRecv(g + o * tpx, (size_t)2 * nt * tpx * 4, ncclFloat32, (int)r, comm_of(c), c->stream),
                         "ncclRecv tiles");
            }
        } else if (mine) {
            VCT_NCCL(ncclSend(g + off * tpx, (size_t)2 * mine * tpx * 4, ncclFloat32, root, comm_of(c), c->stream),
                     "ncclSend tiles");
        }
        VCT_NCCL(ncclGroupEnd(), "ncclGroupEnd");
    }
    if ((int)me != root) return VCT_OK;
    return vct_untile_planes_packed_device(c, (const float*)g, 2, a->width, a->height, R, frames);
}

}  // extern "C"
