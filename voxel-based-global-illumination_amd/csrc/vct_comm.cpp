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
//
// Failure detection (RCCL errors surfaced by ncclCommGetAsyncError).
// The communicator is created non-blocking (ncclConfig_t.blocking = 0): every RCCL
// call may return ncclInProgress, and the library polls ncclCommGetAsyncError until
// the call has been issued, for at most the context's deadline (vct_comm_set_timeout,
// default 300 s).  vct_comm_synchronize waits for the queued work the same way,
// polling the stream and the communicator.  On expiry or on an asynchronous error
// the communicator is aborted (ncclCommAbort) and the call returns VCT_ECOMM, so a
// peer that died or never joined ends the frame loop instead of hanging it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
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

// a non-blocking RCCL call: issued (or the communicator aborted) before going on
#define VCT_NCCL(call, where)                                  \
    do {                                                       \
        vct_status s_ = comm_settle(c, (call), where);         \
        if (s_ != VCT_OK) return s_;                           \
    } while (0)

// a call between ncclGroupStart and ncclGroupEnd: deferred to the group end (nothing to
// poll); on an immediate error the group is closed first (RCCL's thread-local group depth
// would otherwise stay raised for the next vct_comm_init on this thread), then aborted
#define VCT_NCCL_IN_GROUP(call, where)                                                          \
    do {                                                                                        \
        const ncclResult_t r_ = (call);                                                         \
        if (r_ != ncclSuccess && r_ != ncclInProgress) {                                        \
            (void)ncclGroupEnd();                                                               \
            return comm_abort(c, std::string(where) + ": " + ncclGetErrorString(r_));           \
        }                                                                                       \
    } while (0)

#define VCT_HIPC(call, where)                                                                          \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return cfail(c, e_ == hipErrorOutOfMemory ? VCT_ENOMEM : VCT_EDEVICE,                      \
                         std::string(where) + ": " + hipGetErrorName(e_));                             \
    } while (0)

ncclComm_t comm_of(const vct_ctx* c) { return (ncclComm_t)c->comm; }

using Clock = std::chrono::steady_clock;

Clock::time_point deadline_of(const vct_ctx* c) {
    return Clock::now() + std::chrono::milliseconds(c->comm_timeout_ms);
}

// the communicator is unusable: abort it (frees its resources without waiting for peers)
vct_status comm_abort(vct_ctx* c, const std::string& why) {
    if (c->comm) (void)ncclCommAbort(comm_of(c));
    c->comm = nullptr;
    c->comm_rank = 0;
    c->comm_size = 1;
    return cfail(c, VCT_ECOMM, why + " (communicator aborted; vct_comm_init again)");
}

// after a non-blocking RCCL call: poll until it has been issued (ncclInProgress -> done)
vct_status comm_settle(vct_ctx* c, ncclResult_t r, const char* where) {
    if (r != ncclSuccess && r != ncclInProgress) return comm_abort(c, std::string(where) + ": " + ncclGetErrorString(r));
    const Clock::time_point end = deadline_of(c);
    for (;;) {
        ncclResult_t a = ncclSuccess;
        if (ncclCommGetAsyncError(comm_of(c), &a) != ncclSuccess) return comm_abort(c, std::string(where) + ": GetAsyncError failed");
        if (a == ncclSuccess) return VCT_OK;
        if (a != ncclInProgress) return comm_abort(c, std::string(where) + ": " + ncclGetErrorString(a));
        if (Clock::now() > end) return comm_abort(c, std::string(where) + ": timed out");
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

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
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;                  // returns at once; the join is polled below with a deadline
    const ncclResult_t r = ncclCommInitRankConfig(&comm, (int)nranks, uid, (int)rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        if (comm) (void)ncclCommAbort(comm);
        return nccl_fail(c, r, "ncclCommInitRankConfig");
    }
    c->comm = comm;
    c->comm_rank = (int)rank;
    c->comm_size = (int)nranks;
    return comm_settle(c, ncclSuccess, "ncclCommInitRankConfig (waiting for every rank)");
}

vct_status vct_comm_set_timeout(vct_ctx* c, uint32_t timeout_ms) {
    if (!c || timeout_ms == 0) return VCT_EINVAL;
    c->comm_timeout_ms = timeout_ms;
    return VCT_OK;
}

vct_status vct_comm_synchronize(vct_ctx* c) {
    if (!c) return VCT_EINVAL;
    if (!c->comm) return cfail(c, VCT_ESTATE, "comm_synchronize before comm_init");
    VCT_HIPC(hipSetDevice(c->device), "hipSetDevice");
    const Clock::time_point end = deadline_of(c);
    for (;;) {
        // the current stream, and the last frame exchange on any stream (each exchange is
        // ordered after the previous one, so its end event covers them all: xchg_enter)
        hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess && c->xchg_done) q = hipEventQuery(c->xchg_done);
        ncclResult_t a = ncclSuccess;
        if (ncclCommGetAsyncError(comm_of(c), &a) != ncclSuccess || (a != ncclSuccess && a != ncclInProgress))
            return comm_abort(c, std::string("comm_synchronize: ") + ncclGetErrorString(a));
        if (q == hipSuccess) return VCT_OK;
        if (q != hipErrorNotReady) return cfail(c, VCT_EDEVICE, std::string("comm_synchronize: ") + hipGetErrorName(q));
        if (Clock::now() > end) return comm_abort(c, "comm_synchronize: timed out");
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

vct_status vct_comm_frame_layout(uint32_t width, uint32_t height, uint32_t nranks, uint32_t rank, int32_t root,
                                 vct_comm_layout* out) {
    if (!out || nranks == 0 || rank >= nranks || width == 0 || height == 0) return VCT_EINVAL;
    if (root != VCT_ALL_RANKS && (root < 0 || (uint32_t)root >= nranks)) return VCT_EINVAL;
    const bool all = root == VCT_ALL_RANKS;
    const uint32_t T = vct_tiles_for_rank(width, height, 0, 1);
    const uint32_t mine = vct_tiles_for_rank(width, height, rank, nranks);
    const uint32_t maxt = vct_tiles_for_rank(width, height, 0, nranks);
    // packed: [2 planes][tiles(r)] per rank at tile offset 2 * prefix(r); all-gather: [R][2][max_tiles]
    out->buffer_tiles = all ? (uint64_t)nranks * 2 * maxt : (uint64_t)2 * T;
    out->diffuse_tile = all ? (uint64_t)rank * 2 * maxt : (uint64_t)2 * vct_tile_offset(width, height, rank, nranks);
    out->spec_tile = out->diffuse_tile + (all ? maxt : mine);
    out->tiles = mine;
    out->exchange_tiles = all ? 2 * maxt : 2 * mine;
    return VCT_OK;
}

vct_status vct_comm_destroy(vct_ctx* c) {
    if (!c) return VCT_EINVAL;
    if (!c->comm) return VCT_OK;
    VCT_HIPC(hipSetDevice(c->device), "hipSetDevice");
    // flush the issued work (non-blocking: polled with the deadline), then free
    vct_status st = comm_settle(c, ncclCommFinalize(comm_of(c)), "ncclCommFinalize");
    if (st != VCT_OK) return st;           // aborted already
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
    vct_comm_layout L;
    if (vct_comm_frame_layout(a->width, a->height, R, me, root, &L) != VCT_OK) return cfail(c, VCT_EINVAL, "layout");
    VCT_HIPC(hipSetDevice(c->device), "hipSetDevice");
    void* gp = nullptr;
    VCT_HIPC(xchg_enter(c), "stream wait (previous exchange)");
    XchgScope xs{c};                           // every exit below records the exchange's end
    VCT_HIPC(scratch_get(c, 8, L.buffer_tiles * tpx * sizeof(float4) + 256, &gp), "comm gather buffer");
    float4* g = (float4*)gp;
    const uint32_t mine = L.tiles;
    vct_trace_args t = *a;
    t.tile_rank = me;
    t.tile_world = R;
    t.tile_compact = 1;
    t.diffuse4 = (float*)(g + L.diffuse_tile * tpx);
    t.spec4 = (float*)(g + L.spec_tile * tpx);
    vct_status st = VCT_OK;
    if (mine) {
        st = vct_trace_device(c, &t);
        if (st != VCT_OK) return st;
    }
    float* frames[2] = {a->diffuse4, a->spec4};
    if (all) {
        if (R > 1)
            VCT_NCCL(ncclAllGather(g + L.diffuse_tile * tpx, g, (size_t)L.exchange_tiles * tpx * 4, ncclFloat32,
                                   comm_of(c), c->stream),
                     "ncclAllGather tiles");
        st = vct_untile_planes_device(c, (const float*)g, 2, a->width, a->height, R, frames);
    } else {
        if (R > 1) {
            VCT_NCCL(ncclGroupStart(), "ncclGroupStart");
            if ((int)me == root) {
                for (uint32_t r = 0; r < R; ++r) {
                    vct_comm_layout Lr;
                    (void)vct_comm_frame_layout(a->width, a->height, R, r, root, &Lr);
                    if (r == me || Lr.tiles == 0) continue;
                    VCT_NCCL_IN_GROUP(ncclRecv(g + Lr.diffuse_tile * tpx, (size_t)Lr.exchange_tiles * tpx * 4,
                                               ncclFloat32, (int)r, comm_of(c), c->stream),
                                      "ncclRecv tiles");
                }
            } else if (mine) {
                VCT_NCCL_IN_GROUP(ncclSend(g + L.diffuse_tile * tpx, (size_t)L.exchange_tiles * tpx * 4, ncclFloat32,
                                           root, comm_of(c), c->stream),
                                  "ncclSend tiles");
            }
            VCT_NCCL(ncclGroupEnd(), "ncclGroupEnd");
        }
        if ((int)me == root)
            st = vct_untile_planes_packed_device(c, (const float*)g, 2, a->width, a->height, R, frames);
    }
    if (st != VCT_OK) return st;
    VCT_HIPC(xchg_leave(c), "event record (exchange end)");
    xs.done = true;
    return VCT_OK;
}

}  // extern "C"
