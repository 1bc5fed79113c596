// vct_internal.h — context object and kernel launchers behind include/vct.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>
#include "../../include/vct.h"
#include "vct_device.h"
#include "vct_variants.h"

namespace vct {

// Device-resident state of one context.  Everything lives in HBM for the life
// of the context; nothing is re-allocated per frame.
struct Grid {
    uint32_t n = 0, L = 0;
    int aniso = 1;
    float g0[3] = {0, 0, 0};
    float extent = 1.0f;
    float inv_h = 1.0f;
    // radiance pyramid: ONE allocation, level 0 (isotropic) then levels 1..L,
    // each level = faces x n_l^3 float4 texels, linear-Z inside a face volume.
    float4* pyr = nullptr;
    uint64_t lvl_off[kMaxLevels + 1] = {};   // float4 offset of each level
    uint64_t pyr_texels = 0;
    // K1 state
    long long* accum = nullptr;      // [n^3][8] int64: albedo rgb, normal xyz, count, pad
    bool accum_packed = false;       // the last K1 packed its sums (r+2^32 g, b+2^32 nx, ny+2^32 nz, count)
    float4* albedo_occ = nullptr;    // [n^3] (albedo rgb, occupancy)
    float4* normal = nullptr;        // [n^3] (unit normal, 0)
    unsigned long long* occ_bits = nullptr;  // [n^3 / 64] occupancy bitmask
    uint32_t* occ_list = nullptr;            // [n^3] the occupied voxels of the last K1 (k2_list order)
    uint32_t* occ_count = nullptr;           // [1] entries of occ_list
    // K4 empty-space maps (vct_mips.hip, rebuilt by every build_mips): b0 = one bit per
    // level-0 texel, set iff the texel is not +0 (bit order = the texel's index in the brick
    // layout, so byte v = the eight children of level-1 texel v); occ = per level m >= 2 one
    // byte per texel, nonzero iff some level-0 texel under it is; zmap = per level m = 1..zm_levels
    // one bit per position p in [-1, n_m - 1]^3 (stored at p + 1), set iff any level-m texel of
    // p + {0,1}^3 may be nonzero.  A level-l trilinear footprint at corner c lies under the
    // level-(l+1) texels c >> 1 + {0,1}^3, so a clear bit of map l+1 at c >> 1 proves the
    // footprint's texels (every face) are +0.
    static constexpr int kZLevels = 5;
    uint32_t* b0 = nullptr;                  // [n^3 / 32]
    uint8_t* occ = nullptr;                  // levels 2..zm_levels, byte per texel, back to back
    uint64_t occ_off[kZLevels + 1] = {};     // byte offset of level m in occ (m >= 2)
    uint32_t* zmap = nullptr;                // maps 1..zm_levels, back to back
    uint32_t zm_off[kZLevels + 1] = {};      // dword offset of map m
    uint32_t zm_dim[kZLevels + 1] = {};      // n_m + 1 positions per axis
    uint32_t zm_rw[kZLevels + 1] = {};       // dwords per row of map m
    int zm_levels = 0;
    bool zm_valid = false;                   // the maps describe the current pyramid
    // Relight builds (vct_mips.hip launch_mips): after K2, level 0 is nonzero exactly at
    // the occupied voxels (every one gets alpha 1, every other voxel is +0), a pattern only
    // K1 changes.  k3_live[b] = 1 iff K3's first-launch block b (k3_live_bz its depth)
    // holds an occupied voxel.  k3_sparse_ok: the last K3 build ran on such a level 0 for
    // the current occupancy, so every level >= 1 texel and b0 bit above a non-live block is
    // +0 / 0 and the K4 maps are current; the next build from a K2 level 0 may then skip
    // the non-live blocks and the maps.  Cleared by K1 and by any dense level-0 write.
    uint8_t* k3_live = nullptr;              // [n^3 / 256] live flag per block
    uint32_t* k3_live_list = nullptr;        // [n^3 / 1024] + count: the live blocks (any order)
    uint32_t k3_live_count = 0;              // host copy, read back with K1's error word
    int k3_live_bz = 0;
    bool k3_sparse_ok = false;
    // K2's coarse occupancy bits (one per brick of (n/64)^3 voxels, 64-bit rows): from K1's
    // occupancy, so built by the first K2 after each K1 and reused by the next ones
    uint32_t* k2_coarse = nullptr;           // [2 * 64 * 64]
    bool k2_coarse_ok = false;
    bool voxelized = false, injected = false, mipped = false;
    bool l0_dense = false;   // level 0 was replaced densely (upload / device copy): K2 must clear it whole
    bool l0_on_peers = false;   // multi-device: the other devices hold this level 0 (vct_build_mips copies it)
};

struct Mesh {
    float4* tri = nullptr;        // [n_tri][4] : v0, e1 = v1-v0, e2 = v2-v0, (kd rgb, diffuse map as int bits; -1 none)
    float4* uv = nullptr;         // [n_tri][2] : (u0 v0 u1 v1), (u2 v2 0 0)  (textured voxelizations)
    uint32_t n_tri = 0;
    size_t cap = 0, uv_cap = 0;
    bool textured = false;        // the last voxelization had mapped materials (uv is valid)
};

// diffuse maps of vct_set_textures (vct_spec.h "diffuse maps")
struct Textures {
    uint32_t* texels = nullptr;   // every texture's RGBA8 texels, back to back
    TexDesc* desc = nullptr;      // [n] offset / size
    uint32_t n = 0;
    size_t texel_cap = 0, desc_cap = 0;
};

struct Scratch {
    void* p = nullptr;
    size_t bytes = 0;
};

// K4's per-launch scratch, one set per stream: K4 launches on different streams may run
// concurrently (a host that overlaps consecutive frames), so the cone-split hand-over
// and the ray-reorder buffers belong to the stream, not to the context.
enum { kScFlags = 0, kScHand = 1, kScKeys = 2, kScSort = 3, kScOrder = 4, kScN = 5 };
struct StreamScratch {
    hipStream_t s = nullptr;
    bool used = false;
    Scratch sc[kScN];
};
constexpr int kStreamSets = 4;

// K4 candidate choice (vct_trace.hip k4_form).  The default cone trace has two
// bit-identical compiled forms: the four-face-union form (4 waves/SIMD; pays on curved
// surfaces, where a wave's lanes straddle an axis) and the occupancy form (5 waves/SIMD,
// three-face bricks; pays on flat ones); a one-rank full frame may also be traced in
// screen order or with ray reordering (pays on incoherent G-buffers).  Candidate
// c = form | reordered << 1, over the dimensions the variant leaves open.
//
// One entry per workload (frame size, tiling, cone set, grid size, forced bits), kept in
// a small LRU table so that a host alternating workloads (two G-buffers, counting and
// plain launches, two frame sizes) keeps every choice.  A new entry times each candidate
// on its first counter-free launches (HIP events on the ctx stream; while timing, a
// launch first waits for the previous timed launch of that entry, so the choice is made
// within ~7 launches even when the host queues frames far ahead), then keeps the
// fastest.  After that the launch path never blocks: every kWatchEvery-th launch of the
// chosen candidate is timed with an event pair polled by hipEventQuery.  The entry times
// its candidates again only when (a) kDriftRuns consecutive samples run more than kDrift
// times the settled time (the G-buffer or the scene changed what is fastest), or (b) a
// new voxelization (scene) has happened and the entry has run `epoch_wait` launches
// since its last timing; epoch_wait starts at kEpochMin and doubles (up to kEpochMax)
// each time such a re-timing keeps the same winner, so a host that re-voxelizes every
// frame re-times rarely once the choice is stable.  A re-timing keeps the first sample
// of each candidate (its code is loaded already) and drops a candidate after one sample
// that is kCompetitive times slower than the best so far: a much slower candidate
// (screen order on an incoherent G-buffer: 6x) costs one frame per re-timing.
// While timed launches alternate streams (a host overlapping frames, vct.h conventions;
// until 64 launches after the last switch) the entries are not watched (a launch's event
// time then includes whatever share of the chip the neighbouring frames took: measured
// false drifts), and a timing launch first waits for the previous launch of any stream.
// VCT_TUNE_LOG=1 prints every decision to stderr.
struct K4Tuner {
    static constexpr int kSlots = 4;          // event pairs in flight per candidate
    static constexpr int kSamples = 2;        // timed samples per candidate after the first (cold) one
    static constexpr int kEntries = 4;        // workloads remembered (LRU)
    static constexpr uint32_t kWatchEvery = 2;
    static constexpr int kDriftRuns = 3;
    static constexpr float kDrift = 1.35f;
    static constexpr uint32_t kEpochMin = 16, kEpochMax = 4096;
    static constexpr float kCompetitive = 1.5f;
    struct Entry {
        uint64_t key = ~0ull;                 // workload the entry belongs to
        uint64_t used = 0;                    // LRU stamp
        int chosen = -1;                      // the candidate kept; -1 still timing
        float settled = 0.0f;                 // chosen candidate's time when it was chosen, ms
        int drift = 0;                        // consecutive slow watch samples
        uint32_t since = 0;                   // launches since the choice
        uint32_t launches = 0;                // timed launches while choosing
        uint32_t retimes = 0;                 // re-timings after the first choice
        uint32_t epoch = 0;                   // vct_ctx::grid_epoch the choice was made on
        uint32_t epoch_wait = kEpochMin;      // launches before a new scene re-times the entry
        int prev = -1;                        // the winner before this timing (-1: none)
        bool by_epoch = false;                // this timing was started by a new scene
        hipEvent_t ev[4][kSlots][2] = {};
        bool busy[4][kSlots] = {};
        int head[4] = {0, 0, 0, 0};
        int seen[4] = {0, 0, 0, 0};           // completed samples (the first one of a first timing is dropped)
        float best[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // fastest completed sample, ms
        hipEvent_t last = nullptr;            // end event of the previous timed launch while timing
        // longest-first dispatch (launch_trace): the chosen candidate's per-unit wave durations,
        // recorded by every timed launch; the next one dispatches each XCD's units longest first
        uint32_t* hist = nullptr;             // [hist_cap] s_memrealtime ticks per unit (device)
        uint32_t hist_cap = 0, hist_units = 0;
        int hist_cand = -1;                   // candidate (form | order) the durations belong to
        bool hist_ok = false;                 // a recording launch has been queued
    };
    Entry e[kEntries];
    int cur = -1;                             // entry of the last launch (vct_trace_form)
    uint64_t clock = 0;
    // concurrent frames: once timed launches have come on two streams, each one records
    // `prev_end`, and a timing launch first waits for it (samples stay isolated)
    static constexpr uint64_t kMultiLaunches = 64;   // a stream switch counts for this many launches
    hipStream_t prev_stream = nullptr;        // the last timed launch's stream (the null stream is one too)
    bool prev_set = false;                    // prev_stream holds a launch's stream
    hipEvent_t prev_end = nullptr;
    // duration buffers outgrown by a larger workload: a launch on another stream may still
    // write them, so they are freed with the context, not in the launch path
    std::vector<uint32_t*> retired;
    uint64_t multi_until = 0;                 // clock value up to which launches count as overlapped
    bool multi = false;                       // clock < multi_until at the last launch
};

}  // namespace vct

struct vct_ctx {
    vct_config cfg{};
    int device = 0;
    int n_cu = 0;                       // the device's compute units (queried on first use)
    hipStream_t stream = nullptr;
    vct::Grid grid;
    vct::Mesh mesh;
    vct::Textures tex;
    vct::Scratch scratch[12];    // reusable scratch (0 trace host staging, 1 voxelize temps,
                                  // 2-3 G-buffer bins, 4 K2 work list, 7 K1 candidate bucket table,
                                  // 8 multi-device tiles / gather, 9 multi-device step counters)
    vct::StreamScratch k4s[vct::kStreamSets];   // K4 hand-over + reorder scratch per stream (k4_scratch)
    vct::K4Tuner k4tune;                // timed-form choice of the default cone trace
    uint32_t grid_epoch = 0;            // bumped by every voxelization (a new scene for the tuner)
    vct::StepRow* step_tab = nullptr;   // [kMaxStepRows] diffuse-cone step table (device)
    unsigned* spec_keys = nullptr;      // [2 * kSpecSlots]: specular table keys (~0u free), then states
    vct::StepRow* spec_rows = nullptr;  // [kSpecSlots][64] specular step tables (filled by K4)
    const uint32_t* k4_dbg_order = nullptr;   // vct_debug_k4_sched (tools): K4 dispatch order
    uint32_t* k4_dbg_dur = nullptr;           // and per-unit wave durations
    uint64_t k4_lpt_launches = 0;             // launches dispatched longest first (vct_debug_k4_lpt_launches)
    int* k1_err = nullptr;              // device flag of vct_voxelize_device (index out of range)
    // vct_create_multi: this context is device rank 0 and owns one context per
    // further device (ranks 1..n-1); empty for a single-device context
    std::vector<vct_ctx*> peers;
    hipEvent_t ev = nullptr;            // cross-device ordering of the multi-device calls
    // The frame exchanges of trace_multi and vct_comm_trace_frame share scratch slots 8 / 9
    // (and the peers' streams) whatever stream the caller sets: each such call first makes
    // the ctx stream wait for the previous call's end (`xchg_done`, recorded on the stream
    // that call ran on), so frames queued on alternating streams never overlap on the
    // shared buffers; the event of the last call also covers every earlier one
    // (vct_comm_synchronize waits for it).
    hipEvent_t xchg_done = nullptr;
    hipStream_t xchg_stream = nullptr;
    void* comm = nullptr;               // RCCL communicator of vct_comm_init (ncclComm_t), one process per GPU
    int comm_rank = 0, comm_size = 1;
    uint32_t comm_timeout_ms = 300000;  // deadline of every blocking step of vct_comm_* (vct_comm_set_timeout)
    bool own_stream = false;            // stream created by vct_create_multi (destroyed with the ctx)
    std::string err;
};

namespace vct {

// K1
// d_map (device, n_mat entries, may be NULL): diffuse map of each material in c->tex
// (-1 none); uv_offset: byte offset of the TexCoords in a vertex record (read when d_map).
// *d_err (device, zeroed by the caller) collects kK1ErrIndex (an index out of range) and
// kK1ErrRedo (packed sums may have overflowed: repeat with packed = false); nothing is
// read back here, so the launch queues without a synchronisation after the candidate count.
constexpr int kK1ErrIndex = 1, kK1ErrRedo = 2;
hipError_t launch_voxelize(vct_ctx* c, const void* d_verts,
                           uint32_t stride, uint32_t n_verts, const uint32_t* d_idx, uint32_t n_tri,
                           const uint32_t* d_mat, const float4* d_kd, uint32_t n_mat, const int32_t* d_map,
                           uint32_t uv_offset, int* d_err, bool packed = true);
// grid dumps: K1 records [cnt][7] int64 (albedo rgb, normal xyz sums, count) of the voxels
// d_idx (device) -- read out of the accumulators, or written back into them after the
// previous voxelization's sparse reset (bits, occupied list and resolved voxels rebuilt)
hipError_t launch_k1_gather(vct_ctx* c, const uint32_t* d_idx, uint32_t cnt, long long* d_rec);
hipError_t launch_k1_restore(vct_ctx* c, const uint32_t* d_idx, uint32_t cnt, const long long* d_rec);
// K2
hipError_t launch_inject(vct_ctx* c, float lx, float ly, float lz, float cr, float cg, float cb);
// K3 (and the K4 empty-space maps of Grid::zmap)
hipError_t launch_mips(vct_ctx* c);
// K3's live-block list for the occupancy K1 just built (queued on the ctx stream; the count
// reaches g.k3_live_count at the next stream synchronisation)
hipError_t launch_k3_live(vct_ctx* c);
// one nl^3 face volume between the pyramid's texel layout and linear-Z (vct_device.h)
hipError_t launch_relayout(vct_ctx* c, const float4* src, float4* dst, uint32_t nl, bool to_linear);
// K4
hipError_t launch_trace(vct_ctx* c, const vct_trace_args* a);
// ray reordering (variant 0x8000, vct_reorder.hip): *perm = the frame's pixels sorted by the
// Morton code of their cone origin's voxel, background last (device, w * h entries)
// (perm_spec, nullable: a second order for the specular part, by cell and cone aperture)
hipError_t launch_reorder(vct_ctx* c, const vct_trace_args* a, const uint32_t** perm, const uint32_t** perm_spec);
hipError_t launch_untile(vct_ctx* c, const float4* gathered, uint32_t planes, uint32_t w, uint32_t h,
                         uint32_t world, float4* const* frames, bool packed = false);
// composite + present (row f3)
hipError_t launch_composite(vct_ctx* c, const float4* pos, const float4* nrm, const float4* alb,
                            const float4* diff, const float4* spec, uint32_t w, uint32_t h, const float l[3],
                            const float color[3], float4* lin, uint32_t* rgba8);
// G-buffer
hipError_t launch_gbuffer_binned(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h, float rough,
                                 float4* pos, float4* nrm, float4* alb);
hipError_t launch_raycast(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h, float rough,
                          float4* pos, float4* nrm, float4* alb);

uint32_t tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t world);
// dst[j] += sum over i < n of src[2 i + j], j = 0, 1 (a NULL dst is skipped): the
// multi-device trace folds the other devices' step / texel counters into the caller's
hipError_t launch_add_counters(vct_ctx* c, const unsigned long long* src, uint32_t n, unsigned long long* dst0,
                               unsigned long long* dst1);

// K4 step table for aperture tau on an n^3 grid (rows until t > n*sqrt(3), then
// one sentinel row with t = +inf); returns the row count incl. the sentinel, or
// -1 if it exceeds kMaxStepRows
int build_step_table(float tau, uint32_t n, uint32_t L, StepRow* rows);

// scratch helper: grows scratch slot `i` to at least `bytes`
hipError_t scratch_get(vct_ctx* c, int i, size_t bytes, void** out);
// K4 scratch `i` (kSc*) of the ctx's current stream, grown to at least `bytes`; *fresh: it
// was (re)allocated by this call (contents undefined)
hipError_t k4_scratch(vct_ctx* c, int i, size_t bytes, void** out, bool* fresh);
// order a frame exchange (shared slot-8 / 9 scratch) after the previous one on any stream,
// and mark its end (vct_ctx::xchg_done)
hipError_t xchg_enter(vct_ctx* c);
hipError_t xchg_leave(vct_ctx* c);
// an exchange that fails after xchg_enter: record its end anyway, covering the work it
// queued on the ctx stream and the peer streams (XchgScope calls it on every early exit)
void xchg_fail(vct_ctx* c);
struct XchgScope {
    vct_ctx* c;
    bool done = false;                        // set once xchg_leave has succeeded
    ~XchgScope() { if (!done) xchg_fail(c); }
};

}  // namespace vct
