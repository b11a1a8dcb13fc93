// capi.cpp -- the extern "C" boundary of include/atray.h: scene flattening + upload, render
// launches on a HIP stream, progress/wait, and the host prerequisites behind opaque handles.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <fcntl.h>
#include <unistd.h>
#include <cerrno>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "host_scene.h"
#ifdef ATR_DIAG
#include "../../include/atray_diag.h"
#endif

using namespace atr;

extern "C" hipError_t atr_launch_render(const atr::RenderParams& P, int sched, int primary_occ, hipStream_t s);
extern "C" hipError_t atr_launch_traced_finish(unsigned long long* slots, unsigned long long* out, hipStream_t s);
extern "C" hipError_t atr_launch_unpack(const atr::DBlock* blocks, int32_t nblocks, int32_t width,
                                        const uint32_t* packed, uint32_t* image, hipStream_t s);
extern "C" hipError_t atr_launch_path_camera(const atr::PathParams& P, int occ, hipStream_t s);
extern "C" hipError_t atr_launch_path_bounce(const atr::PathParams& P, int ncu, int occ, hipStream_t s);
extern "C" hipError_t atr_launch_path_resolve(const atr::PathParams& P, hipStream_t s);
extern "C" hipError_t atr_launch_path_sort(const atr::PathParams& P, int ncu, hipStream_t s);
extern "C" hipError_t atr_launch_tile_casts(const atr_tile* tiles, int32_t ntiles, int32_t width,
                                            const uint32_t* casts, int64_t* out, hipStream_t s);
extern "C" hipError_t atr_launch_packed_tile_casts(const int32_t* slot_tile, int64_t nslots, const uint32_t* casts,
                                                   int64_t frame_stride, int32_t nframes, int32_t ntiles,
                                                   unsigned long long* out, hipStream_t s);

extern "C" hipError_t atr_launch_plan(const atr::DBlock* base, int32_t nb, unsigned long long* cost,
                                      unsigned long long* cost_last, void* work, atr::DBlock* out, int32_t max_split,
                                      float split2, float split4, hipStream_t s);
extern "C" size_t atr_plan_work_bytes(int32_t nb);
extern "C" hipError_t atr_launch_pack_bgr(const uint32_t* src, int64_t n, uint8_t* dst, hipStream_t s);
extern "C" int64_t atr_masked_chunks(int64_t n);
extern "C" int atr_unpack_max_sources();
extern "C" hipError_t atr_launch_unpack_masked_multi(int32_t n, const atr::DBlock* const* blocks,
                                                     const int32_t* nblocks, const int64_t* own,
                                                     const uint8_t* const* in, const int32_t* raw, int32_t width,
                                                     int32_t nframes, uint32_t* image, int64_t image_stride,
                                                     hipStream_t s);
extern "C" hipError_t atr_launch_unpack_masked(const atr::DBlock* blocks, int32_t nblocks, int32_t width,
                                               const uint8_t* in, int32_t nframes, int64_t own, uint32_t* image,
                                               int64_t image_stride, hipStream_t s);
extern "C" hipError_t atr_launch_pack_bgr_masked(const uint32_t* src, int64_t n, uint32_t bg, uint8_t* out,
                                                 int64_t* nbytes, hipStream_t s);
extern "C" hipError_t atr_launch_scatter_bgr_masked(const uint8_t* in, int64_t n, const int64_t* dst_index,
                                                    uint32_t* image, hipStream_t s);
extern "C" hipError_t atr_launch_scatter_bgr(const uint8_t* src, int64_t n, const int64_t* dst_index,
                                             uint32_t* image, hipStream_t s);

#define HIPCHK(x)                                      \
    do {                                               \
        hipError_t e_ = (x);                           \
        if (e_ != hipSuccess) return -(1000 + int(e_)); \
    } while (0)

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
};

// Blocks for one tile list: the 8x8 cells covering the union of the (inclusive) tile rects,
// each pixel owned exactly once (the reference traces the 1-px overlaps twice, renderer.cpp:429-442).
struct BlockSet {
    std::vector<atr_tile> tiles;
    int32_t width = 0, height = 0;
    std::vector<DBlock> host;
    DevBuf dev;
    DevBuf dev_tiles;
    uint32_t cplan_gen = 0;  // the ctx's cell plan this set was built with
    DevBuf dev_tile;  // owning tile per packed slot (atr_packed_tile_ray_casts; built on first use)
    bool tile_ready = false;
    int64_t packed_pixels = 0;
    // single-frame plan (plan.hip), double-buffered: launch n (parity n & 1) renders from the list
    // planned on the costs of launch n - 2 and writes its per-base-block clocks into its parity's
    // cost half; the plan kernels then run on the context's plan stream, after the render and
    // beside launch n + 1, and rebuild that parity's list from them (plan_ev[parity] after them)
    DevBuf cost, cost_last, plan_work, plan_blocks;
    int32_t max_split = 0;
    bool plan_ready = false;   // a plan was issued on this set (the buffers hold plan state)
    bool plan_valid[2] = {};   // a list is built (or being built) in that parity's half
    hipEvent_t plan_ev[2] = {};
    int plan_par = 0;          // the parity of the next planned launch
    hipStream_t plan_stream = nullptr;
};

// Device scratch freed on every exit path.
struct DevTmp {
    void* p = nullptr;
    ~DevTmp() { if (p) (void)hipFree(p); }
};

uint64_t morton2(uint32_t x, uint32_t y) {
    uint64_t r = 0;
    for (int i = 0; i < 16; ++i) r |= (uint64_t((x >> i) & 1u) << (2 * i)) | (uint64_t((y >> i) & 1u) << (2 * i + 1));
    return r;
}

// first_emit > 0: the pixels of tiles[0, first_emit) are left out (they belong to an earlier
// launch of a progressive render) and only tiles[first_emit, ntiles) emit blocks.
void build_blocks(const atr_tile* tiles, int32_t ntiles, int32_t W, int32_t H, std::vector<DBlock>& out,
                  int64_t& npix, int32_t first_emit = 0, const uint8_t* cplan = nullptr) {
    const int32_t cw = (W + 7) / 8, ch = (H + 7) / 8;
    std::vector<uint64_t> cell(size_t(cw) * size_t(ch), 0), done(first_emit > 0 ? cell.size() : 0, 0);
    // tile order decides the block order: cells are emitted tile by tile (first owner wins)
    std::vector<int32_t> order;
    order.reserve(cell.size());
    std::vector<uint8_t> seen(cell.size(), 0);
    std::vector<int32_t> fresh;
    for (int32_t k = 0; k < ntiles; ++k) {
        atr_tile t = tiles[k];
        fresh.clear();
        if (t.min_x < 0) t.min_x = 0;
        if (t.min_y < 0) t.min_y = 0;
        if (t.max_x > W - 1) t.max_x = W - 1;
        if (t.max_y > H - 1) t.max_y = H - 1;
        if (t.max_x < t.min_x || t.max_y < t.min_y) continue;
        for (int32_t cy = t.min_y / 8; cy <= t.max_y / 8; ++cy)
            for (int32_t cx = t.min_x / 8; cx <= t.max_x / 8; ++cx) {
                const size_t ci = size_t(cy) * size_t(cw) + size_t(cx);
                uint64_t m = 0;
                for (int32_t ly = 0; ly < 8; ++ly) {
                    const int32_t y = cy * 8 + ly;
                    if (y < t.min_y || y > t.max_y) continue;
                    for (int32_t lx = 0; lx < 8; ++lx) {
                        const int32_t x = cx * 8 + lx;
                        if (x >= t.min_x && x <= t.max_x) m |= uint64_t(1) << (ly * 8 + lx);
                    }
                }
                if (k < first_emit) { done[ci] |= m; continue; }
                if (first_emit > 0) m &= ~done[ci];
                if (!m) continue;
                if (!seen[ci]) { seen[ci] = 1; fresh.push_back(int32_t(ci)); }
                cell[ci] |= m;
            }
        // the tile's cells along a Z curve (Morton order): consecutive waves trace a 2D patch and
        // share its leaves in their XCD's L2
        std::stable_sort(fresh.begin(), fresh.end(), [cw](int32_t a, int32_t b) {
                return morton2(uint32_t(a % cw), uint32_t(a / cw)) < morton2(uint32_t(b % cw), uint32_t(b / cw));
            });
        order.insert(order.end(), fresh.begin(), fresh.end());
    }
    out.clear();
    out.reserve(order.size());
    npix = 0;
    bool classes = false;  // some cell has a dispatch class: blocks are reordered after the loop
    for (int32_t ci : order) {
        // cell plan (atr_set_cell_plan): a heavy cell is split into `parts` row bands, one wave
        // each, emitted back to back in lane order (the packed slot order does not change)
        const uint8_t pl = cplan ? cplan[ci] : 0;
        const int parts = (pl & 0xF) >= 2 ? (pl & 0xF) : 1;
        const uint64_t cm = cell[size_t(ci)];
        for (int k = 0; k < parts; ++k) {
            const int rows = 8 / parts;
            const uint64_t band = parts == 1 ? ~uint64_t(0) : ((uint64_t(1) << (8 * rows)) - 1) << (8 * rows * k);
            const uint64_t m = cm & band;
            if (!m) continue;
            DBlock b;
            std::memset(&b, 0, sizeof(b));
            b.x0 = (ci % cw) * 8;
            b.y0 = (ci / cw) * 8;
            b.mask_lo = uint32_t(m);
            b.mask_hi = uint32_t(m >> 32);
            b.out_base = int32_t(npix);
            b.flags = (pl & kPlanPrio) ? kBlockPrio : 0;
            npix += __builtin_popcountll(m);
            out.push_back(b);
            if (pl & kPlanClassMask) classes = true;
        }
    }
    if (classes) {  // dispatch order only: out_base keeps every block's packed slots
        std::stable_sort(out.begin(), out.end(), [&](const DBlock& a, const DBlock& b) {
            return (cplan[size_t(a.y0 / 8) * size_t(cw) + size_t(a.x0 / 8)] & kPlanClassMask) >
                   (cplan[size_t(b.y0 / 8) * size_t(cw) + size_t(b.x0 / 8)] & kPlanClassMask);
        });
    }
    for (size_t i = 0; i < out.size(); ++i) out[i].base = int32_t(i);
}

// load_model_data's pool size (OBJ_loader.cpp:298: one chunk per pool thread): the host's
// hardware threads, at most 16.
int32_t default_parse_threads() {
    const unsigned hw = std::thread::hardware_concurrency();
    return int32_t(std::max(1u, std::min(16u, hw)));
}
#ifndef ATR_MAX_BATCH_LOG2  // experiment builds: 29 to study the 2^29-path cliff
#define ATR_MAX_BATCH_LOG2 28
#endif
#ifndef ATR_PATH_SPLIT_DEFAULT
#define ATR_PATH_SPLIT_DEFAULT 0
#endif
atr_tuning default_tuning() {
    atr_tuning t;
    std::memset(&t, 0, sizeof(t));
    t.xcd_chunk = 16;      // chunks of 16 cells per XCD, interleaved
    t.frame_rotate = 0;    // §4b: rotation measured slower
    t.hybrid_a = 2;        // §4e: sweep optimum
    t.hybrid_b = 0;
    t.path_batch_log2 = 28;  // §4h: 2^28 paths per batch (c4: a frame in one batch, two per batch in flight)
    t.cluster_size = kMaxClusterSize;  // §4b: 8-16 is the flat optimum
    t.frame_plan = 1;      // §4g: single-frame launches dispatch by the previous frame's costs
    t.path_sort_bits = 5;  // §4h: each level's queue in (direction, origin) order, 5 bits per axis
    t.path_split = ATR_PATH_SPLIT_DEFAULT;  // §4h: a one-batch launch as two half batches
    return t;
}
constexpr int kSchedPaths = 10;             // the sample-parallel path engine (paths.hip)
constexpr int kMaxPathBounces = 64;         // bounce launches per batch (AUTO: deeper paths run FLAT)
constexpr int kQueueSlots = 32;             // traced-ray counter sets in flight (ring)
constexpr size_t kTraceBytes = 64 * 128;    // 64 traced-ray counters, 128 B apart (render.hip)

}  // namespace

struct atr_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t last_stream = nullptr;
    // ev_start before every render; its completion event ev_last: the traced-ray set's event of
    // launch_render (one record per launch), or ev_stop for a launch without traced rays
    hipEvent_t ev_start = nullptr, ev_stop = nullptr, ev_last = nullptr;
    bool have_render = false;
    int32_t last_ntiles = 0;
    std::vector<DevBuf> scene_bufs;
    DScene* d_scene = nullptr;
    int64_t scene_bytes = 0;
    int32_t max_nodes = 0, max_depth = 0, nmodels = 0, max_inner = 0;
    float scene_box[6] = {0.f, 0.f, 0.f, 1.f, 1.f, 1.f};  // the models' vertex bounds (lo, hi): queue-sort cells
    atr_tuning tune = default_tuning();  // atr_set_tuning
    int64_t nclusters = 0;
    // per-cell plan (atr_set_cell_plan) for images of cplan_w x cplan_h; cplan_gen invalidates
    // the block cache
    std::vector<uint8_t> cplan;
    int32_t cplan_w = 0, cplan_h = 0;
    uint32_t cplan_gen = 0;
    static constexpr int kBlockSlots = 24;  // tile-list cache: own render + one unpack per rank
    BlockSet blocks[kBlockSlots];
    uint64_t block_use[kBlockSlots] = {};
    uint64_t use_clock = 0;
    int32_t* d_error = nullptr;
    int ncu = 256;
    // path engine workspace per stream (paths.hip: two path queues, the per-path results and the
    // per-level counters), grown on demand
    struct PathWS {
        hipStream_t stream = nullptr;
        DevBuf mem;
        int64_t cap = 0;
        int32_t levels = 0;
        int64_t sort_bins = 0;    // queue-sort buffers for this many bins (PathSort), or none
        hipEvent_t ev = nullptr;  // recorded after the latest launch that used `mem`
        uint64_t last_use = 0;
    };
    static constexpr size_t kMaxPathWS = 4;  // workspaces at most (streams beyond share them)
    // a one-batch PATHS launch runs as two half batches on these streams (fork / join events)
    hipStream_t split_stream[2] = {};
    hipEvent_t split_fork = nullptr, split_join[2] = {};
    uint64_t ws_clock = 0;
    std::vector<PathWS> path_ws;
    // launches' traced-ray counter sets: a ring, each set reused only after the launch that last
    // used it (event) has finished; zeroed by its finish kernel
    void* tring = nullptr;
    hipEvent_t tev[kQueueSlots] = {};
    bool tused[kQueueSlots] = {};
    int tnext = 0;
    // progressive render (atr_render_start_progressive): one launch per tile group, an event
    // after each; prog_end[g] = tiles complete once group g is
    bool prog_active = false;
    std::vector<DevBuf> prog_blocks;
    std::vector<hipEvent_t> prog_ev;
    std::vector<int32_t> prog_end;
    // last launch per stream: everything this context has in flight (scene frees, workspace
    // regrowth and progressive group buffers wait for all of them)
    std::vector<std::pair<hipStream_t, hipEvent_t>> stream_ev;
    int32_t wave_slots = 0;  // CUs x 4 SIMDs x 6 waves (single-frame plan policy), 0 until first use
    hipStream_t plan_side = nullptr;  // the single-frame plan kernels' stream (created on first use)
};

namespace {

// Scheduling knobs of a context (atr_set_tuning); each launch copies them into RenderParams.
void apply_tuning(const atr_ctx* c, RenderParams& P) {
    P.xcd_chunk = c->tune.xcd_chunk;
    P.frame_rotate = 0;
    P.hyb_a = c->tune.hybrid_a;
    P.hyb_b = c->tune.hybrid_b;
}

int dev_upload(atr_ctx* c, const void* src, size_t bytes, void** out) {
    DevBuf b;
    b.n = bytes ? bytes : 16;
    HIPCHK(hipMalloc(&b.p, b.n));
    if (bytes) {
        const hipError_t e = hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(b.p);
            return -(1000 + int(e));
        }
    }
    c->scene_bufs.push_back(b);
    c->scene_bytes += int64_t(b.n);
    *out = b.p;
    return ATR_OK;
}

// Record on stream s, in a (stream, event) list, that work on s is in flight. Entries whose work
// has completed are reused, so a caller that creates a stream per job does not grow the list.
hipError_t note_stream(std::vector<std::pair<hipStream_t, hipEvent_t>>& list, hipStream_t s) {
    for (auto& se : list)
        if (se.first == s) return hipEventRecord(se.second, s);
    for (auto& se : list)
        if (hipEventQuery(se.second) == hipSuccess) {  // finished: take over its event
            se.first = s;
            return hipEventRecord(se.second, s);
        }
    hipEvent_t ev = nullptr;
    hipError_t e;
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    list.emplace_back(s, ev);
    return hipEventRecord(ev, s);
}

// Wait for every entry of a list (all streams).
hipError_t wait_list(const std::vector<std::pair<hipStream_t, hipEvent_t>>& list) {
    for (const auto& se : list) {
        const hipError_t e = hipEventSynchronize(se.second);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Record that a launch on stream s is in flight. (A block set's buffers are rewritten or freed
// only after every stream's latest launch, wait_all: a cache miss or a first per-tile query, rare,
// so launches record no event per block set.) A render whose completion event is one of the
// traced-ray ring's (ring = true) records nothing here: wait_all also waits for every ring event in
// use, and a ring event is re-recorded only on a stream that first waited for its previous record
// (launch_render), so it still covers every launch that recorded it.
hipError_t note_launch(atr_ctx* c, hipStream_t s, bool ring = false) {
    return ring ? hipSuccess : note_stream(c->stream_ev, s);
}

// Wait for every launch of this context still in flight, on any stream.
hipError_t wait_all(atr_ctx* c) {
    hipError_t e = wait_list(c->stream_ev);
    for (int k = 0; e == hipSuccess && k < kQueueSlots; ++k)
        if (c->tused[k]) e = hipEventSynchronize(c->tev[k]);
    return e;
}

void free_scene(atr_ctx* c) {
    for (DevBuf& b : c->scene_bufs) (void)hipFree(b.p);
    c->scene_bufs.clear();
    c->d_scene = nullptr;
    c->scene_bytes = 0;
}

BlockSet* get_blocks(atr_ctx* c, const atr_tile* tiles, int32_t ntiles, int32_t W, int32_t H, int& rc) {
    rc = ATR_OK;
    int lru = 0;
    for (int i = 0; i < atr_ctx::kBlockSlots; ++i) {
        BlockSet& b = c->blocks[i];
        if (b.width == W && b.height == H && int32_t(b.tiles.size()) == ntiles && b.dev.p &&
            b.cplan_gen == c->cplan_gen && (ntiles == 0 || std::memcmp(b.tiles.data(), tiles, sizeof(atr_tile) * size_t(ntiles)) == 0)) {
            c->block_use[i] = ++c->use_clock;
            return &b;
        }
        if (c->block_use[i] < c->block_use[lru]) lru = i;
    }
    BlockSet& b = c->blocks[lru];
    c->block_use[lru] = ++c->use_clock;
    // the slot may still be read by in-flight kernels of earlier renders, on several streams
    {
        const hipError_t e = wait_all(c);
        if (e != hipSuccess) { rc = -(1000 + int(e)); return nullptr; }
    }
    b.tiles.assign(tiles, tiles + ntiles);
    b.tile_ready = false;
    b.plan_ready = false;
    b.width = W;
    b.height = H;
    b.cplan_gen = c->cplan_gen;
    const bool planned = !c->cplan.empty() && c->cplan_w == W && c->cplan_h == H;
    build_blocks(tiles, ntiles, W, H, b.host, b.packed_pixels, 0, planned ? c->cplan.data() : nullptr);
    const size_t need = std::max<size_t>(b.host.size() * sizeof(DBlock), 32);
    if (b.dev.n < need) {
        if (b.dev.p) (void)hipFree(b.dev.p);
        b.dev = DevBuf();
        if (hipMalloc(&b.dev.p, need) != hipSuccess) { rc = ATR_E_NOMEM; return nullptr; }
        b.dev.n = need;
    }
    const size_t tneed = std::max<size_t>(sizeof(atr_tile) * size_t(ntiles), 16);
    if (b.dev_tiles.n < tneed) {
        if (b.dev_tiles.p) (void)hipFree(b.dev_tiles.p);
        b.dev_tiles = DevBuf();
        if (hipMalloc(&b.dev_tiles.p, tneed) != hipSuccess) { rc = ATR_E_NOMEM; return nullptr; }
        b.dev_tiles.n = tneed;
    }
    hipError_t e = hipMemcpy(b.dev.p, b.host.data(), b.host.size() * sizeof(DBlock), hipMemcpyHostToDevice);
    if (e == hipSuccess && ntiles)
        e = hipMemcpy(b.dev_tiles.p, tiles, sizeof(atr_tile) * size_t(ntiles), hipMemcpyHostToDevice);
    if (e != hipSuccess) { rc = -(1000 + int(e)); b.width = -1; return nullptr; }
    return &b;
}

// Grow a device buffer to `bytes` (contents undefined when it grows; zeroed if `zero`).
int ensure_buf(DevBuf& d, size_t bytes, bool zero) {
    if (d.n >= bytes && d.p) return ATR_OK;
    if (d.p) (void)hipFree(d.p);
    d = DevBuf();
    if (hipMalloc(&d.p, bytes) != hipSuccess) return ATR_E_NOMEM;
    d.n = bytes;
    if (zero && hipMemset(d.p, 0, bytes) != hipSuccess) return ATR_E_NOMEM;
    return ATR_OK;
}

// variant (atray.h) -> kernel schedule (render.hip). AUTO = the measured fastest.
// variant (atray.h) -> schedule (render.hip / paths.hip); -1 = not a variant of this build.
int sched_of(int32_t variant) {
    switch (variant) {
        case ATR_KERNEL_LANE: return 0;
        case ATR_KERNEL_FLAT: return 6;
        case ATR_KERNEL_HYBRID: return 7;
        case ATR_KERNEL_PATHS: return kSchedPaths;
        default: return -1;
    }
}

// AUTO: the fastest exact schedule for the camera (measured): primary-only renders
// (one sample, bounce_limit 1, no AA) on HYBRID cells (lane-private leaf scans for coherent rays,
// dealt rounds for the stragglers); everything else on the sample-parallel path engine (a pixel's
// samples side by side, one launch per bounce), or the FLAT cell megakernel for paths deeper than
// its bounce launches.
// -1: not a variant of this build, or a request it cannot run (PATHS beyond its bounce launches):
// every entry point answers ATR_E_INVALID before it changes any state.
int auto_sched(int32_t variant, const atr_camera& cam) {
    if (variant == ATR_KERNEL_PATHS && cam.bounce_limit > kMaxPathBounces) return -1;
    if (variant != ATR_KERNEL_AUTO) return sched_of(variant);
    if (cam.bounce_limit == 1 && !cam.anti_aliasing && cam.samples_per_pixel == 1) return sched_of(ATR_KERNEL_HYBRID);
    return cam.bounce_limit <= kMaxPathBounces ? kSchedPaths : sched_of(ATR_KERNEL_FLAT);
}

// A single-frame launch of a cell schedule with the single-frame plan (tuning frame_plan, plan.hip):
// the render dispatches the block list planned after the previous such launch of this tile list on
// this stream (the base list the first time), adds each cell's clocks into the set's cost buffer,
// and the plan kernels then build the next list from them. Another stream, a user cell plan for the
// size or frame_plan 0 -> the plain base-list launch.
// The render's completion event (ev_last) is recorded right after the render; the plan kernels
// run on the plan stream, so atr_render_wait, atr_last_kernel_ms and the next launch on s do not
// wait for them.
hipError_t launch_render(atr_ctx* c, RenderParams& P, int sched, hipStream_t s, hipEvent_t* done = nullptr);

// One completion record per launch: `done` (the traced-ray set's event launch_render recorded after
// the render) when there is one, else ev_stop.
hipError_t record_stop(atr_ctx* c, hipStream_t s, hipEvent_t done) {
    if (done) {
        c->ev_last = done;
        return hipSuccess;
    }
    c->ev_last = c->ev_stop;
    return hipEventRecord(c->ev_stop, s);
}

int launch_planned(atr_ctx* c, BlockSet* bs, RenderParams& P, int sched, hipStream_t s) {
    const int32_t nb = int32_t(bs->host.size());
    // on top of a user cell plan too: its classes order the base list (and the multi-frame
    // launches), the frame plan re-orders that list for single frames by their measured cost
    const bool use = c->tune.frame_plan && nb > 0 && sched != kSchedPaths &&
                     (!bs->plan_ready || bs->plan_stream == s);
    hipEvent_t done = nullptr;
    if (!use) {
        HIPCHK(launch_render(c, P, sched, s, &done));
        HIPCHK(record_stop(c, s, done));
        return ATR_OK;
    }
    // A launch whose cells fit the chip's wave slots at once (a shard's frame: 4,050 cells of an
    // 8-way c3 plan vs 6,144 slots at 6 waves/SIMD) leaves slots idle while its heaviest cells
    // finish: there the heaviest 3 % take four waves and the next 7 % two, which shortens the
    // frame's critical path at no throughput cost. Larger launches split the heaviest 1 % in two.
    if (!c->wave_slots) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus <= 0)
            cus = 256;
        c->wave_slots = cus * 4 * 6;
    }
    const bool small = nb <= c->wave_slots;
    const float split2 = small ? 0.10f : -1.f, split4 = small ? 0.03f : -1.f;
    const int32_t max_split = std::max<int32_t>(1, small ? nb / 5 : nb / 25);  // spare blocks for splits
    const size_t cap = size_t(nb + max_split);
    int rc;
    const bool fresh = !bs->cost.p;  // the buffers start zeroed; each plan leaves them zeroed
    if ((rc = ensure_buf(bs->cost, 2 * size_t(nb) * sizeof(unsigned long long), true))) return rc;
    if ((rc = ensure_buf(bs->cost_last, size_t(nb) * sizeof(unsigned long long), false))) return rc;
    if ((rc = ensure_buf(bs->plan_work, atr_plan_work_bytes(nb), true))) return rc;
    if ((rc = ensure_buf(bs->plan_blocks, 2 * cap * sizeof(DBlock), false))) return rc;
    if (!c->plan_side) HIPCHK(hipStreamCreateWithFlags(&c->plan_side, hipStreamNonBlocking));
    for (hipEvent_t& e : bs->plan_ev)
        if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!bs->plan_ready && !fresh) {  // a rebuilt set reuses buffers a plan may not have cleared
        HIPCHK(hipMemsetAsync(bs->cost.p, 0, 2 * size_t(nb) * sizeof(unsigned long long), s));
        // and the work area's thresholds (learned on the old list, whose nb and max_split differ):
        // back to the documented zeroed state (class 0, no split) for the first plan on this list
        HIPCHK(hipMemsetAsync(bs->plan_work.p, 0, atr_plan_work_bytes(nb), s));
    }
    if (!bs->plan_ready) {
        bs->plan_valid[0] = bs->plan_valid[1] = false;
        bs->plan_par = 0;
    }
    bs->max_split = max_split;
    const int par = bs->plan_par;
    DBlock* list = static_cast<DBlock*>(bs->plan_blocks.p) + size_t(par) * cap;
    unsigned long long* cost = static_cast<unsigned long long*>(bs->cost.p) + size_t(par) * size_t(nb);
    if (bs->plan_valid[par]) {  // this parity's list, built beside the previous launch, and its cost
        HIPCHK(hipStreamWaitEvent(s, bs->plan_ev[par], 0));  // half cleared by the same kernels
        P.blocks = list;
        P.nblocks = int32_t(cap);
    }
    P.block_cost = cost;
    HIPCHK(launch_render(c, P, sched, s, &done));
    HIPCHK(record_stop(c, s, done));
    HIPCHK(hipStreamWaitEvent(c->plan_side, c->ev_last, 0));
    HIPCHK(atr_launch_plan(static_cast<const DBlock*>(bs->dev.p), nb, cost,
                           static_cast<unsigned long long*>(bs->cost_last.p), bs->plan_work.p, list, max_split,
                           split2, split4, c->plan_side));
    HIPCHK(hipEventRecord(bs->plan_ev[par], c->plan_side));
    HIPCHK(note_stream(c->stream_ev, c->plan_side));
    bs->plan_valid[par] = true;
    bs->plan_par = par ^ 1;
    bs->plan_ready = true;
    bs->plan_stream = s;
    return ATR_OK;
}

// The path engine's workspace for stream s, at least `cap` paths per batch and `levels` bounce
// levels. Each workspace belongs to the stream that used it last; a stream without one takes over
// an idle workspace (its last launch finished), else opens a new one while there are fewer than
// kMaxPathWS, else takes the least recently used one after a GPU-side wait on that workspace's last
// launch. So the total stays bounded however many streams render. Growing a workspace waits for
// its own last launch only. When the device has no memory for it, idle workspaces of other streams
// are released and the allocation retried once; hipErrorOutOfMemory then goes back to the caller
// (launch_paths halves its batch, then drops the queue sort, and launch_kernels falls back to FLAT).
// Queue-sort buffers after the queues and counters (256-B aligned): {key, rank} and the key order
// per entry, then `bins` bins, their starts and block sums.
size_t sort_offset(int64_t cap, int32_t levels) {
    return (size_t(cap) * 16 * (2 * kPathPlanes + 1) + size_t(levels) * sizeof(PathCtl) + 255) & ~size_t(255);
}
size_t sort_bytes(int64_t cap, int64_t bins) {
    return size_t(cap) * 12 + size_t(bins) * 8 + size_t(bins / kSortChunk) * 4;
}

hipError_t path_workspace(atr_ctx* c, hipStream_t s, int64_t cap, int64_t grow_to, int32_t levels, int64_t sort_bins,
                          atr_ctx::PathWS*& out) {
    atr_ctx::PathWS* ws = nullptr;
    hipError_t e;
    for (auto& w : c->path_ws)
        if (w.stream == s) ws = &w;
    if (!ws)
        for (auto& w : c->path_ws)
            if (!ws && w.ev && hipEventQuery(w.ev) == hipSuccess) ws = &w;
    if (!ws && c->path_ws.size() < atr_ctx::kMaxPathWS) {
        c->path_ws.emplace_back();
        ws = &c->path_ws.back();
        if ((e = hipEventCreateWithFlags(&ws->ev, hipEventDisableTiming)) != hipSuccess) return e;
    }
    if (!ws) {
        ws = &c->path_ws[0];
        for (auto& w : c->path_ws)
            if (w.last_use < ws->last_use) ws = &w;
    }
    if (ws->stream != s && ws->mem.p && (e = hipStreamWaitEvent(s, ws->ev, 0)) != hipSuccess) return e;
    ws->stream = s;
    ws->last_use = ++c->ws_clock;
    if (ws->cap < cap || ws->levels < levels || ws->sort_bins < sort_bins) {
        if ((e = hipEventSynchronize(ws->ev)) != hipSuccess) return e;
        if (ws->mem.p && (e = hipFree(ws->mem.p)) != hipSuccess) return e;
        ws->mem = DevBuf();
        // a workspace that already held paths and is too small grows to grow_to (a full batch)
        int64_t ncap = std::max(ws->cap, ws->cap > 0 && ws->cap < cap ? std::max(cap, grow_to) : cap);
        const int32_t nlev = std::max(ws->levels, levels);
        const int64_t nbins = std::max(ws->sort_bins, sort_bins);
        ws->cap = 0;
        ws->levels = 0;
        ws->sort_bins = 0;
        // 2 queues x kPathPlanes planes + the per-path results, 16 B per entry; the level counters;
        // the queue-sort buffers
        auto bytes_for = [&](int64_t n) {
            return nbins ? sort_offset(n, nlev) + sort_bytes(n, nbins)
                         : size_t(n) * 16 * (2 * kPathPlanes + 1) + size_t(nlev) * sizeof(PathCtl);
        };
        size_t bytes = bytes_for(ncap);
        e = hipMalloc(&ws->mem.p, bytes);
        if (e == hipErrorOutOfMemory && ncap > cap) {  // the full batch does not fit: this launch's size
            (void)hipGetLastError();
            ncap = cap;
            bytes = bytes_for(ncap);
            e = hipMalloc(&ws->mem.p, bytes);
        }
        if (e == hipErrorOutOfMemory) {
            (void)hipGetLastError();
            for (auto& w : c->path_ws)
                if (&w != ws && w.mem.p && hipEventQuery(w.ev) == hipSuccess) {
                    (void)hipFree(w.mem.p);
                    w.mem = DevBuf();
                    w.cap = 0;
                    w.levels = 0;
                    w.sort_bins = 0;
                }
            e = hipMalloc(&ws->mem.p, bytes);
        }
        if (e != hipSuccess) {
            (void)hipGetLastError();
            ws->mem = DevBuf();
            return e;
        }
        ws->mem.n = bytes;
        ws->cap = ncap;
        ws->levels = nlev;
        ws->sort_bins = nbins;
    }
    out = ws;
    return hipSuccess;
}

// The sample-parallel path engine (paths.hip) over a cell launch's blocks: the cell list in
// batches of 2^tuning.path_batch_log2 paths, per batch the camera launch, one launch per further
// bounce (persistent waves over the previous level's queue) and the per-pixel resolve, all on s.
hipError_t launch_paths_range(atr_ctx* c, const RenderParams& P, hipStream_t s, int64_t cbeg, int64_t cend) {
    const int64_t spp = P.cam.samples_per_pixel;
    const int32_t bl = P.cam.bounce_limit;
    if (cend <= cbeg) return hipSuccess;
    if (bl > kMaxPathBounces) return hipErrorInvalidValue;
    const int64_t per_cell = 64 * std::max<int64_t>(spp, 1);
    const int32_t levels = std::max(bl, 1);
    // the queue sort pays off only when a level's queue feeds another bounce launch
    int32_t sort_bits = bl >= 2 ? c->tune.path_sort_bits : 0;
    while (sort_bits > 0 && (int64_t(kSortDirs) * kSortDirs << (3 * sort_bits)) > kSortBinsMax) --sort_bits;
    atr_ctx::PathWS* ws = nullptr;
    hipError_t e = hipErrorOutOfMemory;
    int64_t cells = 0;
    // a batch of 2^path_batch_log2 paths, halved while the device cannot hold its workspace (down to
    // 2^16 paths; the outputs do not depend on the batch size); then the same without the queue sort
    for (;;) {
        const int64_t bins = sort_bits > 0 ? int64_t(kSortDirs) * kSortDirs << (3 * sort_bits) : 0;
        for (int32_t lg = c->tune.path_batch_log2; lg >= 16 && e == hipErrorOutOfMemory; --lg) {
            const int64_t batch = std::max<int64_t>(1, (int64_t(1) << lg) / per_cell);
            cells = std::min<int64_t>(batch, cend - cbeg);
            // capacity: this launch's paths rounded up to 2^24 (at most a full batch): a one-frame c4
            // launch holds its 132.7 M paths (21 GB), not a whole 2^28 batch; a workspace that has to
            // grow grows to a full batch at once, so a stream regrows at most once (a regrow inside a
            // timed multi-frame run once measured a 4x slower c4 line, round 6)
            const int64_t need = cells * per_cell, gran = int64_t(1) << 24;
            const int64_t cap = std::max(need, std::min((need + gran - 1) / gran * gran, batch * per_cell));
            e = path_workspace(c, s, cap, std::max(batch * per_cell, cap), std::max(levels, 8), bins, ws);
            if (e == hipSuccess && ws->cap < cap) e = hipErrorOutOfMemory;
        }
        if (e != hipErrorOutOfMemory || sort_bits == 0) break;
        sort_bits = 0;
    }
    if (e != hipSuccess) return e;
    PathParams Q;
    std::memset(&Q, 0, sizeof(Q));
    Q.cam = P.cam;
    Q.scene = P.scene;
    Q.seed = P.seed;
    Q.blocks = P.blocks;
    Q.frame_blocks = P.frame_blocks;
    Q.nblocks = P.nblocks;
    Q.layout = P.layout;
    Q.frame_stride = P.frame_stride;
    Q.framebuffer = P.framebuffer;
    Q.hit_face = P.hit_face;
    Q.hit_t = P.hit_t;
    Q.rgb = P.rgb;
    Q.ray_casts = P.ray_casts;
    Q.traced_rays = P.traced_rays;
    Q.error_flag = P.error_flag;
    Q.block_cost = P.block_cost;
    Q.counters = P.counters;
    float4_t* base = static_cast<float4_t*>(ws->mem.p);
    Q.cap = ws->cap;
    Q.q[0] = base;
    Q.q[1] = base + kPathPlanes * ws->cap;
    Q.out = base + 2 * kPathPlanes * ws->cap;
    Q.ctl = reinterpret_cast<PathCtl*>(base + (2 * kPathPlanes + 1) * ws->cap);
    Q.xcd_chunk = P.xcd_chunk;
    Q.hyb_a = P.hyb_a;
    Q.hyb_b = P.hyb_b;
    Q.nfcam = P.nfcam;
    for (int32_t f = 0; f < P.nfcam; ++f) Q.fcam[f] = P.fcam[f];
    if (sort_bits > 0) {
        PathSort& so = Q.sort;
        so.bits = sort_bits;
        so.nbins = int32_t(kSortDirs * kSortDirs) << (3 * sort_bits);
        const float* box = c->scene_box;
        for (int a = 0; a < 3; ++a) {
            so.lo[a] = box[a];
            const float ext = box[3 + a] - box[a];
            so.sc[a] = ext > 0.0f ? float(1 << sort_bits) / ext : 0.0f;
        }
        char* sb = static_cast<char*>(ws->mem.p) + sort_offset(ws->cap, ws->levels);
        so.kr = reinterpret_cast<uint2_t*>(sb);
        sb += size_t(ws->cap) * 8;
        so.perm = reinterpret_cast<uint32_t*>(sb);
        sb += size_t(ws->cap) * 4;
        so.hist = reinterpret_cast<uint32_t*>(sb);
        so.start = so.hist + ws->sort_bins;
        so.part = so.start + ws->sort_bins;
    }
    const int occ_cam = c->tune.path_camera_occ, occ_bounce = c->tune.path_bounce_occ;
    for (int64_t c0 = cbeg; c0 < cend; c0 += cells) {
        Q.cell0 = int32_t(c0);
        Q.ncells = int32_t(std::min<int64_t>(cells, cend - c0));
        if (bl > 0 && spp > 0) {
            if ((e = hipMemsetAsync(Q.ctl, 0, sizeof(PathCtl) * size_t(levels), s)) != hipSuccess) return e;
            if (sort_bits > 0 &&
                (e = hipMemsetAsync(Q.sort.hist, 0, sizeof(uint32_t) * size_t(Q.sort.nbins), s)) != hipSuccess)
                return e;
            if ((e = atr_launch_path_camera(Q, occ_cam, s)) != hipSuccess) return e;
            for (int32_t k = 1; k < bl; ++k) {
                if (sort_bits > 0) {  // level k - 1's queue in key order (the launches zero the bins)
                    Q.bounce = k - 1;
                    if ((e = atr_launch_path_sort(Q, c->ncu, s)) != hipSuccess) return e;
                }
                Q.bounce = k;
                if ((e = atr_launch_path_bounce(Q, c->ncu, occ_bounce, s)) != hipSuccess) return e;
            }
        }
        if ((e = atr_launch_path_resolve(Q, s)) != hipSuccess) return e;
    }
    return hipEventRecord(ws->ev, s);
}

// The path engine over a launch's cell list. With tuning path_split = 1 a launch that is one batch
// (a single frame: c4's 2 M-pixel frame at 64 spp) runs as two half batches on the context's two
// split streams, forked from and joined back into s, so one half's level tails and queue sorts
// could overlap the other half's tracing; off by default (one c4 frame measured 61.1 vs 60.3 ms,
// DESIGN.md §4h). Outputs do not depend on the batching.
constexpr int64_t kSplitMinCells = 1024;
hipError_t launch_paths(atr_ctx* c, const RenderParams& P, hipStream_t s) {
    if (P.nblocks <= 0) return hipSuccess;
    const int64_t per_cell = 64 * std::max<int64_t>(P.cam.samples_per_pixel, 1);
    const int64_t batch = std::max<int64_t>(1, (int64_t(1) << c->tune.path_batch_log2) / per_cell);
    if (!c->tune.path_split || P.nblocks > batch || P.nblocks < kSplitMinCells || P.counters || P.block_cost)
        return launch_paths_range(c, P, s, 0, P.nblocks);
    hipError_t e;
    if (!c->split_fork) {
        for (int i = 0; i < 2; ++i) {
            if ((e = hipStreamCreateWithFlags(&c->split_stream[i], hipStreamNonBlocking)) != hipSuccess) return e;
            if ((e = hipEventCreateWithFlags(&c->split_join[i], hipEventDisableTiming)) != hipSuccess) return e;
        }
        if ((e = hipEventCreateWithFlags(&c->split_fork, hipEventDisableTiming)) != hipSuccess) return e;
    }
    if ((e = hipEventRecord(c->split_fork, s)) != hipSuccess) return e;
    const int64_t half = (P.nblocks + 1) / 2;
    hipError_t r = hipSuccess;
    for (int i = 0; i < 2; ++i) {
        hipStream_t a = c->split_stream[i];
        if ((e = hipStreamWaitEvent(a, c->split_fork, 0)) != hipSuccess) return e;
        if (r == hipSuccess) r = launch_paths_range(c, P, a, i ? half : 0, i ? P.nblocks : half);
        // joined whatever happened, so a fallback render on s runs after anything queued here
        if ((e = hipEventRecord(c->split_join[i], a)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(s, c->split_join[i], 0)) != hipSuccess) return e;
    }
    return r;
}

hipError_t launch_kernels(atr_ctx* c, RenderParams& P, int sched, hipStream_t s) {
    if (sched == kSchedPaths) {
        hipError_t e = launch_paths(c, P, s);
        if (e != hipErrorOutOfMemory) return e;
        // no memory for a path workspace: the cell megakernel, which needs none (same outputs,
        // DESIGN.md §4). A split launch may have rendered its first half already: every output is
        // rewritten, and the traced-ray counters (always a launch's zeroed ring set of 64 spread
        // counters, launch_render) start again from zero so no ray is counted twice.
        if (P.traced_rays && (e = hipMemsetAsync(P.traced_rays, 0, kTraceBytes, s)) != hipSuccess) return e;
        sched = sched_of(ATR_KERNEL_FLAT);
    }
    return atr_launch_render(P, sched, c->tune.primary_occ, s);
}

// Launch a render schedule; the traced rays go into a zeroed set of 64 spread counters from the
// ring, then one add to the caller's accumulator.
hipError_t launch_render(atr_ctx* c, RenderParams& P, int sched, hipStream_t s, hipEvent_t* done) {
    if (done) *done = nullptr;
    if (!P.traced_rays) return launch_kernels(c, P, sched, s);
    const int k = c->tnext;
    c->tnext = (k + 1) % kQueueSlots;
    hipError_t e;
    if (c->tused[k] && (e = hipStreamWaitEvent(s, c->tev[k], 0)) != hipSuccess) return e;
    unsigned long long* caller = P.traced_rays;
    P.traced_rays = reinterpret_cast<unsigned long long*>(static_cast<char*>(c->tring) + size_t(k) * kTraceBytes);
    e = launch_kernels(c, P, sched, s);
    if (e == hipSuccess) e = atr_launch_traced_finish(P.traced_rays, caller, s);
    P.traced_rays = caller;
    if (e != hipSuccess) return e;
    if ((e = hipEventRecord(c->tev[k], s)) != hipSuccess) return e;
    c->tused[k] = true;
    if (done) *done = c->tev[k];
    return hipSuccess;
}

}  // namespace

extern "C" {

const char* atr_version(void) { return "atray-mi355x 0.2 (gfx950)"; }

// ------------------------------------------------------------------ host prerequisites
int atr_mesh_parse_obj_threaded(const char* text, size_t len, int32_t threads, atr_mesh** out) {
    if (!text || !out || threads < 0) return ATR_E_INVALID;
    if (threads == 0) threads = default_parse_threads();
    atr_mesh* m = new (std::nothrow) atr_mesh();
    if (!m) return ATR_E_NOMEM;
    const int rc = parse_obj_text(text, len, m->m, threads);
    if (rc != ATR_OK) { delete m; return rc; }
    *out = m;
    return ATR_OK;
}

int atr_mesh_parse_obj(const char* text, size_t len, atr_mesh** out) {
    return atr_mesh_parse_obj_threaded(text, len, 1, out);
}

int atr_mesh_load_obj_threaded(const char* path, int32_t threads, atr_mesh** out) {
    if (!path || !out || threads < 0) return ATR_E_INVALID;
    FILE* f = std::fopen(path, "rb");
    if (!f) return ATR_E_IO;
    std::string buf;
    if (std::fseek(f, 0, SEEK_END) == 0) {
        const long sz = std::ftell(f);
        if (sz > 0) buf.reserve(size_t(sz));
        std::rewind(f);
    }
    char tmp[1 << 16];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.append(tmp, n);
    const bool bad = std::ferror(f) != 0;
    std::fclose(f);
    if (bad) return ATR_E_IO;
    return atr_mesh_parse_obj_threaded(buf.data(), buf.size(), threads, out);
}

int atr_mesh_load_obj(const char* path, atr_mesh** out) { return atr_mesh_load_obj_threaded(path, 0, out); }

int atr_mesh_from_arrays(const float* vertices, uint32_t nvertices, const int32_t* face_vertices,
                         uint32_t nfaces, const float* normals, uint32_t nnormals,
                         const int32_t* face_normals, atr_mesh** out) {
    if (!out || (nvertices && !vertices) || (nfaces && !face_vertices)) return ATR_E_INVALID;
    if (nnormals && (!normals || !face_normals)) return ATR_E_INVALID;
    atr_mesh* m = new (std::nothrow) atr_mesh();
    if (!m) return ATR_E_NOMEM;
    for (uint32_t i = 0; i < nvertices; ++i) m->m.vertices.push_back(mk(vertices[3 * i], vertices[3 * i + 1], vertices[3 * i + 2]));
    for (uint32_t i = 0; i < nnormals; ++i) m->m.normals.push_back(mk(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]));
    m->m.face_v.assign(face_vertices, face_vertices + 3 * size_t(nfaces));
    m->m.face_t.assign(3 * size_t(nfaces), -1);
    if (nnormals) m->m.face_n.assign(face_normals, face_normals + 3 * size_t(nfaces));
    else m->m.face_n.assign(3 * size_t(nfaces), -1);
    *out = m;
    return ATR_OK;
}

void atr_mesh_free(atr_mesh* m) { delete m; }

int atr_mesh_info(const atr_mesh* m, uint32_t* nv, uint32_t* nn, uint32_t* nf) {
    if (!m) return ATR_E_INVALID;
    if (nv) *nv = uint32_t(m->m.vertices.size());
    if (nn) *nn = uint32_t(m->m.normals.size());
    if (nf) *nf = uint32_t(m->m.nfaces());
    return ATR_OK;
}

int atr_mesh_export(const atr_mesh* m, float* vertices, float* normals, float* texcoords, uint32_t* ntexcoords,
                    int32_t* face_v, int32_t* face_t, int32_t* face_n) {
    if (!m) return ATR_E_INVALID;
    auto put = [](float* dst, const std::vector<V3>& src) {
        if (!dst) return;
        for (size_t i = 0; i < src.size(); ++i) { dst[3 * i] = src[i].x; dst[3 * i + 1] = src[i].y; dst[3 * i + 2] = src[i].z; }
    };
    put(vertices, m->m.vertices);
    put(normals, m->m.normals);
    put(texcoords, m->m.texcoords);
    if (ntexcoords) *ntexcoords = uint32_t(m->m.texcoords.size());
    if (face_v) std::memcpy(face_v, m->m.face_v.data(), m->m.face_v.size() * sizeof(int32_t));
    if (face_t) std::memcpy(face_t, m->m.face_t.data(), m->m.face_t.size() * sizeof(int32_t));
    if (face_n) std::memcpy(face_n, m->m.face_n.data(), m->m.face_n.size() * sizeof(int32_t));
    return ATR_OK;
}

int atr_mesh_aabb(const atr_mesh* m, float aabb_out[6]) {
    if (!m || !aabb_out) return ATR_E_INVALID;
    mesh_aabb(m->m, aabb_out);
    return ATR_OK;
}

int atr_mesh_translate_to(atr_mesh* m, float aabb[6], atr_vec3 c) {
    if (!m || !aabb) return ATR_E_INVALID;
    mesh_translate(m->m, aabb, mk(c.x, c.y, c.z));
    return ATR_OK;
}

int atr_octree_build(const atr_mesh* m, uint32_t max_faces, atr_octree** out) {
    if (!m || !out) return ATR_E_INVALID;
    atr_octree* t = new (std::nothrow) atr_octree();
    if (!t) return ATR_E_NOMEM;
    const int rc = octree_build(m->m, max_faces, t->t);
    if (rc != ATR_OK) { delete t; return rc; }
    *out = t;
    return ATR_OK;
}

int atr_octree_build_device(const atr_mesh* m, uint32_t max_faces, int32_t device, atr_octree** out,
                            float ms_out[2]) {
    if (!m || !out || device < 0) return ATR_E_INVALID;
    atr_octree* t = new (std::nothrow) atr_octree();
    if (!t) return ATR_E_NOMEM;
    const int rc = octree_build_device(m->m, max_faces, device, t->t, ms_out);
    if (rc != ATR_OK) { delete t; return rc; }
    *out = t;
    return ATR_OK;
}

int atr_octree_from_nodes(int32_t nnodes, const float* bounds, const int32_t* children,
                          const uint32_t* leaf_first, const uint32_t* leaf_count, uint32_t nprims,
                          const float* prim_vertices, const uint32_t* prim_face, atr_octree** out) {
    if (nnodes <= 0 || !bounds || !children || !leaf_first || !leaf_count || !out) return ATR_E_INVALID;
    if (nprims && (!prim_vertices || !prim_face)) return ATR_E_INVALID;
    atr_octree* t = new (std::nothrow) atr_octree();
    if (!t) return ATR_E_NOMEM;
    HostTree& T = t->t;
    T.nnodes = nnodes;
    T.bounds.assign(bounds, bounds + 6 * size_t(nnodes));
    T.children.assign(children, children + nnodes);
    T.leaf_first.assign(leaf_first, leaf_first + nnodes);
    T.leaf_count.assign(leaf_count, leaf_count + nnodes);
    T.prim_vertices.assign(prim_vertices, prim_vertices + 9 * size_t(nprims));
    T.prim_face.assign(prim_face, prim_face + nprims);
    for (int32_t i = 0; i < nnodes; ++i)
        if (children[i] == 0 && uint64_t(leaf_first[i]) + leaf_count[i] > nprims) { delete t; return ATR_E_INVALID; }
    const int rc = octree_finish(T);
    if (rc != ATR_OK) { delete t; return rc; }
    *out = t;
    return ATR_OK;
}

void atr_octree_free(atr_octree* t) { delete t; }

int atr_octree_export(const atr_octree* t, float* bounds, int32_t* children, uint32_t* leaf_first,
                      uint32_t* leaf_count, float* prim_vertices, uint32_t* prim_face) {
    if (!t) return ATR_E_INVALID;
    const HostTree& T = t->t;
    if (bounds) std::memcpy(bounds, T.bounds.data(), T.bounds.size() * sizeof(float));
    if (children) std::memcpy(children, T.children.data(), T.children.size() * sizeof(int32_t));
    if (leaf_first) std::memcpy(leaf_first, T.leaf_first.data(), T.leaf_first.size() * sizeof(uint32_t));
    if (leaf_count) std::memcpy(leaf_count, T.leaf_count.data(), T.leaf_count.size() * sizeof(uint32_t));
    if (prim_vertices) std::memcpy(prim_vertices, T.prim_vertices.data(), T.prim_vertices.size() * sizeof(float));
    if (prim_face) std::memcpy(prim_face, T.prim_face.data(), T.prim_face.size() * sizeof(uint32_t));
    return ATR_OK;
}

int atr_octree_stats(const atr_octree* t, int64_t s[7]) {
    if (!t || !s) return ATR_E_INVALID;
    octree_stats(t->t, s);
    return ATR_OK;
}

int atr_camera_set(atr_camera* cm, atr_vec3 eye, atr_vec3 facing, int32_t w, int32_t h, int32_t aa,
                   uint32_t spp, int32_t bounces, float h_fov) {
    if (!cm || w <= 0 || h <= 0) return ATR_E_INVALID;
    camera_set(*cm, mk(eye.x, eye.y, eye.z), mk(facing.x, facing.y, facing.z), w, h, aa, spp, bounces, h_fov);
    return ATR_OK;
}

namespace {
void put_le(uint8_t* p, uint32_t v, int n) {
    for (int i = 0; i < n; ++i) p[i] = uint8_t(v >> (8 * i));
}
}  // namespace

int atr_write_bmp(const uint32_t* pixels, int32_t width, int32_t height, const char* name, char* out_path,
                  int32_t out_cap) {
    if (!pixels || !name || width <= 0 || height <= 0) return ATR_E_INVALID;
    const size_t len = std::strlen(name);
    if (len + 8 > 1024) return ATR_E_INVALID;  // the reference's new_name[1024]
    const uint64_t bytes = uint64_t(width) * uint64_t(height) * 4;
    if (bytes + 70 > 0x7FFFFFFFull) return ATR_E_INVALID;  // int32 total_file_size
    uint8_t hdr[70] = {};
    hdr[0] = 'B';
    hdr[1] = 'M';
    put_le(hdr + 2, uint32_t(70 + bytes), 4);  // total size; reserved1/2 = 0
    put_le(hdr + 10, 70, 4);                   // pixel offset = 14 + 56
    uint8_t* d = hdr + 14;
    put_le(d + 0, 56, 4);
    put_le(d + 4, uint32_t(width), 4);
    put_le(d + 8, uint32_t(height), 4);  // positive: bottom-up rows, matching row 0 = bottom
    put_le(d + 12, 1, 2);                // planes
    put_le(d + 14, 32, 2);               // bits per pixel
    put_le(d + 16, 3, 4);                // BI_BITFIELDS
    put_le(d + 20, uint32_t(bytes), 4);
    put_le(d + 24, 197, 4);  // ppm x, y as the reference sets them
    put_le(d + 28, 39, 4);
    put_le(d + 40, 0x00FF0000u, 4);  // clr_used/clr_important (32, 36) = 0; R, G, B, A masks
    put_le(d + 44, 0x0000FF00u, 4);
    put_le(d + 48, 0x000000FFu, 4);
    put_le(d + 52, 0, 4);
    std::string path;
    int fd = -1;
    for (uint32_t id = 0; id < 100 && fd < 0; ++id) {  // "%s_%u.bmp" fits len + 8 bytes for ids < 100
        path = std::string(name) + "_" + std::to_string(id) + ".bmp";
        fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_EXCL, 0644);
        if (fd < 0 && errno != EEXIST) return ATR_E_IO;
    }
    if (fd < 0) return ATR_E_IO;
    bool ok = ::write(fd, hdr, sizeof(hdr)) == ssize_t(sizeof(hdr));
    const uint8_t* src = reinterpret_cast<const uint8_t*>(pixels);
    for (uint64_t off = 0; ok && off < bytes;) {
        const ssize_t w = ::write(fd, src + off, size_t(std::min<uint64_t>(bytes - off, 1ull << 30)));
        ok = w > 0;
        off += ok ? uint64_t(w) : 0;
    }
    ok = (::close(fd) == 0) && ok;
    if (!ok) return ATR_E_IO;
    if (out_path && out_cap > 0) {
        std::strncpy(out_path, path.c_str(), size_t(out_cap) - 1);
        out_path[out_cap - 1] = 0;
    }
    return ATR_OK;
}

int32_t atr_make_tiles(int32_t w, int32_t h, int32_t threads, atr_tile* out, int32_t cap) {
    return reference_tiles(w, h, threads, out, out ? cap : 0);
}

int32_t atr_make_shard_tiles(int32_t w, int32_t h, int32_t side, int32_t rank, int32_t world, atr_tile* out,
                             int32_t cap) {
    return shard_tiles(w, h, side, rank, world, out, out ? cap : 0);
}

int32_t atr_balance_shard_tiles(int32_t w, int32_t h, int32_t side, int32_t world, const int64_t* costs,
                                int64_t rank0_extra, int32_t* owner_out) {
    return balance_shard_tiles(w, h, side, world, costs, rank0_extra, owner_out);
}

// ------------------------------------------------------------------ device engine
int atr_create(int device, atr_ctx** out) {
    if (!out) return ATR_E_INVALID;
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(device));
    atr_ctx* c = new (std::nothrow) atr_ctx();
    if (!c) return ATR_E_NOMEM;
    c->device = device;
    const int rc = [&]() -> int {  // any failure below releases what was created (atr_destroy)
        HIPCHK(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreate(&c->ev_start));
        HIPCHK(hipEventCreate(&c->ev_stop));
        HIPCHK(hipMalloc(&c->d_error, 16));
        HIPCHK(hipMemset(c->d_error, 0, 16));
        HIPCHK(hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device));
        HIPCHK(hipMalloc(&c->tring, kQueueSlots * kTraceBytes));
        HIPCHK(hipMemset(c->tring, 0, kQueueSlots * kTraceBytes));
        for (hipEvent_t& e : c->tev) HIPCHK(hipEventCreate(&e));  // timed: a launch's ev_last
        return ATR_OK;
    }();
    if (rc != ATR_OK) {
        atr_destroy(c);
        return rc;
    }
    *out = c;
    return ATR_OK;
}

void atr_default_tuning(atr_tuning* out) {
    if (out) *out = default_tuning();
}

int atr_set_tuning(atr_ctx* c, const atr_tuning* t) {
    if (!c || !t) return ATR_E_INVALID;
    if (t->xcd_chunk < 0 || t->xcd_chunk > 4096 || t->frame_rotate < 0 || t->frame_rotate > 1024 ||
        t->hybrid_a < -4096 || t->hybrid_a > 4096 || t->hybrid_b < -4096 || t->hybrid_b > 4096 ||
        t->path_batch_log2 < 12 || t->path_batch_log2 > ATR_MAX_BATCH_LOG2 || t->cluster_size < 1 || t->cluster_size > kMaxClusterSize ||
        t->frame_plan < 0 || t->frame_plan > 1 || (t->path_camera_occ != 0 && (t->path_camera_occ < 5 || t->path_camera_occ > 7)) ||
        (t->path_bounce_occ != 0 && (t->path_bounce_occ < 5 || t->path_bounce_occ > 7)) ||
        (t->primary_occ != 0 && (t->primary_occ < 6 || t->primary_occ > 8)) ||
        (t->path_sort_bits != 0 && (t->path_sort_bits < 2 || t->path_sort_bits > kMaxSortBits)) ||
        t->path_split < 0 || t->path_split > 1)
        return ATR_E_INVALID;
    for (int32_t r : t->reserved)  // room for later knobs: must be zero
        if (r != 0) return ATR_E_INVALID;
    c->tune = *t;
    return ATR_OK;
}

int atr_get_tuning(atr_ctx* c, atr_tuning* out) {
    if (!c || !out) return ATR_E_INVALID;
    *out = c->tune;
    return ATR_OK;
}

int atr_destroy(atr_ctx* c) {
    if (!c) return ATR_E_INVALID;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    free_scene(c);
    for (BlockSet& b : c->blocks) {
        if (b.dev.p) (void)hipFree(b.dev.p);
        if (b.dev_tiles.p) (void)hipFree(b.dev_tiles.p);
        if (b.dev_tile.p) (void)hipFree(b.dev_tile.p);
        for (DevBuf* d : {&b.cost, &b.cost_last, &b.plan_work, &b.plan_blocks})
            if (d->p) (void)hipFree(d->p);
        for (hipEvent_t e : b.plan_ev)
            if (e) (void)hipEventDestroy(e);
    }
    for (auto& se : c->stream_ev) (void)hipEventDestroy(se.second);
    for (auto& w : c->path_ws) {
        if (w.mem.p) (void)hipFree(w.mem.p);
        if (w.ev) (void)hipEventDestroy(w.ev);
    }
    if (c->d_error) (void)hipFree(c->d_error);
    for (DevBuf& b : c->prog_blocks)
        if (b.p) (void)hipFree(b.p);
    for (hipEvent_t e : c->prog_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->tev)
        if (e) (void)hipEventDestroy(e);
    if (c->tring) (void)hipFree(c->tring);
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->plan_side) (void)hipStreamDestroy(c->plan_side);
    for (int i = 0; i < 2; ++i) {
        if (c->split_stream[i]) (void)hipStreamDestroy(c->split_stream[i]);
        if (c->split_join[i]) (void)hipEventDestroy(c->split_join[i]);
    }
    if (c->split_fork) (void)hipEventDestroy(c->split_fork);
    delete c;
    return ATR_OK;
}

int atr_scene_upload(atr_ctx* c, const atr_material* mats, int32_t nmats, const atr_model* models,
                     int32_t nmodels, const atr_sphere* spheres, int32_t nspheres, const atr_plane* planes,
                     int32_t nplanes) {
    if (!c || !mats || nmats <= 0 || nmats > kMaxMaterials || nmodels < 0 || nmodels > kMaxModels ||
        (nmodels && !models) || nspheres < 0 || nplanes < 0 || (nspheres && !spheres) || (nplanes && !planes))
        return ATR_E_INVALID;
    for (int32_t i = 0; i < nspheres; ++i)  // shading indexes mats[material] on the device
        if (spheres[i].material < 0 || spheres[i].material >= nmats) return ATR_E_INVALID;
    for (int32_t i = 0; i < nplanes; ++i)
        if (planes[i].material < 0 || planes[i].material >= nmats) return ATR_E_INVALID;
    for (int32_t i = 0; i < nmodels; ++i) {
        const atr_model& md = models[i];
        if (!md.mesh || md.material < 0 || md.material >= nmats) return ATR_E_INVALID;
        if (md.tree) {
            for (int32_t d : md.tree->t.depth)
                if (d >= kMaskLevels) return ATR_E_TREE_DEPTH;
        }
    }
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(wait_all(c));  // kernels on any stream may still read the old scene
    free_scene(c);
    DScene S;
    std::memset(&S, 0, sizeof(S));
    for (int32_t i = 0; i < nmats; ++i) {
        const atr_material& m = mats[i];
        S.mats[i] = DMaterial{m.emission.x, m.emission.y, m.emission.z, m.reflection.x, m.reflection.y,
                              m.reflection.z, m.scatter, 0.f};
    }
    S.nmats = nmats;
    S.nmodels = nmodels;
    c->max_nodes = 0;
    c->max_depth = 0;
    c->max_inner = 0;
    c->nclusters = 0;
    float box[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int32_t i = 0; i < nmodels; ++i)
        for (const V3& v : models[i].mesh->m.vertices) {
            box[0] = std::min(box[0], v.x), box[1] = std::min(box[1], v.y), box[2] = std::min(box[2], v.z);
            box[3] = std::max(box[3], v.x), box[4] = std::max(box[4], v.y), box[5] = std::max(box[5], v.z);
        }
    for (int32_t i = 0; i < nspheres; ++i) {  // a sphere's bounds (planes are unbounded: left out)
        const atr_sphere& sp = spheres[i];
        const float r = std::fabs(sp.radius);
        box[0] = std::min(box[0], sp.center.x - r), box[1] = std::min(box[1], sp.center.y - r);
        box[2] = std::min(box[2], sp.center.z - r), box[3] = std::max(box[3], sp.center.x + r);
        box[4] = std::max(box[4], sp.center.y + r), box[5] = std::max(box[5], sp.center.z + r);
    }
    // the queue sort's origin cells span this box; a scene with nothing bounded gets the unit box
    // (not the previous upload's)
    const float unit[6] = {0.f, 0.f, 0.f, 1.f, 1.f, 1.f};
    const bool finite = std::isfinite(box[0]) && std::isfinite(box[1]) && std::isfinite(box[2]) &&
                        std::isfinite(box[3]) && std::isfinite(box[4]) && std::isfinite(box[5]);
    std::memcpy(c->scene_box, finite && box[0] <= box[3] && box[1] <= box[4] && box[2] <= box[5] ? box : unit,
                sizeof(box));
    for (int32_t i = 0; i < nmodels; ++i) {
        const atr_model& md = models[i];
        const HostMesh& M = md.mesh->m;
        DModel& dm = S.models[i];
        std::memset(&dm, 0, sizeof(dm));
        const size_t nf = M.nfaces();
        dm.nfaces = uint32_t(nf);
        dm.material = md.material;
        std::memcpy(dm.aabb, md.surrounding_aabb, sizeof(dm.aabb));
        dm.smooth = M.normals.empty() ? 0 : 1;
        // per-face shading record (renderer.cpp:124-149)
        std::vector<float> shade(9 * (nf ? nf : 1), 0.f);
        for (size_t f = 0; f < nf; ++f) {
            for (int k = 0; k < 3; ++k) {
                V3 v = mk(0.f, 0.f, 0.f);
                if (dm.smooth) {
                    const int32_t ni = M.face_n[3 * f + size_t(k)];
                    if (ni >= 0 && size_t(ni) < M.normals.size()) v = M.normals[size_t(ni)];
                } else {
                    const int32_t vi = M.face_v[3 * f + size_t(k)];
                    if (vi >= 0 && size_t(vi) < M.vertices.size()) v = M.vertices[size_t(vi)];
                }
                shade[9 * f + 3 * size_t(k)] = v.x;
                shade[9 * f + 3 * size_t(k) + 1] = v.y;
                shade[9 * f + 3 * size_t(k) + 2] = v.z;
            }
        }
        void* p = nullptr;
        int rc = dev_upload(c, shade.data(), shade.size() * sizeof(float), &p);
        if (rc) return rc;
        dm.shade = static_cast<const float*>(p);
        if (md.tree) {
            const HostTree& T = md.tree->t;
            PackedTree PT;  // every device table of the model (host_scene.cpp pack_tree)
            if ((rc = pack_tree(T, c->tune.cluster_size, PT))) return rc;
            c->max_depth = std::max(c->max_depth, PT.max_depth);
            auto up = [&](const auto& v, auto*& dst) {
                void* q = nullptr;
                const int r = dev_upload(c, v.data(), v.size() * sizeof(v[0]), &q);
                dst = static_cast<std::remove_reference_t<decltype(dst)>>(q);
                return r;
            };
            dm.ninner = PT.ninner;
            if (dm.ninner > c->max_inner) c->max_inner = dm.ninner;
            if ((rc = up(PT.inner, dm.inner)) || (rc = up(PT.t0, dm.t0)) || (rc = up(PT.t1, dm.t1)) ||
                (rc = up(PT.t2, dm.t2)) || (rc = up(PT.tface, dm.tface)))
                return rc;
            const float4_t* clus = nullptr;
            if ((rc = up(PT.clus, clus))) return rc;
            dm.clus = clus;
            dm.cnrm = reinterpret_cast<const uint4_t*>(dm.clus + 2);
            if ((rc = up(PT.cl_range, dm.cl_range)) || (rc = up(PT.prim, dm.prim))) return rc;
            c->nclusters += int64_t(PT.nclusters);
            if ((rc = up(PT.nodes, dm.nodes)) || (rc = up(PT.leaf_range, dm.leaf_range))) return rc;
            if (PT.tris.empty()) PT.tris.resize(1);
            if ((rc = up(PT.tris, dm.tris))) return rc;
            dm.has_tree = 1;
            dm.root_leaf = T.children[0] == 0;
            dm.near_ok = PT.near_ok;
            if (T.nnodes > c->max_nodes) c->max_nodes = T.nnodes;
        } else {  // brute force: face-ordered triangles straight from the mesh (renderer.cpp:61-66)
            std::vector<DTri> tris(nf);
            for (size_t f = 0; f < nf; ++f) {
                float v[9];
                for (int k = 0; k < 3; ++k) {
                    const int32_t vi = M.face_v[3 * f + size_t(k)];
                    if (vi < 0 || size_t(vi) >= M.vertices.size()) return ATR_E_INVALID;
                    const V3 q = M.vertices[size_t(vi)];
                    v[3 * k] = q.x; v[3 * k + 1] = q.y; v[3 * k + 2] = q.z;
                }
                tris[f] = make_tri(v, uint32_t(f));
            }
            if ((rc = dev_upload(c, tris.data(), tris.size() * sizeof(DTri), &p))) return rc;
            dm.tris = static_cast<const DTri*>(p);
            dm.has_tree = 0;
        }
    }
    {
        std::vector<DSphere> sp(size_t(nspheres) + 1);
        for (int32_t i = 0; i < nspheres; ++i)
            sp[size_t(i)] = DSphere{spheres[i].center.x, spheres[i].center.y, spheres[i].center.z,
                                    spheres[i].radius, spheres[i].material, 0, 0, 0};
        std::vector<DPlane> pl(size_t(nplanes) + 1);
        for (int32_t i = 0; i < nplanes; ++i)
            pl[size_t(i)] = DPlane{planes[i].normal.x, planes[i].normal.y, planes[i].normal.z,
                                   planes[i].distance, planes[i].material, 0, 0, 0};
        void* p = nullptr;
        int rc;
        if ((rc = dev_upload(c, sp.data(), sp.size() * sizeof(DSphere), &p))) return rc;
        S.spheres = static_cast<const DSphere*>(p);
        if ((rc = dev_upload(c, pl.data(), pl.size() * sizeof(DPlane), &p))) return rc;
        S.planes = static_cast<const DPlane*>(p);
        S.nspheres = nspheres;
        S.nplanes = nplanes;
        if ((rc = dev_upload(c, &S, sizeof(S), &p))) return rc;
        c->d_scene = static_cast<DScene*>(p);
    }
    c->nmodels = nmodels;
    return ATR_OK;
}

int atr_scene_info(atr_ctx* c, int64_t* bytes, int32_t* max_nodes, int32_t* max_depth) {
    if (!c) return ATR_E_INVALID;
    if (bytes) *bytes = c->scene_bytes;
    if (max_nodes) *max_nodes = c->max_nodes;
    if (max_depth) *max_depth = c->max_depth;
    return ATR_OK;
}

int atr_workspace_info(atr_ctx* c, int32_t* workspaces, int64_t* bytes) {
    if (!c) return ATR_E_INVALID;
    int32_t n = 0;
    int64_t b = 0;
    for (const auto& w : c->path_ws)
        if (w.mem.p) { ++n; b += int64_t(w.mem.n); }
    if (workspaces) *workspaces = n;
    if (bytes) *bytes = b;
    return ATR_OK;
}

int64_t atr_render_packed_size(const atr_tile* tiles, int32_t ntiles) {
    if (!tiles || ntiles <= 0) return 0;
    int32_t W = 0, H = 0;
    for (int32_t i = 0; i < ntiles; ++i) {
        if (tiles[i].max_x + 1 > W) W = tiles[i].max_x + 1;
        if (tiles[i].max_y + 1 > H) H = tiles[i].max_y + 1;
    }
    std::vector<DBlock> b;
    int64_t n = 0;
    build_blocks(tiles, ntiles, W, H, b, n);
    return n;
}

int64_t atr_packed_pixel_map(const atr_tile* tiles, int32_t ntiles, int32_t W, int32_t H, int64_t* out,
                             int64_t cap) {
    if (ntiles < 0 || (ntiles && !tiles) || W <= 0 || H <= 0) return ATR_E_INVALID;
    std::vector<DBlock> b;
    int64_t n = 0;
    build_blocks(tiles, ntiles, W, H, b, n);
    if (out) {
        int64_t k = 0;
        for (const DBlock& blk : b) {
            const uint64_t m = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
            for (int lane = 0; lane < 64; ++lane)
                if ((m >> lane) & 1) {
                    if (k < cap) out[k] = int64_t(blk.y0 + (lane >> 3)) * W + (blk.x0 + (lane & 7));
                    ++k;
                }
        }
    }
    return n;
}

int atr_render_start_ex(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                        const atr_frame* fr, uint64_t seed, void* stream, int32_t variant) {
    if (!c || !cam || !fr || !fr->framebuffer || ntiles < 0 || (ntiles && !tiles)) return ATR_E_INVALID;
    if (cam->width <= 0 || cam->height <= 0 || cam->width > (1 << 16) || cam->height > (1 << 16)) return ATR_E_INVALID;
    if (fr->layout != ATR_LAYOUT_IMAGE && fr->layout != ATR_LAYOUT_PACKED) return ATR_E_INVALID;
    if (!c->d_scene) return ATR_E_NOSCENE;
    HIPCHK(hipSetDevice(c->device));
    const int wave = auto_sched(variant, *cam);
    if (wave < 0) return ATR_E_INVALID;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream (HIP convention)
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, cam->width, cam->height, rc);
    if (!bs) return rc;
    c->prog_active = false;
    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.cam = *cam;
    P.scene = c->d_scene;
    P.seed = seed;
    P.blocks = static_cast<const DBlock*>(bs->dev.p);
    P.nblocks = int32_t(bs->host.size());
    P.layout = fr->layout;
    P.framebuffer = fr->framebuffer;
    P.hit_face = fr->hit_face;
    P.hit_t = fr->hit_t;
    P.rgb = fr->rgb;
    P.ray_casts = fr->ray_casts;
    P.traced_rays = fr->traced_rays;
    P.error_flag = c->d_error;
    P.counters = nullptr;
    apply_tuning(c, P);
    HIPCHK(hipEventRecord(c->ev_start, s));
    if ((rc = launch_planned(c, bs, P, wave, s))) return rc;
    HIPCHK(note_launch(c, s, c->ev_last != c->ev_stop));  // a ring event covers it
    c->have_render = true;
    c->last_stream = s;
    c->last_ntiles = ntiles;
    return ATR_OK;
}

namespace {
// Frames in flight in one launch (atr_render_start_frames / _cameras): ncams == 1 -> every frame
// renders cams[0]; ncams == nframes -> frame f renders cams[f].
int start_frames(atr_ctx* c, const atr_camera* cams, int32_t ncams, const atr_tile* tiles, int32_t ntiles,
                 const atr_frame* fr, int32_t nframes, int64_t frame_stride, uint64_t seed, void* stream,
                 int32_t variant) {
    if (!c || !cams || !fr || !fr->framebuffer || ntiles < 0 || (ntiles && !tiles) || nframes < 1 || nframes > 64)
        return ATR_E_INVALID;
    if (ncams != 1 && (ncams != nframes || nframes > kMaxFrameCams)) return ATR_E_INVALID;
    const atr_camera* cam = cams;
    if (cam->width <= 0 || cam->height <= 0 || cam->width > (1 << 16) || cam->height > (1 << 16)) return ATR_E_INVALID;
    for (int32_t f = 1; f < ncams; ++f) {  // one block list and one kernel specialization per launch
        const atr_camera& q = cams[f];
        if (q.width != cam->width || q.height != cam->height || q.samples_per_pixel != cam->samples_per_pixel ||
            q.bounce_limit != cam->bounce_limit || q.anti_aliasing != cam->anti_aliasing)
            return ATR_E_INVALID;
    }
    if (fr->layout != ATR_LAYOUT_IMAGE && fr->layout != ATR_LAYOUT_PACKED) return ATR_E_INVALID;
    const int sched = auto_sched(variant, *cam);
    if (sched < 0) return ATR_E_INVALID;
    if (!c->d_scene) return ATR_E_NOSCENE;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, cam->width, cam->height, rc);
    if (!bs) return rc;
    const int64_t per_frame = fr->layout == ATR_LAYOUT_IMAGE ? int64_t(cam->width) * cam->height : bs->packed_pixels;
    if (nframes > 1 && frame_stride < per_frame) return ATR_E_INVALID;
    const int32_t nb = int32_t(bs->host.size());
    if (int64_t(nb) * nframes > (int64_t(1) << 30)) return ATR_E_INVALID;
    c->prog_active = false;
    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.cam = *cam;
    P.scene = c->d_scene;
    P.seed = seed;
    P.blocks = static_cast<const DBlock*>(bs->dev.p);
    P.layout = fr->layout;
    P.framebuffer = fr->framebuffer;
    P.hit_face = fr->hit_face;
    P.hit_t = fr->hit_t;
    P.rgb = fr->rgb;
    P.ray_casts = fr->ray_casts;
    P.traced_rays = fr->traced_rays;
    P.error_flag = c->d_error;
    apply_tuning(c, P);
    HIPCHK(hipEventRecord(c->ev_start, s));
    if (nframes == 1) {  // one frame: the single-frame plan applies
        P.nblocks = nb;
        P.frame_stride = frame_stride;
        if ((rc = launch_planned(c, bs, P, sched, s))) return rc;
    } else {  // one launch over frames x blocks (render_kernel / paths: fidx)
        P.nblocks = nb * nframes;
        P.frame_blocks = nb;
        P.frame_stride = frame_stride;
        P.frame_rotate = c->tune.frame_rotate;
        if (ncams > 1) {
            P.nfcam = ncams;
            for (int32_t f = 0; f < ncams; ++f) P.fcam[f] = cams[f];
        }
        hipEvent_t done = nullptr;
        HIPCHK(launch_render(c, P, sched, s, &done));
        HIPCHK(record_stop(c, s, done));
    }
    HIPCHK(note_launch(c, s, c->ev_last != c->ev_stop));  // a ring event covers it
    c->have_render = true;
    c->last_stream = s;
    c->last_ntiles = ntiles;
    return ATR_OK;
}
}  // namespace

int atr_render_start_frames(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                            const atr_frame* fr, int32_t nframes, int64_t frame_stride, uint64_t seed, void* stream,
                            int32_t variant) {
    return start_frames(c, cam, 1, tiles, ntiles, fr, nframes, frame_stride, seed, stream, variant);
}

int atr_render_start_cameras(atr_ctx* c, const atr_camera* cams, int32_t nframes, const atr_tile* tiles,
                             int32_t ntiles, const atr_frame* fr, int64_t frame_stride, uint64_t seed, void* stream,
                             int32_t variant) {
    return start_frames(c, cams, nframes, tiles, ntiles, fr, nframes, frame_stride, seed, stream, variant);
}

#ifdef ATR_DIAG
int atr_render_wave_trace(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                          uint64_t seed, int32_t variant, uint64_t* out, int64_t cap, int64_t* nblocks) {
    if (!c || !cam || !nblocks || ntiles < 0 || (ntiles && !tiles)) return ATR_E_INVALID;
    if (!c->d_scene) return ATR_E_NOSCENE;
    HIPCHK(hipSetDevice(c->device));
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, cam->width, cam->height, rc);
    if (!bs) return rc;
    const size_t nb = bs->host.size();
    *nblocks = int64_t(nb);
    if (!out || cap < int64_t(3 * nb)) return ATR_OK;  // size query
    DevTmp fb;
    DevTmp tr;
    HIPCHK(hipMalloc(&fb.p, std::max<size_t>(1, size_t(bs->packed_pixels)) * 4));
    HIPCHK(hipMalloc(&tr.p, std::max<size_t>(1, 3 * nb) * sizeof(unsigned long long)));
    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.cam = *cam;
    P.scene = c->d_scene;
    P.seed = seed;
    P.blocks = static_cast<const DBlock*>(bs->dev.p);
    P.nblocks = int32_t(nb);
    P.layout = ATR_LAYOUT_PACKED;
    P.framebuffer = static_cast<uint32_t*>(fb.p);
    P.error_flag = c->d_error;
    P.wave_trace = static_cast<unsigned long long*>(tr.p);
    apply_tuning(c, P);
    const int ts = sched_of(variant);  // per-cell trace: 8x8-cell schedules only
    HIPCHK(atr_launch_render(P, ts < 0 || ts == kSchedPaths ? 7 : ts, 0, nullptr));
    HIPCHK(hipDeviceSynchronize());
    if (nb) HIPCHK(hipMemcpy(out, tr.p, 3 * nb * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return ATR_OK;
}

#endif  // ATR_DIAG

// One instrumented (COUNT) render; h = the 16 device counters (render.hip: [0..9] work counters,
// [10..15] phase clocks, zero unless built with -DATR_PHASE_CLOCKS).
constexpr int kCounterSlots = 32;
static int count_launch(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles, uint64_t seed,
                        int32_t variant, unsigned long long h[kCounterSlots]) {
    if (!c || !cam || ntiles < 0 || (ntiles && !tiles)) return ATR_E_INVALID;
    if (!c->d_scene) return ATR_E_NOSCENE;
    HIPCHK(hipSetDevice(c->device));
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, cam->width, cam->height, rc);
    if (!bs) return rc;
    DevTmp fb;
    DevTmp ctr;
    HIPCHK(hipMalloc(&fb.p, size_t(cam->width) * size_t(cam->height) * 4));
    HIPCHK(hipMalloc(&ctr.p, kCounterSlots * sizeof(unsigned long long)));
    HIPCHK(hipMemset(ctr.p, 0, kCounterSlots * sizeof(unsigned long long)));
    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.cam = *cam;
    P.scene = c->d_scene;
    P.seed = seed;
    P.blocks = static_cast<const DBlock*>(bs->dev.p);
    P.nblocks = int32_t(bs->host.size());
    P.layout = ATR_LAYOUT_IMAGE;
    P.framebuffer = static_cast<uint32_t*>(fb.p);
    P.error_flag = c->d_error;
    P.counters = static_cast<unsigned long long*>(ctr.p);
    apply_tuning(c, P);  // the product's HYBRID thresholds (the counts do not depend on them, the clocks do)
    const int sc = auto_sched(variant, *cam);
    if (sc < 0) return ATR_E_INVALID;
    HIPCHK(launch_render(c, P, sc, nullptr));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(h, ctr.p, kCounterSlots * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return ATR_OK;
}

int atr_render_counters(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                        uint64_t seed, int32_t variant, int64_t out[10]) {
    if (!out) return ATR_E_INVALID;
    unsigned long long h[kCounterSlots];
    const int rc = count_launch(c, cam, tiles, ntiles, seed, variant, h);
    if (rc != ATR_OK) return rc;
    for (int k = 0; k < 10; ++k) out[k] = int64_t(h[k]);
    return ATR_OK;
}

#ifdef ATR_DIAG
int atr_render_phase_clocks(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                            uint64_t seed, int32_t variant, int64_t out[6]) {
    if (!out) return ATR_E_INVALID;
    unsigned long long h[kCounterSlots];
    const int rc = count_launch(c, cam, tiles, ntiles, seed, variant, h);
    if (rc != ATR_OK) return rc;
    for (int k = 0; k < 6; ++k) out[k] = int64_t(h[10 + k]);
    return ATR_OK;
}

int atr_render_path_counters(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                             uint64_t seed, int32_t variant, int64_t out[6]) {
    if (!out) return ATR_E_INVALID;
    unsigned long long h[kCounterSlots];
    const int rc = count_launch(c, cam, tiles, ntiles, seed, variant, h);
    if (rc != ATR_OK) return rc;
    for (int k = 0; k < 6; ++k) out[k] = int64_t(h[16 + k]);
    return ATR_OK;
}

int atr_render_simd_counters(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                             uint64_t seed, int32_t variant, int64_t out[7]) {
    if (!out) return ATR_E_INVALID;
    unsigned long long h[kCounterSlots];
    const int rc = count_launch(c, cam, tiles, ntiles, seed, variant, h);
    if (rc != ATR_OK) return rc;
    out[0] = int64_t(h[22]);  // candidate-loop wave iterations
    out[1] = int64_t(h[2]);   // full triangle tests (lane level)
    for (int k = 0; k < 4; ++k) out[2 + k] = int64_t(h[23 + k]);
    out[6] = int64_t(h[0]);   // traced rays
    return ATR_OK;
}

#endif  // ATR_DIAG

int atr_render_tile_costs(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                          uint64_t seed, int64_t* cost_out) {
    if (!c || !cam || (ntiles && (!tiles || !cost_out)) || ntiles < 0) return ATR_E_INVALID;
    if (!c->d_scene) return ATR_E_NOSCENE;
    HIPCHK(hipSetDevice(c->device));
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, cam->width, cam->height, rc);
    if (!bs) return rc;
    const size_t nb = bs->host.size();
    DevTmp fb;
    DevTmp cost;
    HIPCHK(hipMalloc(&fb.p, std::max<size_t>(1, size_t(bs->packed_pixels)) * 4));
    HIPCHK(hipMalloc(&cost.p, std::max<size_t>(1, nb) * sizeof(unsigned long long)));
    HIPCHK(hipMemset(cost.p, 0, std::max<size_t>(1, nb) * sizeof(unsigned long long)));  // atomically added
    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.cam = *cam;
    P.scene = c->d_scene;
    P.seed = seed;
    P.blocks = static_cast<const DBlock*>(bs->dev.p);
    P.nblocks = int32_t(nb);
    P.layout = ATR_LAYOUT_PACKED;
    P.framebuffer = static_cast<uint32_t*>(fb.p);
    P.error_flag = c->d_error;
    P.block_cost = static_cast<unsigned long long*>(cost.p);
    apply_tuning(c, P);
    HIPCHK(launch_render(c, P, auto_sched(ATR_KERNEL_AUTO, *cam), nullptr));  // per-cell clocks, AUTO's kernels
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(nb);
    if (nb) HIPCHK(hipMemcpy(h.data(), cost.p, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // a block (one 8x8 cell of the image grid) belongs to the first tile (list order) that
    // overlaps it: paint cell owners in list order, first writer wins
    const int32_t cw = (cam->width + 7) / 8, chh = (cam->height + 7) / 8;
    std::vector<int32_t> owner(size_t(cw) * size_t(chh), -1);
    for (int32_t t = 0; t < ntiles; ++t) {
        const atr_tile& T = tiles[t];
        const int32_t x0 = std::max(0, T.min_x) / 8, x1 = std::min(cam->width - 1, T.max_x) / 8;
        const int32_t y0 = std::max(0, T.min_y) / 8, y1 = std::min(cam->height - 1, T.max_y) / 8;
        for (int32_t cy = y0; cy <= y1; ++cy)
            for (int32_t cx = x0; cx <= x1; ++cx) {
                int32_t& o = owner[size_t(cy) * size_t(cw) + size_t(cx)];
                if (o < 0) o = t;
            }
    }
    for (int32_t t = 0; t < ntiles; ++t) cost_out[t] = 0;
    for (size_t k = 0; k < nb; ++k) {
        const DBlock& b = bs->host[k];
        const int32_t o = owner[size_t(b.y0 / 8) * size_t(cw) + size_t(b.x0 / 8)];
        if (o >= 0) cost_out[o] += int64_t(h[k]);
    }
    return ATR_OK;
}

int atr_render_start_progressive(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                                 const atr_frame* fr, uint64_t seed, void* stream, int32_t variant,
                                 int32_t tiles_per_launch) {
    if (!c || !cam || !fr || !fr->framebuffer || ntiles < 0 || (ntiles && !tiles) || tiles_per_launch < 1)
        return ATR_E_INVALID;
    if (cam->width <= 0 || cam->height <= 0 || cam->width > (1 << 16) || cam->height > (1 << 16)) return ATR_E_INVALID;
    if (fr->layout != ATR_LAYOUT_IMAGE) return ATR_E_INVALID;
    const int sched = auto_sched(variant, *cam);
    if (sched < 0) return ATR_E_INVALID;
    if (!c->d_scene) return ATR_E_NOSCENE;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIPCHK(wait_all(c));  // group buffers are reused
    const int32_t ngroups = (ntiles + tiles_per_launch - 1) / tiles_per_launch;
    while (int32_t(c->prog_ev.size()) < ngroups) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->prog_ev.push_back(e);
    }
    c->prog_blocks.resize(std::max<size_t>(c->prog_blocks.size(), size_t(ngroups)));
    c->prog_end.assign(size_t(ngroups), 0);
    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.cam = *cam;
    P.scene = c->d_scene;
    P.seed = seed;
    P.layout = ATR_LAYOUT_IMAGE;
    P.framebuffer = fr->framebuffer;
    P.hit_face = fr->hit_face;
    P.hit_t = fr->hit_t;
    P.rgb = fr->rgb;
    P.ray_casts = fr->ray_casts;
    P.traced_rays = fr->traced_rays;
    P.error_flag = c->d_error;
    apply_tuning(c, P);
    HIPCHK(hipEventRecord(c->ev_start, s));
    for (int32_t g = 0; g < ngroups; ++g) {
        const int32_t a = g * tiles_per_launch, e = std::min(ntiles, a + tiles_per_launch);
        std::vector<DBlock> blocks;
        int64_t npix = 0;
        build_blocks(tiles, e, cam->width, cam->height, blocks, npix, a);  // tiles[a, e), new pixels
        DevBuf& d = c->prog_blocks[size_t(g)];
        const size_t need = std::max<size_t>(blocks.size() * sizeof(DBlock), 32);
        if (d.n < need) {
            if (d.p) HIPCHK(hipFree(d.p));
            d = DevBuf();
            HIPCHK(hipMalloc(&d.p, need));
            d.n = need;
        }
        if (!blocks.empty()) HIPCHK(hipMemcpy(d.p, blocks.data(), blocks.size() * sizeof(DBlock), hipMemcpyHostToDevice));
        P.blocks = static_cast<const DBlock*>(d.p);
        P.nblocks = int32_t(blocks.size());
        HIPCHK(launch_render(c, P, sched, s));
        HIPCHK(hipEventRecord(c->prog_ev[size_t(g)], s));
        c->prog_end[size_t(g)] = e;
    }
    HIPCHK(record_stop(c, s, nullptr));
    HIPCHK(note_launch(c, s));
    c->have_render = true;
    c->prog_active = true;
    c->last_stream = s;
    c->last_ntiles = ntiles;
    return ATR_OK;
}

int atr_render_start(atr_ctx* c, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                     const atr_frame* fr, uint64_t seed, void* stream) {
    return atr_render_start_ex(c, cam, tiles, ntiles, fr, seed, stream, ATR_KERNEL_AUTO);
}

int atr_render_wait(atr_ctx* c, uint32_t timeout_ms, int32_t* tiles_done) {
    if (!c) return ATR_E_INVALID;
    if (tiles_done) *tiles_done = 0;
    if (!c->have_render) { return ATR_OK; }
    HIPCHK(hipSetDevice(c->device));
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(c->ev_last);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) return -(1000 + int(q));
        const auto el = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
        if (uint32_t(el.count()) >= timeout_ms) {
            if (tiles_done && c->prog_active) {  // tiles of the leading groups already complete
                size_t g = 0;
                for (; g < c->prog_end.size(); ++g) {
                    const hipError_t qg = hipEventQuery(c->prog_ev[g]);
                    if (qg != hipSuccess) break;
                    *tiles_done = c->prog_end[g];
                }
                // every group finished since ev_last was queried: the render is done (ev_last
                // follows the last group on the same stream), report it as done, not running
                if (g == c->prog_end.size() && !c->prog_end.empty()) {
                    HIPCHK(hipEventSynchronize(c->ev_last));
                    break;
                }
            }
            return 1;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    int32_t err = 0;
    HIPCHK(hipMemcpy(&err, c->d_error, sizeof(err), hipMemcpyDeviceToHost));
    if (err) {
        HIPCHK(hipMemset(c->d_error, 0, sizeof(int32_t)));
        // bit 1: a queue-sort slot outside its level (paths.hip path_sort_rank; never expected)
        return (err & 2) ? -(1000 + int(hipErrorUnknown)) : ATR_E_TREE_DEPTH;
    }
    if (tiles_done) *tiles_done = c->last_ntiles;
    return ATR_OK;
}

int atr_last_kernel_ms(atr_ctx* c, float* ms) {
    if (!c || !ms || !c->have_render) return ATR_E_INVALID;
    HIPCHK(hipEventSynchronize(c->ev_last));
    HIPCHK(hipEventElapsedTime(ms, c->ev_start, c->ev_last));
    return ATR_OK;
}

int atr_unpack(atr_ctx* c, const atr_tile* tiles, int32_t ntiles, int32_t width, const uint32_t* packed,
               uint32_t* image, void* stream) {
    if (!c || !packed || !image || width <= 0 || ntiles < 0 || (ntiles && !tiles)) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    int32_t H = 0;
    for (int32_t i = 0; i < ntiles; ++i) if (tiles[i].max_y + 1 > H) H = tiles[i].max_y + 1;
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, width, H, rc);
    if (!bs) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream (HIP convention)
    HIPCHK(atr_launch_unpack(static_cast<const DBlock*>(bs->dev.p), int32_t(bs->host.size()), width, packed, image, s));
    HIPCHK(note_launch(c, s));
    return ATR_OK;
}

int atr_tile_ray_casts(atr_ctx* c, const atr_tile* tiles, int32_t ntiles, int32_t width,
                       const uint32_t* casts, int64_t* out, void* stream) {
    if (!c || !casts || !out || width <= 0 || ntiles < 0 || (ntiles && !tiles)) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream (HIP convention)
    void* dt = nullptr;
    HIPCHK(hipMallocAsync(&dt, sizeof(atr_tile) * size_t(ntiles ? ntiles : 1), s));
    HIPCHK(hipMemcpyAsync(dt, tiles, sizeof(atr_tile) * size_t(ntiles), hipMemcpyHostToDevice, s));
    HIPCHK(atr_launch_tile_casts(static_cast<const atr_tile*>(dt), ntiles, width, casts, out, s));
    HIPCHK(hipFreeAsync(dt, s));
    HIPCHK(hipStreamSynchronize(s));
    return ATR_OK;
}

int atr_packed_tile_ray_casts(atr_ctx* c, const atr_tile* tiles, int32_t ntiles, int32_t width, int32_t height,
                              const uint32_t* casts, int32_t nframes, int64_t frame_stride, int64_t* out,
                              void* stream) {
    if (!c || !casts || !out || width <= 0 || height <= 0 || ntiles < 0 || (ntiles && !tiles) || nframes < 0 ||
        nframes > 65535)
        return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, width, height, rc);  // the render's cached set
    if (!bs) return rc;
    if (nframes > 1 && frame_stride < bs->packed_pixels) return ATR_E_INVALID;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream (HIP convention)
    const int64_t n = bs->packed_pixels;
    if (!bs->tile_ready) {  // owner of every pixel = the first tile holding it (packed: traced once)
        std::vector<int32_t> owner(size_t(width) * size_t(height), -1);
        for (int32_t k = 0; k < ntiles; ++k) {
            const int32_t x0 = std::max(tiles[k].min_x, 0), x1 = std::min(tiles[k].max_x, width - 1);
            const int32_t y0 = std::max(tiles[k].min_y, 0), y1 = std::min(tiles[k].max_y, height - 1);
            for (int32_t y = y0; y <= y1; ++y)
                for (int32_t x = x0; x <= x1; ++x) {
                    int32_t& o = owner[size_t(y) * size_t(width) + size_t(x)];
                    if (o < 0) o = k;
                }
        }
        std::vector<int32_t> st(size_t(n > 0 ? n : 1), -1);
        for (const DBlock& blk : bs->host) {  // slots out_base.. in lane order (not list order)
            const uint64_t m = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
            size_t k = size_t(blk.out_base);
            for (int lane = 0; lane < 64; ++lane)
                if ((m >> lane) & 1)
                    st[k++] = owner[size_t(blk.y0 + (lane >> 3)) * size_t(width) + size_t(blk.x0 + (lane & 7))];
        }
        // a hipMemcpy below may overwrite a buffer a kernel on another stream still reads
        HIPCHK(wait_all(c));
        const size_t need = st.size() * sizeof(int32_t);
        if (bs->dev_tile.n < need) {
            if (bs->dev_tile.p) (void)hipFree(bs->dev_tile.p);
            bs->dev_tile = DevBuf();
            if (hipMalloc(&bs->dev_tile.p, need) != hipSuccess) return ATR_E_NOMEM;
            bs->dev_tile.n = need;
        }
        HIPCHK(hipMemcpy(bs->dev_tile.p, st.data(), need, hipMemcpyHostToDevice));
        bs->tile_ready = true;
    }
    HIPCHK(hipMemsetAsync(out, 0, sizeof(int64_t) * size_t(nframes) * size_t(ntiles), s));
    HIPCHK(atr_launch_packed_tile_casts(static_cast<const int32_t*>(bs->dev_tile.p), n, casts, frame_stride, nframes,
                                        ntiles, reinterpret_cast<unsigned long long*>(out), s));
    HIPCHK(note_launch(c, s));
    return ATR_OK;
}

int atr_pack_bgr(atr_ctx* c, const uint32_t* framebuffer, int64_t npixels, uint8_t* out, void* stream) {
    if (!c || npixels < 0 || (npixels && (!framebuffer || !out))) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(atr_launch_pack_bgr(framebuffer, npixels, out, static_cast<hipStream_t>(stream)));
    return ATR_OK;
}

int atr_scatter_bgr(atr_ctx* c, const uint8_t* packed, int64_t npixels, const int64_t* dst_index, uint32_t* image,
                    void* stream) {
    if (!c || npixels < 0 || (npixels && (!packed || !dst_index || !image))) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(atr_launch_scatter_bgr(packed, npixels, dst_index, image, static_cast<hipStream_t>(stream)));
    return ATR_OK;
}

int64_t atr_pack_bgr_masked_bound(int64_t npixels) {
    if (npixels < 0) return ATR_E_INVALID;
    const int64_t nc = atr_masked_chunks(npixels);
    return 16 + 4 * nc + 1024 * nc + 512 * nc + 3 * npixels;  // header, chunk offsets, masks, group offsets
}

int atr_pack_bgr_masked(atr_ctx* c, const uint32_t* framebuffer, int64_t npixels, uint32_t background, uint8_t* out,
                        int64_t* nbytes, void* stream) {
    if (!c || npixels < 0 || npixels >= (int64_t(1) << 32) || !out || !nbytes || (npixels && !framebuffer))
        return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(atr_launch_pack_bgr_masked(framebuffer, npixels, background, out, nbytes, static_cast<hipStream_t>(stream)));
    return ATR_OK;
}

int atr_scatter_bgr_masked(atr_ctx* c, const uint8_t* packed, int64_t npixels, const int64_t* dst_index,
                           uint32_t* image, void* stream) {
    if (!c || npixels < 0 || npixels >= (int64_t(1) << 32) || (npixels && (!packed || !dst_index || !image)))
        return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(atr_launch_scatter_bgr_masked(packed, npixels, dst_index, image, static_cast<hipStream_t>(stream)));
    return ATR_OK;
}

int atr_unpack_masked(atr_ctx* c, const atr_tile* tiles, int32_t ntiles, int32_t width, int32_t height,
                      const uint8_t* packed, int32_t nframes, uint32_t* image, int64_t image_stride, void* stream) {
    if (!c || !packed || !image || width <= 0 || height <= 0 || ntiles < 0 || (ntiles && !tiles) || nframes < 0 ||
        image_stride < int64_t(width) * height)
        return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, width, height, rc);  // the render's cached set
    if (!bs) return rc;
    const int64_t own = bs->packed_pixels;
    if (nframes == 0 || own == 0) return ATR_OK;
    if (int64_t(nframes) * own >= (int64_t(1) << 32)) return ATR_E_INVALID;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream (HIP convention)
    HIPCHK(atr_launch_unpack_masked(static_cast<const DBlock*>(bs->dev.p), int32_t(bs->host.size()), width, packed,
                                    nframes, own, image, image_stride, s));
    HIPCHK(note_launch(c, s));
    return ATR_OK;
}

int atr_unpack_masked_ranks(atr_ctx* c, int32_t nsrc, const atr_tile* const* tiles, const int32_t* ntiles,
                            int32_t width, int32_t height, const uint8_t* const* packed, const int32_t* raw,
                            int32_t nframes, uint32_t* image, int64_t image_stride, void* stream) {
    if (!c || nsrc < 0 || (nsrc && (!tiles || !ntiles || !packed)) || !image || width <= 0 || height <= 0 ||
        nframes < 0 || image_stride < int64_t(width) * height)
        return ATR_E_INVALID;
    for (int32_t i = 0; i < nsrc; ++i)
        if (ntiles[i] < 0 || (ntiles[i] && !tiles[i]) || !packed[i]) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    if (nsrc == 0 || nframes == 0) return ATR_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream (HIP convention)
    const int32_t kMax = atr_unpack_max_sources();
    for (int32_t i0 = 0; i0 < nsrc; i0 += kMax) {  // one launch pair per kMax sources
        const int32_t n = std::min(kMax, nsrc - i0);
        std::vector<const DBlock*> blocks(size_t(n), nullptr);
        std::vector<int32_t> nb(size_t(n), 0);
        std::vector<int64_t> own(size_t(n), 0);
        for (int32_t k = 0; k < n; ++k) {
            int rc = ATR_OK;
            // the renders' cached sets (the most recently used slots: a later lookup here does not
            // evict an earlier one of this batch)
            BlockSet* bs = get_blocks(c, tiles[i0 + k], ntiles[i0 + k], width, height, rc);
            if (!bs) return rc;
            blocks[size_t(k)] = static_cast<const DBlock*>(bs->dev.p);
            nb[size_t(k)] = int32_t(bs->host.size());
            own[size_t(k)] = bs->packed_pixels;
            if (int64_t(nframes) * own[size_t(k)] >= (int64_t(1) << 32)) return ATR_E_INVALID;
        }
        HIPCHK(atr_launch_unpack_masked_multi(n, blocks.data(), nb.data(), own.data(), packed + i0,
                                              raw ? raw + i0 : nullptr, width, nframes, image, image_stride, s));
    }
    HIPCHK(note_launch(c, s));
    return ATR_OK;
}

int atr_render_plan_info(atr_ctx* c, const atr_tile* tiles, int32_t ntiles, int32_t width, int32_t height,
                         int32_t* base_out, uint32_t* mask_hi_lo_out, int64_t cap, uint64_t* cost_out,
                         int64_t* nplanned) {
    if (!c || !nplanned || width <= 0 || height <= 0 || ntiles < 0 || (ntiles && !tiles)) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, tiles, ntiles, width, height, rc);
    if (!bs) return rc;
    *nplanned = 0;
    if (!bs->plan_ready) return ATR_OK;
    HIPCHK(wait_all(c));  // the plan stream's kernels too
    const int64_t nb = int64_t(bs->host.size()), np = nb + bs->max_split;
    *nplanned = np;
    if (cap < np) return ATR_OK;  // size query
    std::vector<DBlock> h(static_cast<size_t>(np));
    // the list built last (from the last planned launch's costs, in that launch's parity half)
    const DBlock* last = static_cast<const DBlock*>(bs->plan_blocks.p) + size_t(bs->plan_par ^ 1) * size_t(np);
    HIPCHK(hipMemcpy(h.data(), last, size_t(np) * sizeof(DBlock), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < np; ++i) {
        if (base_out) base_out[i] = h[size_t(i)].base;
        if (mask_hi_lo_out) {
            mask_hi_lo_out[2 * i] = h[size_t(i)].mask_lo;
            mask_hi_lo_out[2 * i + 1] = h[size_t(i)].mask_hi;
        }
    }
    if (cost_out) HIPCHK(hipMemcpy(cost_out, bs->cost_last.p, size_t(nb) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return ATR_OK;
}

int atr_set_cell_plan(atr_ctx* c, int32_t width, int32_t height, const uint8_t* plan) {
    if (!c || (plan && (width <= 0 || height <= 0))) return ATR_E_INVALID;
    const int32_t cw = (width + 7) / 8, ch = (height + 7) / 8;
    if (plan) {
        for (size_t i = 0; i < size_t(cw) * size_t(ch); ++i) {
            const int p = plan[i] & 0xF;
            if (!(p == 0 || p == 1 || p == 2 || p == 4 || p == 8)) return ATR_E_INVALID;
        }
        c->cplan.assign(plan, plan + size_t(cw) * size_t(ch));
        c->cplan_w = width;
        c->cplan_h = height;
    } else {
        c->cplan.clear();
        c->cplan_w = c->cplan_h = 0;
    }
    ++c->cplan_gen;  // cached block lists are rebuilt on their next use
    return ATR_OK;
}

int atr_render_cell_costs(atr_ctx* c, const atr_camera* cam, uint64_t seed, int32_t variant, int64_t* out) {
    if (!c || !cam || !out || cam->width <= 0 || cam->height <= 0) return ATR_E_INVALID;
    if (!c->d_scene) return ATR_E_NOSCENE;
    HIPCHK(hipSetDevice(c->device));
    const int32_t cw = (cam->width + 7) / 8, ch = (cam->height + 7) / 8;
    const atr_tile full = {0, 0, cam->width - 1, cam->height - 1};
    int rc = ATR_OK;
    BlockSet* bs = get_blocks(c, &full, 1, cam->width, cam->height, rc);
    if (!bs) return rc;
    const size_t nb = bs->host.size();
    DevTmp fb;
    DevTmp cost;
    HIPCHK(hipMalloc(&fb.p, std::max<size_t>(1, size_t(bs->packed_pixels)) * 4));
    HIPCHK(hipMalloc(&cost.p, std::max<size_t>(1, nb) * sizeof(unsigned long long)));
    HIPCHK(hipMemset(cost.p, 0, std::max<size_t>(1, nb) * sizeof(unsigned long long)));  // atomically added
    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.cam = *cam;
    P.scene = c->d_scene;
    P.seed = seed;
    P.blocks = static_cast<const DBlock*>(bs->dev.p);
    P.nblocks = int32_t(nb);
    P.layout = ATR_LAYOUT_PACKED;
    P.framebuffer = static_cast<uint32_t*>(fb.p);
    P.error_flag = c->d_error;
    P.block_cost = static_cast<unsigned long long*>(cost.p);
    apply_tuning(c, P);
    const int sched = auto_sched(variant, *cam);
    if (sched < 0) return ATR_E_INVALID;
    HIPCHK(launch_render(c, P, sched, nullptr));
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(nb);
    if (nb) HIPCHK(hipMemcpy(h.data(), cost.p, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < size_t(cw) * size_t(ch); ++i) out[i] = 0;
    for (size_t k = 0; k < nb; ++k)  // a split cell's waves add up
        out[size_t(bs->host[k].y0 / 8) * size_t(cw) + size_t(bs->host[k].x0 / 8)] += int64_t(h[k]);
    return ATR_OK;
}

int atr_device_alloc(atr_ctx* c, size_t bytes, void** p) {
    if (!c || !p) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMalloc(p, bytes ? bytes : 16));
    return ATR_OK;
}
int atr_device_free(atr_ctx* c, void* p) {
    if (!c) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipFree(p));
    return ATR_OK;
}
int atr_memcpy_d2h(atr_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c || !dst || !src) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return ATR_OK;
}
int atr_memcpy_h2d(atr_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c || !dst || !src) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());  // a render may still read the destination
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return ATR_OK;
}
int atr_memset_d(atr_ctx* c, void* p, int v, size_t bytes) {
    if (!c || !p) return ATR_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemset(p, v, bytes));
    return ATR_OK;
}

}  // extern "C"
