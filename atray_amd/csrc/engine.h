// engine.h -- internal types shared by the host side (scene prep, C-ABI) and the HIP kernels.
// Everything here is plain data; f32 helpers are __host__ __device__ so host-side
// precomputation and the kernels evaluate the same expressions in the same order
// (reference op order: PL/PL_math.h:106-123,416-422). Built with -ffp-contract=off.
#pragma once
#include <math.h>
#include <stdint.h>

#include "../../include/atray.h"

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define ATR_HD __host__ __device__ __forceinline__
#else
#define ATR_HD inline
#endif

namespace atr {

struct alignas(16) float4_t { float x, y, z, w; };
struct alignas(16) uint4_t { uint32_t x, y, z, w; };
struct alignas(8) float2_t { float x, y; };
struct alignas(8) uint2_t { uint32_t x, y; };

constexpr float kMaxFloat = 3.402823466e+38F;     // PL_base_defs.h:72
constexpr float kInvU32Max = 2.328306437e-10F;    // PL_base_defs.h:75
constexpr float kTol = 0.0001f;                   // ray.h:5
constexpr int kMaskLevels = 16;                   // traversal mask-stack depth (8 bits/level)
constexpr int kMaxMaterials = 32;
#ifndef ATR_MAX_FRAME_CAMS  // experiment builds: more cameras per launch (kernel argument size)
#define ATR_MAX_FRAME_CAMS 24
#endif
constexpr int kMaxFrameCams = ATR_MAX_FRAME_CAMS;  // distinct cameras per multi-frame launch (kernel argument)
constexpr int kMaxModels = 8;
// Primitive slots per leaf cluster (atr_tuning.cluster_size <= this) and 16-B words per cluster
// block (one 128-B line: record (2), screen normals (6)). 32 slots in 256-B blocks measured slower
// (DESIGN.md §4b); the layout code is written for either.
constexpr int kMaxClusterSize = 16;
constexpr int kClusterBlock = 8;
constexpr int kNormWords = kMaxClusterSize + kMaxClusterSize / 2;  // u32 screen-normal words per cluster

struct V3 { float x, y, z; };
ATR_HD V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
ATR_HD V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
ATR_HD V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
ATR_HD V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
ATR_HD V3 scale(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
ATR_HD V3 divs(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
ATR_HD V3 had(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
ATR_HD float dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
ATR_HD V3 cross(V3 a, V3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
ATR_HD float len2(V3 v) { return (v.x * v.x) + (v.y * v.y) + (v.z * v.z); }
// normalize (PL_math.h:387-392). SVML _mm_invsqrt_ps is declared as 1/sqrtf.
ATR_HD V3 unit(V3 v) { float inv = 1.0f / sqrtf(len2(v)); return scale(v, inv); }
ATR_HD V3 lerp3(V3 s, V3 t, float k) { return add(scale(sub(t, s), k), s); }
ATR_HD float pl_max(float a, float b) { return a > b ? a : b; }
ATR_HD float pl_min(float a, float b) { return a > b ? b : a; }
ATR_HD V3 from(atr_vec3 v) { return mk(v.x, v.y, v.z); }

// PCG-XSH-RR (PL_math.h:506-516)
ATR_HD uint32_t pcg_next(uint64_t& state, uint64_t stream) {
    uint64_t old = state;
    state = old * 6364136223846793005ULL + (stream | 1ULL);
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
}
ATR_HD float rand_bi(uint64_t& state, uint64_t stream) {  // PL_math.h:525-541
    float rd = (float)pcg_next(state, stream) * kInvU32Max;
    return -1.0f + 2.0f * rd;
}
// One PCG stream per (pixel, sample) (deviation from renderer.cpp:376-378's rdtsc*thread seeding,
// DESIGN.md §2): state = splitmix64(seed ^ pixel ^ sample << 40), increment 2 pixel + 1. A pixel's
// samples are independent paths, so they can run in parallel (paths.hip); sample 0's stream is the
// round-1..3 per-pixel stream.
ATR_HD void path_stream(uint64_t seed, int64_t pixel, uint32_t sample, uint64_t& state, uint64_t& stream) {
    uint64_t x = seed ^ (uint64_t)pixel ^ ((uint64_t)sample << 40);
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    state = x ^ (x >> 31);
    stream = ((uint64_t)pixel << 1) | 1ULL;
}

// ---------------------------------------------------------------- device scene layout
// Octree node, 32 B: two float4 loads. children = children_start_position (0 = leaf),
// parent = index of the parent node (-1 for the root), used by the stackless DFS.
struct alignas(16) DNode {
    float lo_x, lo_y, lo_z, hi_x;
    float hi_y, hi_z;
    int32_t children;
    int32_t parent;
};
static_assert(sizeof(DNode) == 32, "DNode layout");

// Leaf primitive / brute-force triangle, 48 B: a, ab = b - a, ac = c - a (the first two
// subtractions of model.h:77-78, done once on the host: same IEEE f32 results), face index.
struct alignas(16) DTri {
    float ax, ay, az, abx;
    float aby, abz, acx, acy;
    float acz;
    uint32_t face;
    float pad0, pad1;
};
static_assert(sizeof(DTri) == 48, "DTri layout");

// Per-model device view. has_tree == 0 selects the brute-force branch (renderer.cpp:58-82).
struct DModel {
    const DNode* nodes;          // octree nodes in reference order (root = 0)
    // inner nodes only: 3 float4 = {lo.xyz, v.x}{v.yz, hi.xy}{hi.z, bits(first
    // child node), bits(parent inner id), bits((inner id of first inner child << 8) | leaf mask)};
    // the children boxes are derived from lo, v, hi (kd_tree.cpp:116-148)
    const float4_t* inner;
    int32_t ninner;
    const uint32_t* leaf_range;  // 2 u32 per node: first DTri, count (leaves only)
    const DTri* tris;            // leaf-ordered primitives (tree) or face-ordered (brute force)
    // the same primitives as SoA streams for per-lane loads: t0 = {a.xyz, ab.x},
    // t1 = {ab.yz, ac.xy}, t2 = ac.z (36 B per test); tface read only for the final hit
    const float4_t* t0;
    const float4_t* t1;
    const float* t2;
    const uint32_t* tface;
    // leaf clusters, 2 float4 per cluster: {lo.xyz, bound of |ab||ac| with
    // (n - 1) in its low 5 mantissa bits}, {hi.xyz, q}; cl_range = first cluster, count per
    // node. Cluster c owns the primitive slots [16 c, 16 c + n) and the 128-B block clus[8 c ..]:
    // its record (2 words), then (cnrm = clus + 2) 6 words of its screen normals
    // n = ab x ac as f16 integer multiples of q (the screen, cluster.h); prim = 48 B per slot:
    // {a.xyz, ab.x}{ab.yz, ac.xy}{ac.z, bits(leaf rank), bits(face index), 0}
    const float4_t* clus;
    const uint32_t* cl_range;
    const uint4_t* cnrm;
    const float4_t* prim;
    const float* shade;          // 9 f32 per face: smooth -> na, nb, nc; flat -> v0, v1, v2
    uint32_t nfaces;
    int32_t has_tree;
    int32_t root_leaf;           // root never split (kd_tree.cpp:344-361)
    int32_t near_ok;             // depth <= 8 and < 2^16 inner nodes: near-first passes (trace.h)
    int32_t smooth;              // normals.size > 0 (renderer.cpp:129)
    int32_t material;
    float aabb[6];               // Model::surrounding_aabb
};

struct DMaterial { float ex, ey, ez, rx, ry, rz, scatter, pad; };
struct DSphere { float cx, cy, cz, r; int32_t material, pad0, pad1, pad2; };
struct DPlane { float nx, ny, nz, d; int32_t material, pad0, pad1, pad2; };

// Scene-wide device data, uploaded once by atr_scene_upload (read via scalar loads).
struct DScene {
    DMaterial mats[kMaxMaterials];
    DModel models[kMaxModels];
    int32_t nmats, nmodels, nspheres, nplanes;
    const DSphere* spheres;
    const DPlane* planes;
};

// A work block: one wavefront, an 8x8 pixel cell at (x0, y0); lane l -> (x0 + (l & 7),
// y0 + (l >> 3)); only lanes whose bit is set in `mask` own a pixel of the render.
struct alignas(16) DBlock {
    int32_t x0, y0;
    uint32_t mask_lo, mask_hi;
    int32_t out_base;  // PACKED layout: output slot of the block's first owned pixel
    int32_t flags;     // kBlockPrio: the wave raises its issue priority (cell plan, atr_set_cell_plan)
    int32_t base;      // index of the block in its tile list's base block list (per-block cost slot)
    int32_t pad;
};
static_assert(sizeof(DBlock) == 32, "DBlock layout");
constexpr int32_t kBlockPrio = 1;
// cell plan byte (atr_set_cell_plan): low nibble = waves per cell (0/1, 2, 4, 8); bits 4-6 = the
// cell's dispatch class (blocks of class 7 lead the block list, then 6, ..., 0; Morton order within
// a class; their packed slots do not move); kPlanPrio = its waves issue at raised priority
constexpr int kPlanClassShift = 4;
constexpr uint8_t kPlanClassMask = 0x70, kPlanPrio = 0x80;

// Per-render kernel argument (by value, no dynamic indexing into it).
struct RenderParams {
    atr_camera cam;
    const DScene* scene;
    uint64_t seed;
    const DBlock* blocks;
    int32_t nblocks;
    int32_t layout;
    uint32_t* framebuffer;
    uint32_t* hit_face;
    float* hit_t;
    float* rgb;
    uint32_t* ray_casts;
    // 64 traced-ray counters 128 B apart (a zeroed 8-KB slot of the context's ring, capi.cpp
    // launch_render); the kernel adds each wave's count to slot (block & 63). Never a caller's
    // single accumulator: atr_launch_render rejects it together with `counters`.
    unsigned long long* traced_rays;
    int32_t* error_flag;  // set to 1 if a ray hit a traversal limit (never for depth <= 16)
    unsigned long long* counters;  // non-null -> instrumented kernel (10 u64, see render.hip)
    unsigned long long* block_cost;  // non-null -> shader clocks added per base block (blocks[b].base)
    unsigned long long* wave_trace;  // non-null -> per block: start, end (100 MHz clock), HW_ID | XCC_ID << 32
    int32_t xcd_chunk;  // 0: contiguous block range per XCD; k > 0: k-workgroup chunks dealt round-robin
    int32_t frame_blocks;  // > 0: nblocks = frames x frame_blocks, one launch renders every frame
    int64_t frame_stride;  // output elements between consecutive frames (rgb: 3 x this)
    int32_t frame_rotate;  // frame f's blocks start f / frames x frame_rotate / 1024 into its list
    int32_t hyb_a, hyb_b;  // HYBRID: a step's leaves are dealt in rounds when max clusters > a x rounds + b
    int32_t nfcam;         // > 0: frame f renders with fcam[f] instead of cam (same size/spp/bounces)
    atr_camera fcam[kMaxFrameCams];
};

// Sample-parallel path engine (paths.hip): one lane per (pixel, sample) path. A batch
// is a contiguous range [cell0, cell0 + ncells) of the launch's cell list (frames interleaved as in
// RenderParams: cell c renders block c / nf of frame c % nf). The camera launch's wavefront w of
// the batch takes paths r = 64 w .. 64 w + 63 of cell w / spp (r -> pixel lane r / spp, sample
// r % spp: a pixel's samples side by side), so a wavefront lies in one cell. Path records between
// bounces are four float4 planes of `cap` entries each:
//   p0 = {o.xyz, d.x}, p1 = {d.y, d.z, bits(pixel), bits(g)}, p2 = {ret.xyz, w.x},
//   p3 = {w.y, w.z, bits(rng lo), bits(rng hi)};
// a finished path leaves {colour.xyz, bits(ray_casts)} in its result slot
// out[g], g = (c - cell0) x 64 spp + sample x 64 + pixel lane.
constexpr int kPathPlanes = 4;
// Per bounce level k of a batch (zeroed before the batch): the launch of level k (0 = the camera
// rays) appends its surviving paths to queue k & 1 (tail); the bounce launch k + 1 reads them,
// its persistent waves claiming 64 at a time (head of level k + 1).
struct PathCtl {
    uint32_t tail;
    uint32_t head;
};
// Queue sort (tuning path_sort_bits = b > 0): the queues are entry-major (an entry's
// four records together, q[4 e + i], 64 B) and every queued path also records {key, rank} in `kr`:
// key = the ray's coarse direction cell (4 x 4 of the 16 x 16 octahedral cells), a Morton code of
// its origin quantised to b bits per axis over the scene box (lo, sc = 2^b / extent), then its fine
// direction cell within the coarse one (paths.hip path_sort_key), rank = its arrival
// in the key's bin (atomicAdd on hist). The sort launches turn hist into bin starts and write the
// level's key order perm[start[key] + rank] = entry; the next bounce launch's waves claim positions
// of that order, so a wavefront takes rays of one direction cell and one region together (a
// counting sort of 4-B indices; the entries never move; the order within a bin is arrival order,
// and no output depends on queue order).
#ifndef ATR_SORT_DIRS
#define ATR_SORT_DIRS 16
#endif
constexpr int kSortDirs = ATR_SORT_DIRS;  // direction cells per side of the octahedral map
constexpr int kMaxSortBits = 7;
constexpr int64_t kSortBinsMax = int64_t(1) << 26;  // 256 direction cells x 6 bits per axis
constexpr int32_t kSortChunk = 4096;  // bins per block of the bin scan
static_assert((kSortDirs * kSortDirs << 6) % kSortChunk == 0, "the fewest bins (2 bits per axis) fill whole scan blocks");
static_assert((kSortBinsMax / kSortChunk) <= 32768, "path_sort_part_scan: one workgroup, 32 sums per lane");
struct PathSort {
    int32_t bits;      // 0: off
    int32_t nbins;     // kSortDirs^2 << 3 bits
    float lo[3], sc[3];
    uint2_t* kr;       // {key, rank} per entry of the level being written
    uint32_t* perm;    // the previous level's key order (entry per position)
    uint32_t* hist;    // nbins arrival counters (zero between levels)
    uint32_t* start;   // nbins bin starts
    uint32_t* part;    // nbins / kSortChunk block sums
};

struct PathParams {
    atr_camera cam;
    const DScene* scene;
    uint64_t seed;
    const DBlock* blocks;
    int32_t frame_blocks;  // blocks per frame (the launch's frames: nf = nblocks / frame_blocks)
    int32_t nblocks;       // cells of the launch (all frames)
    int32_t cell0, ncells; // this batch
    int32_t layout;
    int64_t frame_stride;
    uint32_t* framebuffer;
    uint32_t* hit_face;
    float* hit_t;
    float* rgb;
    uint32_t* ray_casts;
    unsigned long long* traced_rays;  // 64 spread counters (a ring slot), or null
    int32_t* error_flag;
    unsigned long long* block_cost;   // non-null -> shader clocks per base block (calibration)
    float4_t* q[2];   // path queues, kPathPlanes planes of cap entries each
    int64_t cap;      // entries per plane (>= the batch's paths)
    float4_t* out;    // per path: colour and ray_casts of the finished path
    PathCtl* ctl;     // one per bounce level
    unsigned long long* counters;  // non-null -> instrumented kernels (counters [0..9] of render.hip)
    int32_t bounce;   // bounce launch: this bounce (1 .. bounce_limit - 1)
    int32_t xcd_chunk;
    int32_t hyb_a, hyb_b;
    int32_t nfcam;
    PathSort sort;
    atr_camera fcam[kMaxFrameCams];
};

}  // namespace atr
