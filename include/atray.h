/*
 * atray.h -- C-ABI of the MI355X (gfx950) intersection engine for ATRay's per-pixel render
 * loop. Drop-in boundary under the reference's render API (Source/engine/renderer/renderer.h):
 *
 *   prep_scene(Scene&, uint32&)                        renderer.h:35 / renderer.cpp:264-291
 *       -> atr_mesh_load_obj + atr_octree_build (host prerequisites, or the caller's own
 *          build_KD_tree output flattened by atr_octree_from_nodes) + atr_scene_upload
 *   start_render_from_camera(RenderInfo&, ThreadPool&) renderer.h:32 / renderer.cpp:403-455
 *       -> atr_make_tiles + atr_render_start (async on a HIP stream)
 *   wait_for_render_from_camera_to_finish(...)         renderer.h:33 / renderer.cpp:457-471
 *       -> atr_render_wait (TRUE/1 = still running, FALSE/0 = done, <0 = error)
 *
 * Plain C types and pointers only; every entry point returns an int status (0 = ok,
 * negative = ATR_E_* or -(1000 + hipError_t)). No exceptions cross the ABI. One context per
 * GPU; a context is used by one host thread at a time.
 */
#ifndef ATRAY_H
#define ATRAY_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 2 (round 6): atr_tuning gained reserved[4] (zero; room for later knobs without a size
   change); ABI 1's last two words became path_sort_bits and path_split in round 5. */
#define ATR_ABI_VERSION 2

enum {
    ATR_OK = 0,
    ATR_E_INVALID = -1,     /* bad argument */
    ATR_E_IO = -2,          /* file could not be read */
    ATR_E_NOMEM = -3,
    ATR_E_NOSCENE = -4,     /* render before atr_scene_upload */
    ATR_E_TREE_DEPTH = -5,  /* octree deeper than the traversal's mask stack (16 levels) */
    ATR_E_TREE_LAYOUT = -6, /* children boxes are not the parent's split-point octants
                               (build_oct_kd_tree makes them so, kd_tree.cpp:116-148) */
    ATR_E_HIP = -1000       /* -(1000 + hipError_t) */
};

typedef struct { float x, y, z; } atr_vec3;

/* Material (material.h:4-8). materials[0] is the sky (renderer.cpp:154). */
typedef struct { atr_vec3 emission, reflection; float scatter; } atr_material;

/* Host mesh = ModelData (model.h:15-23) with 0-based indices (OBJ_loader.cpp:229-267). */
typedef struct atr_mesh atr_mesh;
/* Host octree = KD_Tree (kd_tree.h:38-47) flattened in reference node order. */
typedef struct atr_octree atr_octree;

/* load_model_data (OBJ_loader.h:6): custom parse_f64 (parser.h:113-191), faces keep the first
   triangle of each polygon, negative indices relative to the end. atr_mesh_load_obj parses on
   the host's threads (threads = min(hardware threads, 16)); atr_mesh_parse_obj on one. */
int atr_mesh_load_obj(const char* path, atr_mesh** out);
int atr_mesh_parse_obj(const char* text, size_t len, atr_mesh** out);
/* The reference's parallel load (OBJ_loader.cpp:298-340): the text split into `threads`
   newline-aligned chunks parsed concurrently and joined in order (join_chunks, :190-227), then
   the relative indices resolved (prep_model_data, :229-267). threads = 0 picks the default.
   The mesh is bit-identical for every thread count. */
int atr_mesh_load_obj_threaded(const char* path, int32_t threads, atr_mesh** out);
int atr_mesh_parse_obj_threaded(const char* text, size_t len, int32_t threads, atr_mesh** out);
/* ModelData from caller arrays (copied). normals may be NULL (flat shading). */
int atr_mesh_from_arrays(const float* vertices, uint32_t nvertices, const int32_t* face_vertices,
                         uint32_t nfaces, const float* normals, uint32_t nnormals,
                         const int32_t* face_normals, atr_mesh** out);
void atr_mesh_free(atr_mesh* m);
int atr_mesh_info(const atr_mesh* m, uint32_t* nvertices, uint32_t* nnormals, uint32_t* nfaces);
/* Copy ModelData out (any pointer may be NULL): 3 floats per vertex / normal / texcoord, 3 ints
   per face for each index array (0-based, -1 = absent). ntexcoords (may be NULL) receives the
   texcoord count. */
int atr_mesh_export(const atr_mesh* m, float* vertices, float* normals, float* texcoords, uint32_t* ntexcoords,
                    int32_t* face_v, int32_t* face_t, int32_t* face_n);
/* get_AABB (model.h:41-61): min xyz, max xyz padded by 1e-4. */
int atr_mesh_aabb(const atr_mesh* m, float aabb_out[6]);
/* translate_to (model.h:136-152): moves the vertices and the caller's AABB (in/out). */
int atr_mesh_translate_to(atr_mesh* m, float aabb_inout[6], atr_vec3 new_center);

/* build_KD_tree (kd_tree.cpp:20-64) -> build_oct_kd_tree (:67-288), SAH-named split, leaf
   size max_faces (app.cpp:77 uses 300). Result is bit-identical to the reference's tree. */
int atr_octree_build(const atr_mesh* m, uint32_t max_faces, atr_octree** out);
/* A tree the caller already built (e.g. the reference's own KD_Tree walked into arrays):
   per node 6 floats (min, max) and children_start_position (0 = leaf); per leaf node its
   primitive range into prim_vertices (9 floats each) / prim_face. */
int atr_octree_from_nodes(int32_t nnodes, const float* node_bounds, const int32_t* node_children,
                          const uint32_t* leaf_first, const uint32_t* leaf_count, uint32_t nprims,
                          const float* prim_vertices, const uint32_t* prim_face, atr_octree** out);
/* f3: the same build on GPU `device` (atray_amd/csrc/build.hip): level-synchronous
   split sums and ordered vertex-in-box partitions as HIP kernels, nodes numbered in the
   reference's LIFO order on the host. Result bit-identical to atr_octree_build. ms_out (may be
   NULL): [0] wall time of the call incl. transfers, [1] device time of the build kernels. */
int atr_octree_build_device(const atr_mesh* m, uint32_t max_faces, int32_t device, atr_octree** out,
                            float ms_out[2]);
void atr_octree_free(atr_octree* t);
/* Copy the flattened tree out (any pointer may be NULL): 6 floats and children_start_position
   per node, leaf primitive range per node, 9 floats + face index per leaf primitive. */
int atr_octree_export(const atr_octree* t, float* node_bounds, int32_t* node_children,
                      uint32_t* leaf_first, uint32_t* leaf_count, float* prim_vertices,
                      uint32_t* prim_face);
/* nodes, inner, leaves, empty leaves, leaf primitive refs, max leaf, depth */
int atr_octree_stats(const atr_octree* t, int64_t stats_out[7]);

/* Model (model.h:66-71). tree == NULL selects the brute-force branch (renderer.cpp:58-82). */
typedef struct {
    const atr_mesh* mesh;
    const atr_octree* tree;
    float surrounding_aabb[6];
    int32_t material;
} atr_model;
typedef struct { atr_vec3 center; float radius; int32_t material; } atr_sphere; /* sphere.h:5-10 */
typedef struct { atr_vec3 normal; float distance; int32_t material; } atr_plane; /* plane.h:5-10 */

/* Camera (camera.h:9-21) + RenderSettings (settings.h:4-10). atr_camera_set = set_camera. */
typedef struct {
    int32_t width, height;
    int32_t anti_aliasing;
    uint32_t samples_per_pixel;
    int32_t bounce_limit;
    float aspect_ratio;
    atr_vec3 camera_z, camera_x, camera_y, eye, frame_center;
    float h_fov, half_pixel_width, half_pixel_height;
} atr_camera;
int atr_camera_set(atr_camera* cm, atr_vec3 eye, atr_vec3 facing, int32_t width, int32_t height,
                   int32_t anti_aliasing, uint32_t spp, int32_t bounce_limit, float h_fov);

/* Tile (PL_math.h:147-149,185): inclusive pixel rect, row 0 = bottom. */
typedef struct { int32_t min_x, min_y, max_x, max_y; } atr_tile;
/* Reference tile grid (renderer.cpp:406-445): side W/threads (or H/threads), rects overlap by
   one pixel. Returns the tile count; writes at most cap tiles. */
int32_t atr_make_tiles(int32_t width, int32_t height, int32_t threads, atr_tile* out, int32_t cap);
/* Engine tiling for sharding: non-overlapping side x side tiles, tile k owned by rank
   k % world (interleaved for load balance). Returns the count written for `rank`. */
int32_t atr_make_shard_tiles(int32_t width, int32_t height, int32_t side, int32_t rank,
                             int32_t world, atr_tile* out, int32_t cap);
/* Cost-balanced alternative: the same side x side grid (row-major, costs[i] per grid tile, e.g.
   from atr_render_tile_costs) dealt longest-first to the least loaded rank; rank 0 starts with
   rank0_extra (its frame assembly). Writes owner_out[i] per grid tile; returns the tile count. */
int32_t atr_balance_shard_tiles(int32_t width, int32_t height, int32_t side, int32_t world,
                                const int64_t* costs, int64_t rank0_extra, int32_t* owner_out);

/* Live-view output (texture.cpp:66-115, Write_To_File): the BGRX u32 image (row 0 = bottom) as a
   32-bit BI_BITFIELDS BMP, 14-byte file header + 56-byte header, written to the first of
   "<name>_0.bmp", "<name>_1.bmp", ... that does not exist yet (created exclusively). The path
   taken goes to out_path (out_cap bytes, may be NULL). Like the reference's name buffer of
   strlen(name) + 8 bytes, ids stop at 99: ATR_E_IO once <name>_0 .. <name>_99 all exist, or the
   file cannot be created. Host memory only; no device needed. */
int atr_write_bmp(const uint32_t* pixels, int32_t width, int32_t height, const char* name, char* out_path,
                  int32_t out_cap);

/* ---------------------------------------------------------------- device engine */
typedef struct atr_ctx atr_ctx;
int atr_create(int device, atr_ctx** out);
int atr_destroy(atr_ctx* ctx);
const char* atr_version(void);

/* Scheduling knobs of a context. They change launch order and work distribution only, never an
   output bit (every value is covered by the GPU parity tests). atr_default_tuning fills the
   measured defaults; atr_set_tuning validates and copies (ATR_E_INVALID on an out
   of range field); cluster_size takes effect at the next
   atr_scene_upload, the others at the next launch. */
typedef struct {
    int32_t xcd_chunk;      /* cell schedules: consecutive workgroups per XCD chunk (0 = one
                               contiguous range per XCD), 0..4096; default 16 */
    int32_t frame_rotate;   /* multi-frame launches: frame f's cell list starts f/F x this/1024 of
                               the way in, 0..1024; default 0 */
    int32_t hybrid_a, hybrid_b; /* HYBRID: a leaf step is dealt over the lanes when the largest
                               cluster count exceeds a x rounds + b, -4096..4096; default 2, 0 */
    int32_t path_batch_log2; /* PATHS: paths per batch = 2^this (the path queues hold one batch,
                               144 B per path, 156 with the queue sort), 12..28; default 28
                               (1920x1080 at 64 spp: a frame in one batch). A workspace holds the
                               launch's paths rounded up to 2^24, at most one batch: 20.9 GB for a
                               1920x1080 64-spp frame, 42 GB at most (4 per context: 167 GB);
                               a workspace too small for a later launch grows to a whole batch.
                               2^29 measured 5-7x slower */
    int32_t cluster_size;   /* primitives per leaf cluster, 1..16; default 16 */
    int32_t frame_plan;     /* 1: a single-frame launch on the stream of the previous ones
                               dispatches its tiles' cells by the measured cost of the launch two
                               before it, heaviest first, the heaviest 1 % over two waves (built on
                               the GPU on the context's plan stream after each such launch, beside
                               the next one); 0: list order; default 1. With an
                               atr_set_cell_plan plan for the image size it re-orders that plan's
                               block list */
    int32_t path_camera_occ; /* PATHS: waves/SIMD of the camera-ray and bounce launches, 5..7, */
    int32_t path_bounce_occ; /* or 0 = the measured default */
    int32_t primary_occ;    /* HYBRID primary cell launches: waves/SIMD 6, 7 or 8, or 0 = the
                               measured default (8 for one frame, 7 for frames in flight;
                               DESIGN.md §4e) */
    int32_t path_sort_bits; /* PATHS: 2..7 = each level's queue is put in the order of (the ray's
                               direction cell, 16 x 16 octahedral; its origin's cell, this many
                               bits per axis of the scene box) before the next bounce launch, so a
                               wavefront takes rays that walk the same tree nodes (6 at most is
                               used); 0 = queue order; default 5 */
    int32_t path_split;     /* PATHS: 1 = a launch that is one batch (a single frame) runs as two
                               half batches on two internal streams, forked from and joined back
                               into the render's stream; 0 = one stream */
    int32_t reserved[4];    /* must be 0 (ATR_E_INVALID otherwise) */
} atr_tuning;
void atr_default_tuning(atr_tuning* out);
int atr_set_tuning(atr_ctx* ctx, const atr_tuning* tuning);
int atr_get_tuning(atr_ctx* ctx, atr_tuning* out);

/* Flatten + upload the scene (copies; the caller keeps its buffers). prep_scene's tree build
   happens before this call (atr_octree_build); upload is not part of the render timing. */
int atr_scene_upload(atr_ctx* ctx, const atr_material* materials, int32_t nmaterials,
                     const atr_model* models, int32_t nmodels, const atr_sphere* spheres,
                     int32_t nspheres, const atr_plane* planes, int32_t nplanes);
/* device bytes of the uploaded scene, per-model node count and max tree depth */
int atr_scene_info(atr_ctx* ctx, int64_t* device_bytes, int32_t* max_nodes, int32_t* max_depth);
/* Path-engine workspaces held by the context (PATHS: two path queues + per-path results, 144 B per
   path of a batch): how many (at most 4, whatever the number of streams rendering: a stream without
   one takes an idle or the least recently used one) and their device bytes. When the device cannot
   hold a batch's workspace the engine halves the batch (down to 2^16 paths), then renders on FLAT,
   which needs none; outputs are identical either way. */
int atr_workspace_info(atr_ctx* ctx, int32_t* workspaces, int64_t* device_bytes);

/* Output layout of a render. IMAGE: pixel (x,y) at y*width + x. PACKED: the pixels of the
   render's work blocks back to back (atr_render_packed_size); atr_unpack scatters them. */
enum { ATR_LAYOUT_IMAGE = 0, ATR_LAYOUT_PACKED = 1 };

/* Per-pixel outputs; DEVICE pointers (hipMalloc / torch cuda tensors). Optional ones may be
   NULL. framebuffer: BGRX u32 (texture.h:27-38). hit_face/hit_t: primary-ray closest hit of
   sample 0 (face index, 0xFFFFFFFF = miss; t = 3.402823466e38 on miss). rgb: 3 floats per pixel,
   the spp average before clamp (renderer.cpp:358). ray_casts: the reference's per-pixel
   non-sky bounce count (renderer.cpp:260). traced_rays: one u64 accumulator (+= every
   get_intersection_data-equivalent call). */
typedef struct {
    int32_t layout;
    uint32_t* framebuffer;
    uint32_t* hit_face;
    float* hit_t;
    float* rgb;
    uint32_t* ray_casts;
    unsigned long long* traced_rays;
} atr_frame;

/* Kernel variant: AUTO picks the fastest exact variant (HYBRID for primary-only renders -- one
   sample, bounce_limit 1, no AA -- else PATHS, or FLAT beyond 64 bounces). All variants are
   bit-identical; any other value is ATR_E_INVALID. (Codes 2-7 were round-1..3 schedules measured
   slower and removed) */
enum { ATR_KERNEL_AUTO = 0,
       ATR_KERNEL_LANE = 1 /* the reference's exact work: every triangle of every scanned leaf */,
       ATR_KERNEL_FLAT = 8 /* cell megakernel: clustered scan, the wavefront's (ray, cluster) work
                              dealt over its lanes in rounds, a pixel's samples in sequence */,
       ATR_KERNEL_HYBRID = 9 /* cell kernel, per leaf step: lane-private scans when the rays' cluster
                                counts are alike, FLAT rounds when one ray's leaf dominates */,
       ATR_KERNEL_PATHS = 10 /* sample-parallel path engine: one lane per (pixel, sample) path, one
                                launch per bounce over a queue of the live paths (<= 64 bounces) */ };

/* start_render_from_camera: renders the pixels of `tiles` (inclusive rects; overlapping pixels
   are traced once) into `frame`, enqueued on `stream` (hipStream_t; NULL = the null stream, HIP's
   convention). RNG: one deterministic PCG stream per (pixel, sample) from `seed`.
   Returns immediately. */
int atr_render_start(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                     const atr_frame* frame, uint64_t seed, void* stream);
/* Progressive start for a live view (app.cpp:162-186): the tiles are rendered in list order,
   tiles_per_launch per launch, so atr_render_wait's tiles_done grows while the render runs and
   the finished tiles of the IMAGE framebuffer can be shown. Each pixel is still traced once (a
   pixel of overlapping tiles belongs to the first), and every output equals atr_render_start's. */
int atr_render_start_progressive(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                                 const atr_frame* frame, uint64_t seed, void* stream, int32_t variant,
                                 int32_t tiles_per_launch);
/* Like atr_render_start with an explicit kernel variant. */
int atr_render_start_ex(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                        const atr_frame* frame, uint64_t seed, void* stream, int32_t variant);
/* Frames in flight in one launch (throughput, e.g. a live view rendering ahead): nframes renders
   of the same camera and tiles; frame f's outputs start frame_stride elements after frame f-1's
   (rgb: 3 x frame_stride floats; frame_stride >= the layout's pixels per frame). The cell
   schedules run all frames as one grid, so one frame's slow cells overlap the next frame's; the
   path engine runs the frames' cells as one list. Every frame equals atr_render_start_ex's
   output. */
int atr_render_start_frames(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                            const atr_frame* frame, int32_t nframes, int64_t frame_stride, uint64_t seed,
                            void* stream, int32_t variant);
/* The same with one camera per frame (an animation, a camera path): frame f renders cams[f]
   (1 <= nframes <= 24). All cameras must share width, height, samples_per_pixel, bounce_limit
   and anti_aliasing (ATR_E_INVALID otherwise); eye, facing and field of view may differ. Every
   frame equals atr_render_start_ex's output for its camera. */
int atr_render_start_cameras(atr_ctx* ctx, const atr_camera* cams, int32_t nframes, const atr_tile* tiles,
                             int32_t ntiles, const atr_frame* frame, int64_t frame_stride, uint64_t seed,
                             void* stream, int32_t variant);
/* Load-balance calibration, synchronous: renders `tiles` once (default kernel) and returns the
   GPU shader clocks spent per tile (sum over the 8x8 blocks whose area first falls in the tile,
   list order). Used to deal shard tiles to GPUs by measured cost (atray_amd/shard.py). */
int atr_render_tile_costs(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                          uint64_t seed, int64_t* cost_out);
/* Diagnostic, synchronous: an instrumented render of the same work that returns
   [0] traced rays, [1] box tests, [2] triangle tests, [3] leaves scanned -- the reference's own
   per-ray work on this input (kd_tree.cpp:337-465) for every variant but the clustered ones,
   whose [2] counts the full triangle tests they still run -- and the engine's [4] wave-level
   triangle iterations, [5] DFS passes, [6] all octree box tests, [7] wavefronts, [8] cluster
   boxes tested and [9] primitives screened by the clustered scan. */
int atr_render_counters(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                        uint64_t seed, int32_t variant, int64_t counters_out[10]);
/* Number of pixels a PACKED render of these tiles writes. */
int64_t atr_render_packed_size(const atr_tile* tiles, int32_t ntiles);
/* Host-only: pixel index (y * width + x) of every slot of a PACKED render of these tiles, in
   slot order (lets a host consumer read packed buffers). Returns the slot count. */
int64_t atr_packed_pixel_map(const atr_tile* tiles, int32_t ntiles, int32_t width, int32_t height,
                             int64_t* out, int64_t cap);
/* Scatter a PACKED buffer (u32 per pixel) of these tiles into an IMAGE buffer (device). */
int atr_unpack(atr_ctx* ctx, const atr_tile* tiles, int32_t ntiles, int32_t width,
               const uint32_t* packed, uint32_t* image, void* stream);
/* Per-tile sum of an IMAGE ray_casts buffer over inclusive (possibly overlapping) tile rects
   -> the reference's RenderTile::ray_casts (renderer.h:11-15); out is a device int64 array. */
int atr_tile_ray_casts(atr_ctx* ctx, const atr_tile* tiles, int32_t ntiles, int32_t width,
                       const uint32_t* ray_casts_image, int64_t* out, void* stream);
/* Per-tile sums of a PACKED ray_casts buffer holding `nframes` frames (frame f at f *
   frame_stride elements) rendered with these tiles at width x height -- the reference's
   RenderTile::ray_casts (renderer.h:11-15, summed at renderer.cpp:465-468) for a shard's tiles
   without an IMAGE copy: out[f * ntiles + i] = sum over the pixels of tile i (a pixel of
   overlapping tiles counts in the first tile holding it: the packed layout traces it once).
   Asynchronous on `stream`; out is a device int64 array, zeroed here. */
int atr_packed_tile_ray_casts(atr_ctx* ctx, const atr_tile* tiles, int32_t ntiles, int32_t width,
                              int32_t height, const uint32_t* packed_ray_casts, int32_t nframes,
                              int64_t frame_stride, int64_t* out, void* stream);
/* Multi-GPU frame exchange in 3 bytes per pixel (the framebuffer's X byte is always 0,
   texture.h:27-38). atr_pack_bgr: npixels BGRX u32 -> 3 * npixels bytes (B, G, R per pixel).
   atr_scatter_bgr: the inverse with a scatter, image[dst_index[i]] = B | G << 8 | R << 16 for
   pixel i of `packed` (e.g. rank 0's gathered shard frames and their assembly index). Device
   pointers; asynchronous on `stream`. */
int atr_pack_bgr(atr_ctx* ctx, const uint32_t* framebuffer, int64_t npixels, uint8_t* out, void* stream);
int atr_scatter_bgr(atr_ctx* ctx, const uint8_t* packed, int64_t npixels, const int64_t* dst_index, uint32_t* image,
                    void* stream);
/* Lossless masked exchange (round 6): frames that are mostly one background value (a c3 frame is
   86% sky) travel as a bit per pixel plus 3 bytes for each pixel that differs from `background`
   (any value is correct; the common one compresses best): ~0.54 B per c3 pixel instead of 3.
   Stream: a 16-byte header {magic "ATRN", background, chunks, payload pixels}, one u32 payload
   offset per 8192-pixel chunk, 1 KB of mask bits per chunk, 512 B of group offsets per chunk (the
   payload offset of every 64 pixels, so decoders need no scan), then B, G, R of every
   non-background pixel in order. atr_pack_bgr_masked_bound(n) = the largest stream for n pixels (host, no device;
   size `out` by it); atr_pack_bgr_masked writes the stream and its exact byte count to the DEVICE
   int64 *nbytes (the sender ships that many bytes); atr_scatter_bgr_masked decodes a stream of
   npixels into image[dst_index[i]] (as atr_scatter_bgr). Device pointers; async on `stream`;
   npixels < 2^32. */
int64_t atr_pack_bgr_masked_bound(int64_t npixels);
int atr_pack_bgr_masked(atr_ctx* ctx, const uint32_t* framebuffer, int64_t npixels, uint32_t background, uint8_t* out,
                        int64_t* nbytes, void* stream);
int atr_scatter_bgr_masked(atr_ctx* ctx, const uint8_t* packed, int64_t npixels, const int64_t* dst_index,
                           uint32_t* image, void* stream);
/* The masked stream of a PACKED render of these tiles (nframes frames, as atr_pack_bgr_masked wrote
   it from that render's framebuffer) straight into IMAGE frames: frame f's pixel (x, y) at
   image[f * image_stride + y * width + x]. Positions come from the tile list's 8x8 blocks (as
   atr_unpack) instead of an index per pixel: ~5 B of traffic per pixel instead of ~13. */
int atr_unpack_masked(atr_ctx* ctx, const atr_tile* tiles, int32_t ntiles, int32_t width, int32_t height,
                      const uint8_t* packed, int32_t nframes, uint32_t* image, int64_t image_stride, void* stream);
/* Several masked streams into the same IMAGE frames in one call (rank 0's received shards, one
   source per rank): source i is the PACKED render of tiles[i] (ntiles[i] tiles, the list it was
   rendered with), its stream at packed[i] (device), nframes frames each, image_stride apart; with
   raw[i] nonzero (raw may be NULL) packed[i] is that render's u32 PACKED framebuffer itself (rank
   0's own frames), copied in by the same launch. The same pixels as atr_unpack_masked (or
   atr_unpack) per source, from one decode launch per 16 sources instead of a launch and an event
   per source. Asynchronous on `stream`. */
int atr_unpack_masked_ranks(atr_ctx* ctx, int32_t nsrc, const atr_tile* const* tiles, const int32_t* ntiles,
                            int32_t width, int32_t height, const uint8_t* const* packed, const int32_t* raw,
                            int32_t nframes, uint32_t* image, int64_t image_stride, void* stream);
/* Per-cell launch plan for renders of width x height (NULL clears): one byte per 8x8 cell (row
   major, ceil(W/8) x ceil(H/8)). Low nibble: the number of waves the cell is split into (0/1 =
   one, 2, 4 or 8 row bands: a heavy cell's rays then share their dealt leaf scans with 2-8x as
   many lanes and its dependent chain shortens). Bits 4-6: the cell's dispatch class c (0-7):
   cells of class 7 are dispatched first, then 6, ..., then 0 (list order within a class), e.g.
   the heaviest cells of the previous frame first (ATR_PLAN_CLASS(c) = c << 4). ATR_PLAN_PRIO:
   its waves issue at raised priority on their SIMD. Only scheduling changes: outputs and the
   PACKED slot order are identical with any plan. */
#define ATR_PLAN_CLASS(c) ((uint8_t)(((c) & 7) << 4))
enum { ATR_PLAN_PRIO = 0x80 };
int atr_set_cell_plan(atr_ctx* ctx, int32_t width, int32_t height, const uint8_t* plan);
/* Diagnostic, synchronous: the single-frame plan of a tile list (tuning frame_plan) built last,
   from the last planned launch's costs (the list the launch after next dispatches by): *nplanned =
   the planned block list's length (0 = no plan yet; a size query when cap is too small); per
   planned block its base block index (base_out) and lane mask (2 u32, lo then hi); cost_out = the
   clocks per base block of the last measured launch (the base list's length). */
int atr_render_plan_info(atr_ctx* ctx, const atr_tile* tiles, int32_t ntiles, int32_t width, int32_t height,
                         int32_t* base_out, uint32_t* mask_hi_lo_out, int64_t cap, uint64_t* cost_out,
                         int64_t* nplanned);
/* Measured cost (shader clocks) of every 8x8 cell of a full-frame render of `cam` with `variant`
   (cell kernels only): out has ceil(W/8) x ceil(H/8) entries, row major. Synchronous. */
int atr_render_cell_costs(atr_ctx* ctx, const atr_camera* cam, uint64_t seed, int32_t variant,
                          int64_t* out);
/* wait_for_render_from_camera_to_finish: 1 = still running after timeout_ms, 0 = done,
   <0 = error. tiles_done (optional) = tiles of the last render known complete (progress). */
int atr_render_wait(atr_ctx* ctx, uint32_t timeout_ms, int32_t* tiles_done);

/* Device-time of the last render's trace kernel(s) in milliseconds (HIP events recorded on the
   launch stream around the kernel). Valid after atr_render_wait returned 0. */
int atr_last_kernel_ms(atr_ctx* ctx, float* ms);

/* device memory helpers for C callers without a framework */
int atr_device_alloc(atr_ctx* ctx, size_t bytes, void** dptr);
int atr_device_free(atr_ctx* ctx, void* dptr);
int atr_memcpy_d2h(atr_ctx* ctx, void* dst, const void* src, size_t bytes);
int atr_memcpy_h2d(atr_ctx* ctx, void* dptr, const void* src, size_t bytes);
int atr_memset_d(atr_ctx* ctx, void* dptr, int value, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif
