/*
 * atr_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ATRay's per-pixel render path (AdhavanT/ATRay @ /root/reference).
 * This is the parity CHECKER for the MI355X engine in atray_amd/: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * path never links or calls it.
 *
 * Parity pin: the reference itself is unbuildable in this image without stand-in
 * headers (MSVC <intrin.h>/SVML, Win32, the un-vendored ATP submodule), so this
 * restatement is pinned against outputs of the reference recorded by the survey
 * (per-pixel (face, t-bits) FNV hashes and hit counts for
 * Cube 256x256 and Monkey 1280x720, Monkey brute-force hit counts). See DESIGN.md.
 *
 * Declared semantic at the one boundary no reference test pins: normalize() uses
 * SVML _mm_invsqrt_ps (PL/PL_math.h:387-392); here it is 1.0f/sqrtf(m2),
 * correctly rounded ("parity unpinned" at that boundary).
 */
#ifndef ATR_ORACLE_H
#define ATR_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } ov3;

/* ModelData (Source/engine/renderer/model.h:15-23), indices already 0-based. */
typedef struct {
    ov3* vertices;   uint32_t nv;
    ov3* normals;    uint32_t nn;
    ov3* texcoords;  uint32_t nt;
    int32_t* face_v;   /* 3 per face: FaceVertices::vertex_indices      */
    int32_t* face_tc;  /* 3 per face: FaceData::tex_coord_indices       */
    int32_t* face_n;   /* 3 per face: FaceData::vertex_normals_indices  */
    uint32_t nf;
} om_mesh;

/* KD_Node (kd_tree.h:26-37) restated with index-based primitive lists. */
typedef struct {
    float bmin[3], bmax[3];
    int32_t children;     /* children_start_position; 0 <=> leaf (has_children == FALSE) */
    uint32_t prim_off;    /* leaves: first entry in om_tree.prim_* */
    uint32_t prim_cnt;
} om_node;

typedef struct {
    om_node* nodes;  int32_t nnodes;
    float* prim_tri;      /* 9 floats (a,b,c) per leaf primitive, leaf order */
    uint32_t* prim_face;  /* face index per leaf primitive */
    uint32_t nprims;
    uint32_t max_faces;
} om_tree;

typedef struct { ov3 emission, reflection; float scatter; } om_material;

typedef struct { ov3 center; float radius; int32_t material; } om_sphere;
typedef struct { ov3 normal; float distance; int32_t material; } om_plane;

typedef struct {
    const om_mesh* mesh;
    const om_tree* tree;          /* NULL -> brute force branch (renderer.cpp:58-82) */
    float surrounding_aabb[6];    /* Model::surrounding_aabb (min xyz, max xyz) */
    int32_t material;             /* index into om_scene.materials */
} om_model;

typedef struct {
    const om_material* materials; int32_t nmaterials;   /* materials[0] = sky */
    const om_model* models;       int32_t nmodels;
    const om_sphere* spheres;     int32_t nspheres;
    const om_plane* planes;       int32_t nplanes;
} om_scene;

/* Camera (camera.h:9-21) + RenderSettings (settings.h:4-10) */
typedef struct {
    int32_t width, height;
    int32_t anti_aliasing;
    uint32_t spp;
    int32_t bounce_limit;
    float aspect_ratio;
    ov3 camera_z, camera_x, camera_y, eye, frame_center;
    float h_fov, half_pixel_width, half_pixel_height;
} om_camera;

typedef struct { uint64_t n_rays, n_box, n_tri, n_leaf, n_hit, n_raycasts_ref; } om_counters;

/* ---- loader / model prep ---- */
int  om_parse_obj(const char* buf, size_t len, om_mesh* out);
int  om_load_obj(const char* path, om_mesh* out);
void om_free_mesh(om_mesh* m);
void om_get_aabb(const om_mesh* m, float out[6]);
void om_translate_to(om_mesh* m, float aabb[6], ov3 new_center);

/* ---- octree ---- */
int  om_build_tree(const om_mesh* m, uint32_t max_faces, om_tree* out);
void om_free_tree(om_tree* t);

/* ---- camera ---- */
void om_set_camera(om_camera* cm, ov3 eye, ov3 facing, int32_t w, int32_t h, int32_t aa,
                   uint32_t spp, int32_t bounces, float h_fov);

/* ---- hot path ---- */
/* Primary-ray census over pixel rows [y0,y1): face (0xFFFFFFFF miss) and t bits per pixel. */
void om_primary_hits(const om_scene* s, const om_camera* cm, int32_t y0, int32_t y1,
                     uint32_t* face_out, float* t_out, om_counters* ctr);
/* Per-pixel trace of the primary ray's work: leaves scanned (in order, up to cap per pixel,
   -1 padded) and triangle tests. Diagnostic for schedule modelling. */
void om_primary_leaf_trace(const om_scene* s, const om_camera* cm, int32_t y0, int32_t y1,
                           int32_t cap, int32_t* leaves_out, uint32_t* ntri_out);
/* Arbitrary rays (origin+dir per ray, dir already normalized). */
void om_trace_rays(const om_scene* s, const float* orig, const float* dir, int64_t n,
                   uint32_t* face_out, float* t_out, float* uv_out, om_counters* ctr);
/* Full render of pixel set: deterministic per-pixel PCG stream.
   rgb_out: 3 floats/pixel (sum/spp before clamp), fb_out: BGRX u32, casts_out: per-pixel
   reference-style ray_casts (non-sky bounces summed over samples). Any out may be NULL. */
void om_render_rows(const om_scene* s, const om_camera* cm, uint64_t seed, int32_t y0, int32_t y1,
                    float* rgb_out, uint32_t* fb_out, uint32_t* casts_out, om_counters* ctr);
/* Reference tile scheduler (renderer.cpp:403-455) on `threads` pthreads with atomic tile
   claim; returns wall seconds of the render (load/build excluded). */
double om_render_threaded(const om_scene* s, const om_camera* cm, uint64_t seed, int32_t threads,
                          uint32_t* fb_out, int64_t* total_ray_casts, uint64_t* traced_rays);
/* CPU-baseline sample: rows row0 + k * row_step (k < nrows), full spp / bounces, claimed a row at
   a time by `threads` pthreads; returns wall seconds, traced rays and ray_casts of the sample. */
double om_render_rows_threaded(const om_scene* s, const om_camera* cm, uint64_t seed, int32_t threads,
                               int32_t row0, int32_t row_step, int32_t nrows, uint64_t* traced_rays,
                               int64_t* ray_casts);
/* Tile grid of renderer.cpp:403-445 (inclusive rects). Returns count; writes 4 ints/tile. */
int32_t om_make_tiles(int32_t width, int32_t height, int32_t threads, int32_t* tiles_out, int32_t cap);

uint32_t om_pcg_u32(uint64_t* state, uint64_t stream);
void om_path_rng(uint64_t seed, int64_t pixel_index, uint32_t sample, uint64_t* state, uint64_t* stream);

#ifdef __cplusplus
}
#endif
#endif
