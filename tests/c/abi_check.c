/* abi_check.c -- a plain C caller of include/atray.h (the surface a reference-side binding links,
 * INTEGRATION.md). Built by gcc (atray_amd/csrc/Makefile) against libatray_hip.so.
 *
 *   abi_check layout         sizeof/offsetof of every ABI struct as one JSON line (the Python
 *                            ctypes mirrors are checked against it, tests/test_capi_c.py)
 *   abi_check host <Cube.obj> host entry points only: load, AABB, translate, octree stats,
 *                            camera, reference tiles (no GPU needed)
 *   abi_check gpu <Cube.obj>  the renderer.h flow from C: atr_create -> atr_scene_upload ->
 *                            atr_render_start -> atr_render_wait, Cube 256x256 primary hits,
 *                            FNV-1a hash of (face, t bits) as the survey computed it
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/atray.h"

#define OFF(T, f) printf("\"%s.%s\": %zu, ", #T, #f, offsetof(T, f))
#define SZ(T) printf("\"sizeof(%s)\": %zu, ", #T, sizeof(T))

static int layout(void) {
    printf("{");
    SZ(atr_vec3); OFF(atr_vec3, x); OFF(atr_vec3, y); OFF(atr_vec3, z);
    SZ(atr_material); OFF(atr_material, emission); OFF(atr_material, reflection); OFF(atr_material, scatter);
    SZ(atr_model); OFF(atr_model, mesh); OFF(atr_model, tree); OFF(atr_model, surrounding_aabb);
    OFF(atr_model, material);
    SZ(atr_sphere); OFF(atr_sphere, center); OFF(atr_sphere, radius); OFF(atr_sphere, material);
    SZ(atr_plane); OFF(atr_plane, normal); OFF(atr_plane, distance); OFF(atr_plane, material);
    SZ(atr_camera); OFF(atr_camera, width); OFF(atr_camera, height); OFF(atr_camera, anti_aliasing);
    OFF(atr_camera, samples_per_pixel); OFF(atr_camera, bounce_limit); OFF(atr_camera, aspect_ratio);
    OFF(atr_camera, camera_z); OFF(atr_camera, camera_x); OFF(atr_camera, camera_y); OFF(atr_camera, eye);
    OFF(atr_camera, frame_center); OFF(atr_camera, h_fov); OFF(atr_camera, half_pixel_width);
    OFF(atr_camera, half_pixel_height);
    SZ(atr_tile); OFF(atr_tile, min_x); OFF(atr_tile, min_y); OFF(atr_tile, max_x); OFF(atr_tile, max_y);
    SZ(atr_frame); OFF(atr_frame, layout); OFF(atr_frame, framebuffer); OFF(atr_frame, hit_face);
    OFF(atr_frame, hit_t); OFF(atr_frame, rgb); OFF(atr_frame, ray_casts); OFF(atr_frame, traced_rays);
    SZ(atr_tuning); OFF(atr_tuning, xcd_chunk); OFF(atr_tuning, frame_rotate); OFF(atr_tuning, hybrid_a);
    OFF(atr_tuning, hybrid_b); OFF(atr_tuning, path_batch_log2); OFF(atr_tuning, cluster_size);
    OFF(atr_tuning, frame_plan); OFF(atr_tuning, path_camera_occ); OFF(atr_tuning, path_bounce_occ); OFF(atr_tuning, primary_occ);
    OFF(atr_tuning, path_sort_bits); OFF(atr_tuning, path_split); OFF(atr_tuning, reserved);
    printf("\"abi_version\": %d}\n", ATR_ABI_VERSION);
    return 0;
}

#define CHECK(x)                                                        \
    do {                                                                \
        int rc_ = (x);                                                  \
        if (rc_ < 0) {                                                  \
            fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, rc_); \
            return 1;                                                   \
        }                                                               \
    } while (0)

/* app.cpp framing of the Cube: centre (-0.256, 0.22, -3.56), app camera */
static int load_scene(const char* obj, atr_mesh** m, atr_octree** t, float box[6]) {
    atr_vec3 c = {-0.256f, 0.22f, -3.56f};
    CHECK(atr_mesh_load_obj(obj, m));
    CHECK(atr_mesh_aabb(*m, box));
    CHECK(atr_mesh_translate_to(*m, box, c));
    CHECK(atr_octree_build(*m, 300, t));
    return 0;
}

static int host(const char* obj) {
    atr_mesh* m = NULL;
    atr_octree* t = NULL;
    float box[6];
    if (load_scene(obj, &m, &t, box)) return 1;
    uint32_t nv = 0, nn = 0, nf = 0;
    int64_t st[7];
    CHECK(atr_mesh_info(m, &nv, &nn, &nf));
    CHECK(atr_octree_stats(t, st));
    atr_camera cam;
    atr_vec3 eye = {0.1f, 2.0f, 0.0f}, facing = {-0.1f, -0.5f, -1.0f};
    CHECK(atr_camera_set(&cam, eye, facing, 256, 256, 0, 1, 1, 1.0f));
    int32_t ntiles = atr_make_tiles(1280, 720, 8, NULL, 0);
    printf("{\"version\": \"%s\", \"nv\": %u, \"nn\": %u, \"nf\": %u, \"nodes\": %lld, \"leaf_refs\": %lld, "
           "\"aabb\": [%.9g, %.9g, %.9g, %.9g, %.9g, %.9g], \"aspect\": %.9g, \"frame_center\": [%.9g, %.9g, %.9g], "
           "\"tiles_1280x720_8\": %d}\n",
           atr_version(), nv, nn, nf, (long long)st[0], (long long)st[4], box[0], box[1], box[2], box[3], box[4],
           box[5], cam.aspect_ratio, cam.frame_center.x, cam.frame_center.y, cam.frame_center.z, ntiles);
    atr_octree_free(t);
    atr_mesh_free(m);
    return 0;
}

static int gpu(const char* obj) {
    const int32_t W = 256, H = 256;
    atr_mesh* m = NULL;
    atr_octree* t = NULL;
    float box[6];
    if (load_scene(obj, &m, &t, box)) return 1;
    atr_ctx* ctx = NULL;
    CHECK(atr_create(0, &ctx));
    atr_material mats[2] = {{{0.3f, 0.4f, 0.5f}, {0.2f, 0.3f, 0.4f}, 0.3f},    /* sky (app.cpp:91) */
                            {{0.4f, 0.2f, 0.2f}, {0.92f, 0.5f, 0.0f}, 0.3f}};  /* model (app.cpp:96) */
    atr_model model;
    memset(&model, 0, sizeof(model));
    model.mesh = m;
    model.tree = t;
    memcpy(model.surrounding_aabb, box, sizeof(box));
    model.material = 1;
    CHECK(atr_scene_upload(ctx, mats, 2, &model, 1, NULL, 0, NULL, 0));
    atr_camera cam;
    atr_vec3 eye = {0.1f, 2.0f, 0.0f}, facing = {-0.1f, -0.5f, -1.0f};
    CHECK(atr_camera_set(&cam, eye, facing, W, H, 0, 1, 1, 1.0f));
    atr_tile tiles[64];
    const int32_t ntiles = atr_make_tiles(W, H, 8, tiles, 64);
    void *fb = NULL, *face = NULL, *tt = NULL, *casts = NULL, *traced = NULL;
    const size_t n = (size_t)W * (size_t)H;
    CHECK(atr_device_alloc(ctx, 4 * n, &fb));
    CHECK(atr_device_alloc(ctx, 4 * n, &face));
    CHECK(atr_device_alloc(ctx, 4 * n, &tt));
    CHECK(atr_device_alloc(ctx, 4 * n, &casts));
    CHECK(atr_device_alloc(ctx, 8, &traced));
    CHECK(atr_memset_d(ctx, traced, 0, 8));
    atr_frame fr = {ATR_LAYOUT_IMAGE, (uint32_t*)fb, (uint32_t*)face, (float*)tt, NULL, (uint32_t*)casts,
                    (unsigned long long*)traced};
    CHECK(atr_render_start(ctx, &cam, tiles, ntiles, &fr, 0x853C49E6748FEA9BULL, NULL));
    int32_t done = 0;
    int rc;
    while ((rc = atr_render_wait(ctx, 33, &done)) == 1) {
    }
    CHECK(rc);
    uint32_t* hf = (uint32_t*)malloc(4 * n);
    uint32_t* ht = (uint32_t*)malloc(4 * n);
    unsigned long long ntr = 0;
    CHECK(atr_memcpy_d2h(ctx, hf, face, 4 * n));
    CHECK(atr_memcpy_d2h(ctx, ht, tt, 4 * n));
    CHECK(atr_memcpy_d2h(ctx, &ntr, traced, 8));
    uint64_t hsh = 1469598103934665603ULL;
    int64_t hits = 0;
    for (size_t i = 0; i < n; ++i) {
        hsh = (hsh ^ hf[i]) * 1099511628211ULL;
        hsh = (hsh ^ ht[i]) * 1099511628211ULL;
        hits += hf[i] != 0xFFFFFFFFu;
    }
    printf("{\"hash\": \"%016llx\", \"hits\": %lld, \"traced\": %llu, \"tiles_done\": %d, \"ntiles\": %d}\n",
           (unsigned long long)hsh, (long long)hits, ntr, done, ntiles);
    free(hf);
    free(ht);
    CHECK(atr_device_free(ctx, fb));
    CHECK(atr_device_free(ctx, face));
    CHECK(atr_device_free(ctx, tt));
    CHECK(atr_device_free(ctx, casts));
    CHECK(atr_device_free(ctx, traced));
    CHECK(atr_destroy(ctx));
    atr_octree_free(t);
    atr_mesh_free(m);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && !strcmp(argv[1], "layout")) return layout();
    if (argc >= 3 && !strcmp(argv[1], "host")) return host(argv[2]);
    if (argc >= 3 && !strcmp(argv[1], "gpu")) return gpu(argv[2]);
    fprintf(stderr, "usage: abi_check layout | host <obj> | gpu <obj>\n");
    return 2;
}
