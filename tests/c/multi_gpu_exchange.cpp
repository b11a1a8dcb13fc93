// multi_gpu_exchange.cpp -- the reference-side multi-GPU flow of INTEGRATION.md §"Several GPUs",
// compiled: what a maintainer adds beside the renderer.h binding to render one frame over N GPUs
// (one process per GPU) with RCCL directly, using only include/atray.h and <rccl/rccl.h>.
//
//   start_render_from_camera (renderer.cpp:403-455)  -> every rank: the cost-balanced shard plan
//       (atr_render_tile_costs on rank 0, ncclBroadcast, atr_balance_shard_tiles), its tiles rendered
//       PACKED (atr_render_start)
//   wait_for_render_from_camera_to_finish (:457-471) -> atr_render_wait; per-tile ray_casts
//       (atr_packed_tile_ray_casts); the pixels and the tile sums to rank 0 (grouped ncclSend /
//       ncclRecv), rank 0 assembles the framebuffer (atr_unpack, or atr_unpack_masked_ranks for the
//       masked exchange) and sums total_ray_casts (:465-468)
//
// usage: multi_gpu_exchange OBJ W H SPP BOUNCES [--exchange u32|masked] [--side S] [--out FILE]
//        [--check]
// env: RANK, WORLD_SIZE, LOCAL_RANK (default 0, 1, RANK); ATR_NCCL_ID: a path the ranks share for
// the ncclUniqueId (rank 0 writes it). Rank 0 prints one JSON line; --out writes the assembled BGRX
// frame (W x H u32, row 0 = bottom); --check compares it and total_ray_casts with a one-GPU render.
// tests/test_gpu_rccl_cpp.py runs it at world size 1 on C4 against the oracle's whole-frame digest.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "atray.h"

namespace {

int die(const char* what, long long rc) {
    std::fprintf(stderr, "multi_gpu_exchange: %s failed (%lld)\n", what, rc);
    std::exit(1);
}
#define ATR(x) do { const int rc_ = (x); if (rc_ != ATR_OK) die(#x, rc_); } while (0)
#define NCCL(x) do { const ncclResult_t rc_ = (x); if (rc_ != ncclSuccess) die(#x, rc_); } while (0)
#define HIP(x) do { const hipError_t rc_ = (x); if (rc_ != hipSuccess) die(#x, rc_); } while (0)

int env_int(const char* k, int dflt) {
    const char* v = std::getenv(k);
    return v ? std::atoi(v) : dflt;
}

// The communicator: rank 0 makes the id and publishes it through a shared file (renamed into place
// so a reader never sees half of it); the others wait for the file.
ncclComm_t make_comm(int rank, int world) {
    ncclUniqueId id;
    if (rank == 0) NCCL(ncclGetUniqueId(&id));
    if (world > 1) {
        const char* path = std::getenv("ATR_NCCL_ID");
        if (!path) die("ATR_NCCL_ID (a file path shared by the ranks) for world > 1", 0);
        if (rank == 0) {
            const std::string tmp = std::string(path) + ".tmp";
            FILE* f = std::fopen(tmp.c_str(), "wb");
            if (!f || std::fwrite(&id, sizeof(id), 1, f) != 1) die("writing the nccl id", 0);
            std::fclose(f);
            if (std::rename(tmp.c_str(), path) != 0) die("publishing the nccl id", 0);
        } else {
            for (int k = 0;; ++k) {
                FILE* f = std::fopen(path, "rb");
                if (f) {
                    const bool ok = std::fread(&id, sizeof(id), 1, f) == 1;
                    std::fclose(f);
                    if (ok) break;
                }
                if (k > 6000) die("waiting for the nccl id", 0);
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            }
        }
    }
    ncclComm_t comm;
    NCCL(ncclCommInitRank(&comm, world, id, rank));
    return comm;
}

template <class T>
T* dalloc(atr_ctx* ctx, size_t n) {
    void* p = nullptr;
    ATR(atr_device_alloc(ctx, std::max<size_t>(1, n) * sizeof(T), &p));
    return static_cast<T*>(p);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s OBJ W H SPP BOUNCES [--exchange u32|masked] [--side S] [--out FILE] [--check]\n",
                     argv[0]);
        return 2;
    }
    const char* obj = argv[1];
    const int32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    const uint32_t spp = uint32_t(std::atoi(argv[4]));
    const int32_t bounces = std::atoi(argv[5]);
    std::string exchange = "u32", out_path;
    int32_t side = 32;
    bool check = false;
    for (int i = 6; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--exchange" && i + 1 < argc) exchange = argv[++i];
        else if (a == "--side" && i + 1 < argc) side = std::atoi(argv[++i]);
        else if (a == "--out" && i + 1 < argc) out_path = argv[++i];
        else if (a == "--check") check = true;
        else { std::fprintf(stderr, "unknown argument %s\n", a.c_str()); return 2; }
    }
    if (exchange != "u32" && exchange != "masked") { std::fprintf(stderr, "--exchange u32|masked\n"); return 2; }
    const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1);
    const int local = env_int("LOCAL_RANK", rank);
    const uint64_t seed = 0x853C49E6748FEA9BULL;

    // ---- prep_scene (renderer.cpp:264-291) on every rank: the scene is replicated
    int ndev = 0;
    HIP(hipGetDeviceCount(&ndev));
    const int device = local % std::max(1, ndev);
    HIP(hipSetDevice(device));  // RCCL binds the communicator to the current device
    atr_ctx* ctx = nullptr;
    ATR(atr_create(device, &ctx));
    ncclComm_t comm = make_comm(rank, world);
    atr_mesh* mesh = nullptr;
    ATR(atr_mesh_load_obj(obj, &mesh));
    float box[6];
    ATR(atr_mesh_aabb(mesh, box));
    ATR(atr_mesh_translate_to(mesh, box, atr_vec3{0.0f, -15.0f, -38.0f}));  // app.cpp:73
    atr_octree* tree = nullptr;
    ATR(atr_octree_build(mesh, 300, &tree));  // app.cpp:76-77
    const atr_material mats[2] = {{{0.3f, 0.4f, 0.5f}, {0.2f, 0.3f, 0.4f}, 0.3f},   // sky (app.cpp:91-105)
                                  {{0.4f, 0.2f, 0.2f}, {0.92f, 0.5f, 0.0f}, 0.3f}};
    atr_model model = {};
    model.mesh = mesh;
    model.tree = tree;
    std::memcpy(model.surrounding_aabb, box, sizeof(box));
    model.material = 1;
    ATR(atr_scene_upload(ctx, mats, 2, &model, 1, nullptr, 0, nullptr, 0));
    atr_camera cam;
    ATR(atr_camera_set(&cam, atr_vec3{0.1f, 2.0f, 0.0f}, atr_vec3{-0.1f, -0.5f, -1.0f}, W, H, 0, spp, bounces, 1.0f));

    // ---- the shard plan: rank 0 measures every grid tile's cost, every rank deals the same plan
    const int32_t ngrid = atr_make_shard_tiles(W, H, side, 0, 1, nullptr, 0);
    std::vector<atr_tile> grid(static_cast<size_t>(ngrid));
    atr_make_shard_tiles(W, H, side, 0, 1, grid.data(), ngrid);
    std::vector<int64_t> cost(size_t(ngrid), 0);
    if (rank == 0) ATR(atr_render_tile_costs(ctx, &cam, grid.data(), ngrid, seed, cost.data()));
    int64_t* d_cost = dalloc<int64_t>(ctx, size_t(ngrid));
    ATR(atr_memcpy_h2d(ctx, d_cost, cost.data(), sizeof(int64_t) * size_t(ngrid)));
    NCCL(ncclBroadcast(d_cost, d_cost, size_t(ngrid), ncclInt64, 0, comm, nullptr));
    ATR(atr_memcpy_d2h(ctx, cost.data(), d_cost, sizeof(int64_t) * size_t(ngrid)));
    std::vector<int32_t> owner(static_cast<size_t>(ngrid));
    atr_balance_shard_tiles(W, H, side, world, cost.data(), 0, owner.data());
    std::vector<int32_t> by_cost(static_cast<size_t>(ngrid));
    std::iota(by_cost.begin(), by_cost.end(), 0);
    std::stable_sort(by_cost.begin(), by_cost.end(), [&](int32_t a, int32_t b) { return cost[size_t(a)] > cost[size_t(b)]; });
    std::vector<std::vector<atr_tile>> tiles_of(static_cast<size_t>(world));  // each rank's tiles, heaviest first
    std::vector<std::vector<int32_t>> gid_of(static_cast<size_t>(world));
    for (int32_t t : by_cost) {
        tiles_of[size_t(owner[size_t(t)])].push_back(grid[size_t(t)]);
        gid_of[size_t(owner[size_t(t)])].push_back(t);
    }
    std::vector<int64_t> n_of(static_cast<size_t>(world));
    for (int r = 0; r < world; ++r)
        n_of[size_t(r)] = tiles_of[size_t(r)].empty() ? 0 : atr_render_packed_size(tiles_of[size_t(r)].data(),
                                                                                     int32_t(tiles_of[size_t(r)].size()));
    const std::vector<atr_tile>& mine = tiles_of[size_t(rank)];
    const int64_t n = n_of[size_t(rank)];
    const int32_t nmine = int32_t(mine.size());

    // ---- start_render_from_camera: this rank's tiles, PACKED
    uint32_t* d_fb = dalloc<uint32_t>(ctx, size_t(n));
    uint32_t* d_casts = dalloc<uint32_t>(ctx, size_t(n));
    int64_t* d_tile_casts = dalloc<int64_t>(ctx, size_t(nmine));
    atr_frame f = {ATR_LAYOUT_PACKED, d_fb, nullptr, nullptr, nullptr, d_casts, nullptr};
    const auto t0 = std::chrono::steady_clock::now();
    if (nmine) ATR(atr_render_start(ctx, &cam, mine.data(), nmine, &f, seed, nullptr));
    // ---- wait_for_render_from_camera_to_finish: done, then the tile counters and the exchange
    int32_t done = 0;
    while (atr_render_wait(ctx, 1000, &done) == 1) {}
    if (nmine) ATR(atr_packed_tile_ray_casts(ctx, mine.data(), nmine, W, H, d_casts, 1, n, d_tile_casts, nullptr));

    // rank 0's receive buffers: every rank's pixels (its own through a self send/recv as well, so
    // world size 1 exercises the same calls) and its per-tile ray_casts
    std::vector<void*> d_recv(size_t(world), nullptr);
    std::vector<int64_t*> d_rtc(size_t(world), nullptr);
    std::vector<int64_t> bytes_of(size_t(world), 0);
    uint8_t* d_enc = nullptr;
    if (exchange == "masked") {  // phase 1: each rank's stream length to rank 0
        // the background: this rank's most common pixel (the sky's colour); any value is exact
        uint32_t background = 0;
        if (n) {
            std::vector<uint32_t> px(static_cast<size_t>(n));
            ATR(atr_memcpy_d2h(ctx, px.data(), d_fb, px.size() * 4));
            std::sort(px.begin(), px.end());
            size_t best = 0;
            for (size_t i = 0, j; i < px.size(); i = j) {
                for (j = i; j < px.size() && px[j] == px[i]; ++j) {}
                if (j - i > best) { best = j - i; background = px[i]; }
            }
        }
        d_enc = dalloc<uint8_t>(ctx, size_t(atr_pack_bgr_masked_bound(n)));
        int64_t* d_nb = dalloc<int64_t>(ctx, 1);
        ATR(atr_pack_bgr_masked(ctx, d_fb, n, background, d_enc, d_nb, nullptr));
        int64_t* d_sizes = rank == 0 ? dalloc<int64_t>(ctx, size_t(world)) : nullptr;
        NCCL(ncclGroupStart());
        if (rank == 0)
            for (int r = 0; r < world; ++r) NCCL(ncclRecv(d_sizes + r, 1, ncclInt64, r, comm, nullptr));
        NCCL(ncclSend(d_nb, 1, ncclInt64, 0, comm, nullptr));
        NCCL(ncclGroupEnd());
        ATR(atr_memcpy_d2h(ctx, &bytes_of[size_t(rank)], d_nb, sizeof(int64_t)));
        if (rank == 0) ATR(atr_memcpy_d2h(ctx, bytes_of.data(), d_sizes, sizeof(int64_t) * size_t(world)));
    }
    if (rank == 0)
        for (int r = 0; r < world; ++r) {
            const size_t bytes = exchange == "masked" ? size_t(bytes_of[size_t(r)]) : size_t(n_of[size_t(r)]) * 4;
            d_recv[size_t(r)] = dalloc<uint8_t>(ctx, bytes);
            d_rtc[size_t(r)] = dalloc<int64_t>(ctx, tiles_of[size_t(r)].size());
        }
    NCCL(ncclGroupStart());  // phase 2: the pixels and the tile sums, exact sizes
    if (rank == 0)
        for (int r = 0; r < world; ++r) {
            if (exchange == "masked") NCCL(ncclRecv(d_recv[size_t(r)], size_t(bytes_of[size_t(r)]), ncclUint8, r, comm, nullptr));
            else if (n_of[size_t(r)]) NCCL(ncclRecv(d_recv[size_t(r)], size_t(n_of[size_t(r)]), ncclUint32, r, comm, nullptr));
            if (!tiles_of[size_t(r)].empty())
                NCCL(ncclRecv(d_rtc[size_t(r)], tiles_of[size_t(r)].size(), ncclInt64, r, comm, nullptr));
        }
    if (exchange == "masked") NCCL(ncclSend(d_enc, size_t(bytes_of[size_t(rank)]), ncclUint8, 0, comm, nullptr));
    else if (n) NCCL(ncclSend(d_fb, size_t(n), ncclUint32, 0, comm, nullptr));
    if (nmine) NCCL(ncclSend(d_tile_casts, size_t(nmine), ncclInt64, 0, comm, nullptr));
    NCCL(ncclGroupEnd());

    int rc = 0;
    if (rank == 0) {  // assembly: the framebuffer and total_ray_casts (renderer.cpp:465-468)
        uint32_t* d_image = dalloc<uint32_t>(ctx, size_t(W) * size_t(H));
        ATR(atr_memset_d(ctx, d_image, 0x7F, size_t(W) * size_t(H) * 4));
        int64_t total_ray_casts = 0;
        std::vector<int64_t> grid_casts(size_t(ngrid), 0);  // RenderTile::ray_casts per grid tile
        if (exchange == "masked") {  // every rank's stream in one call, positions from its tile blocks
            std::vector<const atr_tile*> tp;
            std::vector<int32_t> tn;
            std::vector<const uint8_t*> pp;
            for (int r = 0; r < world; ++r)
                if (!tiles_of[size_t(r)].empty()) {
                    tp.push_back(tiles_of[size_t(r)].data());
                    tn.push_back(int32_t(tiles_of[size_t(r)].size()));
                    pp.push_back(static_cast<const uint8_t*>(d_recv[size_t(r)]));
                }
            ATR(atr_unpack_masked_ranks(ctx, int32_t(tp.size()), tp.data(), tn.data(), W, H, pp.data(), nullptr, 1,
                                        d_image, int64_t(W) * H, nullptr));
        }
        for (int r = 0; r < world; ++r) {
            const std::vector<atr_tile>& tr = tiles_of[size_t(r)];
            if (tr.empty()) continue;
            if (exchange != "masked") {
                ATR(atr_unpack(ctx, tr.data(), int32_t(tr.size()), W, static_cast<const uint32_t*>(d_recv[size_t(r)]),
                               d_image, nullptr));
            }
            std::vector<int64_t> tc(tr.size());
            ATR(atr_memcpy_d2h(ctx, tc.data(), d_rtc[size_t(r)], sizeof(int64_t) * tc.size()));
            for (size_t i = 0; i < tc.size(); ++i) {
                grid_casts[size_t(gid_of[size_t(r)][i])] = tc[i];
                total_ray_casts += tc[i];
            }
        }
        std::vector<uint32_t> image(size_t(W) * size_t(H));
        ATR(atr_memcpy_d2h(ctx, image.data(), d_image, image.size() * 4));
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        long long mism = -1, full_casts = -1;
        if (check) {  // the same frame on this GPU alone: one IMAGE launch of the whole frame
            uint32_t* d_ref = dalloc<uint32_t>(ctx, image.size());
            uint32_t* d_refc = dalloc<uint32_t>(ctx, image.size());
            int64_t* d_sum = dalloc<int64_t>(ctx, 1);
            const atr_tile whole = {0, 0, W - 1, H - 1};
            atr_frame fr = {ATR_LAYOUT_IMAGE, d_ref, nullptr, nullptr, nullptr, d_refc, nullptr};
            ATR(atr_render_start(ctx, &cam, &whole, 1, &fr, seed, nullptr));
            while (atr_render_wait(ctx, 1000, &done) == 1) {}
            ATR(atr_tile_ray_casts(ctx, &whole, 1, W, d_refc, d_sum, nullptr));
            std::vector<uint32_t> ref(image.size());
            int64_t sum = 0;
            ATR(atr_memcpy_d2h(ctx, ref.data(), d_ref, ref.size() * 4));
            ATR(atr_memcpy_d2h(ctx, &sum, d_sum, 8));
            mism = 0;
            for (size_t i = 0; i < ref.size(); ++i) mism += ref[i] != image[i];
            full_casts = sum;
            if (mism != 0 || full_casts != total_ray_casts) rc = 3;
        }
        if (!out_path.empty()) {
            FILE* fo = std::fopen(out_path.c_str(), "wb");
            if (!fo || std::fwrite(image.data(), 4, image.size(), fo) != image.size()) die("writing --out", 0);
            std::fclose(fo);
        }
        int64_t wire = 0;
        for (int r = 1; r < world; ++r) wire += exchange == "masked" ? bytes_of[size_t(r)] : 4 * n_of[size_t(r)];
        std::printf("{\"world\": %d, \"exchange\": \"%s\", \"W\": %d, \"H\": %d, \"spp\": %u, \"bounces\": %d, "
                    "\"total_ray_casts\": %lld, \"shard_pixels\": [", world, exchange.c_str(), W, H, spp, bounces,
                    (long long)total_ray_casts);
        for (int r = 0; r < world; ++r) std::printf("%s%lld", r ? ", " : "", (long long)n_of[size_t(r)]);
        std::printf("], \"rank0_stream_bytes\": %lld, \"bytes_into_rank0\": %lld, \"render_to_assembled_ms\": %.3f, "
                    "\"check_mismatched_pixels\": %lld, \"check_total_ray_casts\": %lld, "
                    "\"grid_tiles_with_casts\": %lld}\n",
                    (long long)(exchange == "masked" ? bytes_of[0] : 4 * n_of[0]), (long long)wire, ms, mism, full_casts,
                    (long long)std::count_if(grid_casts.begin(), grid_casts.end(), [](int64_t v) { return v > 0; }));
    }
    NCCL(ncclCommDestroy(comm));
    atr_octree_free(tree);
    atr_mesh_free(mesh);
    ATR(atr_destroy(ctx));
    return rc;
}
