// Host-side scene preparation under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only;
// tests/test_host_sanitize.py builds this with the engine's host sources and runs it).
//
// Exercises the C++ code the engine runs before any GPU work, on the committed OBJ assets and on
// deterministic mutations of them (truncations, byte flips, injected numbers / indices):
//   parse_obj_text  (load_model_data, OBJ_loader.cpp:278-360) at 1, 3 and 8 threads -- the meshes
//                   must be identical;
//   mesh_aabb / mesh_translate, octree_build (build_oct_kd_tree, kd_tree.cpp:67-288),
//   octree_finish, octree_stats, leaf_clusters (8 and 16 slots), inner_table, pack_tree (the
//   device tables atr_scene_upload uploads: sizes and every stored index checked);
//   reference_tiles (renderer.cpp:403-455), shard_tiles, balance_shard_tiles, camera_set.
// A sanitizer report aborts the process (halt_on_error); the final line "host_sanitize ok N"
// says how many cases ran.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../atray_amd/csrc/host_scene.h"

using namespace atr;

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint32_t rnd() {  // xorshift64*
    g_rng ^= g_rng >> 12; g_rng ^= g_rng << 25; g_rng ^= g_rng >> 27;
    return uint32_t((g_rng * 0x2545F4914F6CDD1Dull) >> 32);
}

int g_cases = 0;

#define CHECK(c)                                                                \
    do {                                                                        \
        if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); std::exit(1); } \
    } while (0)

bool same_mesh(const HostMesh& a, const HostMesh& b) {
    auto eqv = [](const std::vector<V3>& x, const std::vector<V3>& y) {
        return x.size() == y.size() && (x.empty() || !std::memcmp(x.data(), y.data(), x.size() * sizeof(V3)));
    };
    return eqv(a.vertices, b.vertices) && eqv(a.normals, b.normals) && eqv(a.texcoords, b.texcoords) &&
           a.face_v == b.face_v && a.face_t == b.face_t && a.face_n == b.face_n;
}

bool g_verbose = false;

uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// pack_tree (atr_scene_upload's device tables): every array sized as the kernels assume and every
// stored index inside the table it indexes.
void pack_case(const HostTree& T, size_t nfaces, int cluster_size) {
    PackedTree P;
    if (pack_tree(T, cluster_size, P) != ATR_OK) return;  // ATR_E_TREE_LAYOUT and the like
    ++g_cases;
    const size_t nprims = T.prim_face.size(), ncl = P.nclusters, nleafr = P.leaf_range.size() / 2;
    CHECK(P.nodes.size() == size_t(T.nnodes));
    CHECK(P.inner.size() == 3 * size_t(std::max(1, P.ninner)));
    CHECK(P.tris.size() == nprims && P.t0.size() == std::max<size_t>(1, nprims) && P.t1.size() == P.t0.size() &&
          P.t2.size() == P.t0.size() && P.tface.size() == P.t0.size());
    CHECK(P.clus.size() == std::max<size_t>(1, ncl) * 4 * kClusterBlock);
    CHECK(P.prim.size() == 3 * std::max<size_t>(1, ncl) * kMaxClusterSize);
    CHECK(P.cl_range.size() == P.leaf_range.size() && P.leaf_range.size() >= 2);
    for (size_t k = 0; k < nleafr; ++k) {
        CHECK(uint64_t(P.leaf_range[2 * k]) + P.leaf_range[2 * k + 1] <= nprims);
        CHECK(uint64_t(P.cl_range[2 * k]) + P.cl_range[2 * k + 1] <= ncl);
    }
    for (size_t c = 0; c < ncl; ++c) {
        const uint32_t n = (P.clus[4 * kClusterBlock * c + 3] & 31u) + 1u;
        CHECK(n <= uint32_t(cluster_size) && n <= uint32_t(kMaxClusterSize));
        for (uint32_t i = 0; i < n; ++i) {
            const float4_t r = P.prim[3 * (c * kMaxClusterSize + i) + 2];
            CHECK(bits(r.z) < nfaces);                  // face id
            CHECK(bits(r.y) < uint32_t(1u << 30));      // leaf rank of the primitive
        }
        for (uint32_t i = n; i < uint32_t(kMaxClusterSize); ++i) {  // unused slots stay zero
            const float4_t r = P.prim[3 * (c * kMaxClusterSize + i) + 2];
            CHECK(bits(r.y) == 0 && bits(r.z) == 0);
        }
    }
    for (int32_t i = 0; i < P.ninner; ++i) {
        const float4_t w = P.inner[3 * size_t(i) + 2];
        CHECK(bits(w.y) < uint32_t(std::max<size_t>(1, nleafr)));              // first leaf child's rank
        CHECK(int32_t(bits(w.z)) >= -1 && int32_t(bits(w.z)) < P.ninner);      // parent inner id
        CHECK((bits(w.w) >> 8) < uint32_t(P.ninner));                           // first inner child id
    }
    CHECK(P.near_ok == (P.max_depth <= 8 && P.ninner < 65536));
}

void scene_case(const std::string& text, uint32_t max_faces) {
    ++g_cases;
    if (g_verbose) std::fprintf(stderr, "case %d: %zu bytes, max_faces %u\n", g_cases, text.size(), max_faces);
    HostMesh m1, m3, m8;
    CHECK(parse_obj_text(text.data(), text.size(), m1, 1) == ATR_OK);
    CHECK(parse_obj_text(text.data(), text.size(), m3, 3) == ATR_OK);
    CHECK(parse_obj_text(text.data(), text.size(), m8, 8) == ATR_OK);
    CHECK(same_mesh(m1, m3) && same_mesh(m1, m8));
    float box[6];
    mesh_aabb(m1, box);
    HostTree T;
    if (octree_build(m1, max_faces, T) != ATR_OK) return;  // out-of-range face indices
    CHECK(octree_finish(T) == ATR_OK);
    int64_t st[7];
    octree_stats(T, st);
    for (int size : {8, 16}) {
        LeafClusters C;
        leaf_clusters(T, size, C);
    }
    std::vector<float4_t> inner;
    std::vector<int32_t> leaf_rank;
    inner_table(T, inner, leaf_rank);
    for (int size : {16, 5}) pack_case(T, m1.nfaces(), size);
    if (!m1.vertices.empty()) {
        mesh_translate(m1, box, mk(1.f, -2.f, 3.f));
        mesh_aabb(m1, box);
    }
}

std::string mutate(const std::string& src) {
    static const char* kInject[] = {"99999999999999999999", "1e400", "-1e-400", "-0", "f 1\n", "f -5 -6 -7\n",
                                    "f 1/2/3 4//5 6/7\n", "v\n", "vn 1 2\n", "vt\n", "f 0 0 0\n",
                                    "f 2147483647 -2147483648 3\n", ".e-e+9", "\n\n", "\t", "f"};
    static const char kChars[] = "vtnf/-+0123456789 .eE\n\t#";
    std::string s = src;
    const int edits = 1 + int(rnd() % 6);
    for (int e = 0; e < edits && !s.empty(); ++e) {
        const size_t at = rnd() % s.size();
        switch (rnd() % 4) {
            case 0: s.resize(at); break;
            case 1: s[at] = kChars[rnd() % (sizeof(kChars) - 1)]; break;
            case 2: s.insert(at, kInject[rnd() % (sizeof(kInject) / sizeof(kInject[0]))]); break;
            default: s.erase(at, 1 + rnd() % 16); break;
        }
    }
    return s;
}

void tile_cases() {
    const int32_t dims[][2] = {{1, 1}, {7, 5}, {64, 64}, {65, 33}, {256, 256}, {1920, 1080}, {3840, 2160}};
    for (auto& d : dims) {
        const int32_t W = d[0], H = d[1];
        for (int32_t threads : {1, 3, 16, 64, 1000}) {
            ++g_cases;
            const int32_t n = reference_tiles(W, H, threads, nullptr, 0);
            CHECK(n >= 0);
            std::vector<atr_tile> t(size_t(n) + 1);
            CHECK(reference_tiles(W, H, threads, t.data(), n) == n);
            if (n > 1) reference_tiles(W, H, threads, t.data(), n / 2);  // short buffer: no overrun
        }
        for (int32_t side : {1, 16, 32, 64, 100}) {
            if (int64_t(W / side + 1) * (H / side + 1) > 200000) continue;
            for (int32_t world = 1; world <= 9; ++world) {
                ++g_cases;
                int64_t total = 0;
                for (int32_t r = 0; r < world; ++r) {
                    const int32_t n = shard_tiles(W, H, side, r, world, nullptr, 0);
                    CHECK(n >= 0);
                    std::vector<atr_tile> t(size_t(n) + 1);
                    CHECK(shard_tiles(W, H, side, r, world, t.data(), n) == n);
                    for (int32_t i = 0; i < n; ++i)
                        total += int64_t(t[size_t(i)].max_x - t[size_t(i)].min_x + 1) *
                                 (t[size_t(i)].max_y - t[size_t(i)].min_y + 1);
                }
                CHECK(total == int64_t(W) * H);  // the ranks' tiles cover the frame exactly
                const int64_t gx = (W + side - 1) / side, gy = (H + side - 1) / side;
                std::vector<int64_t> cost(size_t(gx * gy));
                for (int64_t& c : cost) c = int64_t(rnd() % 1000);
                std::vector<int32_t> owner(cost.size(), -1);
                const int64_t extra = (world & 1) ? int64_t(rnd() % 5000) : 0;
                if (balance_shard_tiles(W, H, side, world, cost.data(), extra, owner.data()) >= 0)
                    for (int32_t o : owner) CHECK(o >= 0 && o < world);
            }
        }
    }
    for (int aa : {0, 1}) {
        atr_camera cm;
        std::memset(&cm, 0, sizeof(cm));
        camera_set(cm, mk(0.f, 1.f, 5.f), mk(0.f, 0.f, -1.f), 1920, 1080, aa, 4, 5, 60.f);
        camera_set(cm, mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), 1, 1, aa, 1, 1, 0.f);  // degenerate
        ++g_cases;
    }
}

std::string read_file(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path); std::exit(2); }
    std::string s;
    char buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, n);
    std::fclose(f);
    return s;
}

}  // namespace

int main(int argc, char** argv) {
    // argv: <mutations per asset> <asset.obj> ...
    if (argc < 3) { std::fprintf(stderr, "usage: host_sanitize MUTATIONS asset.obj ...\n"); return 2; }
    const int mutations = std::atoi(argv[1]);
    g_verbose = std::getenv("HOST_SANITIZE_VERBOSE") != nullptr;
    tile_cases();
    if (g_verbose) std::fprintf(stderr, "tiles done (%d cases)\n", g_cases);
    scene_case("", 8);
    scene_case("v 0 0 0\nv 0 0 0\nv 0 0 0\nf 1 2 3\nf 1 2 3\n", 1);  // zero-area faces
    scene_case("v 1 2 3", 8);                                        // no final newline
    for (int i = 2; i < argc; ++i) {
        const std::string text = read_file(argv[i]);
        // the reference's default leaf size and a small one (leaves far below 32 faces grow the
        // reference's octree without bound on Monkey.obj: straddling faces enter every child)
        scene_case(text, 300);
        scene_case(text, 32);
        // mutations of big assets are cut to their first 16 KB so a case stays fast under ASan
        const std::string base = text.size() > 16384 ? text.substr(0, text.rfind('\n', 16384) + 1) : text;
        for (int k = 0; k < mutations; ++k) scene_case(mutate(base), 64);
    }
    std::printf("host_sanitize ok %d\n", g_cases);
    return 0;
}
