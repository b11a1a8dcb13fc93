// host_scene.cpp -- host prerequisites of the render path (not timed by the benchmark):
// OBJ loading with the reference's number parser, model AABB/translation, the octree build
// and its flattening into the device layout of engine.h. Reference: OBJ_loader.cpp:278-360,
// utilities/parser.h, model.h:41-61,136-152, kd_tree.cpp:1-288, camera.h, renderer.cpp:403-445.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "engine.h"
#include "host_scene.h"

using namespace atr;

// OBJ text parsing (load_model_data, parse_f64): obj_parse.cpp

void atr::mesh_aabb(const HostMesh& m, float out[6]) {  // get_AABB (model.h:41-61)
    float lo[3] = {kMaxFloat, kMaxFloat, kMaxFloat}, hi[3] = {-kMaxFloat, -kMaxFloat, -kMaxFloat};
    for (const V3& v : m.vertices) {
        const float c[3] = {v.x, v.y, v.z};
        for (int a = 0; a < 3; ++a) {
            hi[a] = pl_max(hi[a], c[a]);
            lo[a] = pl_min(lo[a], c[a]);
        }
    }
    for (int a = 0; a < 3; ++a) {
        out[a] = lo[a] - kTol;
        out[3 + a] = hi[a] + kTol;
    }
}

void atr::mesh_translate(HostMesh& m, float box[6], V3 c) {  // translate_to (model.h:136-152)
    V3 lo = mk(box[0], box[1], box[2]), hi = mk(box[3], box[4], box[5]);
    V3 old_center = add(lo, divs(sub(hi, lo), 2.0f));
    V3 d = sub(c, old_center);
    for (V3& v : m.vertices) v = add(v, d);
    hi = add(hi, d);
    lo = add(lo, d);
    box[0] = lo.x; box[1] = lo.y; box[2] = lo.z;
    box[3] = hi.x; box[4] = hi.y; box[5] = hi.z;
}

// ------------------------------------------------------------------ octree
namespace {
struct Tri9 { V3 a, b, c; uint32_t face; };

inline bool pt_in(const V3& p, const float* lo, const float* hi) {  // aabb.h:19-27 (closed)
    return (p.x >= lo[0] && p.x <= hi[0]) && (p.y >= lo[1] && p.y <= hi[1]) &&
           (p.z >= lo[2] && p.z <= hi[2]);
}
}  // namespace

// build_KD_tree (kd_tree.cpp:20-64) + build_oct_kd_tree (kd_tree.cpp:67-288).
// Node numbering follows the reference exactly: a LIFO work list, children appended as a
// contiguous block of 8 at the current tree length, in the order bb/bf/tb/tf x left/right.
int atr::octree_build(const HostMesh& m, uint32_t max_faces, HostTree& T) {
    struct Work { float lo[3], hi[3]; int32_t children = 0; int32_t parent = -1; int depth = 0;
                  std::vector<Tri9> prims; };
    std::vector<Work> nodes(1);
    float box[6];
    mesh_aabb(m, box);
    std::memcpy(nodes[0].lo, box, 12);
    std::memcpy(nodes[0].hi, box + 3, 12);
    const size_t nf = m.face_v.size() / 3;
    nodes[0].prims.resize(nf);
    for (size_t i = 0; i < nf; ++i) {
        const int32_t* f = &m.face_v[3 * i];
        for (int k = 0; k < 3; ++k)
            if (f[k] < 0 || size_t(f[k]) >= m.vertices.size()) return ATR_E_INVALID;
        nodes[0].prims[i] = Tri9{m.vertices[f[0]], m.vertices[f[1]], m.vertices[f[2]], uint32_t(i)};
    }
    std::vector<int32_t> todo{0};
    while (!todo.empty()) {
        const int32_t id = todo.back();
        todo.pop_back();
        if (nodes[id].prims.size() <= max_faces || nodes[id].depth >= 64) continue;  // leaf
        // "SAH" split point = area-weighted centroid (kd_tree.cpp:93-114); f32 sum, f64 area sum
        V3 acc = mk(0.f, 0.f, 0.f);
        double area_sum = 0.0;
        for (const Tri9& t : nodes[id].prims) {
            V3 centroid = divs(add(add(t.a, t.b), t.c), 3.0f);
            V3 ab = sub(t.a, t.b), ac = sub(t.a, t.c);
            float area = std::sqrt(len2(cross(ac, ab))) / 2.0f;  // area_of_triangle (:3-8)
            acc = add(acc, scale(centroid, area));
            area_sum += double(area);
        }
        const V3 s = divs(acc, float(area_sum));
        if (!pt_in(s, nodes[id].lo, nodes[id].hi)) continue;  // degenerate split -> leaf
        const float* L = nodes[id].lo;
        const float* H = nodes[id].hi;
        // child k: x from bit 2 (left/right), y from bit 1 (bottom/top), z from bit 0 (back/front)
        float cb[8][6];
        for (int k = 0; k < 8; ++k) {
            const bool xr = (k >> 2) & 1, yt = (k >> 1) & 1, zf = k & 1;
            cb[k][0] = xr ? s.x : L[0]; cb[k][3] = xr ? H[0] : s.x;
            cb[k][1] = yt ? s.y : L[1]; cb[k][4] = yt ? H[1] : s.y;
            cb[k][2] = zf ? s.z : L[2]; cb[k][5] = zf ? H[2] : s.z;
        }
        std::vector<Tri9> parts[8];
        for (const Tri9& t : nodes[id].prims)  // vertex-in-box assignment (:10-17, :181-228)
            for (int k = 0; k < 8; ++k)
                if (pt_in(t.a, cb[k], cb[k] + 3) || pt_in(t.b, cb[k], cb[k] + 3) ||
                    pt_in(t.c, cb[k], cb[k] + 3))
                    parts[k].push_back(t);
        const int32_t first = int32_t(nodes.size());
        const int depth = nodes[id].depth;
        nodes[id].prims.clear();
        nodes[id].prims.shrink_to_fit();
        nodes[id].children = first;
        for (int k = 0; k < 8; ++k) {
            Work w;
            std::memcpy(w.lo, cb[k], 12);
            std::memcpy(w.hi, cb[k] + 3, 12);
            w.parent = id;
            w.depth = depth + 1;
            w.prims.swap(parts[k]);
            nodes.push_back(std::move(w));
        }
        for (int k = 0; k < 8; ++k) todo.push_back(first + k);
    }
    T = HostTree();
    T.nnodes = int32_t(nodes.size());
    T.bounds.resize(6 * nodes.size());
    T.children.resize(nodes.size());
    T.parent.resize(nodes.size());
    T.leaf_first.assign(nodes.size(), 0);
    T.leaf_count.assign(nodes.size(), 0);
    T.depth.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) {
        std::memcpy(&T.bounds[6 * i], nodes[i].lo, 12);
        std::memcpy(&T.bounds[6 * i + 3], nodes[i].hi, 12);
        T.children[i] = nodes[i].children;
        T.parent[i] = nodes[i].parent;
        T.depth[i] = nodes[i].depth;
        if (nodes[i].children == 0) {
            T.leaf_first[i] = uint32_t(T.prim_face.size());
            T.leaf_count[i] = uint32_t(nodes[i].prims.size());
            for (const Tri9& t : nodes[i].prims) {
                const float v[9] = {t.a.x, t.a.y, t.a.z, t.b.x, t.b.y, t.b.z, t.c.x, t.c.y, t.c.z};
                T.prim_vertices.insert(T.prim_vertices.end(), v, v + 9);
                T.prim_face.push_back(t.face);
            }
        }
    }
    return ATR_OK;
}

int atr::leaf_clusters(const HostTree& T, int size, LeafClusters& C) {
    if (size < 1 || size > 32) return ATR_E_INVALID;
    const size_t np = T.prim_face.size();
    C = LeafClusters();
    C.order.reserve(np);
    C.rank.reserve(np);
    C.range.assign(2 * size_t(T.nnodes), 0u);
    const float* V = T.prim_vertices.data();
    for (size_t k = 0; k < 9 * np; ++k) C.max_abs = std::max(C.max_abs, std::fabs(V[k]));
    std::vector<uint32_t> idx;
    std::vector<double> cen;
    for (int32_t n = 0; n < T.nnodes; ++n) {
        if (T.children[size_t(n)]) continue;
        const uint32_t first = T.leaf_first[size_t(n)], cnt = T.leaf_count[size_t(n)];
        C.range[2 * size_t(n)] = uint32_t(C.rec.size() / 8);
        if (!cnt) continue;
        idx.resize(cnt);
        cen.resize(3 * size_t(cnt));
        for (uint32_t i = 0; i < cnt; ++i) {
            idx[i] = i;
            const float* v = V + 9 * size_t(first + i);
            for (int a = 0; a < 3; ++a) cen[3 * i + a] = (double(v[a]) + v[3 + a] + v[6 + a]) / 3.0;
        }
        // explicit stack of [lo, hi) ranges; children pushed right-first so clusters come out
        // left to right
        std::vector<std::pair<uint32_t, uint32_t>> st{{0u, cnt}};
        while (!st.empty()) {
            const auto [lo, hi] = st.back();
            st.pop_back();
            const uint32_t m = hi - lo;
            if (m > uint32_t(size)) {
                double bl[3] = {1e300, 1e300, 1e300}, bh[3] = {-1e300, -1e300, -1e300};
                for (uint32_t i = lo; i < hi; ++i)
                    for (int a = 0; a < 3; ++a) {
                        bl[a] = std::min(bl[a], cen[3 * idx[i] + a]);
                        bh[a] = std::max(bh[a], cen[3 * idx[i] + a]);
                    }
                int ax = 0;
                for (int a = 1; a < 3; ++a)
                    if (bh[a] - bl[a] > bh[ax] - bl[ax]) ax = a;
                const uint32_t nclus = (m + uint32_t(size) - 1) / uint32_t(size);
                const uint32_t left = ((nclus + 1) / 2) * uint32_t(size);
                std::nth_element(idx.begin() + lo, idx.begin() + lo + left, idx.begin() + hi,
                                 [&](uint32_t x, uint32_t y) {
                                     const double cx = cen[3 * x + ax], cy = cen[3 * y + ax];
                                     return cx < cy || (cx == cy && x < y);
                                 });
                st.push_back({lo + left, hi});
                st.push_back({lo, lo + left});
                continue;
            }
            std::sort(idx.begin() + lo, idx.begin() + hi);  // leaf order inside a cluster
            float bl[3] = {INFINITY, INFINITY, INFINITY}, bh[3] = {-INFINITY, -INFINITY, -INFINITY};
            double pmax = 0.0;
            const uint32_t slot0 = uint32_t(C.order.size());
            for (uint32_t i = lo; i < hi; ++i) {
                const float* v = V + 9 * size_t(first + idx[i]);
                for (int c = 0; c < 3; ++c)
                    for (int a = 0; a < 3; ++a) {
                        bl[a] = std::min(bl[a], v[3 * c + a]);
                        bh[a] = std::max(bh[a], v[3 * c + a]);
                    }
                // ab, ac exactly as the device holds them (f32 b - a, c - a)
                double ab[3], ac[3];
                for (int a = 0; a < 3; ++a) {
                    ab[a] = double(v[3 + a] - v[a]);
                    ac[a] = double(v[6 + a] - v[a]);
                }
                const double n[3] = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2],
                                     ab[0] * ac[1] - ab[1] * ac[0]};
                pmax = std::max(pmax, std::sqrt(ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2]) *
                                          std::sqrt(ac[0] * ac[0] + ac[1] * ac[1] + ac[2] * ac[2]));
                // the culled test's det = ab . (d x ac) = -(d . n)
                for (int a = 0; a < 3; ++a) C.normal.push_back(float(n[a]));
                C.order.push_back(first + idx[i]);
                C.rank.push_back(idx[i]);
            }
            // count (n - 1) rides in the low 5 mantissa bits of the |ab||ac| bound, rounded up
            // first so the stored value is still an upper bound
            float pf = float(pmax * (1.0 + 1e-5) + 1e-30);
            uint32_t pb;
            std::memcpy(&pb, &pf, 4);
            pb = (pb & ~31u) + 32u;
            pb |= (m - 1);
            std::memcpy(&pf, &pb, 4);
            float sf;
            std::memcpy(&sf, &slot0, 4);
            const float r[8] = {bl[0], bl[1], bl[2], pf, bh[0], bh[1], bh[2], sf};
            C.rec.insert(C.rec.end(), r, r + 8);
        }
        C.range[2 * size_t(n) + 1] = uint32_t(C.rec.size() / 8) - C.range[2 * size_t(n)];
    }
    return ATR_OK;
}

int atr::inner_table(const HostTree& T, std::vector<float4_t>& out, std::vector<int32_t>& leaf_rank) {
    const int32_t n = T.nnodes;
    std::vector<int32_t> rank(size_t(n), -1);
    int32_t ninner = 0;
    for (int32_t i = 0; i < n; ++i)
        if (T.children[size_t(i)]) rank[size_t(i)] = ninner++;
    // Static discovery order of the leaves: the traversal examines all children of a node (leaf
    // children found in child order) before descending, and descends into the inner children
    // highest first, each subtree completely before the next (the LIFO hit stack,
    // kd_tree.cpp:363-435). Any single pass discovers its leaves in this order restricted to the
    // ones it reaches, so the rank replaces the per-pass discovery index as the tie key.
    leaf_rank.assign(size_t(n), -1);
    if (n > 0) {
        int32_t next = 0;
        std::vector<int32_t> stack{0};
        if (T.children[0] == 0) leaf_rank[0] = next++;
        while (!stack.empty()) {
            const int32_t x = stack.back();
            stack.pop_back();
            const int32_t c = T.children[size_t(x)];
            if (!c) continue;
            if (c < 0 || c + 8 > n) return ATR_E_INVALID;
            for (int k = 0; k < 8; ++k)
                if (T.children[size_t(c + k)] == 0) {
                    if (leaf_rank[size_t(c + k)] >= 0) return ATR_E_INVALID;  // shared child: not a tree
                    leaf_rank[size_t(c + k)] = next++;
                }
            for (int k = 0; k < 8; ++k)
                if (T.children[size_t(c + k)]) {
                    if (int32_t(stack.size()) > n) return ATR_E_INVALID;
                    stack.push_back(c + k);
                }
        }
    }
    out.assign(3 * size_t(ninner), float4_t{0.f, 0.f, 0.f, 0.f});
    auto same = [](float a, float b) { return std::memcmp(&a, &b, sizeof(float)) == 0; };
    for (int32_t i = 0; i < n; ++i) {
        const int32_t c = T.children[size_t(i)];
        if (!c) continue;
        if (c < 0 || c + 8 > n) return ATR_E_INVALID;
        const float* b = &T.bounds[6 * size_t(i)];
        const float* b0 = &T.bounds[6 * size_t(c)];
        const float lo[3] = {b[0], b[1], b[2]}, hi[3] = {b[3], b[4], b[5]};
        const float v[3] = {b0[3], b0[4], b0[5]};  // bb_left.aabb.max = division point
        uint32_t leafm = 0;
        int32_t base = -1, leaf0 = -1;
        for (int k = 0; k < 8; ++k) {
            const float* cb = &T.bounds[6 * size_t(c + k)];
            const int bit[3] = {k >> 2, (k >> 1) & 1, k & 1};  // x: left/right, y: bottom/top, z: back/front
            for (int a = 0; a < 3; ++a) {
                const float mn = bit[a] ? v[a] : lo[a], mx = bit[a] ? hi[a] : v[a];
                if (!same(cb[a], mn) || !same(cb[3 + a], mx)) return ATR_E_TREE_LAYOUT;
            }
            if (T.children[size_t(c + k)] == 0) {
                leafm |= 1u << k;
                if (leaf0 < 0) leaf0 = leaf_rank[size_t(c + k)];
                if (leaf_rank[size_t(c + k)] != leaf0 + __builtin_popcount(leafm) - 1) return ATR_E_INVALID;
            } else if (base < 0) {
                base = rank[size_t(c + k)];
            }
        }
        if (base < 0) base = 0;
        if (leaf0 < 0) leaf0 = 0;
        const int32_t par = T.parent.empty() || T.parent[size_t(i)] < 0 ? -1 : rank[size_t(T.parent[size_t(i)])];
        const uint32_t bm = (uint32_t(base) << 8) | leafm;
        float w[3];
        std::memcpy(&w[0], &leaf0, 4);
        std::memcpy(&w[1], &par, 4);
        std::memcpy(&w[2], &bm, 4);
        float4_t* r = &out[3 * size_t(rank[size_t(i)])];
        r[0] = float4_t{lo[0], lo[1], lo[2], v[0]};
        r[1] = float4_t{v[1], v[2], hi[0], hi[1]};
        r[2] = float4_t{hi[2], w[0], w[1], w[2]};
    }
    return ATR_OK;
}

int atr::octree_finish(HostTree& T) {  // parents/depths for a caller-provided tree
    const int32_t n = T.nnodes;
    T.parent.assign(size_t(n), -1);
    T.depth.assign(size_t(n), 0);
    for (int32_t i = 0; i < n; ++i) {
        const int32_t c = T.children[size_t(i)];
        if (c == 0) continue;
        if (c < 0 || c + 8 > n) return ATR_E_INVALID;
        for (int k = 0; k < 8; ++k) T.parent[size_t(c + k)] = i;
    }
    for (int32_t i = 0; i < n; ++i) {  // depth by walking parents (children follow parents)
        int d = 0;
        for (int32_t p = T.parent[size_t(i)]; p >= 0; p = T.parent[size_t(p)]) {
            if (++d > n) return ATR_E_INVALID;  // cycle
        }
        T.depth[size_t(i)] = d;
    }
    return ATR_OK;
}

void atr::octree_stats(const HostTree& T, int64_t s[7]) {
    int64_t inner = 0, leaves = 0, empty = 0, refs = 0, maxleaf = 0, depth = 0;
    for (int32_t i = 0; i < T.nnodes; ++i) {
        if (T.children[size_t(i)]) { ++inner; }
        else {
            ++leaves;
            const int64_t c = T.leaf_count[size_t(i)];
            refs += c;
            if (!c) ++empty;
            if (c > maxleaf) maxleaf = c;
        }
        if (T.depth[size_t(i)] > depth) depth = T.depth[size_t(i)];
    }
    s[0] = T.nnodes; s[1] = inner; s[2] = leaves; s[3] = empty; s[4] = refs; s[5] = maxleaf; s[6] = depth;
}

// ------------------------------------------------------------------ camera / tiles
void atr::camera_set(atr_camera& cm, V3 eye, V3 facing, int32_t w, int32_t h, int32_t aa,
                     uint32_t spp, int32_t bounces, float h_fov) {  // set_camera (camera.h:23-45)
    std::memset(&cm, 0, sizeof(cm));
    cm.h_fov = h_fov;
    cm.width = w;
    cm.height = h;
    cm.anti_aliasing = aa;
    cm.samples_per_pixel = spp;
    cm.bounce_limit = bounces;
    cm.aspect_ratio = float(w) / float(h);
    const V3 f = unit(facing);
    const V3 fc = add(eye, f);
    const V3 z = neg(f);
    const V3 x = unit(cross(mk(0.f, 1.f, 0.f), z));
    const V3 y = unit(cross(z, x));
    cm.eye = atr_vec3{eye.x, eye.y, eye.z};
    cm.frame_center = atr_vec3{fc.x, fc.y, fc.z};
    cm.camera_z = atr_vec3{z.x, z.y, z.z};
    cm.camera_x = atr_vec3{x.x, x.y, x.z};
    cm.camera_y = atr_vec3{y.x, y.y, y.z};
    cm.half_pixel_width = (0.5f * cm.h_fov) / float(w);
    cm.half_pixel_height = 0.5f / float(h);
}

int32_t atr::reference_tiles(int32_t W, int32_t H, int32_t threads, atr_tile* out, int32_t cap) {
    if (W <= 0 || H <= 0 || threads <= 0) return 0;
    int32_t side = W / threads;  // renderer.cpp:406-411
    if (side > H) side = H / threads;
    if (side <= 0) side = 1;
    const int32_t nx = (W + side - 1) / side, ny = (H + side - 1) / side;
    int32_t n = 0;
    for (int32_t ty = 0; ty < ny; ++ty)
        for (int32_t tx = 0; tx < nx; ++tx, ++n) {
            if (n >= cap) continue;
            atr_tile t;
            t.min_x = tx * side;
            t.min_y = ty * side;
            t.max_x = t.min_x + side < W - 1 ? t.min_x + side : W - 1;  // inclusive, clipped
            t.max_y = t.min_y + side < H - 1 ? t.min_y + side : H - 1;
            out[n] = t;
        }
    return n;
}

int32_t atr::shard_tiles(int32_t W, int32_t H, int32_t side, int32_t rank, int32_t world,
                         atr_tile* out, int32_t cap) {
    if (W <= 0 || H <= 0 || side <= 0 || world <= 0 || rank < 0 || rank >= world) return 0;
    const int32_t nx = (W + side - 1) / side, ny = (H + side - 1) / side;
    int32_t n = 0, k = 0;
    for (int32_t ty = 0; ty < ny; ++ty)
        for (int32_t tx = 0; tx < nx; ++tx, ++k) {
            if (k % world != rank) continue;
            if (n < cap) {
                atr_tile t;
                t.min_x = tx * side;
                t.min_y = ty * side;
                t.max_x = (tx + 1) * side - 1 < W - 1 ? (tx + 1) * side - 1 : W - 1;
                t.max_y = (ty + 1) * side - 1 < H - 1 ? (ty + 1) * side - 1 : H - 1;
                out[n] = t;
            }
            ++n;
        }
    return n;
}

// Longest-processing-time-first deal of the shard grid (side x side tiles, row-major) to
// `world` ranks by measured cost: tiles in descending cost (ties: grid order) go to the least
// loaded rank (ties: lowest rank); rank 0 starts with `rank0_extra` (its frame assembly work).
int32_t atr::balance_shard_tiles(int32_t W, int32_t H, int32_t side, int32_t world, const int64_t* costs,
                                 int64_t rank0_extra, int32_t* owner) {
    if (W <= 0 || H <= 0 || side <= 0 || world <= 0 || !costs || !owner) return -1;
    const int32_t nx = (W + side - 1) / side, ny = (H + side - 1) / side, n = nx * ny;
    std::vector<int32_t> order(static_cast<size_t>(n));
    for (int32_t i = 0; i < n; ++i) order[size_t(i)] = i;
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return costs[a] > costs[b]; });
    std::vector<int64_t> load(size_t(world), 0);
    load[0] = rank0_extra;
    for (int32_t i : order) {
        int32_t best = 0;
        for (int32_t r = 1; r < world; ++r)
            if (load[size_t(r)] < load[size_t(best)]) best = r;
        owner[i] = best;
        load[size_t(best)] += costs[i];
    }
    return n;
}

// ------------------------------------------------------------------ device tables of an octree model
namespace {
// IEEE binary16 bits of an integer |v| <= 2047 (exact).
uint16_t half_of_int(int32_t v) {
    if (v == 0) return 0;
    const uint32_t sign = v < 0 ? 0x8000u : 0u;
    uint32_t m = uint32_t(v < 0 ? -v : v);
    int e = 31 - __builtin_clz(m);
    return uint16_t(sign | (uint32_t(e + 15) << 10) | ((m << (10 - e)) & 0x3FFu));
}
}  // namespace

atr::DTri atr::make_tri(const float* v, uint32_t face) {
    DTri t;
    std::memset(&t, 0, sizeof(t));
    const V3 a = mk(v[0], v[1], v[2]), b = mk(v[3], v[4], v[5]), c = mk(v[6], v[7], v[8]);
    const V3 ab = sub(b, a), ac = sub(c, a);  // model.h:77-78, once per primitive
    t.ax = a.x; t.ay = a.y; t.az = a.z;
    t.abx = ab.x; t.aby = ab.y; t.abz = ab.z;
    t.acx = ac.x; t.acy = ac.y; t.acz = ac.z;
    t.face = face;
    return t;
}

int atr::pack_tree(const HostTree& T, int cluster_size, PackedTree& P) {
    P = PackedTree();
    if (T.nnodes <= 0 || T.bounds.size() != 6 * size_t(T.nnodes) || T.children.size() != size_t(T.nnodes) ||
        T.parent.size() != size_t(T.nnodes) || T.depth.size() != size_t(T.nnodes) ||
        T.leaf_first.size() != size_t(T.nnodes) || T.leaf_count.size() != size_t(T.nnodes) ||
        T.prim_vertices.size() != 9 * T.prim_face.size())
        return ATR_E_INVALID;
    const size_t nprims = T.prim_face.size();
    P.nodes.resize(size_t(T.nnodes));
    std::vector<uint32_t> range(2 * size_t(T.nnodes), 0);
    for (int32_t n = 0; n < T.nnodes; ++n) {
        DNode& d = P.nodes[size_t(n)];
        const float* b = &T.bounds[6 * size_t(n)];
        d.lo_x = b[0]; d.lo_y = b[1]; d.lo_z = b[2];
        d.hi_x = b[3]; d.hi_y = b[4]; d.hi_z = b[5];
        d.children = T.children[size_t(n)];
        d.parent = T.parent[size_t(n)];
        if (!T.children[size_t(n)] && uint64_t(T.leaf_first[size_t(n)]) + T.leaf_count[size_t(n)] > nprims)
            return ATR_E_INVALID;
        range[2 * size_t(n)] = T.leaf_first[size_t(n)];
        range[2 * size_t(n) + 1] = T.children[size_t(n)] ? 0u : T.leaf_count[size_t(n)];
        P.max_depth = std::max(P.max_depth, T.depth[size_t(n)]);
    }
    // leaves are addressed by their static discovery rank on the device (inner_table)
    std::vector<int32_t> leaf_rank;
    int rc;
    if ((rc = inner_table(T, P.inner, leaf_rank))) return rc;
    P.ninner = int32_t(P.inner.size() / 3);
    if (P.inner.empty()) P.inner.assign(3, float4_t{0.f, 0.f, 0.f, 0.f});
    auto by_rank = [&](const std::vector<uint32_t>& per_node) {
        std::vector<uint32_t> out(std::max<size_t>(2, per_node.size()), 0u);
        for (int32_t n = 0; n < T.nnodes; ++n) {
            const int32_t k = leaf_rank[size_t(n)];
            if (k < 0) continue;
            out[2 * size_t(k)] = per_node[2 * size_t(n)];
            out[2 * size_t(k) + 1] = per_node[2 * size_t(n) + 1];
        }
        return out;
    };
    P.leaf_range = by_rank(range);
    P.tris.resize(nprims);
    for (size_t k = 0; k < nprims; ++k) P.tris[k] = make_tri(&T.prim_vertices[9 * k], T.prim_face[k]);
    const size_t np = nprims ? nprims : 1;
    P.t0.assign(np, float4_t{0.f, 0.f, 0.f, 0.f});
    P.t1.assign(np, float4_t{0.f, 0.f, 0.f, 0.f});
    P.t2.assign(np, 0.f);
    P.tface.assign(np, 0u);
    for (size_t k = 0; k < nprims; ++k) {
        const DTri& t = P.tris[k];
        P.t0[k] = float4_t{t.ax, t.ay, t.az, t.abx};
        P.t1[k] = float4_t{t.aby, t.abz, t.acx, t.acy};
        P.t2[k] = t.acz;
        P.tface[k] = t.face;
    }
    // clustered copy of the leaf primitives
    LeafClusters C;
    if ((rc = leaf_clusters(T, cluster_size, C))) return rc;
    // every cluster owns kMaxClusterSize consecutive slots (its first slot is 16 c), so the
    // record's last word can carry the screen normals' step instead
    const size_t ncl = C.rec.size() / 8;
    P.nclusters = ncl;
    const size_t ns = std::max<size_t>(1, ncl) * kMaxClusterSize;
    // full-test records, 48 B per slot (cluster.h load_prim)
    P.prim.assign(3 * ns, float4_t{0.f, 0.f, 0.f, 0.f});
    // screen normals, kNormWords u32 per cluster: (nx, ny) of slot k as f16 in word k, then
    // (nz of slot 2i, nz of slot 2i + 1) in word kMaxClusterSize + i (cluster.h)
    std::vector<uint32_t> nw(std::max<size_t>(1, ncl) * kNormWords, 0u);
    for (size_t cl = 0; cl < ncl; ++cl) {
        uint32_t pw, first;
        std::memcpy(&pw, &C.rec[8 * cl + 3], 4);
        std::memcpy(&first, &C.rec[8 * cl + 7], 4);
        const uint32_t n = (pw & 31u) + 1u;
        if (n > uint32_t(kMaxClusterSize) || size_t(first) + n > C.order.size()) return ATR_E_INVALID;
        // screen normals: a step q >= max |n component| / 511 and each normal as round(n / q),
        // integers of at most 511 (exact in f16; |n - q p| <= q / 2)
        double mx = 0.0;
        for (uint32_t k = first; k < first + n; ++k)
            for (int a = 0; a < 3; ++a) mx = std::max(mx, std::fabs(double(C.normal[3 * size_t(k) + size_t(a)])));
        float q = float(mx / 511.0);
        while (double(q) * 511.0 < mx) q = std::nextafter(q, INFINITY);
        if (!(q > 0.f)) q = 1e-30f;
        C.rec[8 * cl + 7] = q;
        for (uint32_t i = 0; i < n; ++i) {
            const size_t k = first + i, slot = cl * kMaxClusterSize + i;
            if (C.order[k] >= nprims) return ATR_E_INVALID;
            const DTri& t = P.tris[C.order[k]];
            float rk, fc;
            std::memcpy(&rk, &C.rank[k], 4);
            std::memcpy(&fc, &t.face, 4);
            P.prim[3 * slot] = float4_t{t.ax, t.ay, t.az, t.abx};
            P.prim[3 * slot + 1] = float4_t{t.aby, t.abz, t.acx, t.acy};
            P.prim[3 * slot + 2] = float4_t{t.acz, rk, fc, 0.f};
            uint16_t h[3];
            for (int a = 0; a < 3; ++a) {
                const double r = double(C.normal[3 * k + size_t(a)]) / double(q);
                long v = std::isfinite(r) ? std::lround(std::max(-1e6, std::min(1e6, r))) : 0L;
                v = std::max(-511L, std::min(511L, v));
                h[a] = half_of_int(int32_t(v));
            }
            nw[kNormWords * cl + i] = uint32_t(h[0]) | (uint32_t(h[1]) << 16);
            nw[kNormWords * cl + kMaxClusterSize + i / 2] |= uint32_t(h[2]) << (16 * (i & 1));
        }
    }
    // one 128-B block per cluster: record {lo, P}{hi, q}, then its kNormWords normal words
    static_assert(8 + kNormWords == 4 * kClusterBlock, "cluster block layout");
    P.clus.assign(std::max<size_t>(1, ncl) * 4 * kClusterBlock, 0u);
    for (size_t cl = 0; cl < ncl; ++cl) {
        std::memcpy(&P.clus[4 * kClusterBlock * cl], &C.rec[8 * cl], 8 * sizeof(float));
        std::memcpy(&P.clus[4 * kClusterBlock * cl + 8], &nw[kNormWords * cl], kNormWords * sizeof(uint32_t));
    }
    P.cl_range = by_rank(C.range);
    P.near_ok = P.max_depth <= 8 && P.ninner < 65536;  // traverse_pass_near's register stack
    return ATR_OK;
}
