// bounce_sim.cpp -- offline work model of the clustered scan for BOUNCE rays (analysis tool, not
// product). Where do a bounce ray's full triangle tests go?
//
// Builds the Dragon surrogate's octree and leaf clusters with the product's host code, traces the
// camera rays of every `step`-th pixel of a 1920x1080 frame, and from each hit one bounce ray per
// sample (the reference's bounce: renderer.cpp:231-258 with the interpolated normal replaced by
// the geometric one, a PCG-like hash for the three rand_bi draws). Each bounce ray is traced with
// the kernel's clustered scan (loose + tight padded boxes, det screen; the reference leaf order)
// and every full test is classified:
//   hit       accepted (t > kTol, u, v in range)
//   behind    plane parameter t <= kTol (the triangle's plane is at or behind the origin: the
//             origin's own surface patch)
//   far       plane t beyond the best t so far
//   uv        plane t in (kTol, best) but the line misses the triangle (u, v out of range)
//   culled    det below kTol (the screen's band kept it)
// and the would-be rejections of cheaper per-primitive screens are counted: the plane test with
// f32 normals (behind / far) and a bounding sphere around the triangle.
//
// g++ -O2 -std=c++17 -ffp-contract=off -I atray_amd/csrc tools/bounce_sim.cpp
//     atray_amd/csrc/host_scene.cpp -o build/bounce_sim && build/bounce_sim OBJ [step] [spp]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

#include "engine.h"
#include "host_scene.h"

using namespace atr;

namespace {

struct TriOut { float t, u, v, det; bool acc; };
TriOut tri(V3 o, V3 d, V3 a, V3 ab, V3 ac) {
    TriOut r{0, 0, 0, 0, false};
    const V3 pvec = cross(d, ac);
    r.det = dot(ab, pvec);
    if (r.det < kTol) return r;
    const float det_inv = 1 / r.det;
    const V3 tvec = sub(o, a);
    r.u = dot(tvec, pvec) * det_inv;
    const V3 qvec = cross(tvec, ab);
    r.v = dot(d, qvec) * det_inv;
    r.t = dot(qvec, ac) * det_inv;
    r.acc = !(r.u < 0 || r.u > 1 || r.v < 0 || r.u + r.v > 1);
    return r;
}

bool box_check(V3 o, V3 inv, const float* b) {
    const int s0 = inv.x < 0, s1 = inv.y < 0, s2 = inv.z < 0;
    float tmin = ((s0 ? b[3] : b[0]) - o.x) * inv.x, tmax = ((s0 ? b[0] : b[3]) - o.x) * inv.x;
    const float tymin = ((s1 ? b[4] : b[1]) - o.y) * inv.y, tymax = ((s1 ? b[1] : b[4]) - o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = ((s2 ? b[5] : b[2]) - o.z) * inv.z, tzmax = ((s2 ? b[2] : b[5]) - o.z) * inv.z;
    return !((tmin > tzmax) || (tzmin > tmax));
}
float box_entry(V3 o, V3 inv, const float* b) {
    const int s0 = inv.x < 0, s1 = inv.y < 0, s2 = inv.z < 0;
    float tmin = ((s0 ? b[3] : b[0]) - o.x) * inv.x, tmax = ((s0 ? b[0] : b[3]) - o.x) * inv.x;
    const float tymin = ((s1 ? b[4] : b[1]) - o.y) * inv.y, tymax = ((s1 ? b[1] : b[4]) - o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = ((s2 ? b[5] : b[2]) - o.z) * inv.z, tzmax = ((s2 ? b[2] : b[5]) - o.z) * inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    if (tmin > 0) return tmin;
    if (tmax > 0) return tmax;
    return 0;
}

uint64_t hash64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
float rbi(uint64_t& s) { s = hash64(s + 0x9E3779B97F4A7C15ull); return float(s >> 40) / float(1 << 24) * 2.f - 1.f; }

struct Cls { double rays = 0, leaves = 0, crec = 0, cpass = 0, screen = 0, full = 0, hit = 0, behind = 0, far = 0,
             uv = 0, culled = 0, plane_keep = 0, sphere_keep = 0, both_keep = 0, origin_leaf_full = 0; };

struct Scene {
    HostTree T;
    LeafClusters C;
    std::vector<float> sph;  // per slot: bounding sphere centre + radius (f32, exact enough for a model)
    std::vector<int32_t> rank;          // leaf node -> static discovery rank (inner_table)
    std::vector<int32_t> rlo, rhi;      // node -> smallest / largest leaf rank below it
};

struct Walk { double rays = 0, ref_visits = 0, lazy_visits = 0, lazy_pq_visits = 0, k8_visits = 0, lr_visits = 0, lr_passes = 0, k8_passes = 0; };
Walk g_walk[3];
int g_level = 0;
int g_min_safe = 1;  // lazy_restart: safe leaves a pass returns at least (argv[4])
// per traced ray of the current level, for the wave model: the kernel's passes (visits, leaves
// consumed) and the lazy walk's visits before each leaf it scans
struct RaySeq { std::vector<std::pair<int, int>> k8; std::vector<int> lazy; std::vector<int32_t> p1; float o[3], d[3]; int oleaf = -1; };
std::vector<RaySeq> g_seq[3];

// Inner-node visits of three traversal schedules for the same query (the leaf set and order are the
// reference's; only the visiting differs):
//   ref   the reference DFS (every discovered node examined);
//   k8    near-first passes into an 8-leaf buffer with subtree skipping once full, re-walks after
//         the buffer's last leaf (the kernel's traverse_pass_near);
//   lazy  near-first DFS that scans a leaf as soon as no pending subtree can hold a leaf before it
//         in (distance, rank) order, and stops at the leaf that ends the query; lazy_pq the same
//         with the pending subtrees in a priority queue (a lower bound).
void walk_model(const Scene& S, V3 o, V3 d, int improving, const std::vector<std::pair<float, int>>& ref_leaves);

// One query with the kernel's clustered scan; returns best t (kMaxFloat none) and the hit slot.
float trace(const Scene& S, V3 o, V3 d, Cls* cls, uint32_t& hit_slot) {
    const HostTree& T = S.T;
    const LeafClusters& C = S.C;
    const V3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
    hit_slot = 0xFFFFFFFFu;
    if (cls) cls->rays += 1;
    if (!box_check(o, inv, &T.bounds[0])) return kMaxFloat;
    std::vector<std::pair<float, int>> leaves;
    std::vector<int32_t> stack(1, 0);
    while (!stack.empty()) {
        const int32_t cur = stack.back();
        stack.pop_back();
        const int32_t ch = T.children[size_t(cur)];
        int hit = 0;
        for (int i = 0; i < 8 && hit <= 4; ++i) {
            const int32_t c = ch + i;
            if (T.children[size_t(c)]) {
                if (box_check(o, inv, &T.bounds[6 * size_t(c)])) { ++hit; stack.push_back(c); }
            } else {
                const float dis = box_entry(o, inv, &T.bounds[6 * size_t(c)]);
                if (dis > 0) {
                    ++hit;
                    auto it = std::upper_bound(leaves.begin(), leaves.end(), dis,
                                               [](float v, const std::pair<float, int>& e) { return v < e.first; });
                    leaves.insert(it, {dis, c});
                }
            }
        }
    }
    float best = kMaxFloat;
    bool first_leaf = true;
    int improving = -1;  // node id of the leaf that ended the query (-1: none)
    for (auto& lf : leaves) {
        if (cls) cls->leaves += 1;
        const uint32_t c0 = C.range[2 * size_t(lf.second)], nc = C.range[2 * size_t(lf.second) + 1];
        bool improved = false;
        for (uint32_t c = c0; c < c0 + nc; ++c) {
            if (cls) cls->crec += 1;
            const float* r = &C.rec[8 * size_t(c)];
            const float eps = 5.9604645e-8f, tau = 3e-3f;
            const float ex = r[4] - r[0], ey = r[5] - r[1], ez = r[6] - r[2];
            const float fx = std::max(std::fabs(r[0] - o.x), std::fabs(r[4] - o.x));
            const float fy = std::max(std::fabs(r[1] - o.y), std::fabs(r[5] - o.y));
            const float fz = std::max(std::fabs(r[2] - o.z), std::fabs(r[6] - o.z));
            const float W = std::sqrt(fx * fx + fy * fy + fz * fz) * 1.0000005f + (ex + ey + ez);
            const float P = r[3];
            auto pad = [&](float D) { return W * (P * (36 * eps / (0.9f * D)) + 12 * eps); };
            auto hitbox = [&](float g) {
                float bb[6];
                for (int q = 0; q < 3; ++q) { bb[q] = r[q] - g; bb[3 + q] = r[4 + q] + g; }
                return box_check(o, inv, bb) && !(box_entry(o, inv, bb) > best);
            };
            const float mg = 16 * eps * P;
            const float dlo = kTol - mg;
            float dhi = 1e30f;
            if (!hitbox(pad(kTol))) continue;
            if (!hitbox(pad(tau))) dhi = tau + mg;
            if (cls) cls->cpass += 1;
            uint32_t pw, fs;
            std::memcpy(&pw, &C.rec[8 * c + 3], 4);
            std::memcpy(&fs, &C.rec[8 * c + 7], 4);
            const uint32_t n = (pw & 31u) + 1u;
            for (uint32_t k = fs; k < fs + n; ++k) {
                if (cls) cls->screen += 1;
                const float* nn = &C.normal[3 * k];
                const float det = -(d.x * nn[0] + d.y * nn[1] + d.z * nn[2]);
                if (!(det >= dlo && det < dhi)) continue;
                const float* v = &T.prim_vertices[9 * size_t(C.order[k])];
                const V3 a = mk(v[0], v[1], v[2]);
                const TriOut to = tri(o, d, a, sub(mk(v[3], v[4], v[5]), a), sub(mk(v[6], v[7], v[8]), a));
                const bool accepted = to.det >= kTol && to.acc && to.t > kTol && to.t < best;
                if (cls) {
                    cls->full += 1;
                    if (first_leaf) cls->origin_leaf_full += 1;
                    // plane parameter in double
                    const double n0 = nn[0], n1 = nn[1], n2 = nn[2];
                    const double num = (double(a.x) - o.x) * n0 + (double(a.y) - o.y) * n1 + (double(a.z) - o.z) * n2;
                    const double den = double(d.x) * n0 + double(d.y) * n1 + double(d.z) * n2;
                    const double tp = den != 0 ? num / den : 1e30;
                    if (to.det < kTol) cls->culled += 1;
                    else if (accepted || (to.acc && to.t > kTol)) cls->hit += 1;
                    else if (tp <= kTol) cls->behind += 1;
                    else if (tp >= best) cls->far += 1;
                    else cls->uv += 1;
                    // would a per-primitive plane screen keep it? (margin 1e-5 relative + 1e-6)
                    const bool pk = !(tp <= kTol * 0.5 || tp > double(best) * 1.001 + 1e-5);
                    // bounding sphere (f32 centre, radius + rounding pad): does the line pass within R?
                    const float* sp = &S.sph[4 * size_t(k)];
                    const double w[3] = {sp[0] - double(o.x), sp[1] - double(o.y), sp[2] - double(o.z)};
                    const double tc = w[0] * d.x + w[1] * d.y + w[2] * d.z;
                    const double cx = w[1] * d.z - w[2] * d.y, cy = w[2] * d.x - w[0] * d.z, cz = w[0] * d.y - w[1] * d.x;
                    const double R = sp[3] * 1.001 + pad(det >= tau ? tau : kTol);
                    const bool sk = cx * cx + cy * cy + cz * cz <= R * R && tc + R > kTol && tc - R < best;
                    cls->plane_keep += pk;
                    cls->sphere_keep += sk;
                    cls->both_keep += pk && sk;
                }
                if (accepted) { best = to.t; hit_slot = k; improved = true; }
            }
        }
        first_leaf = false;
        if (improved) { improving = lf.second; break; }
    }
    if (cls) walk_model(S, o, d, improving, leaves);
    return best;
}

struct Pend { float bound; int32_t rlo; int32_t node; };
bool lex_less(float d, int32_t r, float d2, int32_t r2) { return d < d2 || (d == d2 && r < r2); }

// near-first child order: children in the ray's crossing order (index mirrored by the direction's
// signs, as traverse_pass_near), examined with the reference's first-5-hits rule in child order.
struct Examined { std::vector<std::pair<float, int32_t>> leaves; std::vector<Pend> inner; };
Examined examine(const Scene& S, V3 o, V3 inv, int32_t node) {
    const HostTree& T = S.T;
    Examined e;
    const int32_t ch = T.children[size_t(node)];
    int hit = 0;
    bool hitv[8] = {};
    for (int i = 0; i < 8 && hit <= 4; ++i) {
        const int32_t c = ch + i;
        const float* b = &T.bounds[6 * size_t(c)];
        if (T.children[size_t(c)]) {
            if (box_check(o, inv, b)) { ++hit; hitv[i] = true; }
        } else {
            const float dis = box_entry(o, inv, b);
            if (dis > 0) { ++hit; hitv[i] = true; }
        }
    }
    const int sm = (inv.x < 0) * 4 + (inv.y < 0) * 2 + (inv.z < 0);
    for (int k = 0; k < 8; ++k) {
        const int i = k ^ sm;
        if (!hitv[i]) continue;
        const int32_t c = ch + i;
        const float* b = &T.bounds[6 * size_t(c)];
        if (T.children[size_t(c)]) {
            // lower bound of the leaf distances below: the box entry if in front, else 0
            const int s0 = inv.x < 0, s1 = inv.y < 0, s2 = inv.z < 0;
            float tmin = ((s0 ? b[3] : b[0]) - o.x) * inv.x;
            tmin = std::max(tmin, ((s1 ? b[4] : b[1]) - o.y) * inv.y);
            tmin = std::max(tmin, ((s2 ? b[5] : b[2]) - o.z) * inv.z);
            float tmax = ((s0 ? b[0] : b[3]) - o.x) * inv.x;
            tmax = std::min(tmax, ((s1 ? b[1] : b[4]) - o.y) * inv.y);
            tmax = std::min(tmax, ((s2 ? b[2] : b[5]) - o.z) * inv.z);
            if (tmax <= 0) continue;  // nothing in front
            e.inner.push_back({std::max(tmin, 0.f), S.rlo[size_t(c)], c});
        } else {
            e.leaves.push_back({box_entry(o, inv, b), S.rank[size_t(c)]});
        }
    }
    return e;
}

void walk_model(const Scene& S, V3 o, V3 d, int improving, const std::vector<std::pair<float, int>>& ref_leaves) {
    const HostTree& T = S.T;
    Walk& W = g_walk[g_level];
    W.rays += 1;
    const V3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
    if (!box_check(o, inv, &T.bounds[0]) || T.children[0] == 0) return;
    const int32_t stop_rank = improving >= 0 ? S.rank[size_t(improving)] : -1;
    // ref: every inner node the reference DFS examines
    {
        std::vector<int32_t> st(1, 0);
        while (!st.empty()) {
            const int32_t cur = st.back();
            st.pop_back();
            W.ref_visits += 1;
            const int32_t ch = T.children[size_t(cur)];
            int hit = 0;
            for (int i = 0; i < 8 && hit <= 4; ++i) {
                const int32_t c = ch + i;
                if (T.children[size_t(c)]) {
                    if (box_check(o, inv, &T.bounds[6 * size_t(c)])) { ++hit; st.push_back(c); }
                } else if (box_entry(o, inv, &T.bounds[6 * size_t(c)]) > 0) ++hit;
            }
        }
    }
    // lazy (DFS stack order) and lazy_pq (priority queue)
    for (int pq = 0; pq < 2; ++pq) {
        std::vector<Pend> pend{{0.f, S.rlo[0], 0}};
        std::vector<std::pair<float, int32_t>> found;  // sorted (dist, rank)
        double visits = 0;
        int since = 0;  // visits since the last leaf scan
        std::vector<int> seq;
        bool done = false;
        while (!done) {
            // scan every safe leaf
            while (!found.empty()) {
                bool safe = true;
                for (const Pend& p : pend)
                    if (!lex_less(found[0].first, found[0].second, p.bound, p.rlo)) { safe = false; break; }
                if (!safe) break;
                seq.push_back(since);
                since = 0;
                if (found[0].second == stop_rank) { done = true; break; }
                found.erase(found.begin());
            }
            if (done || pend.empty()) break;
            size_t pick = pend.size() - 1;
            if (pq)
                for (size_t i = 0; i < pend.size(); ++i)
                    if (lex_less(pend[i].bound, pend[i].rlo, pend[pick].bound, pend[pick].rlo)) pick = i;
            const Pend p = pend[pick];
            pend.erase(pend.begin() + long(pick));
            visits += 1;
            ++since;
            Examined e = examine(S, o, inv, p.node);
            for (auto& lf : e.leaves) {
                auto it = std::lower_bound(found.begin(), found.end(), lf, [](const std::pair<float, int32_t>& a,
                                                                               const std::pair<float, int32_t>& b) {
                    return lex_less(a.first, a.second, b.first, b.second);
                });
                found.insert(it, lf);
            }
            // DFS order: push the far children first so the nearest is on top
            for (auto it = e.inner.rbegin(); it != e.inner.rend(); ++it) pend.push_back(*it);
        }
        (pq ? W.lazy_pq_visits : W.lazy_visits) += visits;
        if (!pq) {
            while (!found.empty() && !done) {  // no pending subtree left: the rest are safe
                seq.push_back(since);
                since = 0;
                if (found[0].second == stop_rank) break;
                found.erase(found.begin());
            }
            g_seq[g_level].emplace_back();
            RaySeq& rs = g_seq[g_level].back();
            rs.lazy = seq;
            rs.o[0] = o.x; rs.o[1] = o.y; rs.o[2] = o.z;
            rs.d[0] = d.x; rs.d[1] = d.y; rs.d[2] = d.z;
            // the leaf holding the origin (the first leaf of the reference order whose box contains o)
            for (int32_t n = 0; n < T.nnodes && rs.oleaf < 0; ++n) {
                if (T.children[size_t(n)]) continue;
                const float* b = &T.bounds[6 * size_t(n)];
                if (o.x >= b[0] && o.x <= b[3] && o.y >= b[1] && o.y <= b[4] && o.z >= b[2] && o.z <= b[5]) rs.oleaf = n;
            }
        }
    }
    // lazy_restart: near-first passes that return as soon as some found leaf is safe (every safe leaf,
    // at most K), the leaves scanned, then a re-walk from the root after the last returned leaf
    // (no traversal state kept across the leaf scans); inner children whose exit is at or before
    // the re-walk bound are not entered (the kernel's cull rule)
    {
        const int K = 8;
        float bd = -1e30f;
        int32_t bi = -1;
        double visits = 0, passes = 0;
        for (;;) {
            passes += 1;
            std::vector<Pend> pend{{0.f, S.rlo[0], 0}};
            std::vector<std::pair<float, int32_t>> found;
            std::vector<std::pair<float, int32_t>> out;
            for (;;) {
                while (!found.empty() && (int)out.size() < K) {
                    bool safe = true;
                    for (const Pend& p : pend)
                        if (!lex_less(found[0].first, found[0].second, p.bound, p.rlo)) { safe = false; break; }
                    if (!safe) break;
                    out.push_back(found[0]);
                    found.erase(found.begin());
                }
                if ((int)out.size() >= g_min_safe || pend.empty()) break;
                const Pend p = pend.back();
                pend.pop_back();
                visits += 1;
                Examined e = examine(S, o, inv, p.node);
                for (auto& lf : e.leaves) {
                    if (!lex_less(bd, bi, lf.first, lf.second)) continue;
                    auto it = std::lower_bound(found.begin(), found.end(), lf, [](const std::pair<float, int32_t>& a,
                                                                               const std::pair<float, int32_t>& b) {
                        return lex_less(a.first, a.second, b.first, b.second);
                    });
                    found.insert(it, lf);
                }
                for (auto it = e.inner.rbegin(); it != e.inner.rend(); ++it) pend.push_back(*it);
            }
            bool stop = out.empty();
            for (auto& lf : out)
                if (lf.second == stop_rank) stop = true;
            if (stop) break;
            bd = out.back().first;
            bi = out.back().second;
        }
        W.lr_visits += visits;
        W.lr_passes += passes;
    }
    // k8: near-first passes with an 8-leaf buffer, subtree skip when full, re-walk after the buffer
    {
        const int K = 8;
        float bd = -1e30f;
        int32_t bi = -1;
        double visits = 0;
        std::vector<std::pair<int, int>> passes;
        for (;;) {
            W.k8_passes += 1;
            const double v0 = visits;
            std::vector<std::pair<float, int32_t>> buf;  // sorted, at most K
            bool more = false;
            std::vector<Pend> st{{0.f, S.rlo[0], 0}};
            while (!st.empty()) {
                const Pend p = st.back();
                st.pop_back();
                if ((int)buf.size() == K && !lex_less(p.bound, p.rlo, buf.back().first, buf.back().second)) {
                    more = true;
                    continue;
                }
                visits += 1;
                if (passes.empty()) g_seq[g_level].back().p1.push_back(p.node);  // first pass's nodes
                Examined e = examine(S, o, inv, p.node);
                for (auto& lf : e.leaves) {
                    if (!lex_less(bd, bi, lf.first, lf.second)) continue;  // at or before the re-walk bound
                    auto it = std::lower_bound(buf.begin(), buf.end(), lf, [](const std::pair<float, int32_t>& a,
                                                                             const std::pair<float, int32_t>& b) {
                        return lex_less(a.first, a.second, b.first, b.second);
                    });
                    buf.insert(it, lf);
                    if ((int)buf.size() > K) { buf.pop_back(); more = true; }
                }
                for (auto it = e.inner.rbegin(); it != e.inner.rend(); ++it) st.push_back(*it);
            }
            bool stop = false;
            int used = 0;
            for (auto& lf : buf) {
                ++used;
                if (lf.second == stop_rank) { stop = true; break; }
            }
            passes.push_back({int(visits - v0), used});
            if (stop || !more || buf.empty()) break;
            bd = buf.back().first;
            bi = buf.back().second;
        }
        W.k8_visits += visits;
        g_seq[g_level].back().k8 = passes;
    }
    (void)ref_leaves;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: bounce_sim OBJ [step] [spp]\n"); return 2; }
    const int step = argc > 2 ? std::atoi(argv[2]) : 8;
    const int spp = argc > 3 ? std::atoi(argv[3]) : 4;
    if (argc > 4) g_min_safe = std::atoi(argv[4]);
    std::ifstream f(argv[1], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    HostMesh M;
    if (parse_obj_text(text.data(), text.size(), M)) return 1;
    float box[6];
    mesh_aabb(M, box);
    mesh_translate(M, box, mk(0.f, -15.f, -38.f));
    Scene S;
    if (octree_build(M, 300, S.T)) return 1;
    if (leaf_clusters(S.T, 16, S.C)) return 1;
    {
        std::vector<float4_t> inner;
        if (inner_table(S.T, inner, S.rank)) return 1;
        const int32_t nn = S.T.nnodes;
        S.rlo.assign(size_t(nn), 1 << 30);
        S.rhi.assign(size_t(nn), -1);
        for (int32_t n = nn - 1; n >= 0; --n) {  // children come after their parent in node order
            if (S.T.children[size_t(n)] == 0) { S.rlo[size_t(n)] = S.rhi[size_t(n)] = S.rank[size_t(n)]; continue; }
            for (int i = 0; i < 8; ++i) {
                const int32_t c = S.T.children[size_t(n)] + i;
                S.rlo[size_t(n)] = std::min(S.rlo[size_t(n)], S.rlo[size_t(c)]);
                S.rhi[size_t(n)] = std::max(S.rhi[size_t(n)], S.rhi[size_t(c)]);
            }
        }
    }
    const size_t nslots = S.C.order.size();
    S.sph.resize(4 * nslots);
    for (size_t k = 0; k < nslots; ++k) {
        const float* v = &S.T.prim_vertices[9 * size_t(S.C.order[k])];
        double cc[3], rr = 0;
        for (int q = 0; q < 3; ++q) cc[q] = (double(v[q]) + v[3 + q] + v[6 + q]) / 3.0;
        for (int j = 0; j < 3; ++j) {
            double d2 = 0;
            for (int q = 0; q < 3; ++q) d2 += (v[3 * j + q] - cc[q]) * (v[3 * j + q] - cc[q]);
            rr = std::max(rr, std::sqrt(d2));
        }
        for (int q = 0; q < 3; ++q) S.sph[4 * k + q] = float(cc[q]);
        S.sph[4 * k + 3] = float(rr);
    }
    atr_camera cm;
    camera_set(cm, mk(0.1f, 2.f, 0.f), mk(-0.1f, -0.5f, -1.f), 1920, 1080, 0, 1, 1, 1.f);
    const V3 eye = from(cm.eye), fc = from(cm.frame_center), cx = from(cm.camera_x), cy = from(cm.camera_y);
    Cls cam, b1, b2;
    for (int y = 0; y < cm.height; y += step)
        for (int x = 0; x < cm.width; x += step) {
            const float film_y = -1.0f + 2.0f * (float(y) / float(cm.height));
            const float film_x = ((-1.0f + 2.0f * (float(x) / float(cm.width))) * cm.h_fov) * cm.aspect_ratio;
            const V3 d0 = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));
            uint32_t slot;
            g_level = 0;
            const float t0 = trace(S, eye, d0, &cam, slot);
            if (slot == 0xFFFFFFFFu) continue;
            for (int s = 0; s < spp; ++s) {
                uint64_t st = hash64((uint64_t(y) << 32) ^ uint64_t(x) ^ (uint64_t(s) << 48));
                V3 o = add(eye, scale(d0, t0)), d = d0;
                uint32_t sl = slot;
                for (int level = 1; level <= 2; ++level) {
                    const float* nn = &S.C.normal[3 * sl];
                    V3 n = unit(mk(nn[0], nn[1], nn[2]));
                    if (dot(neg(d), n) < 0) n = neg(n);
                    const V3 rnd = unit(add(mk(rbi(st), rbi(st), rbi(st)), n));
                    const V3 pure = unit(sub(d, scale(n, 2 * dot(d, n))));
                    d = unit(add(scale(rnd, 0.7f), scale(pure, 0.3f)));  // lerp(rnd, pure, 0.3)
                    g_level = level;
                    const float t = trace(S, o, d, level == 1 ? &b1 : &b2, sl);
                    if (sl == 0xFFFFFFFFu) break;
                    o = add(o, scale(d, t));
                }
            }
        }
    auto pr = [](const char* name, const Cls& c) {
        const double a = c.rays;
        std::printf("%-8s rays %.0f: leaves %.2f  cluster recs %.1f  passed %.1f  screened %.1f  full %.1f"
                    " [hit %.2f behind %.1f far %.1f uv %.1f culled %.2f; origin leaf %.1f]"
                    "  plane screen keeps %.2f, sphere keeps %.2f, both %.2f\n",
                    name, a, c.leaves / a, c.crec / a, c.cpass / a, c.screen / a, c.full / a, c.hit / a, c.behind / a,
                    c.far / a, c.uv / a, c.culled / a, c.origin_leaf_full / a, c.plane_keep / a, c.sphere_keep / a,
                    c.both_keep / a);
    };
    // wave model: rays in generation order, 64 per wave (level 1: a pixel's samples side by side)
    for (int l = 1; l < 3; ++l)
      for (int order = 0; order < 11; ++order) {
        // 0: queue order; 1: sorted by (origin leaf, direction octant); 2: by direction octant then
        // origin leaf; 3: by a 64-bin direction cell (octant x 8 sub-cells) then origin leaf
        std::vector<RaySeq> R = g_seq[l];
        auto oct = [](const RaySeq& r) { return (r.d[0] < 0) * 4 + (r.d[1] < 0) * 2 + (r.d[2] < 0); };
        auto cell = [&](const RaySeq& r) {
            const float ax = std::fabs(r.d[0]), ay = std::fabs(r.d[1]), az = std::fabs(r.d[2]);
            const int major = ax >= ay && ax >= az ? 0 : (ay >= az ? 1 : 2);
            return oct(r) * 8 + major * 2 + (std::max(ax, std::max(ay, az)) > 0.85f);
        };
        if (order == 1) std::stable_sort(R.begin(), R.end(), [&](const RaySeq& a, const RaySeq& b) {
            return a.oleaf != b.oleaf ? a.oleaf < b.oleaf : oct(a) < oct(b); });
        if (order == 2) std::stable_sort(R.begin(), R.end(), [&](const RaySeq& a, const RaySeq& b) {
            return oct(a) != oct(b) ? oct(a) < oct(b) : a.oleaf < b.oleaf; });
        if (order == 3) std::stable_sort(R.begin(), R.end(), [&](const RaySeq& a, const RaySeq& b) {
            return cell(a) != cell(b) ? cell(a) < cell(b) : a.oleaf < b.oleaf; });
        // 4..7: the direction cell, then a Morton code of the origin at 3..6 bits per axis over the
        // origins' bounding box (what a GPU key can compute without a point location)
        if (order >= 4) {
            float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
            for (const auto& r : R)
                for (int a = 0; a < 3; ++a) lo[a] = std::min(lo[a], r.o[a]), hi[a] = std::max(hi[a], r.o[a]);
            const int bits = order >= 8 ? 4 : order - 1;
            auto morton = [&](const RaySeq& r) {
                uint32_t m = 0;
                int q[3];
                for (int a = 0; a < 3; ++a)
                    q[a] = std::min((1 << bits) - 1, std::max(0, int((r.o[a] - lo[a]) / (hi[a] - lo[a] + 1e-20f) * float(1 << bits))));
                for (int b = bits - 1; b >= 0; --b)
                    for (int a = 0; a < 3; ++a) m = (m << 1) | ((q[a] >> b) & 1);
                return m;
            };
            // 8..10: an octahedral direction cell of 8x8, 16x16, 32x32 instead of the 64-bin cell
            const int oc = order == 8 ? 8 : order == 9 ? 16 : 32;
            auto ocell = [&](const RaySeq& r) {
                const float s = std::fabs(r.d[0]) + std::fabs(r.d[1]) + std::fabs(r.d[2]);
                float u = r.d[0] / s, v = r.d[1] / s;
                if (r.d[2] < 0) {
                    const float uu = (1 - std::fabs(v)) * (u >= 0 ? 1 : -1), vv = (1 - std::fabs(u)) * (v >= 0 ? 1 : -1);
                    u = uu, v = vv;
                }
                const int iu = std::min(oc - 1, int((u * 0.5f + 0.5f) * oc)), iv = std::min(oc - 1, int((v * 0.5f + 0.5f) * oc));
                return iv * oc + iu;
            };
            if (order < 8)
                std::stable_sort(R.begin(), R.end(), [&](const RaySeq& a, const RaySeq& b) {
                    return cell(a) != cell(b) ? cell(a) < cell(b) : morton(a) < morton(b); });
            else
                std::stable_sort(R.begin(), R.end(), [&](const RaySeq& a, const RaySeq& b) {
                    return ocell(a) != ocell(b) ? ocell(a) < ocell(b) : morton(a) < morton(b); });
        }
        double k8_iters = 0, k8_steps = 0, lz_iters = 0, lz_steps = 0, waves = 0;
        double p1_max = 0, p1_mean = 0, p1_union = 0, p1_uniform = 0;
        for (size_t w0 = 0; w0 + 64 <= R.size(); w0 += 64) {
            waves += 1;
            {   // first passes: per-lane walks (wave iterations = the longest) vs one wave-walked
                // near-first pass for a common direction-sign octant (iterations = the union)
                std::vector<int32_t> all;
                size_t mx = 0, sum = 0, n = 0;
                int sm0 = -1;
                bool uni = true;
                for (int i = 0; i < 64; ++i) {
                    const auto& v = R[w0 + i].p1;
                    if (v.empty()) continue;
                    const int sm = (R[w0 + i].d[0] < 0) * 4 + (R[w0 + i].d[1] < 0) * 2 + (R[w0 + i].d[2] < 0);
                    if (sm0 < 0) sm0 = sm;
                    uni = uni && sm == sm0;
                    mx = std::max(mx, v.size());
                    sum += v.size();
                    ++n;
                    all.insert(all.end(), v.begin(), v.end());
                }
                std::sort(all.begin(), all.end());
                p1_union += double(std::unique(all.begin(), all.end()) - all.begin());
                p1_max += double(mx);
                p1_mean += n ? double(sum) / double(n) : 0.0;
                p1_uniform += uni ? 1.0 : 0.0;
            }
            {   // the kernel: a pass phase whenever a lane needs a pass (all lanes wait), then a leaf step
                std::vector<size_t> p(64, 0);
                std::vector<int> c(64, 0);
                std::vector<char> need(64, 1), done(64, 0);
                for (int i = 0; i < 64; ++i) if (R[w0 + i].k8.empty()) done[i] = 1, need[i] = 0;
                for (;;) {
                    int mx = 0, live = 0;
                    for (int i = 0; i < 64; ++i)
                        if (!done[i] && need[i]) { mx = std::max(mx, R[w0 + i].k8[p[i]].first); need[i] = 0; }
                    for (int i = 0; i < 64; ++i) live += !done[i];
                    if (!live) break;
                    k8_iters += mx;
                    k8_steps += 1;
                    for (int i = 0; i < 64; ++i) {
                        if (done[i]) continue;
                        const auto& ps = R[w0 + i].k8;
                        if (++c[i] >= ps[p[i]].second) {
                            if (p[i] + 1 < ps.size()) { ++p[i]; c[i] = 0; need[i] = 1; }
                            else done[i] = 1;
                        }
                    }
                }
            }
            {   // lazy: before each leaf step, every live lane walks until its next leaf is safe
                std::vector<size_t> q(64, 0);
                for (;;) {
                    int mx = 0, live = 0;
                    for (int i = 0; i < 64; ++i) {
                        const auto& z = R[w0 + i].lazy;
                        if (q[i] < z.size()) { ++live; mx = std::max(mx, z[q[i]]); }
                    }
                    if (!live) break;
                    lz_iters += mx;
                    lz_steps += 1;
                    for (int i = 0; i < 64; ++i) if (q[i] < R[w0 + i].lazy.size()) ++q[i];
                }
            }
        }
        std::printf("level %d order %d wave model (%.0f waves): DFS wave iterations %.1f -> %.1f lazy; leaf steps %.1f -> %.1f;"
                    " first pass nodes: lane mean %.1f, wave max %.1f, wave union %.1f, one octant %.2f\n",
                    l, order, waves, k8_iters / waves, lz_iters / waves, k8_steps / waves, lz_steps / waves,
                    p1_mean / waves, p1_max / waves, p1_union / waves, p1_uniform / waves);
    }
    for (int l = 0; l < 3; ++l) {
        const Walk& w = g_walk[l];
        std::printf("level %d inner-node visits per ray: reference %.2f  k8 passes %.2f (%.2f passes)  lazy %.2f  lazy (priority) %.2f"
                    "  lazy with restarts %.2f (%.2f passes)\n",
                    l, w.ref_visits / w.rays, w.k8_visits / w.rays, w.k8_passes / w.rays, w.lazy_visits / w.rays,
                    w.lazy_pq_visits / w.rays, w.lr_visits / w.rays, w.lr_passes / w.rays);
    }
    pr("camera", cam);
    pr("bounce1", b1);
    pr("bounce2", b2);
    return 0;
}
