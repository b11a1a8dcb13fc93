// super_sim.cpp -- would a second level of cluster boxes (groups of G consecutive clusters of a
// leaf) let a primary-ray wave skip clusters none of its rays needs? (analysis tool, not product)
// Derived from cluster_sim.cpp: same scene, same rounding-padded loose box as the kernel.
//
// Builds the Dragon surrogate's octree and leaf clusters with the product's host code, traces
// the primary rays of a 1920x1080 frame (every `step`-th pixel) on the CPU with the reference
// leaf order (kd_tree.cpp:337-465) and counts, per ray, the work of several leaf-scan
// strategies: cluster records read, primitives screened, full triangle tests. The strategies
// differ only in which clusters they read and in which order, never in the result.
//
// g++ -O2 -std=c++17 -ffp-contract=off -I atray_amd/csrc tools/cluster_sim.cpp
//     atray_amd/csrc/host_scene.cpp -o build/cluster_sim && build/cluster_sim OBJ [step]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <map>
#include <vector>

#include "engine.h"
#include "host_scene.h"

using namespace atr;

static float tri_hit(V3 o, V3 d, V3 a, V3 ab, V3 ac) {
    const V3 pvec = cross(d, ac);
    const float det = dot(ab, pvec);
    if (det < kTol) return 0;
    const float det_inv = 1 / det;
    const V3 tvec = sub(o, a);
    const float u = dot(tvec, pvec) * det_inv;
    if (u < 0 || u > 1) return 0;
    const V3 qvec = cross(tvec, ab);
    const float v = dot(d, qvec) * det_inv;
    if (v < 0 || u + v > 1) return 0;
    return dot(qvec, ac) * det_inv;
}

static float box_entry(V3 o, V3 inv, const float* b) {
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
static bool box_check(V3 o, V3 inv, const float* b) {
    const int s0 = inv.x < 0, s1 = inv.y < 0, s2 = inv.z < 0;
    float tmin = ((s0 ? b[3] : b[0]) - o.x) * inv.x, tmax = ((s0 ? b[0] : b[3]) - o.x) * inv.x;
    const float tymin = ((s1 ? b[4] : b[1]) - o.y) * inv.y, tymax = ((s1 ? b[1] : b[4]) - o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = ((s2 ? b[5] : b[2]) - o.z) * inv.z, tzmax = ((s2 ? b[2] : b[5]) - o.z) * inv.z;
    return !((tmin > tzmax) || (tzmin > tmax));
}


int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: super_sim OBJ [G]\n"); return 2; }
    const int G = argc > 2 ? std::atoi(argv[2]) : 4;
    std::ifstream f(argv[1], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    HostMesh M;
    if (parse_obj_text(text.data(), text.size(), M)) return 1;
    float box[6];
    mesh_aabb(M, box);
    mesh_translate(M, box, mk(0.f, -15.f, -38.f));
    HostTree T;
    if (octree_build(M, 300, T)) return 1;
    LeafClusters C;
    if (leaf_clusters(T, 16, C)) return 1;
    atr_camera cm;
    camera_set(cm, mk(0.1f, 2.f, 0.f), mk(-0.1f, -0.5f, -1.f), 1920, 1080, 0, 1, 1, 1.f);
    const V3 eye = from(cm.eye), fc = from(cm.frame_center), cx = from(cm.camera_x), cy = from(cm.camera_y);
    const float eps = 5.9604645e-8f;
    auto loose_hit = [&](const float* r, V3 o, V3 inv, float best) {
        const float ex = r[4] - r[0], ey = r[5] - r[1], ez = r[6] - r[2];
        const float fx = std::max(std::fabs(r[0] - o.x), std::fabs(r[4] - o.x));
        const float fy = std::max(std::fabs(r[1] - o.y), std::fabs(r[5] - o.y));
        const float fz = std::max(std::fabs(r[2] - o.z), std::fabs(r[6] - o.z));
        const float W = std::sqrt(fx * fx + fy * fy + fz * fz) * 1.0000005f + (ex + ey + ez);
        const float g = W * (r[3] * (36 * eps / (0.9f * kTol)) + 12 * eps);
        float bb[6];
        for (int q = 0; q < 3; ++q) { bb[q] = r[q] - g; bb[3 + q] = r[4 + q] + g; }
        return box_check(o, inv, bb) && !(box_entry(o, inv, bb) > best);
    };
    double iters_now = 0, iters_super = 0, leaf_steps = 0, union_clusters = 0;
    std::vector<std::pair<int, int>> cell_steps;  // per cell: wave leaf steps now / with tail speculation
    std::vector<std::pair<float, int>> leaves;
    std::vector<int32_t> stack;
    const int cw = (cm.width + 7) / 8, chh = (cm.height + 7) / 8;
    for (int cyi = 0; cyi < chh; ++cyi)
        for (int cxi = 0; cxi < cw; ++cxi) {
            // per leaf scanned by any ray of the cell: which clusters some ray passes
            std::map<int, std::vector<char>> used;
            std::vector<int> nleaves;  // per active ray: leaves scanned (the query's leaf steps)
            for (int ly = 0; ly < 8; ++ly)
                for (int lx = 0; lx < 8; ++lx) {
                    const int x = cxi * 8 + lx, y = cyi * 8 + ly;
                    if (x >= cm.width || y >= cm.height) continue;
                    const float film_y = -1.0f + 2.0f * (float(y) / float(cm.height));
                    const float film_x = ((-1.0f + 2.0f * (float(x) / float(cm.width))) * cm.h_fov) * cm.aspect_ratio;
                    const V3 d = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));
                    const V3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
                    if (!box_check(eye, inv, &T.bounds[0])) continue;
                    leaves.clear();
                    stack.assign(1, 0);
                    while (!stack.empty()) {
                        const int32_t cur = stack.back();
                        stack.pop_back();
                        const int32_t ch = T.children[size_t(cur)];
                        int hit = 0;
                        for (int i = 0; i < 8 && hit <= 4; ++i) {
                            const int32_t c = ch + i;
                            if (T.children[size_t(c)]) {
                                if (box_check(eye, inv, &T.bounds[6 * size_t(c)])) { ++hit; stack.push_back(c); }
                            } else {
                                const float dis = box_entry(eye, inv, &T.bounds[6 * size_t(c)]);
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
                    int scanned = 0;
                    for (auto& lf : leaves) {
                        ++scanned;
                        const uint32_t c0 = C.range[2 * size_t(lf.second)], nc = C.range[2 * size_t(lf.second) + 1];
                        auto& u = used[lf.second];
                        u.resize(nc, 0);
                        bool improved = false;
                        for (uint32_t c = c0; c < c0 + nc; ++c) {
                            const float* r = &C.rec[8 * size_t(c)];
                            if (!loose_hit(r, eye, inv, best)) continue;
                            u[c - c0] = 1;
                            uint32_t pw, fs;
                            std::memcpy(&pw, &C.rec[8 * c + 3], 4);
                            std::memcpy(&fs, &C.rec[8 * c + 7], 4);
                            for (uint32_t k = fs; k < fs + (pw & 31u) + 1u; ++k) {
                                const float* v = &T.prim_vertices[9 * size_t(C.order[k])];
                                const V3 a = mk(v[0], v[1], v[2]);
                                const float t = tri_hit(eye, d, a, sub(mk(v[3], v[4], v[5]), a), sub(mk(v[6], v[7], v[8]), a));
                                if (t > kTol && t < best) { best = t; improved = true; }
                            }
                        }
                        if (improved) break;
                    }
                    nleaves.push_back(scanned);
                }
            // wave step model: every live ray scans one leaf per step (now), or, once at most T rays
            // are live, up to min(8, 64 / live) leaves each (tail speculation); a pass every 8 leaves
            if (!nleaves.empty()) {
                auto steps = [&](bool tail) {
                    std::vector<int> left = nleaves, pos(nleaves.size(), 0);
                    int st = 0;
                    for (;;) {
                        int live = 0;
                        for (int x : left) live += x > 0;
                        if (!live) break;
                        ++st;
                        const int S = tail && live <= 8 ? std::min(8, 64 / live) : 1;
                        for (size_t i = 0; i < left.size(); ++i) {
                            if (left[i] <= 0) continue;
                            const int take = std::min(S, 8 - pos[i] % 8);  // not past the pass's buffer
                            left[i] -= take;
                            pos[i] += take;
                        }
                    }
                    return st;
                };
                const int a = steps(false), b = steps(true);
                cell_steps.push_back({a, b});
            }
            for (auto& kv : used) {
                const int nc = int(kv.second.size());
                leaf_steps += 1;
                iters_now += nc;
                int ns = 0, inner = 0, uc = 0;
                for (int g = 0; g < nc; g += G) {
                    ++ns;
                    bool any = false;
                    for (int k = g; k < std::min(nc, g + G); ++k) { any |= kv.second[size_t(k)] != 0; uc += kv.second[size_t(k)]; }
                    if (any) inner += std::min(nc, g + G) - g;
                }
                iters_super += ns + inner;
                union_clusters += uc;
            }
        }
    std::sort(cell_steps.begin(), cell_steps.end());
    const size_t nc = cell_steps.size();
    double sa = 0, sb = 0;
    for (auto& p : cell_steps) { sa += p.first; sb += p.second; }
    std::printf("cells %zu: leaf steps per cell %.2f now, %.2f with tail speculation; slowest 1%%:", nc, sa / nc, sb / nc);
    double ta = 0, tb = 0;
    for (size_t k = nc - nc / 100; k < nc; ++k) { ta += cell_steps[k].first; tb += cell_steps[k].second; }
    std::printf(" %.1f -> %.1f; max %d -> %d\n", ta / (nc / 100), tb / (nc / 100), cell_steps.back().first, cell_steps.back().second);
    std::printf("G=%d  leaf steps (cell, leaf) %.0f: cluster iterations now %.0f (%.2f per step), with superclusters %.0f (%.2f per step),"
                " clusters some ray passes %.2f per step\n", G, leaf_steps, iters_now, iters_now / leaf_steps, iters_super,
                iters_super / leaf_steps, union_clusters / leaf_steps);
    return 0;
}
