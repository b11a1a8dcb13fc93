// cluster.h -- the clustered leaf scan: one leaf's result from a fraction of
// the reference's triangle tests, bit-identical.
//
// Each leaf's primitives are regrouped into spatial clusters of <= 16 with a bounding box, and a
// primitive is skipped only when it provably cannot be accepted with t <= the best so far:
//   * rounding (first order): an accepted hit of the culled test (computed
//     det >= kTol; u, v in range) has its true line within D_lat of the triangle and its
//     computed t within D_t of the true t, D_lat + D_t <= W (29 eps |ab||ac| / det + 6 eps),
//     W >= |o - a| + |edge|: the u, v, t numerators carry ~7.5 eps |tvec| |ac| (resp. |ab|,
//     |ab||ac|) of cancellation, det ~6.5 eps |ab||ac|. A box grown by that much (36 and
//     12 eps here, with the slab's own rounding) is entered no later than the computed t of any
//     acceptable primitive inside and left no earlier.
//   * D depends on det, which is not known per cluster: the box is grown twice, for det >= kTol
//     (loose) and det >= kTau (tight). Missing the loose box skips the cluster. Inside the
//     tight box every front-facing primitive is a candidate. In between, only primitives whose
//     det could lie in [kTol, kTau) are: the det estimate -(d . n) (n = ab x ac, one 16-B
//     load) is within 16 eps |ab||ac| of the computed det, which sets the screen's margins.
//     Back-facing primitives (det < kTol) are screened out the same way in both cases.
//   * inside the leaf the reference keeps the FIRST primitive (leaf order) with the smallest t
//     below the incoming best (strict <, kd_tree.cpp:440-456); clusters change the visiting
//     order, so equal t is resolved by the leaf rank, and a best carried in from an earlier
//     leaf never loses a tie.
#pragma once
#include "trace.h"

namespace atr {

constexpr float kTau = 3e-3f;
constexpr float kEps = 5.9604645e-8f;  // 2^-24
constexpr float kPadRel = 36.0f * kEps, kPadAbs = 12.0f * kEps;

// Best hit of one leaf scan in progress: t, primitive slot, barycentrics, leaf rank of the hit
// taken in THIS leaf (-1: the best was carried in), whether this leaf improved it.
struct LeafHit {
    float t;
    uint32_t slot;
    float u, v;
    int32_t rank;
    bool improved;
};

template <bool COUNT>
__device__ __forceinline__ void cluster_tri(const Ray& r, const DModel& m, uint32_t k, float acz, LeafHit& h,
                                            Ctr& ct) {
    if constexpr (COUNT) ct.tri += 1;
    const float4_t q0 = m.c0[k], q1 = m.c1[k];
    float u = 0.f, v = 0.f;
    const float dist = tri_hit(r, mk(q0.x, q0.y, q0.z), mk(q0.w, q1.x, q1.y), mk(q1.z, q1.w, acz), u, v);
    if (dist <= h.t && dist > kTol) {
        const int32_t rk = int32_t(m.crank[k]);
        if (dist < h.t || (h.rank >= 0 && rk < h.rank)) {
            h.t = dist;
            h.slot = k;
            h.u = u;
            h.v = v;
            h.rank = rk;
            h.improved = true;
        }
    }
}

// One cluster (record lo = {lo.xyz, P | (n - 1)}, hi = {hi.xyz, first slot}) of the current
// leaf: padded box tests, then the screen and the full tests of its primitives.
template <bool COUNT>
__device__ __forceinline__ void cluster_step(const Ray& r, const DModel& m, float4_t lo, float4_t hi, LeafHit& h,
                                             Ctr& ct) {
    const float ax = fabsf(r.inv.x), ay = fabsf(r.inv.y), az = fabsf(r.inv.z);
    const float ex = hi.x - lo.x, ey = hi.y - lo.y, ez = hi.z - lo.z;
    const float fx = fmaxf(fabsf(lo.x - r.o.x), fabsf(hi.x - r.o.x));
    const float fy = fmaxf(fabsf(lo.y - r.o.y), fabsf(hi.y - r.o.y));
    const float fz = fmaxf(fabsf(lo.z - r.o.z), fabsf(hi.z - r.o.z));
    // W >= |o - a| + |edge| for every primitive inside (far corner; L1 extent >= diagonal)
    const float W = __builtin_sqrtf(fx * fx + fy * fy + fz * fz) * 1.0000005f + (ex + ey + ez);
    const float P = lo.w;  // >= |ab||ac| of every primitive inside
    const float gl = W * (P * (kPadRel / (0.9f * kTol)) + kPadAbs);
    const float gt = W * (P * (kPadRel / (0.9f * kTau)) + kPadAbs);
    // slab entry/exit of the unpadded box per axis, then widened by g |inv| per axis
    const float x0 = (lo.x - r.o.x) * r.inv.x, x1 = (hi.x - r.o.x) * r.inv.x;
    const float y0 = (lo.y - r.o.y) * r.inv.y, y1 = (hi.y - r.o.y) * r.inv.y;
    const float z0 = (lo.z - r.o.z) * r.inv.z, z1 = (hi.z - r.o.z) * r.inv.z;
    const float nx = fminf(x0, x1), fx1 = fmaxf(x0, x1), ny = fminf(y0, y1), fy1 = fmaxf(y0, y1),
                nz = fminf(z0, z1), fz1 = fmaxf(z0, z1);
    float tn = fmaxf(fmaxf(nx - gl * ax, ny - gl * ay), nz - gl * az);
    float tf = fminf(fminf(fx1 + gl * ax, fy1 + gl * ay), fz1 + gl * az);
    if (tn > tf || tf < 0.f || tn > h.t) return;
    tn = fmaxf(fmaxf(nx - gt * ax, ny - gt * ay), nz - gt * az);
    tf = fminf(fminf(fx1 + gt * ax, fy1 + gt * ay), fz1 + gt * az);
    const bool tight = !(tn > tf || tf < 0.f || tn > h.t);
#ifdef ATR_EXP_SKIP_LOOSE
    if (!tight) return;  // EXPERIMENT ONLY (not exact): cost of the loose-only screens
#endif
    const float mg = 16.0f * kEps * P;
    const float dlo = kTol - mg, dhi = tight ? __builtin_inff() : kTau + mg;
    const uint32_t first = __float_as_uint(hi.w);
    const uint32_t n = (__float_as_uint(lo.w) & 31u) + 1u, last = first + n - 1;
    if constexpr (COUNT) ct.screen += n;
    // screen four primitives per step (their normal loads in flight together)
    for (uint32_t k = first; k <= last; k += 4) {
        const uint32_t k1 = k + 1 <= last ? k + 1 : last, k2 = k + 2 <= last ? k + 2 : last,
                       k3 = k + 3 <= last ? k + 3 : last;
        const float4_t n0 = m.c2[k], n1 = m.c2[k1], n2 = m.c2[k2], n3 = m.c2[k3];
        const float d0 = -(r.d.x * n0.x + r.d.y * n0.y + r.d.z * n0.z);
        const float d1 = -(r.d.x * n1.x + r.d.y * n1.y + r.d.z * n1.z);
        const float d2 = -(r.d.x * n2.x + r.d.y * n2.y + r.d.z * n2.z);
        const float d3 = -(r.d.x * n3.x + r.d.y * n3.y + r.d.z * n3.z);
        if (d0 >= dlo && d0 < dhi) cluster_tri<COUNT>(r, m, k, n0.w, h, ct);
        if (k + 1 <= last && d1 >= dlo && d1 < dhi) cluster_tri<COUNT>(r, m, k + 1, n1.w, h, ct);
        if (k + 2 <= last && d2 >= dlo && d2 < dhi) cluster_tri<COUNT>(r, m, k + 2, n2.w, h, ct);
        if (k + 3 <= last && d3 >= dlo && d3 < dhi) cluster_tri<COUNT>(r, m, k + 3, n3.w, h, ct);
    }
}

}  // namespace atr
