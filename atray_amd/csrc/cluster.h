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
//     det could lie in [kTol, kTau) are: the det estimate -(d . n) (n = ab x ac, stored per
//     cluster as f16 integer multiples of one step) is within a bounded margin of the computed det
//     (cluster_step), which widens the screen's band.
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

// The full-test operands of slot k, one 48-B record {a.xyz, ab.x}{ab.yz, ac.xy}{ac.z, bits(leaf
// rank), bits(face), 0}: one cache line (at most two) per test. (Round 3's three SoA streams
// touched three lines per test; incoherent bounce rays miss in L2 on most of them)
__device__ __forceinline__ void load_prim(const DModel& m, uint32_t k, float4_t& a0, float4_t& a1, float4_t& a2) {
    a0 = m.prim[3 * size_t(k)];
    a1 = m.prim[3 * size_t(k) + 1];
    a2 = m.prim[3 * size_t(k) + 2];
}

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

// Which scan flavours load the first screen normals with the box test (cluster_cands EARLY): bit 0
// primary-only rays, bit 1 camera rays of the path engine, bit 2 bounce rays (experiment builds
// set others; 0 = every flavour loads them after the box test passes). Not the camera rays: their
// 6-wave kernel then spills 20 dwords instead of 5 and writes 4 GB more per c4 frame, for no time
// measured (c4 3,824-3,826 Mrays/s without, 3,828-3,834 with)
#ifndef ATR_EARLY_NRM
#define ATR_EARLY_NRM 5
#endif

// Ray-side constants of the cluster screen, once per ray (f16 direction, its L1 norm).
struct ScreenRay {
    float ax, ay, az, sd;
    h2_t dxy, dz_lo, dz_hi;
};
__device__ __forceinline__ ScreenRay screen_ray(const Ray& r) {
    ScreenRay s;
    s.ax = fabsf(r.inv.x); s.ay = fabsf(r.inv.y); s.az = fabsf(r.inv.z);
    s.sd = fabsf(r.d.x) + fabsf(r.d.y) + fabsf(r.d.z);
    s.dxy = h2_t{(_Float16)r.d.x, (_Float16)r.d.y};
    const _Float16 hz = (_Float16)r.d.z;
    s.dz_lo = h2_t{hz, (_Float16)0.0f};
    s.dz_hi = h2_t{(_Float16)0.0f, hz};
    return s;
}

// Cluster record lo = {lo.xyz, P | (n - 1)}, hi = {hi.xyz, q}: the two rounding-padded box
// tests. False: no primitive inside can be accepted with t <= best. Else the det band
// [dlo, dhi) of the primitives that still need the full test.
__device__ __forceinline__ bool cluster_pads(const Ray& r, const ScreenRay& sr, float4_t lo, float4_t hi, float best,
                                             float& dlo, float& dhi) {
    const float ex = hi.x - lo.x, ey = hi.y - lo.y, ez = hi.z - lo.z;
    const float fx = fmaxf(fabsf(lo.x - r.o.x), fabsf(hi.x - r.o.x));
    const float fy = fmaxf(fabsf(lo.y - r.o.y), fabsf(hi.y - r.o.y));
    const float fz = fmaxf(fabsf(lo.z - r.o.z), fabsf(hi.z - r.o.z));
    // W >= |o - a| + |edge| for every primitive inside (far corner; L1 extent >= diagonal). The
    // hardware square root (v_sqrt_f32, within 1 ulp) instead of the correctly rounded expansion
    // (~15 VALU: denormal scaling, two FMA corrections): W only has to bound the distance from
    // above, the 1 + 2^-21 factor covers 8 ulp, and the 2^-63 term the flushed denormal case
    const float W = (__builtin_amdgcn_sqrtf(fx * fx + fy * fy + fz * fz) + 1.0842022e-19f) * 1.0000005f + (ex + ey + ez);
    const float P = lo.w;  // >= |ab||ac| of every primitive inside
    const float gl = W * (P * (kPadRel / (0.9f * kTol)) + kPadAbs);
    const float gt = W * (P * (kPadRel / (0.9f * kTau)) + kPadAbs);
    // slab entry/exit of the unpadded box per axis, then widened by g |inv| per axis
    const float x0 = (lo.x - r.o.x) * r.inv.x, x1 = (hi.x - r.o.x) * r.inv.x;
    const float y0 = (lo.y - r.o.y) * r.inv.y, y1 = (hi.y - r.o.y) * r.inv.y;
    const float z0 = (lo.z - r.o.z) * r.inv.z, z1 = (hi.z - r.o.z) * r.inv.z;
    const float nx = fminf(x0, x1), fx1 = fmaxf(x0, x1), ny = fminf(y0, y1), fy1 = fmaxf(y0, y1),
                nz = fminf(z0, z1), fz1 = fmaxf(z0, z1);
    float tn = fmaxf(fmaxf(nx - gl * sr.ax, ny - gl * sr.ay), nz - gl * sr.az);
    float tf = fminf(fminf(fx1 + gl * sr.ax, fy1 + gl * sr.ay), fz1 + gl * sr.az);
    if (tn > tf || tf < 0.f || tn > best) return false;
    tn = fmaxf(fmaxf(nx - gt * sr.ax, ny - gt * sr.ay), nz - gt * sr.az);
    tf = fminf(fminf(fx1 + gt * sr.ax, fy1 + gt * sr.ay), fz1 + gt * sr.az);
    const bool tight = !(tn > tf || tf < 0.f || tn > best);
    // screen: det estimate -q (d . p) with the cluster's quantized normals n ~ q p (p integers
    // of at most 511, f16, 96 B per cluster) and d rounded to f16, two f16 dot products per
    // primitive. |n - q p| <= q/2 per component, d's f16 rounding <= 2^-11 |d_a| + 2^-25, the
    // f32 accumulation a few eps: the estimate is within
    //   (|d.x| + |d.y| + |d.z|) q (0.51 + 511 (2^-11 + 8 eps)) + 16 eps 511 q + 2^-20 q
    // of -(d . n), which is within 16 eps |ab||ac| of the computed det; the band is widened by it.
    const float q = hi.w;
    const float mq = sr.sd * (q * (0.51f + 511.0f * (4.8828125e-4f + 8.0f * kEps))) +
                     q * (16.0f * kEps * 511.0f + 9.5367432e-7f) + 16.0f * kEps * P;
    dlo = kTol - mq;
    dhi = tight ? __builtin_inff() : kTau + mq;
    return true;
}

// Screen of 8 primitives g .. g + 7 of n: words a0, a1 hold (nx, ny) of slots g .. g + 7 as f16,
// z the nz of slots g .. g + 7 (two per word). Bit j: slot g + j needs the full test.
// Bit j set iff the f16 dot D_j of slot g + j lies in (blo, ahi]: the det band mapped back through
// the cluster's step by the caller (cluster_cands). (The slots past n are masked off once per
// cluster by the caller, not per primitive.)
#ifndef ATR_SCREEN_TWO_CMP
// The band as one comparison: |D - mid| <= half. mid enters as the z dot's accumulator, so each
// primitive costs two dots and one compare (|.| is an operand modifier). Every dot D lies within
// +-3 x 511 x 1.0005 < 1600 (f16 direction, integer normals of at most 511), so the band is first
// clipped to [-1600, 1600] -- the tight band (blo = -inf) and bands beyond every D keep exactly
// the D they kept -- which also bounds mid and half. half covers the closed band plus the
// rounding of mid and of the accumulation with mid in it (<= 2^-22 (1600 + |mid|)): the screen
// only grows. An empty band stays empty (half < 0); NaN ends open the band.
__device__ __forceinline__ void screen_band(float blo, float ahi, float& mid, float& half) {
    const float lo = fmaxf(blo, -1600.0f), hi = fminf(ahi, 1600.0f);
    mid = 0.5f * (lo + hi);
    half = 0.5f * (hi - lo) * 1.000001f + (fabsf(mid) + 2048.0f) * 4.7683716e-7f;  // 2^-21
}
__device__ __forceinline__ uint32_t screen8(const ScreenRay& sr, float nmid, float half, uint4_t a0, uint4_t a1,
                                            uint4_t z) {
    const uint32_t xy[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const uint32_t zz[4] = {z.x, z.y, z.z, z.w};
    uint32_t gc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const h2_t pxy = __builtin_bit_cast(h2_t, xy[j]), pz = __builtin_bit_cast(h2_t, zz[j / 2]);
        float dz;
        asm("v_dot2_f32_f16 %0, %1, %2, %3" : "=v"(dz) : "v"((j & 1) ? sr.dz_hi : sr.dz_lo), "v"(pz), "v"(nmid));
        const float e = __builtin_amdgcn_fdot2(sr.dxy, pxy, dz, false);
        if (fabsf(e) <= half) gc |= 1u << j;
    }
    return gc;
}
#else
__device__ __forceinline__ uint32_t screen8(const ScreenRay& sr, float blo, float ahi, uint4_t a0, uint4_t a1,
                                            uint4_t z) {
    const uint32_t xy[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const uint32_t zz[4] = {z.x, z.y, z.z, z.w};
    uint32_t gc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const h2_t pxy = __builtin_bit_cast(h2_t, xy[j]), pz = __builtin_bit_cast(h2_t, zz[j / 2]);
        // the z term with a zero accumulator operand (VOP3P v_dot2_f32_f16 ..., 0): the builtin
        // selects v_dot2c_f32_f16, whose accumulator is its destination, plus a v_mov of the zero
        float dz;
        asm("v_dot2_f32_f16 %0, %1, %2, 0" : "=v"(dz) : "v"((j & 1) ? sr.dz_hi : sr.dz_lo), "v"(pz));
        const float e = __builtin_amdgcn_fdot2(sr.dxy, pxy, dz, false);
        if (e > blo && e <= ahi) gc |= 1u << j;
    }
    return gc;
}
#endif

// Cluster c of a leaf: the padded box tests and the screen against the bound `best`. Returns the
// mask of the primitives (slot 16 c + bit) that still need the full test.
template <bool COUNT, bool EARLY = true>
__device__ __forceinline__ uint32_t cluster_cands(const Ray& r, const DModel& m, uint32_t c, float4_t lo, float4_t hi,
                                                  float best, Ctr& ct) {
    // the screen constants (7 values) are recomputed for every cluster from an opaque copy of the
    // ray instead of being hoisted out of the scan loops and held through the passes and rounds:
    // ~10 VALU per cluster for 7 VGPRs, what lets HYBRID run 6 waves/SIMD
    Ray rr = r;
    asm volatile("" : "+v"(rr.d.x), "+v"(rr.d.y), "+v"(rr.d.z), "+v"(rr.inv.x), "+v"(rr.inv.y), "+v"(rr.inv.z));
    const ScreenRay sr = screen_ray(rr);
    const uint4_t* nb = m.cnrm + kClusterBlock * size_t(c);
    // EARLY: the first 8 slots' screen normals are loaded together with the box test instead of
    // after it passes -- one dependent memory round trip less per cluster on the dealt rounds' chain,
    // at 12 VGPRs held through the pads (c3 +1.2%, c4 +0.7%, round 6)
    uint4_t e0, e1, ez;
    if constexpr (EARLY) {
        e0 = nb[0], e1 = nb[1], ez = nb[kMaxClusterSize / 4];
    }
    float dlo, dhi;
    if (!cluster_pads(r, sr, lo, hi, best, dlo, dhi)) return 0;
    const uint32_t n = (__float_as_uint(lo.w) & 31u) + 1u;
    if constexpr (COUNT) ct.screen += n;
    const uint32_t slots = (2u << (n - 1)) - 1u;  // [0, n), 1 <= n <= 16
    const float q = hi.w;
    if (!(q >= 1.1754944e-38f)) return slots;  // zero or subnormal step (degenerate normals): no screen
    // The band dlo <= -q D < dhi of the estimate, as a band of the dot D itself: D in
    // (-dhi / q, -dlo / q] (one reciprocal per cluster instead of a product per primitive). The
    // ends are widened by 2^-20 relative -- the hardware reciprocal (1 ulp) and the products'
    // rounding are below 2^-22 -- and by 2^-126 absolute (flushed subnormals), so every primitive
    // whose rounded product fell in the band still passes: the screen only grows.
    const float rq = __builtin_amdgcn_rcpf(q);
    const float a = -dlo * rq, b = -dhi * rq;  // b = -inf for the tight case (dhi = inf)
    const float ahi = a + fabsf(a) * 9.5367432e-7f + 1.1754944e-38f;
    const float blo = b - fabsf(b) * 9.5367432e-7f - 1.1754944e-38f;
    uint32_t cand = 0;
#ifndef ATR_SCREEN_TWO_CMP
    float mid, half;
    screen_band(blo, ahi, mid, half);
    if constexpr (EARLY) {
        cand = screen8(sr, -mid, half, e0, e1, ez);
        if (n > 8) cand |= screen8(sr, -mid, half, nb[2], nb[3], nb[kMaxClusterSize / 4 + 1]) << 8;
    } else {
        for (uint32_t g = 0; g < n; g += 8)  // eight primitives per step: (nx, ny) x 8, nz x 8
            cand |= screen8(sr, -mid, half, nb[g / 4], nb[g / 4 + 1], nb[kMaxClusterSize / 4 + g / 8]) << g;
    }
#else
    for (uint32_t g = 0; g < n; g += 8)
        cand |= screen8(sr, blo, ahi, nb[g / 4], nb[g / 4 + 1], nb[kMaxClusterSize / 4 + g / 8]) << g;
#endif
    return cand & slots;
}

}  // namespace atr
