// shade.h -- the tail of get_intersection_data (renderer.cpp:86-160): spheres, planes and the
// hit record (type, normal, material) once the models' closest triangle is known.
#pragma once
#include "trace.h"

namespace atr {

enum { T_NONE = 0, T_TRI = 1, T_SPHERE = 2, T_PLANE = 3, T_SKY = 4 };

struct Isect {
    int type;
    float t;
    V3 normal;
    int32_t material;
    uint32_t face;
};

// best/face/fu/fv/nm: the closest model hit so far (nm = -1: none).
__device__ __forceinline__ void scene_finish(const DScene* __restrict__ S, V3 o, V3 d, float best, uint32_t face,
                                             float fu, float fv, int32_t nm, Isect& id) {
    int32_t ns = -1, np = -1;
    const int32_t nspheres = __builtin_amdgcn_readfirstlane(S->nspheres), nplanes = __builtin_amdgcn_readfirstlane(S->nplanes);
    for (int32_t i = 0; i < nspheres; ++i) {  // sphere.h:12-39
        const DSphere& sp = uniform_global(S->spheres)[i];
        const V3 pc = sub(o, mk(sp.cx, sp.cy, sp.cz));
        const float pcs = len2(pc);
        const float b = 2 * (dot(d, pc));
        const float bs = b * b;
        const float c = pcs - sp.r * sp.r;
        const float dmt = bs - (4 * c);
        float t = 0;
        if (!(dmt < 0)) {
            const float ta = (-b + sqrtf(dmt)) * 0.5f;
            const float tb = (-b - sqrtf(dmt)) * 0.5f;
            if (ta <= 0 && tb <= 0) t = 0;
            else if (tb > 0) t = tb;
            else t = ta;
        }
        if (t > kTol && t < best) { best = t; ns = i; }
    }
    for (int32_t i = 0; i < nplanes; ++i) {  // plane.h:12-22
        const DPlane& pl = uniform_global(S->planes)[i];
        const V3 n = mk(pl.nx, pl.ny, pl.nz);
        const float denom = dot(n, d);
        float t = 0;
        if (!(denom > -kTol && denom < kTol)) t = (pl.d - dot(o, n)) / denom;
        if (t > kTol && t < best) { np = i; best = t; }
    }
    id.t = best;
    id.face = 0xFFFFFFFFu;
    if (np >= 0) {
        const DPlane& pl = as_global(S->planes)[np];
        id.type = T_PLANE;
        id.normal = mk(pl.nx, pl.ny, pl.nz);
        id.material = pl.material;
    } else if (ns >= 0) {
        const DSphere& sp = as_global(S->spheres)[ns];
        id.type = T_SPHERE;
        id.normal = sub(add(o, scale(d, best)), mk(sp.cx, sp.cy, sp.cz));  // Ray::at (ray.h:10-13)
        id.material = sp.material;
    } else if (nm >= 0) {
        const DModel& m = S->models[nm];
        id.type = T_TRI;
        id.face = face;
        const float* sh = as_global(m.shade) + 9 * size_t(face);
        if (m.smooth) {  // interpolated vertex normals (:129-138)
            const V3 na = mk(sh[0], sh[1], sh[2]), nb = mk(sh[3], sh[4], sh[5]), nc = mk(sh[6], sh[7], sh[8]);
            id.normal = add(add(scale(na, (1 - fu - fv)), scale(nb, fu)), scale(nc, fv));
        } else {  // flat (:140-146)
            const V3 v0 = mk(sh[0], sh[1], sh[2]), v1 = mk(sh[3], sh[4], sh[5]), v2 = mk(sh[6], sh[7], sh[8]);
            id.normal = cross(sub(v0, v1), sub(v0, v2));
        }
        id.material = m.material;
    } else {
        id.type = T_SKY;
        id.material = 0;
    }
    if (id.type != T_SKY) id.normal = unit(id.normal);  // :157
}

}  // namespace atr
