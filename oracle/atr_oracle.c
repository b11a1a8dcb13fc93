/*
 * atr_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker; see atr_oracle.h header).
 *
 * Plain-C restatement of AdhavanT/ATRay's render path. Every function cites the
 * reference file:line it follows (paths relative to /root/reference/Source).
 * f32 expressions keep the reference's evaluation order (left-to-right vec3f ops,
 * PL/PL_math.h:106-123,416-422); build with -ffp-contract=off and no -ffast-math.
 */
#define _GNU_SOURCE
#include "atr_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#define OM_MAX_FLOAT 3.402823466e+38F      /* PL/PL_base_defs.h:72 */
#define OM_INV_UINT32_MAX 2.328306437e-10F /* PL/PL_base_defs.h:75 */
#define OM_TOL 0.0001f                     /* engine/renderer/ray.h:5 */

/* ------------------------------------------------------------------ vec3f (PL_math.h:82-129) */
static inline ov3 v3(float x, float y, float z) { ov3 r = {x, y, z}; return r; }
static inline ov3 vadd(ov3 a, ov3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline ov3 vsub(ov3 a, ov3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline ov3 vneg(ov3 a) { return v3(-a.x, -a.y, -a.z); }
static inline ov3 vmul(ov3 a, float n) { return v3(a.x * n, a.y * n, a.z * n); }
static inline ov3 vdiv(ov3 a, float n) { return v3(a.x / n, a.y / n, a.z / n); }
static inline float vdot(ov3 p, ov3 n) { return (p.x * n.x) + (p.y * n.y) + (p.z * n.z); } /* :416 */
static inline ov3 vhad(ov3 a, ov3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }         /* :419 */
static inline ov3 vcross(ov3 a, ov3 b) {                                                      /* :422 */
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float vmag2(ov3 v) { return (v.x * v.x) + (v.y * v.y) + (v.z * v.z); } /* :377-380 */
static inline float vmag(ov3 v) { return sqrtf(vmag2(v)); }                           /* :382-385 */
/* normalize (PL_math.h:387-392): v * invsqrt(mag2). SVML stand-in = 1/sqrtf (declared). */
static inline ov3 vnormalize(ov3 v) { float inv = 1.0f / sqrtf(vmag2(v)); return vmul(v, inv); }
static inline ov3 vlerp(ov3 s, ov3 t, float k) { return vadd(vmul(vsub(t, s), k), s); } /* :439-442 */
static inline float fmaxr(float a, float b) { return a > b ? a : b; } /* PL_math.h:335-338 */
static inline float fminr(float a, float b) { return a > b ? b : a; } /* PL_math.h:329-333 */

/* ------------------------------------------------------------------ parser (utilities/parser.h) */
static const uint64_t INT_POWER_10[20] = {
    1ULL, 10ULL, 100ULL, 1000ULL, 10000ULL, 100000ULL, 1000000ULL, 10000000ULL, 100000000ULL,
    1000000000ULL, 10000000000ULL, 100000000000ULL, 1000000000000ULL, 10000000000000ULL,
    100000000000000ULL, 1000000000000000ULL, 10000000000000000ULL, 100000000000000000ULL,
    1000000000000000000ULL, 10000000000000000000ULL}; /* PL_math.h:6-28 */
static const double F64_POWER_10[48] = {
    1.0e-28, 1.0e-27, 1.0e-26, 1.0e-25, 1.0e-24, 1.0e-23, 1.0e-22, 1.0e-21, 1.0e-20,
    1.0e-19, 1.0e-18, 1.0e-17, 1.0e-16, 1.0e-15, 1.0e-14, 1.0e-13, 1.0e-12, 1.0e-11,
    1.0e-10, 1.0e-9,  1.0e-8,  1.0e-7,  1.0e-6,  1.0e-5,  1.0e-4,  1.0e-3,  1.0e-2,
    1.0e-1,  1.0e0,   1.0e1,   1.0e2,   1.0e3,   1.0e4,   1.0e5,   1.0e6,   1.0e7,
    1.0e8,   1.0e9,   1.0e10,  1.0e11,  1.0e12,  1.0e13,  1.0e14,  1.0e15,  1.0e16,
    1.0e17,  1.0e18,  1.0e19}; /* PL_math.h:33-41, offset 28 = 1.0e0 (:30) */

static inline int is_ws(char c) { return c == ' ' || c == '\t' || c == '\r'; } /* parser.h:4-7 */
static inline int is_dig(char c) { return c >= '0' && c <= '9'; }
static inline const char* skip_ws(const char* p) { while (is_ws(*p)) p++; return p; }

/* parse_int (parser.h:38-65) */
static const char* parse_i32(const char* p, int32_t* val) {
    p = skip_ws(p);
    int32_t sign = 1;
    if (*p == '+') { p++; } else if (*p == '-') { sign = -1; p++; }
    uint32_t v = 0; /* int32 wrap emulated in u32 (reference overflow is UB) */
    while (is_dig(*p)) { v = v * 10u + (uint32_t)(*p - '0'); p++; }
    *val = (int32_t)(v * (uint32_t)sign);
    return p;
}

/* parse_f64 (parser.h:113-191): u64 mantissa, f64 multiply by the power-of-ten table. */
static const char* parse_f64(const char* p, double* val) {
    double sign = 1.0;
    p = skip_ws(p);
    if (*p == '+') { p++; } else if (*p == '-') { sign = -1.0; p++; }
    uint64_t front = 0;
    while (is_dig(*p)) { front = front * 10u + (uint64_t)(*p - '0'); p++; }
    if (*p == '.') p++;
    uint64_t frac = 0; int32_t frac_prec = 0;
    while (is_dig(*p)) { frac_prec++; frac = frac * 10u + (uint64_t)(*p - '0'); p++; }
    /* reference indexes INT_POWER_10[frac_prec] unchecked (UB past 19 digits); clamp here */
    front *= INT_POWER_10[frac_prec > 19 ? 19 : frac_prec];
    front += frac;
    int32_t exponent = 0;
    if (*p == 'e' || *p == 'E') {
        p++;
        int32_t es = 1;
        if (*p == '+') { p++; } else if (*p == '-') { es = -1; p++; }
        while (is_dig(*p)) { exponent = 10 * exponent + (*p - '0'); p++; }
        exponent *= es;
    }
    exponent -= frac_prec;
    double v = (double)front;
    v = v * sign;
    exponent = (exponent >= -28 && exponent <= 19) ? exponent : 0;
    v *= F64_POWER_10[exponent + 28];
    *val = v;
    return p;
}

/* parse_vec3f (parser.h:194-205) */
static const char* parse_v3(const char* p, ov3* out) {
    double d;
    p = parse_f64(p, &d); out->x = (float)d;
    p = parse_f64(p, &d); out->y = (float)d;
    p = parse_f64(p, &d); out->z = (float)d;
    return p;
}

typedef struct { void* p; size_t n, cap, esz; } dyn;
static void dyn_push(dyn* d, const void* e) {
    if (d->n == d->cap) { d->cap = d->cap ? d->cap * 2 : 256; d->p = realloc(d->p, d->cap * d->esz); }
    memcpy((char*)d->p + d->n * d->esz, e, d->esz); d->n++;
}

/* one face index group: v, v/vt, v//vn, v/vt/vn (OBJ_loader.cpp:54-110) */
static const char* parse_face_vertex(const char* p, int32_t* v, int32_t* vt, int32_t* vn) {
    p = parse_i32(p, v);
    if (*p == '/') {
        p++;
        if (*p == '/') { p++; p = parse_i32(p, vn); }
        else { p = parse_i32(p, vt); if (*p == '/') { p++; p = parse_i32(p, vn); } }
    }
    return p;
}

/* load_model_data (OBJ_loader.cpp:278-360): the threaded newline-aligned chunking joins
   in order, so it equals one sequential pass over the text + an appended '\n' (:330-331).
   parse_chunks (:32-176), prep_model_data (:229-267). */
int om_parse_obj(const char* buf, size_t len, om_mesh* out) {
    char* text = (char*)malloc(len + 2);
    memcpy(text, buf, len);
    text[len] = '\n'; text[len + 1] = 0;
    const char* cur = text;
    const char* end = text + len + 1;
    dyn V = {0, 0, 0, sizeof(ov3)}, N = {0, 0, 0, sizeof(ov3)}, T = {0, 0, 0, sizeof(ov3)};
    dyn FV = {0, 0, 0, 3 * sizeof(int32_t)}, FT = {0, 0, 0, 3 * sizeof(int32_t)}, FN = {0, 0, 0, 3 * sizeof(int32_t)};
    while (cur < end) {
        if (*cur == 'v') {
            cur++;
            ov3 p3;
            if (*cur == ' ') { cur = parse_v3(cur, &p3); dyn_push(&V, &p3); }
            else if (*cur == 't') { cur++; cur = parse_v3(cur, &p3); dyn_push(&T, &p3); }
            else if (*cur == 'n') { cur++; cur = parse_v3(cur, &p3); dyn_push(&N, &p3); }
        } else if (*cur == 'f') {
            cur++;
            int32_t v[3] = {0, 0, 0}, t[3] = {0, 0, 0}, n[3] = {0, 0, 0};
            for (int k = 0; k < 3; k++) cur = parse_face_vertex(cur, &v[k], &t[k], &n[k]);
            dyn_push(&FT, t); dyn_push(&FN, n); dyn_push(&FV, v);
        }
        /* 'u'semtl, '#', '\n', default: nothing (:129-150) */
        while (*cur != '\n') cur++; /* skip_to_new_line */
        cur++;
    }
    free(text);
    memset(out, 0, sizeof(*out));
    out->vertices = (ov3*)V.p; out->nv = (uint32_t)V.n;
    out->normals = (ov3*)N.p; out->nn = (uint32_t)N.n;
    out->texcoords = (ov3*)T.p; out->nt = (uint32_t)T.n;
    out->face_v = (int32_t*)FV.p; out->face_tc = (int32_t*)FT.p; out->face_n = (int32_t*)FN.p;
    out->nf = (uint32_t)FV.n;
    /* prep_model_data: negative -> relative to end (+1), then remove the +1 offset */
    for (uint32_t i = 0; i < out->nf; i++) {
        for (int j = 0; j < 3; j++) {
            int32_t* tc = &out->face_tc[3 * i + j]; int32_t* nn = &out->face_n[3 * i + j];
            int32_t* vv = &out->face_v[3 * i + j];
            if (*tc < 0) *tc = (int32_t)out->nt + *tc + 1;
            if (*nn < 0) *nn = (int32_t)out->nn + *nn + 1;
            if (*vv < 0) *vv = (int32_t)out->nv + *vv + 1;
        }
        for (int j = 0; j < 3; j++) { out->face_tc[3 * i + j]--; out->face_v[3 * i + j]--; out->face_n[3 * i + j]--; }
    }
    return 0;
}

int om_load_obj(const char* path, om_mesh* out) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    char* buf = (char*)malloc((size_t)sz + 1);
    size_t rd = fread(buf, 1, (size_t)sz, f);
    fclose(f);
    if (rd != (size_t)sz) { free(buf); return -2; }
    int r = om_parse_obj(buf, (size_t)sz, out);
    free(buf);
    return r;
}

void om_free_mesh(om_mesh* m) {
    free(m->vertices); free(m->normals); free(m->texcoords);
    free(m->face_v); free(m->face_tc); free(m->face_n);
    memset(m, 0, sizeof(*m));
}

/* get_AABB (model.h:41-61): running max/min with PL max/min, then +/- tolerance. */
void om_get_aabb(const om_mesh* m, float o[6]) {
    float xM = -OM_MAX_FLOAT, xm = OM_MAX_FLOAT, yM = -OM_MAX_FLOAT, ym = OM_MAX_FLOAT,
          zM = -OM_MAX_FLOAT, zm = OM_MAX_FLOAT;
    for (uint32_t i = 0; i < m->nv; i++) {
        ov3 v = m->vertices[i];
        xM = fmaxr(xM, v.x); xm = fminr(xm, v.x);
        yM = fmaxr(yM, v.y); ym = fminr(ym, v.y);
        zM = fmaxr(zM, v.z); zm = fminr(zm, v.z);
    }
    o[3] = xM + OM_TOL; o[4] = yM + OM_TOL; o[5] = zM + OM_TOL;
    o[0] = xm - OM_TOL; o[1] = ym - OM_TOL; o[2] = zm - OM_TOL;
}

/* translate_to (model.h:136-152) */
void om_translate_to(om_mesh* m, float a[6], ov3 c) {
    ov3 mn = v3(a[0], a[1], a[2]), mx = v3(a[3], a[4], a[5]);
    ov3 old_center = vadd(mn, vdiv(vsub(mx, mn), 2.0f));
    ov3 tr = vsub(c, old_center);
    for (uint32_t i = 0; i < m->nv; i++) m->vertices[i] = vadd(m->vertices[i], tr);
    mx = vadd(mx, tr); mn = vadd(mn, tr);
    a[0] = mn.x; a[1] = mn.y; a[2] = mn.z; a[3] = mx.x; a[4] = mx.y; a[5] = mx.z;
}

/* ------------------------------------------------------------------ octree build (kd_tree.cpp:1-288) */
typedef struct { ov3 a, b, c; uint32_t face; } prim_t; /* KD_Primitive (kd_tree.h:18-24) */
typedef struct { float bmin[3], bmax[3]; int32_t children; prim_t* prims; uint32_t n; } bnode;

static inline int inside_pt(ov3 p, const float* mn, const float* mx) { /* aabb.h:19-27 */
    int xc = (p.x >= mn[0]) && (p.x <= mx[0]);
    int yc = (p.y >= mn[1]) && (p.y <= mx[1]);
    int zc = (p.z >= mn[2]) && (p.z <= mx[2]);
    return xc && yc && zc;
}
static inline int inside_tri(const prim_t* t, const float* mn, const float* mx) { /* kd_tree.cpp:10-17 */
    int a = inside_pt(t->a, mn, mx), b = inside_pt(t->b, mn, mx), c = inside_pt(t->c, mn, mx);
    return a || b || c;
}
static inline float tri_area(const prim_t* t) { /* kd_tree.cpp:3-8 */
    ov3 ab = vsub(t->a, t->b), ac = vsub(t->a, t->c);
    return vmag(vcross(ac, ab)) / 2.0f;
}

int om_build_tree(const om_mesh* m, uint32_t max_faces, om_tree* out) {
    size_t cap = 64, len = 0;
    bnode* T = (bnode*)calloc(cap, sizeof(bnode));
    /* build_KD_tree (:20-45): root = get_AABB, all faces in face order */
    float bb[6]; om_get_aabb(m, bb);
    memcpy(T[0].bmin, bb, 12); memcpy(T[0].bmax, bb + 3, 12);
    T[0].n = m->nf;
    T[0].prims = (prim_t*)malloc(sizeof(prim_t) * (m->nf ? m->nf : 1));
    for (uint32_t i = 0; i < m->nf; i++) {
        prim_t* p = &T[0].prims[i];
        p->a = m->vertices[m->face_v[3 * i + 0]];
        p->b = m->vertices[m->face_v[3 * i + 1]];
        p->c = m->vertices[m->face_v[3 * i + 2]];
        p->face = i;
    }
    len = 1;
    /* build_oct_kd_tree (:67-288): LIFO node stack, SAH-named area-weighted centroid split */
    size_t scap = 1024, slen = 0;
    uint32_t* stack = (uint32_t*)malloc(scap * sizeof(uint32_t));
    uint8_t* depth = (uint8_t*)calloc(cap, 1);
    stack[slen++] = 0;
    while (slen > 0) {
        uint32_t ci = stack[--slen];
        if (T[ci].n > max_faces && depth[ci] < 64) { /* depth guard: reference would not terminate */
            ov3 sum = v3(0, 0, 0);
            double sum_areas = 0.0;
            for (uint32_t i = 0; i < T[ci].n; i++) { /* :96-104 */
                const prim_t* p = &T[ci].prims[i];
                ov3 cen = vdiv(vadd(vadd(p->a, p->b), p->c), 3.0f);
                float area = tri_area(p);
                sum = vadd(sum, vmul(cen, area));
                sum_areas += (double)area;
            }
            ov3 v = vdiv(sum, (float)sum_areas); /* :105 */
            if (!inside_pt(v, T[ci].bmin, T[ci].bmax)) { T[ci].children = 0; continue; } /* :107-112 */
            const float* pn = T[ci].bmin; const float* px = T[ci].bmax;
            float cb[8][6] = {
                /* bb_left  */ {pn[0], pn[1], pn[2], v.x, v.y, v.z},
                /* bf_left  */ {pn[0], pn[1], v.z, v.x, v.y, px[2]},
                /* tb_left  */ {pn[0], v.y, pn[2], v.x, px[1], v.z},
                /* tf_left  */ {pn[0], v.y, v.z, v.x, px[1], px[2]},
                /* bb_right */ {v.x, pn[1], pn[2], px[0], v.y, v.z},
                /* bf_right */ {v.x, pn[1], v.z, px[0], v.y, px[2]},
                /* tb_right */ {v.x, v.y, pn[2], px[0], px[1], v.z},
                /* tf_right */ {v.x, v.y, v.z, px[0], px[1], px[2]}}; /* :126-148 */
            prim_t* cp[8]; uint32_t cn[8];
            for (int k = 0; k < 8; k++) { cp[k] = (prim_t*)malloc(sizeof(prim_t) * (T[ci].n ? T[ci].n : 1)); cn[k] = 0; }
            for (uint32_t i = 0; i < T[ci].n; i++) /* :181-228 */
                for (int k = 0; k < 8; k++)
                    if (inside_tri(&T[ci].prims[i], cb[k], cb[k] + 3)) cp[k][cn[k]++] = T[ci].prims[i];
            free(T[ci].prims); T[ci].prims = NULL; T[ci].n = 0; /* :257 */
            if (len + 8 > cap) {
                size_t nc = cap * 2;
                T = (bnode*)realloc(T, nc * sizeof(bnode));
                memset(T + cap, 0, (nc - cap) * sizeof(bnode));
                depth = (uint8_t*)realloc(depth, nc);
                memset(depth + cap, 0, nc - cap);
                cap = nc;
            }
            int32_t start = (int32_t)len; /* :259 children_start_position = tree.length */
            T[ci].children = start;
            for (int k = 0; k < 8; k++) {
                bnode* c = &T[len++];
                memcpy(c->bmin, cb[k], 12); memcpy(c->bmax, cb[k] + 3, 12);
                c->children = 0; c->prims = cp[k]; c->n = cn[k];
                depth[start + k] = (uint8_t)(depth[ci] + 1);
            }
            if (slen + 8 > scap) { scap *= 2; stack = (uint32_t*)realloc(stack, scap * sizeof(uint32_t)); }
            for (int k = 0; k < 8; k++) stack[slen++] = (uint32_t)(start + k); /* :273-280 */
        } else {
            T[ci].children = 0; /* leaf :282-285 */
        }
    }
    free(stack); free(depth);
    /* flatten leaf primitive lists in node order */
    uint64_t total = 0;
    for (size_t i = 0; i < len; i++) if (T[i].children == 0) total += T[i].n;
    memset(out, 0, sizeof(*out));
    out->nodes = (om_node*)calloc(len, sizeof(om_node));
    out->nnodes = (int32_t)len;
    out->nprims = (uint32_t)total;
    out->prim_tri = (float*)malloc(sizeof(float) * 9 * (total ? total : 1));
    out->prim_face = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
    out->max_faces = max_faces;
    uint32_t off = 0;
    for (size_t i = 0; i < len; i++) {
        om_node* o = &out->nodes[i];
        memcpy(o->bmin, T[i].bmin, 12); memcpy(o->bmax, T[i].bmax, 12);
        o->children = T[i].children;
        if (T[i].children == 0) {
            o->prim_off = off; o->prim_cnt = T[i].n;
            for (uint32_t k = 0; k < T[i].n; k++) {
                const prim_t* p = &T[i].prims[k];
                float* d = &out->prim_tri[9 * (size_t)(off + k)];
                d[0] = p->a.x; d[1] = p->a.y; d[2] = p->a.z;
                d[3] = p->b.x; d[4] = p->b.y; d[5] = p->b.z;
                d[6] = p->c.x; d[7] = p->c.y; d[8] = p->c.z;
                out->prim_face[off + k] = p->face;
            }
            off += T[i].n;
        }
        free(T[i].prims);
    }
    free(T);
    return 0;
}

void om_free_tree(om_tree* t) { free(t->nodes); free(t->prim_tri); free(t->prim_face); memset(t, 0, sizeof(*t)); }

/* ------------------------------------------------------------------ camera (camera.h:23-45) */
void om_set_camera(om_camera* cm, ov3 eye, ov3 facing, int32_t w, int32_t h, int32_t aa,
                   uint32_t spp, int32_t bounces, float h_fov) {
    memset(cm, 0, sizeof(*cm));
    cm->h_fov = h_fov;
    cm->width = w; cm->height = h; cm->anti_aliasing = aa; cm->spp = spp; cm->bounce_limit = bounces;
    cm->aspect_ratio = (float)w / (float)h;
    cm->eye = eye;
    facing = vnormalize(facing);
    cm->frame_center = vadd(cm->eye, facing);
    cm->camera_z = vneg(facing);
    cm->camera_x = vnormalize(vcross(v3(0.f, 1.f, 0.f), cm->camera_z));
    cm->camera_y = vnormalize(vcross(cm->camera_z, cm->camera_x));
    cm->half_pixel_width = (0.5f * cm->h_fov) / (float)w;
    cm->half_pixel_height = 0.5f / (float)h;
}

/* ------------------------------------------------------------------ intersection (aabb.h, model.h) */
typedef struct { ov3 o, d, inv; int s[3]; } oray; /* Optimized_Ray (ray.h:16-21) */

static inline float bnd(const float* mn, const float* mx, int sel, int axis) { return sel ? mx[axis] : mn[axis]; }

/* check_ray_AABB_intersection (aabb.h:65-93): no z-merge, no t>0 check */
static inline int check_aabb(const oray* r, const float* mn, const float* mx) {
    float tmin = (bnd(mn, mx, r->s[0], 0) - r->o.x) * r->inv.x;
    float tmax = (bnd(mn, mx, 1 - r->s[0], 0) - r->o.x) * r->inv.x;
    float tymin = (bnd(mn, mx, r->s[1], 1) - r->o.y) * r->inv.y;
    float tymax = (bnd(mn, mx, 1 - r->s[1], 1) - r->o.y) * r->inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (bnd(mn, mx, r->s[2], 2) - r->o.z) * r->inv.z;
    float tzmax = (bnd(mn, mx, 1 - r->s[2], 2) - r->o.z) * r->inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    return 1;
}
/* get_ray_AABB_intersection (aabb.h:29-63): entry t, else exit t if > 0, else 0 */
static inline float get_aabb(const oray* r, const float* mn, const float* mx) {
    float tmin = (bnd(mn, mx, r->s[0], 0) - r->o.x) * r->inv.x;
    float tmax = (bnd(mn, mx, 1 - r->s[0], 0) - r->o.x) * r->inv.x;
    float tymin = (bnd(mn, mx, r->s[1], 1) - r->o.y) * r->inv.y;
    float tymax = (bnd(mn, mx, 1 - r->s[1], 1) - r->o.y) * r->inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (bnd(mn, mx, r->s[2], 2) - r->o.z) * r->inv.z;
    float tzmax = (bnd(mn, mx, 1 - r->s[2], 2) - r->o.z) * r->inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    if (tmin > 0) return tmin;
    else if (tmax > 0) return tmax;
    return 0;
}

/* get_triangle_ray_intersection_culled (model.h:75-103) */
static inline float mt_culled(ov3 o, ov3 d, ov3 a, ov3 b, ov3 c, float* u, float* v) {
    ov3 ab = vsub(b, a), ac = vsub(c, a);
    ov3 pvec = vcross(d, ac);
    float det = vdot(ab, pvec);
    if (det < OM_TOL) return 0;
    float det_inv = 1 / det;
    ov3 tvec = vsub(o, a);
    *u = vdot(tvec, pvec) * det_inv;
    if (*u < 0 || *u > 1) return 0;
    ov3 qvec = vcross(tvec, ab);
    *v = vdot(d, qvec) * det_inv;
    if (*v < 0 || *u + *v > 1) return 0;
    return vdot(qvec, ac) * det_inv;
}

typedef struct { int32_t node; float dist; } leafpair; /* LeafNodePair (kd_tree.h:49-53) */
static __thread int32_t* g_leaf_log = NULL; /* diagnostic leaf trace (om_primary_leaf_trace) */
static __thread int32_t g_leaf_cap = 0, g_leaf_n = 0;

typedef struct {
    int32_t* hit;     /* hit stack (node indices) */
    leafpair* leaf;   /* leaf list with barrier at index 0 */
    int32_t cap;
} trav_ws;

static void ws_init(trav_ws* w, int32_t nnodes) {
    w->cap = nnodes + 2;
    w->hit = (int32_t*)malloc(sizeof(int32_t) * (size_t)w->cap);
    w->leaf = (leafpair*)malloc(sizeof(leafpair) * (size_t)(w->cap + 1));
}
static void ws_free(trav_ws* w) { free(w->hit); free(w->leaf); }

/* scan one leaf's primitive list with the closest/tolerance acceptance (kd_tree.cpp:443-456) */
static inline int scan_leaf(const om_tree* t, const om_node* n, const oray* r, float* closest,
                            uint32_t* face, float* uo, float* vo, om_counters* ctr) {
    int hit = 0;
    for (uint32_t i = 0; i < n->prim_cnt; i++) {
        const float* p = &t->prim_tri[9 * (size_t)(n->prim_off + i)];
        float u = 0, v = 0;
        float dist = mt_culled(r->o, r->d, v3(p[0], p[1], p[2]), v3(p[3], p[4], p[5]), v3(p[6], p[7], p[8]), &u, &v);
        if (dist < *closest && dist > OM_TOL) {
            *closest = dist; *face = t->prim_face[n->prim_off + i]; *uo = u; *vo = v; hit = 1;
        }
    }
    if (ctr) ctr->n_tri += n->prim_cnt;
    return hit;
}

/* get_ray_kd_tree_intersection + traverse_oct_tree_new (kd_tree.cpp:302-465) */
static float tree_intersect(const om_tree* t, const oray* r, trav_ws* w, uint32_t* face, float* u,
                            float* v, om_counters* ctr) {
    float closest = OM_MAX_FLOAT;
    const om_node* N = t->nodes;
    if (ctr) ctr->n_box++;
    if (!check_aabb(r, N[0].bmin, N[0].bmax)) return closest; /* :339-342 */
    if (N[0].children == 0) { /* :344-361 */
        if (ctr) ctr->n_leaf++;
        scan_leaf(t, &N[0], r, &closest, face, u, v, ctr);
        return closest;
    }
    leafpair* lf = w->leaf + 1;
    w->leaf[0].node = -1; w->leaf[0].dist = -OM_MAX_FLOAT; /* barrier (renderer.cpp:386) */
    int32_t nleaf = 0, nhit = 1;
    w->hit[0] = 0;
    while (nhit > 0) { /* :368-435 */
        int32_t cur = w->hit[--nhit];
        int32_t ch = N[cur].children;
        int nodes_hit = 0;
        for (int i = 0; i < 8 && nodes_hit <= 4; i++, ch++) {
            const om_node* c = &N[ch];
            if (ctr) ctr->n_box++;
            if (c->children) {
                if (check_aabb(r, c->bmin, c->bmax)) { nodes_hit++; w->hit[nhit++] = ch; }
            } else {
                float dis = get_aabb(r, c->bmin, c->bmax);
                if (dis > 0.0f) {
                    nodes_hit++;
                    if (nleaf == 0) { lf[0].node = ch; lf[0].dist = dis; nleaf++; }
                    else {
                        int32_t e = nleaf - 1; /* insertion sort, barrier at lf[-1] */
                        while (dis < lf[e].dist) { lf[e + 1] = lf[e]; e--; }
                        lf[e + 1].node = ch; lf[e + 1].dist = dis;
                        nleaf++;
                    }
                }
            }
        }
    }
    for (int32_t j = 0; j < nleaf; j++) { /* :437-462 first improving leaf ends the scan */
        if (ctr) ctr->n_leaf++;
        if (g_leaf_log && g_leaf_n < g_leaf_cap) g_leaf_log[g_leaf_n++] = lf[j].node;
        if (scan_leaf(t, &N[lf[j].node], r, &closest, face, u, v, ctr)) break;
    }
    return closest;
}

/* sphere.h:12-39, plane.h:12-22 */
static inline float sphere_hit(ov3 o, ov3 d, const om_sphere* s) {
    ov3 pc = vsub(o, s->center);
    float pcs = vmag2(pc);
    float b = 2 * (vdot(d, pc));
    float bs = b * b;
    float c = pcs - s->radius * s->radius;
    float dmt = bs - (4 * c);
    if (dmt < 0) return 0;
    float ta = (-b + sqrtf(dmt)) * 0.5f;
    float tb = (-b - sqrtf(dmt)) * 0.5f;
    if (ta <= 0 && tb <= 0) return 0;
    if (tb > 0) return tb;
    return ta;
}
static inline float plane_hit(ov3 o, ov3 d, const om_plane* p) {
    float denom = vdot(p->normal, d);
    if (denom > -OM_TOL && denom < OM_TOL) return 0;
    return (p->distance - vdot(o, p->normal)) / denom;
}

enum { OT_NONE = 0, OT_TRI = 1, OT_SPHERE = 2, OT_PLANE = 3, OT_SKY = 4 };
typedef struct { int type; float t; ov3 normal; int32_t material; uint32_t face; float u, v; } isect;

/* get_intersection_data (renderer.cpp:34-160) */
static void intersect_scene(const om_scene* s, ov3 o, ov3 d, isect* id, trav_ws* w, om_counters* ctr) {
    id->t = OM_MAX_FLOAT;
    int32_t nm = -1, ns = -1, np = -1;
    oray r; r.o = o; r.d = d;
    r.inv = v3(1 / d.x, 1 / d.y, 1 / d.z); /* :43 */
    r.s[0] = r.inv.x < 0; r.s[1] = r.inv.y < 0; r.s[2] = r.inv.z < 0;
    if (ctr) ctr->n_rays++;
    for (int32_t i = 0; i < s->nmodels; i++) {
        const om_model* md = &s->models[i];
        if (md->tree) { /* USE_KD_TREE (:49-57) */
            uint32_t f = 0; float u = 0, v = 0;
            float t = tree_intersect(md->tree, &r, w, &f, &u, &v, ctr);
            if (t > OM_TOL && t < id->t) { id->t = t; id->face = f; id->u = u; id->v = v; nm = i; }
        } else { /* brute force (:58-82) */
            if (ctr) ctr->n_box++;
            if (get_aabb(&r, md->surrounding_aabb, md->surrounding_aabb + 3) != 0) {
                const om_mesh* m = md->mesh;
                for (uint32_t j = 0; j < m->nf; j++) {
                    float u = 0, v = 0;
                    float t = mt_culled(o, d, m->vertices[m->face_v[3 * j]], m->vertices[m->face_v[3 * j + 1]],
                                        m->vertices[m->face_v[3 * j + 2]], &u, &v);
                    if (t > OM_TOL && t < id->t) { id->t = t; id->u = u; id->v = v; id->face = j; nm = i; }
                }
                if (ctr) ctr->n_tri += m->nf;
            }
        }
    }
    for (int32_t i = 0; i < s->nspheres; i++) {
        float t = sphere_hit(o, d, &s->spheres[i]);
        if (t > OM_TOL && t < id->t) { id->t = t; ns = i; }
    }
    for (int32_t i = 0; i < s->nplanes; i++) {
        float t = plane_hit(o, d, &s->planes[i]);
        if (t > OM_TOL && t < id->t) { np = i; id->t = t; }
    }
    if (np >= 0) {
        id->type = OT_PLANE; id->normal = s->planes[np].normal; id->material = s->planes[np].material;
    } else if (ns >= 0) {
        id->type = OT_SPHERE;
        id->normal = vsub(vadd(o, vmul(d, id->t)), s->spheres[ns].center); /* Ray::at (ray.h:10-13) */
        id->material = s->spheres[ns].material;
    } else if (nm >= 0) {
        id->type = OT_TRI;
        const om_mesh* m = s->models[nm].mesh;
        if (m->nn > 0) { /* smooth (:129-138) */
            const int32_t* fn = &m->face_n[3 * id->face];
            ov3 na = m->normals[fn[0]], nb = m->normals[fn[1]], nc = m->normals[fn[2]];
            id->normal = vadd(vadd(vmul(na, (1 - id->u - id->v)), vmul(nb, id->u)), vmul(nc, id->v));
        } else { /* flat (:140-146) */
            const int32_t* fv = &m->face_v[3 * id->face];
            ov3 ab = vsub(m->vertices[fv[0]], m->vertices[fv[1]]);
            ov3 ac = vsub(m->vertices[fv[0]], m->vertices[fv[2]]);
            id->normal = vcross(ab, ac);
        }
        id->material = s->models[nm].material;
        if (ctr) ctr->n_hit++;
    } else {
        id->type = OT_SKY; id->material = 0;
    }
    if (id->type != OT_SKY) id->normal = vnormalize(id->normal); /* :157 (sky normal unused) */
}

/* ------------------------------------------------------------------ RNG (PL_math.h:492-541) */
uint32_t om_pcg_u32(uint64_t* state, uint64_t stream) {
    uint64_t old = *state;
    *state = old * 6364136223846793005ULL + (stream | 1);
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31));
}
static inline float rand_bi(uint64_t* st, uint64_t stream) {
    float rd = (float)om_pcg_u32(st, stream) * OM_INV_UINT32_MAX;
    return -1.0f + 2.0f * rd;
}
/* Deterministic stream per (pixel, sample) (documented deviation from renderer.cpp:376-378, whose
   rdtsc*thread_id seeding makes the reference's multi-bounce RGB non-deterministic): state =
   splitmix64(seed ^ pixel ^ sample << 40), increment 2 pixel + 1. Sample 0's stream is the
   per-pixel stream of rounds 1-3. */
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
void om_path_rng(uint64_t seed, int64_t pixel_index, uint32_t sample, uint64_t* state, uint64_t* stream) {
    *state = splitmix64(seed ^ (uint64_t)pixel_index ^ ((uint64_t)sample << 40));
    *stream = ((uint64_t)pixel_index << 1) | 1ULL;
}

/* ------------------------------------------------------------------ shading (renderer.cpp:213-262) */
static ov3 cast_ray(const om_scene* s, ov3 o, ov3 d, int32_t bounce_limit, uint64_t* st, uint64_t stream,
                    uint32_t* casts, trav_ws* w, om_counters* ctr) {
    ov3 ret = v3(0, 0, 0), weight = v3(1, 1, 1);
    isect id; memset(&id, 0, sizeof(id));
    int i;
    for (i = 0; i < bounce_limit; i++) {
        intersect_scene(s, o, d, &id, w, ctr);
        const om_material* mat = &s->materials[id.material];
        if (id.type == OT_SKY) { ret = vadd(ret, vhad(weight, mat->emission)); break; }
        float att = vdot(vneg(d), id.normal);
        if (att < 0) { id.normal = vneg(id.normal); att = 0; }
        ov3 pure = vsub(d, vmul(id.normal, (2 * vdot(d, id.normal))));
        pure = vnormalize(pure);
        float r0 = rand_bi(st, stream), r1 = rand_bi(st, stream), r2 = rand_bi(st, stream);
        ov3 rnd = vadd(v3(r0, r1, r2), id.normal);
        rnd = vnormalize(rnd);
        o = vadd(o, vmul(d, id.t));
        d = vnormalize(vlerp(rnd, pure, mat->scatter));
        ret = vadd(ret, vhad(weight, mat->emission));
        weight = vhad(weight, vmul(mat->reflection, att));
    }
    *casts += (uint32_t)i;
    if (ctr) ctr->n_raycasts_ref += (uint64_t)i;
    return ret;
}

static inline ov3 primary_dir(const om_camera* cm, float fx, float fy) {
    ov3 pp = vadd(vadd(cm->frame_center, vmul(cm->camera_x, fx)), vmul(cm->camera_y, fy)); /* :350 */
    return vnormalize(vsub(pp, cm->eye)); /* SetRay (ray.h:24-29) */
}
static inline float film_y(const om_camera* cm, int32_t y) { return -1.0f + 2.0f * ((float)y / (float)cm->height); }
static inline float film_x(const om_camera* cm, int32_t x) {
    return ((-1.0f + 2.0f * ((float)x / (float)cm->width)) * cm->h_fov) * cm->aspect_ratio;
}

void om_primary_hits(const om_scene* s, const om_camera* cm, int32_t y0, int32_t y1,
                     uint32_t* face_out, float* t_out, om_counters* ctr) {
    int32_t maxn = 1;
    for (int32_t i = 0; i < s->nmodels; i++) if (s->models[i].tree && s->models[i].tree->nnodes > maxn) maxn = s->models[i].tree->nnodes;
    trav_ws w; ws_init(&w, maxn);
    for (int32_t y = y0; y < y1; y++) {
        float fy = film_y(cm, y);
        for (int32_t x = 0; x < cm->width; x++) {
            ov3 d = primary_dir(cm, film_x(cm, x), fy);
            isect id; memset(&id, 0, sizeof(id));
            intersect_scene(s, cm->eye, d, &id, &w, ctr);
            size_t k = (size_t)(y - y0) * (size_t)cm->width + (size_t)x;
            face_out[k] = id.type == OT_TRI ? id.face : 0xFFFFFFFFu;
            t_out[k] = id.t;
        }
    }
    ws_free(&w);
}

void om_primary_leaf_trace(const om_scene* s, const om_camera* cm, int32_t y0, int32_t y1,
                           int32_t cap, int32_t* leaves_out, uint32_t* ntri_out) {
    int32_t maxn = 1;
    for (int32_t i = 0; i < s->nmodels; i++) if (s->models[i].tree && s->models[i].tree->nnodes > maxn) maxn = s->models[i].tree->nnodes;
    trav_ws w; ws_init(&w, maxn);
    for (int32_t y = y0; y < y1; y++) {
        float fy = film_y(cm, y);
        for (int32_t x = 0; x < cm->width; x++) {
            size_t k = (size_t)(y - y0) * (size_t)cm->width + (size_t)x;
            om_counters c; memset(&c, 0, sizeof(c));
            g_leaf_log = leaves_out + k * (size_t)cap; g_leaf_cap = cap; g_leaf_n = 0;
            for (int32_t q = 0; q < cap; q++) g_leaf_log[q] = -1;
            ov3 d = primary_dir(cm, film_x(cm, x), fy);
            isect id; memset(&id, 0, sizeof(id));
            intersect_scene(s, cm->eye, d, &id, &w, &c);
            ntri_out[k] = (uint32_t)c.n_tri;
        }
    }
    g_leaf_log = NULL;
    ws_free(&w);
}

void om_trace_rays(const om_scene* s, const float* orig, const float* dir, int64_t n,
                   uint32_t* face_out, float* t_out, float* uv_out, om_counters* ctr) {
    int32_t maxn = 1;
    for (int32_t i = 0; i < s->nmodels; i++) if (s->models[i].tree && s->models[i].tree->nnodes > maxn) maxn = s->models[i].tree->nnodes;
    trav_ws w; ws_init(&w, maxn);
    for (int64_t k = 0; k < n; k++) {
        isect id; memset(&id, 0, sizeof(id));
        intersect_scene(s, v3(orig[3 * k], orig[3 * k + 1], orig[3 * k + 2]), v3(dir[3 * k], dir[3 * k + 1], dir[3 * k + 2]), &id, &w, ctr);
        face_out[k] = id.type == OT_TRI ? id.face : 0xFFFFFFFFu;
        t_out[k] = id.t;
        if (uv_out) { uv_out[2 * k] = id.u; uv_out[2 * k + 1] = id.v; }
    }
    ws_free(&w);
}

/* one pixel of render_tile_from_camera (renderer.cpp:317-365) */
static void render_pixel(const om_scene* s, const om_camera* cm, uint64_t seed, int32_t x, int32_t y, trav_ws* w,
                         om_counters* ctr, ov3* rgb, uint32_t* bgrx, uint32_t* casts) {
    float fy = film_y(cm, y), fx = film_x(cm, x);
    uint64_t st, stream;
    const int64_t pix = (int64_t)y * cm->width + x;
    ov3 col = v3(0, 0, 0);
    uint32_t c = 0;
    if (cm->anti_aliasing) { /* :336-347 */
        for (uint32_t i = 0; i < cm->spp; i++) {
            om_path_rng(seed, pix, i, &st, &stream); /* one stream per (pixel, sample) */
            float xo = rand_bi(&st, stream) * cm->half_pixel_width + fx;
            float yo = rand_bi(&st, stream) * cm->half_pixel_height + fy;
            ov3 d = primary_dir(cm, xo, yo);
            col = vadd(col, cast_ray(s, cm->eye, d, cm->bounce_limit, &st, stream, &c, w, ctr));
        }
    } else { /* :348-357 */
        ov3 d = primary_dir(cm, fx, fy);
        for (uint32_t i = 0; i < cm->spp; i++) {
            om_path_rng(seed, pix, i, &st, &stream);
            col = vadd(col, cast_ray(s, cm->eye, d, cm->bounce_limit, &st, stream, &c, w, ctr));
        }
    }
    col = vdiv(col, (float)cm->spp); /* :358 */
    *rgb = col;
    ov3 cl = v3(fmaxr(0.0f, fminr(col.x, 1.0f)), fmaxr(0.0f, fminr(col.y, 1.0f)), fmaxr(0.0f, fminr(col.z, 1.0f)));
    uint32_t r8 = (uint8_t)(int32_t)(cl.x * 255.0f), g8 = (uint8_t)(int32_t)(cl.y * 255.0f), b8 = (uint8_t)(int32_t)(cl.z * 255.0f);
    *bgrx = b8 | (g8 << 8) | (r8 << 16); /* Set_Pixel (texture.h:27-38) */
    *casts = c;
}

void om_render_rows(const om_scene* s, const om_camera* cm, uint64_t seed, int32_t y0, int32_t y1,
                    float* rgb_out, uint32_t* fb_out, uint32_t* casts_out, om_counters* ctr) {
    int32_t maxn = 1;
    for (int32_t i = 0; i < s->nmodels; i++) if (s->models[i].tree && s->models[i].tree->nnodes > maxn) maxn = s->models[i].tree->nnodes;
    trav_ws w; ws_init(&w, maxn);
    for (int32_t y = y0; y < y1; y++)
        for (int32_t x = 0; x < cm->width; x++) {
            ov3 rgb; uint32_t px, c;
            render_pixel(s, cm, seed, x, y, &w, ctr, &rgb, &px, &c);
            size_t k = (size_t)(y - y0) * (size_t)cm->width + (size_t)x;
            if (rgb_out) { rgb_out[3 * k] = rgb.x; rgb_out[3 * k + 1] = rgb.y; rgb_out[3 * k + 2] = rgb.z; }
            if (fb_out) fb_out[k] = px;
            if (casts_out) casts_out[k] = c;
        }
    ws_free(&w);
}

/* ------------------------------------------------------------------ tile scheduler (renderer.cpp:371-471) */
int32_t om_make_tiles(int32_t W, int32_t H, int32_t threads, int32_t* tiles, int32_t cap) {
    int32_t tw = W / threads;                 /* :406 */
    if (tw > H) tw = H / threads;             /* :407-410 */
    if (tw <= 0) tw = 1;
    int32_t th = tw;
    int32_t nx = (W + tw - 1) / tw, ny = (H + th - 1) / th;
    int32_t n = 0;
    for (int32_t y = 0; y < ny; y++)
        for (int32_t x = 0; x < nx; x++) {
            uint32_t minx = (uint32_t)(x * tw), miny = (uint32_t)(y * th), maxx = minx + (uint32_t)tw, maxy = miny + (uint32_t)th;
            if (maxx > (uint32_t)W - 1) maxx = (uint32_t)W - 1;
            if (maxy > (uint32_t)H - 1) maxy = (uint32_t)H - 1;
            if (n < cap) { tiles[4 * n] = (int32_t)minx; tiles[4 * n + 1] = (int32_t)miny; tiles[4 * n + 2] = (int32_t)maxx; tiles[4 * n + 3] = (int32_t)maxy; }
            n++;
        }
    return n;
}

typedef struct {
    const om_scene* s; const om_camera* cm; uint64_t seed;
    const int32_t* tiles; int32_t ntiles; volatile int32_t next;
    uint32_t* fb; int64_t* tile_casts; int32_t maxn;
    volatile uint64_t traced; /* get_intersection_data calls, summed over the threads */
} pool_t;

static void* tile_worker(void* arg) { /* start_tile_render_thread (:371-399) */
    pool_t* p = (pool_t*)arg;
    trav_ws w; ws_init(&w, p->maxn);
    om_counters ctr; memset(&ctr, 0, sizeof(ctr));
    for (;;) {
        int32_t k = __atomic_add_fetch(&p->next, 1, __ATOMIC_SEQ_CST); /* :298-307 */
        if (k > p->ntiles) break;
        const int32_t* t = &p->tiles[4 * (k - 1)];
        int64_t casts = 0;
        for (int32_t y = t[1]; y <= t[3]; y++)
            for (int32_t x = t[0]; x <= t[2]; x++) {
                ov3 rgb; uint32_t px, c;
                render_pixel(p->s, p->cm, p->seed, x, y, &w, &ctr, &rgb, &px, &c);
                p->fb[(size_t)y * p->cm->width + x] = px;
                casts += c;
            }
        p->tile_casts[k - 1] = casts;
    }
    __atomic_add_fetch(&p->traced, ctr.n_rays, __ATOMIC_SEQ_CST);
    ws_free(&w);
    return NULL;
}

/* CPU-baseline sample: rows row0, row0 + row_step, ... (nrows of them) of the frame, claimed one
   row at a time by `threads` workers (the reference's atomic claim, renderer.cpp:298-307, with a
   row as the unit), full spp / bounces per pixel. Returns seconds; traced rays and the
   reference's non-sky ray_casts (renderer.cpp:260) of the sample through the pointers. */
typedef struct {
    const om_scene* s; const om_camera* cm; uint64_t seed;
    int32_t row0, row_step, nrows; volatile int32_t next; int32_t maxn;
    volatile uint64_t traced; volatile int64_t casts;
} rowpool_t;

static void* row_worker(void* arg) {
    rowpool_t* p = (rowpool_t*)arg;
    trav_ws w; ws_init(&w, p->maxn);
    om_counters ctr; memset(&ctr, 0, sizeof(ctr));
    int64_t casts = 0;
    for (;;) {
        int32_t k = __atomic_fetch_add(&p->next, 1, __ATOMIC_SEQ_CST);
        if (k >= p->nrows) break;
        const int32_t y = p->row0 + k * p->row_step;
        for (int32_t x = 0; x < p->cm->width; x++) {
            ov3 rgb; uint32_t px, c;
            render_pixel(p->s, p->cm, p->seed, x, y, &w, &ctr, &rgb, &px, &c);
            casts += c;
        }
    }
    __atomic_add_fetch(&p->traced, ctr.n_rays, __ATOMIC_SEQ_CST);
    __atomic_add_fetch(&p->casts, casts, __ATOMIC_SEQ_CST);
    ws_free(&w);
    return NULL;
}

double om_render_rows_threaded(const om_scene* s, const om_camera* cm, uint64_t seed, int32_t threads,
                               int32_t row0, int32_t row_step, int32_t nrows, uint64_t* traced_rays,
                               int64_t* ray_casts) {
    rowpool_t p; memset(&p, 0, sizeof(p));
    p.s = s; p.cm = cm; p.seed = seed; p.row0 = row0; p.row_step = row_step; p.nrows = nrows;
    p.maxn = 1;
    for (int32_t i = 0; i < s->nmodels; i++) if (s->models[i].tree && s->models[i].tree->nnodes > p.maxn) p.maxn = s->models[i].tree->nnodes;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int32_t i = 0; i < threads; i++) pthread_create(&th[i], NULL, row_worker, &p);
    for (int32_t i = 0; i < threads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (traced_rays) *traced_rays = p.traced;
    if (ray_casts) *ray_casts = p.casts;
    free(th);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

double om_render_threaded(const om_scene* s, const om_camera* cm, uint64_t seed, int32_t threads,
                          uint32_t* fb_out, int64_t* total_ray_casts, uint64_t* traced_rays) {
    int32_t cap = 1 << 16;
    int32_t* tiles = (int32_t*)malloc(sizeof(int32_t) * 4 * (size_t)cap);
    int32_t nt = om_make_tiles(cm->width, cm->height, threads, tiles, cap);
    pool_t p; memset(&p, 0, sizeof(p));
    p.s = s; p.cm = cm; p.seed = seed; p.tiles = tiles; p.ntiles = nt; p.next = 0; p.fb = fb_out;
    p.tile_casts = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
    p.maxn = 1;
    for (int32_t i = 0; i < s->nmodels; i++) if (s->models[i].tree && s->models[i].tree->nnodes > p.maxn) p.maxn = s->models[i].tree->nnodes;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int32_t i = 0; i < threads; i++) pthread_create(&th[i], NULL, tile_worker, &p);
    for (int32_t i = 0; i < threads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    int64_t tot = 0;
    for (int32_t i = 0; i < nt; i++) tot += p.tile_casts[i];
    if (total_ray_casts) *total_ray_casts = tot;
    /* every get_intersection_data call, the 1-px tile overlaps traced twice as the reference's
       threads do */
    if (traced_rays) *traced_rays = p.traced;
    free(th); free(p.tile_casts); free(tiles);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
