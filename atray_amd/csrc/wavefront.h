// wavefront.h -- state of the leaf-major (ray-sorted) schedule, see wavefront.hip.
#pragma once
#include "engine.h"

namespace atr {

// device counters of the wavefront pipeline
struct WFCtl {
    int32_t nact[2];   // active path lists (double-buffered across bounces)
    int32_t npend[2];  // rays with a binned pending leaf (current / next step)
    int32_t nrw;       // rays that need a re-walk of the tree
    int32_t nitems;    // work items of the current step
    int32_t pad[2];
};

// Everything is structure-of-arrays over path slots r in [0, n): slot r renders pixel pix[r].
struct WFParams {
    atr_camera cam;
    const DScene* scene;
    uint64_t seed;
    int32_t n;
    int32_t layout;
    const int32_t* pix;
    // per-path state
    uint64_t* rng;
    float* col;   // 3n accumulated colour over samples
    float* ret;   // 3n colour of the current sample
    float* wt;    // 3n weight of the current sample
    uint32_t* casts;
    uint32_t* traced;
    uint32_t* hface;
    float* ht;
    // current ray
    float* ro;    // 3n
    float* rd;    // 3n
    // closest hit over models (current bounce)
    float* bt;
    float* bu;
    float* bv;
    uint32_t* bface;
    int32_t* bmodel;
    // per-model tree query: 8 buffered leaves per ray + bound of the 8th
    int32_t* ql;  // 8n, [k * n + r]
    float* qd7;
    int32_t* qi7;
    int32_t* qpos;
    int32_t* qnb;
    int32_t* qnc;
    int32_t* pleaf;
    int32_t* pslot;
    // lists
    int32_t* act[2];
    int32_t* pend[2];
    int32_t* rw;
    uint32_t* cnt[2];  // per node
    int32_t* offs;     // per node
    int32_t* items;    // int4 (leaf, bucket start, count, 0)
    int32_t* bucket;
    WFCtl* ctl;
    // outputs
    uint32_t* framebuffer;
    uint32_t* out_hit_face;
    float* out_hit_t;
    float* out_rgb;
    uint32_t* out_ray_casts;
    unsigned long long* traced_rays;
    int32_t* error_flag;
};

}  // namespace atr
