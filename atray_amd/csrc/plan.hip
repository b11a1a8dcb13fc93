// plan.hip -- the single-frame dispatch plan, built on the GPU from the previous frame's measured
// per-cell cost. A live view (app.cpp:158-186) renders one frame per launch, and a
// launch ends with its slowest cells; so the next launch dispatches the cells that were heavy in
// the last one first, graded by cost into 8 classes (Morton order kept inside a class), and splits
// the heaviest 1 % into two row-band waves. Outputs never change: every block keeps its pixels and
// packed slots; only the dispatch order and the number of waves per cell differ.
//
// Two launches after the render, on its stream, no host round trip:
//   plan_count_kernel: the cost histogram, and per 256-block chunk the slots each class takes under
//     the thresholds of the previous plan; its last workgroup derives the next thresholds from the
//     histogram (in parallel) and the class start slots;
//   plan_order_kernel: every block to its slot (class start + earlier chunks + its place in its
//     chunk); its last workgroup promotes the new thresholds.
// The class thresholds lag one plan behind the costs they order (cost levels move slowly between
// consecutive frames); the order itself always follows the latest costs.
#include <hip/hip_runtime.h>

#include "engine.h"

#ifndef ATR_PLAN_SPLIT2
#define ATR_PLAN_SPLIT2 0.01f
#endif
#ifndef ATR_PLAN_SPLIT4
#define ATR_PLAN_SPLIT4 0.0f
#endif

namespace atr {

constexpr int kPlanBuckets = 256;  // cost histogram: 8 buckets per power of two of the clock count
constexpr int kPlanClasses = 8;    // class index 0 (dispatched first) .. 7 (last)
// cumulative fractions of the cells (heaviest first) that end classes 0, 1, ..., 6; the rest is 7
__constant__ float kClassFrac[kPlanClasses - 1] = {0.02f, 0.05f, 0.10f, 0.20f, 0.30f, 0.50f, 0.75f};
// default split fractions: the heaviest ATR_PLAN_SPLIT4 of the cells get four row-band waves, the
// heaviest ATR_PLAN_SPLIT2 two, within the list's spare capacity (max_split extra blocks); the host
// passes larger ones for launches that leave the chip's wave slots idle (capi.cpp launch_planned)
constexpr float kSplit4Frac = ATR_PLAN_SPLIT4, kSplitFrac = ATR_PLAN_SPLIT2;

struct Thresholds {
    int32_t thr[kPlanClasses];      // bucket >= thr[k] (first such k) -> class k
    int32_t split_thr, split4_thr;  // bucket >= split4_thr: 4 waves; >= split_thr: 2
};

struct PlanWork {
    uint32_t hist[kPlanBuckets];
    Thresholds use;   // the thresholds this plan orders by (all zero = one class, no split)
    Thresholds next;  // derived from this plan's histogram, promoted at its end
    uint32_t start[kPlanClasses];     // first slot of each class under `use`
    uint32_t used;                    // slots holding blocks (nb + split waves)
    uint32_t nosplit;                 // the splits under `use` would overflow the list: none this time
    uint32_t done_count, done_order;  // workgroups finished (last-workgroup election)
};
// per 256-block chunk: the slots of each class with the splits, then without (kChunkWords words)
constexpr int kChunkWords = 2 * kPlanClasses;

__device__ __forceinline__ int cost_bucket(unsigned long long c) {
    if (c == 0) return 0;
    const int e = 63 - __clzll(c);  // floor(log2 c)
    const int m = e >= 3 ? int((c >> (e - 3)) & 7) : int((c << (3 - e)) & 7);  // next 3 bits
    const int b = e * 8 + m;
    return b < kPlanBuckets ? b : kPlanBuckets - 1;
}

__device__ __forceinline__ int block_class(const Thresholds& T, int bkt) {
    int k = 0;
    while (k < kPlanClasses - 1 && bkt < T.thr[k]) ++k;
    return k;
}

// a zeroed Thresholds (the first plan) gives class 0 and one wave to every cell: split thresholds
// of 0 are replaced by "no split" (kPlanBuckets) when derived, so 0 only occurs before the first
__device__ __forceinline__ int block_parts(const Thresholds& T, int bkt) {
    if (T.split_thr == 0) return 1;
    return bkt >= T.split4_thr ? 4 : (bkt >= T.split_thr ? 2 : 1);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// The next thresholds from the histogram, one bucket per thread (256 threads): the cells above
// bucket b (a suffix sum) decide its class (the number of class fractions they reach) and whether
// it splits (whole buckets from the top while they fit the fraction and the spare capacity: both
// conditions are monotone in b, so the split buckets are a top range, as a sequential walk would
// take them); thr[k] = the lowest bucket of class k.
__device__ void next_thresholds(const uint32_t* hist, int32_t nb, int32_t max_split, float split2, float split4,
                                Thresholds& T, uint32_t* scratch /* 256 + 16 words of LDS */) {
    const int b = int(threadIdx.x);
    const uint32_t n = hist[b];
    scratch[b] = n;  // inclusive suffix sum: cells in buckets >= b
    __syncthreads();
    for (int off = 1; off < kPlanBuckets; off <<= 1) {
        const uint32_t v = b + off < kPlanBuckets ? scratch[b + off] : 0u;
        __syncthreads();
        scratch[b] += v;
        __syncthreads();
    }
    const uint32_t incl = scratch[b], above = incl - n;
    __syncthreads();
    int32_t* thr = reinterpret_cast<int32_t*>(scratch);  // reused: 8 thresholds, 2 split minima, n4
    if (b < kPlanClasses + 2) thr[b] = kPlanBuckets;
    if (b == kPlanClasses + 2) thr[b] = 0;
    __syncthreads();
    const bool s4 = n && float(incl) <= split4 * float(nb) + 0.5f && 3u * incl <= uint32_t(max_split);
    if (s4) {
        atomicMin(&thr[kPlanClasses + 1], b);
        atomicMax(&thr[kPlanClasses + 2], int32_t(incl));  // cells taking four waves
    }
    __syncthreads();
    const uint32_t n4 = uint32_t(thr[kPlanClasses + 2]);
    const bool s2 = n && !s4 && float(incl) <= split2 * float(nb) + 0.5f &&
                    3u * n4 + (incl - n4) <= uint32_t(max_split);
    if (s2 || s4) atomicMin(&thr[kPlanClasses], b);
    int k = 0;
    while (k < kPlanClasses - 1 && float(above) >= kClassFrac[k] * float(nb)) ++k;
    if (n) atomicMin(&thr[k], b);
    __syncthreads();
    if (b == 0) {
        // classes with no bucket take the previous class's threshold (they match nothing)
        int32_t last = kPlanBuckets;
        for (int j = 0; j < kPlanClasses; ++j) {
            T.thr[j] = thr[j] == kPlanBuckets ? last : thr[j];
            last = T.thr[j];
        }
        T.thr[kPlanClasses - 1] = 0;  // everything else is the last class
        T.split_thr = thr[kPlanClasses] > 0 ? thr[kPlanClasses] : 1;  // 0 is the "first plan" marker
        T.split4_thr = thr[kPlanClasses + 1] > 0 ? thr[kPlanClasses + 1] : 1;
    }
    __syncthreads();
}

// Histogram + per-chunk class slots under W->use; the last workgroup derives W->next, the class
// start slots and the used count, and clears the histogram for the next plan.
__global__ __launch_bounds__(256) void plan_count_kernel(const unsigned long long* __restrict__ cost, int32_t nb,
                                                         int32_t max_split, float split2, float split4,
                                                         PlanWork* __restrict__ W,
                                                         uint32_t* __restrict__ chunk_slots) {
    __shared__ uint32_t h[kPlanBuckets];
    __shared__ uint32_t scratch[kPlanBuckets + 16];
    __shared__ uint32_t cnt[kChunkWords];
    __shared__ Thresholds T;
    __shared__ bool last;
    h[threadIdx.x] = 0;
    if (threadIdx.x < kChunkWords) cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) T = W->use;
    __syncthreads();
    const int32_t i = int32_t(blockIdx.x) * 256 + int32_t(threadIdx.x);
    if (i < nb) {
        const int bkt = cost_bucket(cost[i]);
        const int k = block_class(T, bkt);
        atomicAdd(&h[bkt], 1u);
        atomicAdd(&cnt[k], uint32_t(block_parts(T, bkt)));
        atomicAdd(&cnt[kPlanClasses + k], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&W->hist[threadIdx.x], h[threadIdx.x]);
    if (threadIdx.x < kChunkWords) chunk_slots[size_t(blockIdx.x) * kChunkWords + threadIdx.x] = cnt[threadIdx.x];
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&W->done_count, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    // the last workgroup: every chunk's counts and the whole histogram are visible
    __threadfence();
    h[threadIdx.x] = atomicExch(&W->hist[threadIdx.x], 0u);  // read and clear for the next plan
    if (threadIdx.x < kChunkWords) cnt[threadIdx.x] = 0;
    __syncthreads();
    {
        uint32_t acc[kChunkWords] = {};
        for (uint32_t c = threadIdx.x; c < gridDim.x; c += 256)
#pragma unroll
            for (int j = 0; j < kChunkWords; ++j)
                acc[j] += __atomic_load_n(&chunk_slots[size_t(c) * kChunkWords + j], __ATOMIC_RELAXED);
#pragma unroll
        for (int j = 0; j < kChunkWords; ++j) {
            const uint32_t v = wave_sum(acc[j]);
            if ((threadIdx.x & 63) == 0 && v) atomicAdd(&cnt[j], v);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // the previous plan's split thresholds may select more cells now: over the spare capacity,
        // this plan splits none (the block counts, not the slot counts, then place the blocks)
        uint32_t total = 0;
        for (int j = 0; j < kPlanClasses; ++j) total += cnt[j];
        const uint32_t nosplit = total > uint32_t(nb + max_split) ? 1u : 0u;
        uint32_t s = 0;
        for (int j = 0; j < kPlanClasses; ++j) { W->start[j] = s; s += cnt[nosplit ? kPlanClasses + j : j]; }
        W->used = s;
        W->nosplit = nosplit;
        W->done_count = 0;
    }
    __shared__ Thresholds nx;
    next_thresholds(h, nb, max_split, split2, split4, nx, scratch);
    if (threadIdx.x == 0) W->next = nx;
}

// Every base block to its slot, list order kept within each class: class start + the class's slots
// in earlier chunks + its slots before the block in this chunk (wave ballots, waves in order). A
// split block becomes `parts` waves on row bands of its cell (the later bands' packed slots follow
// the earlier ones'). Slots past `used` get empty blocks (no lanes). The costs are kept in
// cost_last and cleared for the next launch; the last workgroup promotes W->next to W->use.
__global__ __launch_bounds__(256) void plan_order_kernel(const DBlock* __restrict__ base, int32_t nb,
                                                         unsigned long long* __restrict__ cost,
                                                         unsigned long long* __restrict__ cost_last,
                                                         PlanWork* __restrict__ W,
                                                         const uint32_t* __restrict__ chunk_slots,
                                                         DBlock* __restrict__ out, int32_t cap) {
    __shared__ uint32_t before[kPlanClasses];
    __shared__ uint32_t wave_tot[4][kPlanClasses];
    __shared__ Thresholds T;
    __shared__ bool last;
    const int32_t i = int32_t(blockIdx.x) * 256 + int32_t(threadIdx.x);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t nosplit = W->nosplit, col = nosplit ? kPlanClasses : 0;
    if (threadIdx.x < kPlanClasses) before[threadIdx.x] = W->start[threadIdx.x];
    if (threadIdx.x == 0) T = W->use;
    __syncthreads();
    {
        uint32_t acc[kPlanClasses] = {};
        for (uint32_t c = threadIdx.x; c < blockIdx.x; c += 256)
#pragma unroll
            for (int j = 0; j < kPlanClasses; ++j) acc[j] += chunk_slots[size_t(c) * kChunkWords + col + j];
#pragma unroll
        for (int j = 0; j < kPlanClasses; ++j) {
            const uint32_t v = wave_sum(acc[j]);
            if (lane == 0 && v) atomicAdd(&before[j], v);
        }
    }
    int k = -1, parts = 1;
    DBlock b;
    if (i < nb) {
        b = base[i];
        const unsigned long long c = cost[i];
        cost_last[i] = c;  // kept for atr_render_plan_info
        cost[i] = 0;       // the next launch measures afresh
        const int bkt = cost_bucket(c);
        k = block_class(T, bkt);
        parts = nosplit ? 1 : block_parts(T, bkt);
    }
    const uint64_t below = (uint64_t(1) << lane) - 1;
    const uint64_t b2 = __ballot(parts >= 2), b4 = __ballot(parts == 4);  // slots = 1 + [>= 2] + 2 [4]
    uint32_t my_off = 0;
    for (int j = 0; j < kPlanClasses; ++j) {
        const uint64_t bj = __ballot(k == j);
        if (k == j) my_off = uint32_t(__popcll(bj & below) + __popcll(bj & b2 & below) + 2 * __popcll(bj & b4 & below));
        if (lane == 0) wave_tot[wv][j] = uint32_t(__popcll(bj) + __popcll(bj & b2) + 2 * __popcll(bj & b4));
    }
    __syncthreads();
    if (i < nb) {
        uint32_t s = before[k] + my_off;
        for (int w = 0; w < wv; ++w) s += wave_tot[w][k];
        const uint64_t m = uint64_t(b.mask_lo) | (uint64_t(b.mask_hi) << 32);
        const int rows = 8 / parts;
        int32_t ob = b.out_base;
        for (int p = 0; p < parts; ++p) {  // row bands p * rows .. (p + 1) * rows - 1, lane order
            const uint64_t band = parts == 1 ? ~uint64_t(0) : ((uint64_t(1) << (8 * rows)) - 1) << (8 * rows * p);
            DBlock t = b;
            t.mask_lo = uint32_t(m & band);
            t.mask_hi = uint32_t((m & band) >> 32);
            t.out_base = ob;
#ifdef ATR_PLAN_PRIO_CLASSES  // experiment: the heaviest classes' waves at raised issue priority
            if (k < ATR_PLAN_PRIO_CLASSES) t.flags |= kBlockPrio;
#endif
            ob += __popcll(m & band);
            out[s + p] = t;
        }
    }
    const uint32_t used = W->used;
    for (int32_t t = int32_t(used) + i; t < cap; t += int32_t(gridDim.x) * 256) {
        DBlock e;
        e.x0 = 0; e.y0 = 0; e.mask_lo = 0; e.mask_hi = 0; e.out_base = 0; e.flags = 0; e.base = 0; e.pad = 0;
        out[t] = e;
    }
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&W->done_order, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last && threadIdx.x == 0) {  // every workgroup has read W->use
        W->use = W->next;
        W->done_order = 0;
    }
}

}  // namespace atr

// work: PlanWork + the per-chunk class slots, zeroed once at allocation and left ready for the next
// plan by every plan (a zeroed `use` = one class, no split, until the first plan promotes real
// thresholds); cost: the render's per-base-block clocks (cleared again; cost_last keeps them); out:
// cap = nb + max_split blocks.
// split2 / split4 < 0: the defaults (ATR_PLAN_SPLIT2 / ATR_PLAN_SPLIT4).
extern "C" hipError_t atr_launch_plan(const atr::DBlock* base, int32_t nb, unsigned long long* cost,
                                      unsigned long long* cost_last, void* work, atr::DBlock* out, int32_t max_split,
                                      float split2, float split4, hipStream_t s) {
    if (split2 < 0.f) split2 = atr::kSplitFrac;
    if (split4 < 0.f) split4 = atr::kSplit4Frac;
    if (nb <= 0) return hipSuccess;
    atr::PlanWork* W = static_cast<atr::PlanWork*>(work);
    uint32_t* chunk_slots = reinterpret_cast<uint32_t*>(W + 1);
    const unsigned g = unsigned((nb + 255) / 256);
    hipLaunchKernelGGL(atr::plan_count_kernel, dim3(g), dim3(256), 0, s, cost, nb, max_split, split2, split4, W,
                       chunk_slots);
    hipLaunchKernelGGL(atr::plan_order_kernel, dim3(g), dim3(256), 0, s, base, nb, cost, cost_last, W, chunk_slots,
                       out, nb + max_split);
    return hipGetLastError();
}

extern "C" size_t atr_plan_work_bytes(int32_t nb) {
    return sizeof(atr::PlanWork) + size_t((nb + 255) / 256) * atr::kChunkWords * sizeof(uint32_t);
}
