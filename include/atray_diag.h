/*
 * atray_diag.h -- diagnostic entry points of the engine library, compiled only into the
 * diagnostic build (make -C atray_amd/csrc DIAG=1, -DATR_DIAG). The shipping library
 * (include/atray.h) does not export them. Used by the probes under tools/.
 */
#ifndef ATRAY_DIAG_H
#define ATRAY_DIAG_H
#include "atray.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic: one instrumented render; out = wave clocks (s_memtime, summed over waves) spent in
   the FLAT/HYBRID scans' DFS passes, lane-private leaf scans, dealt leaf rounds, in the whole
   wave, in each leaf step's preparation (leaf range, prefix sums, schedule decision), and in the
   whole scan (tree query). The per-phase clocks are compiled only into a diagnostic build
   (make EXTRA=-DATR_PHASE_CLOCKS); the product library reports the whole-wave clocks alone. */
int atr_render_phase_clocks(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                            uint64_t seed, int32_t variant, int64_t out[6]);
/* Diagnostic: one instrumented render; lane use of the bounce loop (cast_ray, renderer.cpp:213-262)
   in the wavefront schedules (WAVE, FLAT, HYBRID): out[0..2] = wave steps of bounce 0, 1 and >= 2
   (a step = one loop iteration some lane of the wave traces in), out[3..5] = lanes tracing in
   them. out[3 + k] / (64 out[k]) is the lane utilisation of bounce bucket k. */
int atr_render_path_counters(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                             uint64_t seed, int32_t variant, int64_t out[6]);
/* Diagnostic: one instrumented render; SIMD efficiency of the clustered scans: out[0] wave-level
   iterations of the full-test candidate loops (two tests each in the paired loops), out[1] full
   triangle tests, out[2] / out[3] DFS loop iterations at wave / lane level, out[4] dealt rounds,
   out[5] the (ray, cluster) items they carried, out[6] traced rays. */
int atr_render_simd_counters(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                             uint64_t seed, int32_t variant, int64_t out[7]);
/* Diagnostic: one render of `tiles` recording, per 8x8 work block (block order), the wave's start
   and end on the 100 MHz device clock and its HW_ID | XCC_ID << 32. out = 3 u64 per block;
   with out == NULL (or cap too small) only *nblocks is set. */
int atr_render_wave_trace(atr_ctx* ctx, const atr_camera* cam, const atr_tile* tiles, int32_t ntiles,
                          uint64_t seed, int32_t variant, uint64_t* out, int64_t cap, int64_t* nblocks);
#ifdef __cplusplus
}
#endif
#endif
