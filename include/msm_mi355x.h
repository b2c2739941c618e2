/*
 * msm_mi355x.h -- C ABI of the MI355X (gfx950) BLS12-381 MSM engine
 * (libmsm_mi355x.so, built from msm_blst_amd/csrc).
 *
 * Drop-in boundary for the hot path of LuoGuiwen/MSM_blst (a blst v0.3.10
 * fork): plain C types and pointers only, layout-identical to
 * bindings/blst.h, so a caller of the reference links this library for the
 * MSM entry points below instead of libblst's.  Each declaration cites the
 * reference interface it replaces.
 *
 * Threading: entry points are thread-safe per call (each blst-named call leases
 * an engine with its own device buffers and stream from a process-wide pool;
 * engine contexts are not shared across threads unless the
 * caller serialises).  Errors: the blst-named functions keep blst's void
 * signatures; by default a HIP failure inside one prints the error and aborts
 * (a silent wrong answer is never returned); after msm_set_abort_on_error(0)
 * such a call returns with its result set to the all-zero point (infinity;
 * blst_p{1,2}s_mult_wbits_precompute: the whole table zeroed, never half written),
 * msm_error_pending() nonzero and the message in msm_last_error().  The msm_*
 * extension API returns MSM_OK or a negative MSM_E* code and msm_last_error()
 * describes it.
 */
#ifndef MSM_MI355X_H
#define MSM_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- types: layout-identical to /root/reference/bindings/blst.h ---- */
typedef uint8_t byte;                                      /* blst.h:53 */
typedef uint64_t limb_t;                                   /* blst.h:54 */
typedef struct { byte b[256 / 8]; } blst_scalar;           /* blst.h:56 */
typedef struct { limb_t l[384 / 8 / sizeof(limb_t)]; } blst_fp;  /* blst.h:58 */
typedef struct { blst_fp fp[2]; } blst_fp2;                /* blst.h:60 */
typedef struct { blst_fp x, y, z; } blst_p1;               /* blst.h:164 */
typedef struct { blst_fp x, y; } blst_p1_affine;           /* blst.h:165 */
typedef struct { blst_fp2 x, y, z; } blst_p2;              /* blst.h:191 */
typedef struct { blst_fp2 x, y; } blst_p2_affine;          /* blst.h:192 */
typedef struct { blst_fp x, y, zzz, zz; } blst_p1xyzz;     /* blst.h:251 */
typedef struct { blst_fp2 x, y, zzz, zz; } blst_p2xyzz;    /* blst.h:252 */
typedef struct { int m; int b; int alpha; } digit_decomposition; /* blst.h:253 */

/* ---- plain Pippenger (replaces src/multi_scalar.c:581-607, blst.h:238-246, :377-384) ----
 * Same semantics as blst: points[] / scalars[] are arrays of pointers; when
 * points[1] (resp. scalars[1]) is NULL the data is one flat array, scalars
 * packed with stride (nbits+7)/8 (multi_scalar.c:393-416).  The low nbits bits
 * of each scalar are used (scalars are not reduced mod r).  The all-zero
 * affine point is infinity and contributes nothing.  ret is a Jacobian point
 * in Montgomery form; any representative (callers normalise with to_affine).
 * scratch is accepted for ABI compatibility and not used (device buffers are
 * the engine's own).  Unlike blst (defect at n=1), any n >= 0 is exact. */
size_t blst_p1s_mult_pippenger_scratch_sizeof(size_t npoints);
void blst_p1s_mult_pippenger(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch);
void blst_p1s_tile_pippenger(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch, size_t bit0,
                             size_t window);
size_t blst_p2s_mult_pippenger_scratch_sizeof(size_t npoints);
void blst_p2s_mult_pippenger(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch);
void blst_p2s_tile_pippenger(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch, size_t bit0,
                             size_t window);

/* ---- blst-level CHES / BGMW95 entry points (replace ref src/multi_scalar.c:584-790,
 * declared at ref bindings/blst.h:249-357; used by ref main_p1.cpp:233-236, :279-282, :384) ----
 * Same names, argument meaning and layouts.  The tile_* and integrate_* calls run on
 * the GPU (entries uploaded, sorted by bucket, accumulated one lane per bucket, then
 * the weighted bucket sum); the per-point helpers run on the host (one point op is
 * far below a kernel launch).  Differences, all toward the mathematically exact sum:
 * the last-element guard of ref multi_scalar.c:461 is applied to the last element's
 * own bucket (SURVEY 8a defect 1); buckets[] is filled with the per-bucket sums as
 * the reference leaves it (xyzz representatives may differ; equal as points). */
size_t blst_p1s_mult_pippenger_scratch_sizeof_CHES(size_t window);  /* multi_scalar.c:584-585 */
size_t blst_p2s_mult_pippenger_scratch_sizeof_CHES(size_t window);
void blst_p1xyzz_dadd_affine(blst_p1xyzz *out, const blst_p1xyzz *in, const blst_p1_affine *p,
                             unsigned char booth_sign);              /* ec_ops.h:710-769 */
void blst_p2xyzz_dadd_affine(blst_p2xyzz *out, const blst_p2xyzz *in, const blst_p2_affine *p,
                             unsigned char booth_sign);
void blst_p1xyzz_dadd(blst_p1xyzz *p3, const blst_p1xyzz *p1, const blst_p1xyzz *p2);  /* ec_ops.h:642-702 */
void blst_p2xyzz_dadd(blst_p2xyzz *p3, const blst_p2xyzz *p1, const blst_p2xyzz *p2);
void blst_p1xyzz_to_Jacobian(blst_p1 *out, const blst_p1xyzz *in);   /* ec_ops.h:771-777 */
void blst_p2xyzz_to_Jacobian(blst_p2 *out, const blst_p2xyzz *in);
void blst_p1_to_xyzz(blst_p1xyzz *out, blst_p1 *in);                /* ec_ops.h:779-785 */
void blst_p2_to_xyzz(blst_p2xyzz *out, blst_p2 *in);
void blst_p1_prefetch_CHES(const blst_p1xyzz buckets[], size_t booth_idx);  /* no-op hint */
void blst_p2_prefetch_CHES(const blst_p2xyzz buckets[], size_t booth_idx);
void blst_p1_bucket_CHES(blst_p1xyzz buckets[], int booth_idx, const blst_p1_affine *p,
                         unsigned char booth_sign);                  /* multi_scalar.c:358-361 */
void blst_p2_bucket_CHES(blst_p2xyzz buckets[], int booth_idx, const blst_p2_affine *p, unsigned char booth_sign);
/* sum_i bucket_set_ascend[i] * buckets[i] (multi_scalar.c:301-321); any non-negative
 * weights are accepted (d_max is not needed by the GPU reduction) */
void blst_p1_integrate_buckets_accumulation_d_CHES(blst_p1 *out, blst_p1xyzz buckets[], int bucket_set_ascend[],
                                                   size_t bucket_set_size, int d_max);
void blst_p2_integrate_buckets_accumulation_d_CHES(blst_p2 *out, blst_p2xyzz buckets[], int bucket_set_ascend[],
                                                   size_t bucket_set_size, int d_max);
/* integral scalar conversion (multi_scalar.c:748-775): standard q-ary digits in
 * nh_scalars[] (carry written into the next slot) -> bucket values, signs, table pointers */
void blst_p1_construct_nh_scalars_nh_points(int nh_scalars[], unsigned char booth_signs[],
                                            blst_p1_affine *nh_points_ptr[], const size_t npoints,
                                            blst_p1_affine precomputation_points_list_3nh[],
                                            const digit_decomposition digit_conversion_hash_table[]);
void blst_p2_construct_nh_scalars_nh_points(int nh_scalars[], unsigned char booth_signs[],
                                            blst_p2_affine *nh_points_ptr[], const size_t npoints,
                                            blst_p2_affine precomputation_points_list_3nh[],
                                            const digit_decomposition digit_conversion_hash_table[]);
/* CHES accumulation + d-reduction (multi_scalar.c:421-463, 643-655) */
void blst_p1_tile_pippenger_d_CHES(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints,
                                   const int scalars[], const unsigned char booth_signs[], blst_p1xyzz buckets[],
                                   int bucket_set_ascend[], int bucket_value_to_its_index[], size_t bucket_set_size,
                                   int d_max);
void blst_p2_tile_pippenger_d_CHES(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints,
                                   const int scalars[], const unsigned char booth_signs[], blst_p2xyzz buckets[],
                                   int bucket_set_ascend[], int bucket_value_to_its_index[], size_t bucket_set_size,
                                   int d_max);
/* buckets indexed by bucket value (multi_scalar.c:466-503); values outside the set weigh 0 */
void blst_p1_tile_pippenger_d_CHES_noindexhash(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints,
                                               const int scalars[], const unsigned char booth_signs[],
                                               blst_p1xyzz buckets[], int bucket_set_ascend[], size_t bucket_set_size,
                                               int d_max);
void blst_p2_tile_pippenger_d_CHES_noindexhash(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints,
                                               const int scalars[], const unsigned char booth_signs[],
                                               blst_p2xyzz buckets[], int bucket_set_ascend[], size_t bucket_set_size,
                                               int d_max);
/* standard q-ary digits in, digit-hash lookup + carry inside (multi_scalar.c:671-744);
 * scalars[] is updated with the carries as the reference does (needs one slot of padding) */
void blst_p1_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar(
    blst_p1 *ret, const blst_p1_affine precomputation_points_list_3nh[], size_t npoints, int scalars[],
    digit_decomposition digit_conversion_hash_table[], blst_p1xyzz buckets[], int bucket_set_ascend[],
    int bucket_value_to_its_index[], size_t bucket_set_size, int d_max);
void blst_p2_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar(
    blst_p2 *ret, const blst_p2_affine precomputation_points_list_3nh[], size_t npoints, int scalars[],
    digit_decomposition digit_conversion_hash_table[], blst_p2xyzz buckets[], int bucket_set_ascend[],
    int bucket_value_to_its_index[], size_t bucket_set_size, int d_max);
/* BGMW95 accumulation + running-sum reduction (multi_scalar.c:506-547); |digits| <= q/2 */
void blst_p1_tile_pippenger_BGMW95(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints,
                                   const int scalars[], const unsigned char booth_signs[], blst_p1xyzz buckets[],
                                   size_t q_exponent);
void blst_p2_tile_pippenger_BGMW95(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints,
                                   const int scalars[], const unsigned char booth_signs[], blst_p2xyzz buckets[],
                                   size_t q_exponent);

/* ---- sum of affine points (replaces ref src/bulk_addition.c:145-164, blst.h:224-225) ----
 * ret = sum of npoints affine points (all-zero = infinity).  Pointer rule of
 * bulk_addition.c:155: a NULL entry means "the point right after the previous one"
 * ({ptr, NULL} = one flat array).  On the GPU: entries spread over buckets of
 * weight 1, one lane per bucket, then the bucket reduction. */
void blst_p1s_add(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints);
void blst_p2s_add(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints);

/* ---- fixed-window MSM with a precomputed table (replaces ref src/multi_scalar.c:63-261,
 * blst.h:228-236 and :367-375; used by the C++ binding's P1_Affines / P2_Affines,
 * ref bindings/blst.hpp:362-430) ----
 * Same semantics and table layout as blst: table row i holds the canonical affine
 * multiples (k+1) P_i, k < 2^(wbits-1), wbits in [2, 14]; precompute may be called
 * with the points stored inside the output table (blst.hpp:383-393); the pointer
 * rules of blst apply to points[] and scalars[] (stride (nbits+7)/8).  On the GPU:
 * precompute builds every row by repeated mixed additions and one batch inversion
 * per point; mult sums the Booth-digit gathers of each window in parallel and
 * combines the window totals on the host.  The table is uploaded on every mult
 * call (the msm_wbits_ctx_* API below keeps it resident).  scratch is not used. */
size_t blst_p1s_mult_wbits_precompute_sizeof(size_t wbits, size_t npoints);
void blst_p1s_mult_wbits_precompute(blst_p1_affine table[], size_t wbits, const blst_p1_affine *const points[],
                                    size_t npoints);
size_t blst_p1s_mult_wbits_scratch_sizeof(size_t npoints);
void blst_p1s_mult_wbits(blst_p1 *ret, const blst_p1_affine table[], size_t wbits, size_t npoints,
                         const byte *const scalars[], size_t nbits, limb_t *scratch);
size_t blst_p2s_mult_wbits_precompute_sizeof(size_t wbits, size_t npoints);
void blst_p2s_mult_wbits_precompute(blst_p2_affine table[], size_t wbits, const blst_p2_affine *const points[],
                                    size_t npoints);
size_t blst_p2s_mult_wbits_scratch_sizeof(size_t npoints);
void blst_p2s_mult_wbits(blst_p2 *ret, const blst_p2_affine table[], size_t wbits, size_t npoints,
                         const byte *const scalars[], size_t nbits, limb_t *scratch);

/* ---- extension API: device-resident contexts (points uploaded once) ---- */
enum {
  MSM_OK = 0,
  MSM_E_ARG = -1,      /* bad argument */
  MSM_E_HIP = -2,      /* HIP runtime failure (message in msm_last_error) */
  MSM_E_NODEV = -3,    /* no gfx950 device visible */
  MSM_E_STATE = -4     /* context not ready (e.g. tables not built) */
};
typedef struct msm_ctx msm_ctx;
const char *msm_last_error(void);
/* void blst-named entry points on failure: 1 = print + abort (default), 0 = return
 * with the all-zero result and raise msm_error_pending(); returns the previous mode */
int msm_set_abort_on_error(int on);
/* nonzero if a blst-named call of this thread failed since the last query (clears it) */
int msm_error_pending(void);
int msm_device_count(void);
/* The VALU ceilings of `device`, measured now by register-resident kernels
 * (extension, no reference counterpart; bench.py prices its roofline with them
 * in the same run): out = {v_mad_u64_u32 lane-ops/s, Fp-mul/s, G1 xyzz madd/s
 * (the accumulation's loop body, rows in cache), device ms spent} */
int msm_valu_probe(int device, double out[4]);
/* Engines behind the blst-named entry points (no caller context: ref
 * multi_scalar.c:581-607) live in a process-wide pool per (device, kind,
 * window): a call leases one, a concurrent call creates another, and a returned
 * engine stays cached while the idle engines of its kind on its device hold at
 * most the cache limit of device memory (default 8 GiB); device memory is thus
 * bounded by the peak number of concurrent calls, not by the number of calling
 * threads.  release: frees every idle engine now.  stats: out[0] engines alive
 * (leased + idle), out[1] idle, out[2] device bytes held by idle engines.
 * set_limit returns the previous limit. */
void msm_release_engine_cache(void);
void msm_engine_cache_stats(size_t out[3]);
size_t msm_set_engine_cache_limit(size_t bytes);
/* Registered host tables (extension for the pointer-array tiles above).  The
 * reference driver hands the SAME host table to every CHES tile call, as one
 * pointer per entry into PRECOMPUTATION_POINTS_LIST_3nh (ref main_p1.cpp:233-236,
 * :279-282; 3 n h rows, built once by init_pippenger_CHES_q_over_5 :128-178).
 * Registering those rows once uploads them to the current device; afterwards a
 * tile call (blst_p{1,2}_tile_pippenger_d_CHES, _noindexhash, _BGMW95) whose
 * pointers all lie on row boundaries inside one registered table sends 4-B row
 * indices instead of gathering and uploading every 96/192-B row (1.2 GB per
 * G1 2^20 call).  Any pointer outside the table falls back to the gather.  A
 * point array registered the same way serves the plain drop-in: a flat
 * {ptr, NULL} blst_p{1,2}s_mult_pippenger / _tile_pippenger call whose npoints
 * points lie inside one registered table reads their device copy instead of
 * uploading 96/192 B per point (ref multi_scalar.c:549-607; callers that
 * multiply one SRS many times).  The
 * caller must not modify or free the rows while they are registered (as with
 * hipHostRegister).  Guard: up to 1024 rows at even strides (first and last
 * included) are sampled at registration; a call whose rows include a sample
 * that no longer matches the host memory re-uploads the table first, so a
 * reused or rewritten buffer is caught (an edit of one unsampled row is not).  group 1 (G1, blst_p1_affine rows) or 2 (G2); registering
 * an already registered base replaces it.  Returns MSM_OK or an error code. */
int msm_register_host_table(int group, const void *rows_affine, size_t nrows);
int msm_unregister_host_table(const void *rows_affine);
/* group 1 (G1) or 2 (G2); points in blst affine layout, host or device memory */
int msm_ctx_create(msm_ctx **ctx, int group, int device, int window_bits);
int msm_ctx_set_points(msm_ctx *ctx, const void *points_affine, size_t npoints, int points_on_device,
                       void *hip_stream);
/* scalars: npoints byte strings with the given stride (32 for blst_scalar arrays),
 * on host or device; ret: blst_p1 / blst_p2 Jacobian (host memory) */
int msm_ctx_mult(msm_ctx *ctx, void *ret, const byte *scalars, size_t stride, size_t nbits, int scalars_on_device,
                 void *hip_stream);
/* `count` MSMs over the context's points in one pipelined call (extension: the
 * shape of a prover committing many polynomials to one SRS; ref
 * main_p1.cpp:470-476 runs 5 scalar arrays back to back): scalar set k at
 * scalars + k * set_stride, each npoints strings of `stride` bytes; rets: count
 * Jacobians.  scalars_on_device = 0: the sets are uploaded first.  Results equal
 * `count` msm_ctx_mult calls. */
int msm_ctx_mult_batch(msm_ctx *ctx, void *rets, const byte *scalars, size_t stride, size_t set_stride,
                       size_t nbits, size_t count, int scalars_on_device, void *hip_stream);
int msm_ctx_set_profiling(msm_ctx *ctx, int on);
/* per-phase device ms of the last msm_ctx_mult (profiling on):
 * [digits, sort, accumulate, reduce, finalize, total] */
int msm_ctx_phase_times(const msm_ctx *ctx, float out[6]);
void msm_ctx_destroy(msm_ctx *ctx);

/* ---- CHES "nh + q/5" bucket-set method, device-resident precomputed table ----
 * Replaces the driver-level CHES path of ref main_p1.cpp: init_pippenger_CHES_q_over_5
 * (:128-178: bucket set, digit hash, table T[3(i h + j) + m - 1] = m q^j P_i) and
 * pippenger_variant_q_over_5_CHES (:192-246: MB digit conversion, accumulation
 * blst_p1_tile_pippenger_d_CHES, reduction :301-321).  The table is built on
 * the GPU (or uploaded) once; each mult takes n 32-byte scalars.  The result is
 * the true sum_i s_i P_i (the reference's last-element guard defect,
 * multi_scalar.c:461, is not reproduced; scalars >= r are reduced mod r where
 * the reference requires s < r). */
typedef struct msm_ches_ctx msm_ches_ctx;
/* the configuration of ref ches_config_files/config_file_n_exp_<n_exp>[_beta].h:
 * out = {n_exp, beta, q_exp, h, a_h, d_max, b_size, q_exp_bgmw, h_bgmw} */
int msm_ches_params(int n_exp, int beta, int out[9]);
int msm_ches_ctx_create(msm_ches_ctx **ctx, int group, int device, int n_exp, int beta);
/* explicit parameters (same 9-int layout; b_size 0 = not checked) */
int msm_ches_ctx_create_params(msm_ches_ctx **ctx, int group, int device, const int params[9]);
/* One MSM over several devices from one process (the reference is
 * single-device, its Go binding splits points x windows over CPU threads,
 * bindings/go/blst.go:2064-2197).  The points are split into ndev contiguous
 * balanced shards, shard g on devices[g] with its own rows of the reference
 * table (the rows of point i are contiguous in main_p1.cpp:155-172's layout, so
 * set/get/save/load_table keep that layout); each mult runs every shard
 * concurrently and folds the 144/288-B partials exactly on the host.  n_exp /
 * beta select the configuration of ONE SHARD (e.g. 2^21 points over 8 devices:
 * n_exp = 18).  Devices may repeat (several shards on one device).  Points,
 * table rows and scalars must be in host memory when ndev > 1. */
int msm_ches_ctx_create_multi(msm_ches_ctx **ctx, int group, const int *devices, int ndev, int n_exp, int beta);
int msm_ches_ctx_shards(const msm_ches_ctx *ctx);
/* 1 if this context's batches exchange their partials over RCCL (opt-in:
 * MSM_MULTI_RCCL=1 with shards on distinct devices; round 6 made it opt-in
 * until a run on several devices has checked it), 0 if each shard is read back */
int msm_ches_ctx_rccl_exchange(const msm_ches_ctx *ctx);
/* base points P_i (blst affine) -> T built on the GPU */
int msm_ches_ctx_build_table(msm_ches_ctx *ctx, const void *points_affine, size_t npoints, int on_device,
                             void *hip_stream);
/* a precomputed T (blst affine, 3 * npoints * h entries, main_p1.cpp:155-172 order) */
int msm_ches_ctx_set_table(msm_ches_ctx *ctx, const void *table_affine, size_t npoints, int on_device,
                           void *hip_stream);
/* T[first, first + count) in blst affine layout, to host memory */
int msm_ches_ctx_get_table(msm_ches_ctx *ctx, void *out_affine, size_t first, size_t count);
/* scalars: npoints 32-byte LE strings with the given stride (>= 32), host or device */
int msm_ches_ctx_mult(msm_ches_ctx *ctx, void *ret, const byte *scalars, size_t stride, int scalars_on_device,
                      void *hip_stream);
/* count MSMs over the same points: scalar set k (npoints strings of `stride` bytes)
 * at scalars + k * set_stride; rets: count Jacobians.  Pipelined on the device:
 * MSM k's latency-bound bucket-reduction tail runs on a second stream beside
 * MSM k+1's digit conversion, sort and accumulation (the batched-MSM shape of a
 * prover committing many polynomials to one SRS).  Results equal count calls
 * of msm_ches_ctx_mult.  Host scalars (scalars_on_device = 0) are copied set by
 * set inside the pipeline, each copy overlapping earlier MSMs' accumulations;
 * pass page-locked memory (hipHostMalloc / hipHostRegister) for the copies to
 * be asynchronous. */
int msm_ches_ctx_mult_batch(msm_ches_ctx *ctx, void *rets, const byte *scalars, size_t stride, size_t set_stride,
                            size_t count, int scalars_on_device, void *hip_stream);
/* table file cache (the reference rebuilds its tables on every run, main_p1.cpp:128-178):
 * 64-byte header + the rows in blst affine layout; load checks group/method/q/h */
int msm_ches_ctx_save_table(msm_ches_ctx *ctx, const char *path);
int msm_ches_ctx_load_table(msm_ches_ctx *ctx, const char *path);
int msm_ches_ctx_set_profiling(msm_ches_ctx *ctx, int on);
int msm_ches_ctx_phase_times(const msm_ches_ctx *ctx, float out[6]);
size_t msm_ches_ctx_bucket_count(const msm_ches_ctx *ctx);
/* accumulation lanes msm_ches_ctx_mult_batch runs (first shard's engine): 1 when
 * one accumulation fills the chip >= 3 wave-slot rounds deep, else 2-3 MSMs
 * accumulate side by side (MSM_BATCH_LANES overrides); 0 on a NULL ctx */
int msm_ches_ctx_batch_lanes(const msm_ches_ctx *ctx);
/* diagnostic (single-device contexts): digits + sort of nsets scalar sets in
 * DEVICE memory (set_stride bytes apart, 32-byte scalars), then the mean ms of
 * reps launches accumulating all nsets sets in one grid, alone on the stream */
int msm_ches_ctx_time_accumulation(msm_ches_ctx *ctx, const byte *scalars_dev, size_t set_stride, int nsets, int reps,
                                   float *ms_per_launch);
void msm_ches_ctx_destroy(msm_ches_ctx *ctx);

/* ---- BGMW95 fixed-base method, device-resident precomputed table ----
 * Replaces ref main_p1.cpp:94-122 init_pippenger_BGMW95 (table T[i h + j] = q^j P_i)
 * and :294-398 pippenger_variant_BGMW95 (signed radix-q digits in (-q/2, q/2],
 * r - s for large top digits, one set of q/2 buckets, tile
 * blst_p1_tile_pippenger_BGMW95 multi_scalar.c:506-547 + integrate :281-297).
 * q = 2^q_exp with q_exp * h >= 255; the reference's per-n choice is
 * msm_ches_params(...)[7..8] (EXPONENT_OF_q_BGMW95, h_BGMW95). */
typedef struct msm_bgmw_ctx msm_bgmw_ctx;
int msm_bgmw_ctx_create(msm_bgmw_ctx **ctx, int group, int device, int q_exp, int h);
int msm_bgmw_ctx_build_table(msm_bgmw_ctx *ctx, const void *points_affine, size_t npoints, int on_device,
                             void *hip_stream);
/* a precomputed T (blst affine, npoints * h entries, main_p1.cpp:109-119 order) */
int msm_bgmw_ctx_set_table(msm_bgmw_ctx *ctx, const void *table_affine, size_t npoints, int on_device,
                           void *hip_stream);
int msm_bgmw_ctx_get_table(msm_bgmw_ctx *ctx, void *out_affine, size_t first, size_t count);
int msm_bgmw_ctx_mult(msm_bgmw_ctx *ctx, void *ret, const byte *scalars, size_t stride, int scalars_on_device,
                      void *hip_stream);
int msm_bgmw_ctx_save_table(msm_bgmw_ctx *ctx, const char *path);
int msm_bgmw_ctx_load_table(msm_bgmw_ctx *ctx, const char *path);
int msm_bgmw_ctx_set_profiling(msm_bgmw_ctx *ctx, int on);
int msm_bgmw_ctx_phase_times(const msm_bgmw_ctx *ctx, float out[6]);
size_t msm_bgmw_ctx_bucket_count(const msm_bgmw_ctx *ctx);
void msm_bgmw_ctx_destroy(msm_bgmw_ctx *ctx);

/* ---- fixed-window (wbits) MSM with the table resident in HBM ---- */
typedef struct msm_wbits_ctx msm_wbits_ctx;
int msm_wbits_ctx_create(msm_wbits_ctx **ctx, int group, int device, int wbits);
/* base points (blst affine, host or device) -> the table, built on the GPU */
int msm_wbits_ctx_precompute(msm_wbits_ctx *ctx, const void *points_affine, size_t npoints, int on_device,
                             void *hip_stream);
/* a table in the reference layout (npoints << (wbits-1) blst affine rows), host or device */
int msm_wbits_ctx_set_table(msm_wbits_ctx *ctx, const void *table_affine, size_t npoints, int on_device,
                            void *hip_stream);
int msm_wbits_ctx_get_table(msm_wbits_ctx *ctx, void *out_affine, size_t first, size_t count);
/* scalars: npoints LE strings of `stride` bytes (>= (nbits+7)/8), host or device; low nbits bits */
int msm_wbits_ctx_mult(msm_wbits_ctx *ctx, void *ret, const byte *scalars, size_t stride, size_t nbits,
                       int scalars_on_device, void *hip_stream);
size_t msm_wbits_ctx_table_rows(const msm_wbits_ctx *ctx);
void msm_wbits_ctx_destroy(msm_wbits_ctx *ctx);

/* host setup logic of the CHES method (no device work):
 * bucket set of ref auxiliaryfunc.h:257-288 (returns |B|; out may be NULL) */
size_t msm_ches_bucket_set(int q, int a_h, int *out, size_t cap);
/* digit hash of ref main_p1.cpp:140-152, q+1 entries in the blst.h:253 layout */
int msm_ches_digit_table(int q, int a_h, digit_decomposition *out);

/* ---- boundary helpers (host; no blst symbols are redefined) ---- */
void msm_gen_scalars(byte *out32, size_t n, uint64_t seed);         /* BASELINE.md sec.3 SplitMix64 */
void msm_p1_fixed_points(blst_p1_affine *out, size_t n);            /* P_i = 2^(i+1) G1 (main_p1.cpp:52-66) */
void msm_p2_fixed_points(blst_p2_affine *out, size_t n);
/* P_{start+i} = 2^(start+i+1) G for i < n: the shard of the same point sequence */
void msm_p1_fixed_points_range(blst_p1_affine *out, size_t start, size_t n);
void msm_p2_fixed_points_range(blst_p2_affine *out, size_t start, size_t n);
void msm_p1_to_affine(blst_p1_affine *out, const blst_p1 *in);      /* e1.c:80-92 */
void msm_p2_to_affine(blst_p2_affine *out, const blst_p2 *in);
void msm_p1_compress(byte out[48], const blst_p1 *in);              /* e1.c:225-234 */
void msm_p2_compress(byte out[96], const blst_p2 *in);
void msm_p1_add(blst_p1 *out, const blst_p1 *a, const blst_p1 *b);  /* Jacobian, doubling aware */
void msm_p2_add(blst_p2 *out, const blst_p2 *a, const blst_p2 *b);

/* ---- device self-test entry points (parity tests of the Fp/Fp2/xyzz layers) ----
 * op: 0 mul, 1 add, 2 sub, 3 sqr; values in blst Montgomery layout */
int msm_test_field(int group, int op, const limb_t *a, const limb_t *b, limb_t *out, size_t n);
/* nseq sequences of len ops (point index | sign<<31, 0xffffffff = skip) -> per sequence
 * two blst Jacobians: acc and acc+acc (via the xyzz+xyzz path) */
int msm_test_xyzz(int group, const void *points_affine, size_t npoints, const uint32_t *ops, int len, size_t nseq,
                  void *out);

#ifdef __cplusplus
}
#endif
#endif
