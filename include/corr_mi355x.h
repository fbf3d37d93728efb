/*
 * corr_mi355x.h — C-ABI of libcorr_mi355x.so, the MI355X (gfx950) E-RAFT correlation hot path.
 *
 * Drop-in boundary for the reference CorrBlock (AhmedHumais/E-RAFT, model/corr.py:12-60).
 * Plain pointers and sizes only; no torch types.  Every pointer argument except the host
 * arrays of level pointers is DEVICE memory on the current HIP device; the caller allocates
 * everything (pyramid, outputs, gradients, workspace) and the library never allocates,
 * frees or synchronises.  All work is enqueued asynchronously on `stream` (a hipStream_t;
 * NULL = the default stream) and calls are graph-capturable.
 *
 * Layouts (fp32, C-contiguous), N = H*W, K = (2*radius+1)^2:
 *   fmap1, fmap2          [B][D][H][W]                       (corr.py:53-56)
 *   pyramid level l       B*N query maps of H_l x W_l cells, H_l = H>>l, W_l = W>>l
 *                         (corr.py:21-27, floor halving), each map TILED: 4x4-cell tiles of 64 B,
 *                         tiles row-major, cells row-major inside a tile:
 *                           cell (y, x) at ((y/4) * ceil(W_l/4) + x/4) * 16 + (y%4) * 4 + x%4,
 *                         corr_map_floats(H_l, W_l) = ceil(H_l/4) * ceil(W_l/4) * 16 floats per
 *                         map, maps consecutive (query q's map at q * corr_map_floats).  Cells
 *                         past W_l / H_l are padding (the builds may write them; never read).
 *                         Level pointers 16-byte aligned.  The reference's [B*N][H_l][W_l]
 *                         (corr.py's corr_pyramid) is corr_pyramid_export's output.
 *   coords                [B][2][H][W], ch0 = x, ch1 = y     (utils.py:24-27, corr.py:31)
 *   lookup output         [B][levels*K][H][W]                (corr.py:46-50)
 *   gradient pyramids     [B*N][H>>l][W>>l] row-major (corr_lookup_bwd, corr_pool_bwd,
 *                         corr_backward's scratch: the reference's layout; level 0 = dC [B*N][N])
 *
 * Return value: CORR_OK (0) or a negative CORR_E* code; corr_last_error() then returns a
 * thread-local message.  The reference performs no validation (torch raises inside
 * avg_pool2d / grid_sample); here bad arguments are rejected up front with CORR_EINVAL.
 * A level of height or width 1 is accepted and, like the reference (utils.py:11-12 divides
 * by W_l - 1 = 0), produces NaN for all of that level's channels and no gradient.
 */
#ifndef CORR_MI355X_H
#define CORR_MI355X_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CORR_OK 0
#define CORR_EINVAL -1       /* bad sizes / null or misaligned pointers            */
#define CORR_EUNSUPPORTED -2 /* valid for the reference, not built here (e.g. lookup_conv r != 4) */
#define CORR_EHIP -3         /* HIP launch / runtime error                          */

#define CORR_MAX_LEVELS 8
#define CORR_MAX_RADIUS 7

/* ABI version (major * 100 + minor).
 *   101: first ABI.
 *   102: corr_lookup_conv's weight argument is the opaque buffer written by
 *        corr_lookup_conv_weights (it was an fp32 [L*K][256] transpose under 101); callers
 *        built against 101 must check this version before calling it.
 *   103: CORR_BUILD_BF16X6, corr_build_region, corr_lookup_conv_bwd (the packed weight buffer
 *        grew: size it with corr_lookup_conv_weights_bytes()).
 *   104: corr_build_bwd_ex / corr_backward accept CORR_BUILD_BF16X6 (backward GEMMs on the exact
 *        bf16 split); E-RAFT's default backward for the BF16X6 build.
 *   200: the value pyramid (the builds' output, the lookups' input) is TILED (see Layouts;
 *        16-B aligned levels, corr_map_floats per map); corr_map_floats, corr_pyramid_export,
 *        corr_pyramid_import.  Gradient pyramids keep the reference layout.
 *   201: corr_backward's fused fold takes the separable closed form by default (dC within ~1e-7
 *        of the staged path, not bitwise); CORR_BACKWARD_EXACT_FOLD restores the bit-exact replay.
 *   202: the CORR_BUILD_BF16X6 backward GEMMs (corr_build_bwd_ex, corr_backward) give the fp32
 *        reference's results for non-finite inputs (+-inf where fp32 has +-inf; NaN only where it
 *        has NaN) instead of NaN for every output an infinity reaches. */
int corr_version(void);

/* Thread-local description of the last error on this thread ("" if none). */
const char *corr_last_error(void);

/* Floats of one query's tiled level map of H_l x W_l cells (ceil(H_l/4) * ceil(W_l/4) * 16). */
size_t corr_map_floats(int Hl, int Wl);

/*
 * The tiled pyramid <-> the reference's layout.  corr_pyramid_export writes every level as
 * [BN][H>>l][W>>l] row-major (the reference's corr_pyramid[l] viewed [B*N, 1, H_l, W_l],
 * corr.py:16,24,27,36); corr_pyramid_import tiles such levels into a pyramid (padding cells
 * zeroed), so a pyramid computed elsewhere can be looked up.  BN = B * NQ query maps; `pyr`,
 * `src`, `out` are host arrays of `levels` device pointers; the tiled side 16-B aligned.
 */
int corr_pyramid_export(const float *const *pyr, int BN, int H, int W, int levels, float *const *out, void *stream);
int corr_pyramid_import(const float *const *src, int BN, int H, int W, int levels, float *const *pyr, void *stream);

/*
 * All-pairs correlation + average-pool pyramid.  Replaces CorrBlock.__init__
 * (model/corr.py:13-27) together with CorrBlock.corr (model/corr.py:52-60):
 *   pyr[0][b*N + n](y, x) = sum_d fmap1[b][d][n] * fmap2[b][d][y*W + x] / sqrt(float(D))
 *   pyr[l][q](y, x)       = avg_pool2d(pyr[l-1], 2, stride 2)[q](y, x)   (floor)
 * (cell (y, x) of query q's tiled map, see Layouts.)  `pyr` is a HOST array of `levels` device
 * pointers.  levels == 1 gives CorrBlock.corr's [B,H,W,1,H,W] volume (export it for that view).  fp32 in / fp32 MFMA accumulate / fp32 out (CORR_BUILD_FP32;
 * corr_build_ex selects the faster CORR_BUILD_BF16X6, no less accurate, or CORR_BUILD_F16X3).
 */
int corr_build(const float *fmap1, const float *fmap2, int B, int D, int H, int W, int levels,
               float *const *pyr, void *stream);

/*
 * Build algorithms for corr_build_ex (same outputs, same pyramid arithmetic; they differ only
 * in how the fp32 dot products are formed — all accumulate in fp32):
 *   CORR_BUILD_FP32   fp32 operands on v_mfma_f32_32x32x2_f32 (the corr_build path).
 *   CORR_BUILD_BF16X6 each fp32 feature is split EXACTLY into three bf16 pieces, x = hi + mid +
 *                     lo (bf16 keeps fp32's exponent range: no scale, no flush — the one floor
 *                     is lo's bf16 subnormal range, |x| < ~2^-110); six bf16 MFMAs per product
 *                     (every piece pair of weight >= 2^-16: lo*hi + hi*lo + mid*mid + mid*hi +
 *                     hi*mid + hi*hi) into two fp32 accumulators (hi*hi; the five smaller ones),
 *                     added once.  The dropped terms are <= 2^-23 of |x_t x_q| and the main
 *                     accumulator rounds D/32 times per dot product (an fp32 fmaf chain: D
 *                     times): no narrower than CORR_BUILD_FP32 (checked per query row against
 *                     an fp64 oracle).  +-inf features split as (inf, 0, 0); a result whose
 *                     hi*hi sum is infinite is that sum, so infinities and NaNs land where the
 *                     fp32 build puts them (one exception: an infinity against a nonzero feature
 *                     below bf16's range, |x| < 2^-133, whose hi is 0: NaN where fp32 gives inf).
 *                     Needs a workspace for the split operands.
 *                     ~2x faster than CORR_BUILD_FP32 on gfx950.
 *   CORR_BUILD_F16X3  each fp32 feature x of pixel n is split as 2^e_n * (hi + lo), f16 hi/lo,
 *                     e_n putting the pixel's largest |x| in [2^14, 2^15); three f16 MFMAs
 *                     (hi*hi + hi*lo + lo*hi) per product into one fp32 accumulator.  Each
 *                     feature is carried to 2^-22 relative (fp32: 2^-24), and each product to
 *                     ~2^-21; features below 2^-38 of their pixel's largest flush to zero.
 *                     Needs a workspace for the packed operands.  ~1.5-1.7x faster on gfx950.
 */
#define CORR_BUILD_FP32 0
#define CORR_BUILD_F16X3 1
#define CORR_BUILD_BF16X6 2
/* Measurement only (OR-ed into CORR_BUILD_F16X3 / _BF16X6): run just one of its two kernels — the
 * operand pack, or the MFMA build from a workspace that already holds this pair's pack — so a
 * benchmark can time each kernel on its own.  The pyramid is complete only after both. */
#define CORR_BUILD_ONLY_PACK 0x100
#define CORR_BUILD_ONLY_MFMA 0x200

/* Bytes of device workspace corr_build_ex(algo, ...) needs (0 for CORR_BUILD_FP32;
 * (size_t)-1 if the algorithm does not support D). */
size_t corr_build_workspace(int algo, int B, int D, int NQ, int H, int W);

/*
 * corr_build_rows with an explicit algorithm and caller-allocated workspace (>= the size
 * corr_build_workspace returns; it may be reused across calls on the same stream).
 * CORR_EUNSUPPORTED if `algo` cannot handle D.
 */
int corr_build_ex(int algo, const float *fmap1_rows, int NQ, const float *fmap2, int B, int D,
                  int H, int W, int levels, float *const *pyr, void *workspace,
                  size_t workspace_bytes, void *stream);

/*
 * One target-row region of corr_build_ex (CORR_BUILD_BF16X6 only): the pyramid entries of target
 * rows [y0, y1) — level l rows [y0 >> l, ceil(y1 / 2^l)) of every query's maps — from a slab
 * fmap2_rows [B][D][y1 - y0][W] holding just those rows of fmap2.  y0 a multiple of 8, y1 a
 * multiple of 8 or H, levels <= 4.  Calls over a partition of [0, H) with the same workspace
 * give the bits of one corr_build_ex call; the first call of a build sets
 * CORR_REGION_PACK_QUERIES (the query operand is packed into the workspace once and reused).
 * Lets a row-sharded caller build from fmap2 chunks as their broadcast arrives.
 */
#define CORR_REGION_PACK_QUERIES 1
int corr_build_region(int algo, const float *fmap1_rows, int NQ, const float *fmap2_rows, int y0, int y1, int B,
                      int D, int H, int W, int levels, float *const *pyr, void *workspace, size_t workspace_bytes,
                      int flags, void *stream);

/*
 * Window lookup.  Replaces CorrBlock.__call__ (model/corr.py:29-50) and bilinear_sampler
 * (model/utils.py:7-21):
 *   out[b][l*K + i*(2r+1) + j][h][w] = grid_sample(pyr[l][b*N + h*W + w],
 *        (x/2^l + i - r, y/2^l + j - r), bilinear, zeros, align_corners=True)
 * with (x, y) = coords[b][:][h][w].  The slow window index i moves x (corr.py:37-43).
 * Bit-identical to the reference on identical pyramids.  `pyr` is a host array.
 */
int corr_lookup(const float *const *pyr, const float *coords, int B, int H, int W, int levels,
                int radius, float *out, void *stream);

/*
 * Input-gradient of corr_lookup (autograd of model/utils.py:15; coords carry no gradient,
 * model/eraft.py:128).  ACCUMULATES into grad_pyr (host array of device pointers, same
 * shapes as the pyramid; zero it once before the first lookup of a build).  Deterministic:
 * a query's contributions stay inside its own map, summed in a fixed order, no atomics.
 */
int corr_lookup_bwd(const float *coords, const float *grad_out, int B, int H, int W, int levels,
                    int radius, float *const *grad_pyr, void *stream);

/*
 * avg_pool2d backward chain (autograd of model/corr.py:25-27), in place, coarse -> fine:
 *   grad_pyr[l-1][q][2y+a][2x+c] += grad_pyr[l][q][y][x] * 0.25      (l = levels-1 .. 1)
 * Afterwards grad_pyr[0] holds dLoss/dcorr.  BN = B*H*W query maps.
 */
int corr_pool_bwd(float *const *grad_pyr, int BN, int H, int W, int levels, void *stream);

/* Bytes of device workspace corr_build_bwd needs for these sizes. */
size_t corr_build_bwd_workspace(int B, int D, int H, int W);

/*
 * Backward of the all-pairs product and its 1/sqrt(D) scale (autograd of
 * model/corr.py:58-60).  grad_c: [B*N][N] (= grad_pyr[0] after corr_pool_bwd);
 *   dfmap1[b][d][n] = sum_m grad_c[b*N+n][m] * fmap2[b][d][m] / sqrt(D)
 *   dfmap2[b][d][m] = sum_n fmap1[b][d][n] * grad_c[b*N+n][m] / sqrt(D)
 * Both outputs are OVERWRITTEN.  Deterministic (split-K partial slabs summed in order).
 */
int corr_build_bwd(const float *grad_c, const float *fmap1, const float *fmap2, int B, int D,
                   int H, int W, float *dfmap1, float *dfmap2, void *workspace,
                   size_t workspace_bytes, void *stream);

/*
 * Row-slab variants, for query-row sharding across GPUs (no reference counterpart: the
 * reference has no multi-GPU CorrBlock).  The queries are NQ consecutive
 * pixels of fmap1 — a block of whole rows, NQ = rows*W — while the targets are all H*W
 * pixels of fmap2:
 *   fmap1_rows [B][D][NQ]; pyramid level l: B*NQ tiled maps of (H>>l) x (W>>l) cells;
 *   coords_rows [B][2][NQ]; out_rows [B][levels*K][NQ]; grad_c [B*NQ][H*W].
 * Every query's arithmetic is identical to the full-size call, so a row partition
 * reproduces the unsharded results bit for bit.  corr_build_bwd_rows writes this slab's
 * dfmap1 rows and its PARTIAL dfmap2 (sum it over the slabs, e.g. with an all-reduce).
 * The reference-shaped functions above are these with NQ = H*W.
 */
int corr_build_rows(const float *fmap1_rows, int NQ, const float *fmap2, int B, int D, int H,
                    int W, int levels, float *const *pyr, void *stream);
int corr_lookup_rows(const float *const *pyr, const float *coords_rows, int B, int NQ, int H,
                     int W, int levels, int radius, float *out_rows, void *stream);
int corr_lookup_bwd_rows(const float *coords_rows, const float *grad_out_rows, int B, int NQ,
                         int H, int W, int levels, int radius, float *const *grad_pyr,
                         void *stream);
size_t corr_build_bwd_rows_workspace(int B, int D, int NQ, int H, int W);
int corr_build_bwd_rows(const float *grad_c, const float *fmap1_rows, int NQ, const float *fmap2,
                        int B, int D, int H, int W, float *dfmap1_rows, float *dfmap2,
                        void *workspace, size_t workspace_bytes, void *stream);

/*
 * Backward GEMMs with an explicit algorithm (the corr_build_ex counterpart of
 * corr_build_bwd_rows; same outputs and contract).  CORR_BUILD_FP32 is corr_build_bwd_rows;
 * CORR_BUILD_BF16X6 splits every element of F1 / F2 / dC EXACTLY into three bf16 pieces while
 * staging it (no scales, no maxima; the one floor as for the build: |x| < ~2^-110) and runs the
 * six piece products of weight >= 2^-16 per product on the bf16 MFMA into one fp32 accumulator
 * (6 roundings per 16 k, an fp32 fmaf chain 16): every element within (3 + 6 ceil(K/16) + splits)
 * u sum|ab| (an fp32 dot product: K u sum|ab|), worst and mean row error below the fp32 GEMMs',
 * checked against fp64 — but with one accumulator not every single row (unlike the build's).
 * Non-finite inputs give the fp32 reference's results: an output the split makes NaN (an
 * infinite element meets zero pieces: inf * 0) is recomputed by the split-K reduce as the
 * reference computes it (dC / sqrt(D), then an fp32 dot product), so it becomes +-inf where
 * fp32 has +-inf and stays NaN where fp32 has NaN; finite inputs are unaffected
 * (tests/test_gpu_parity.py::test_build_bwd_bf16x6_inf_matches_fp32).
 * CORR_BUILD_F16X3 packs F1, F2 (per feature row d) and dC (per query
 * row for dfmap1, per target column for dfmap2) as 2^e (hi + lo) f16 pairs and runs three f16
 * MFMAs per product (~2^-22 relative: narrower than fp32).  Split-K partial sums are reduced in
 * split order (deterministic).
 * Workspace: corr_build_bwd_ex_workspace(algo, ...) bytes ((size_t)-1: unknown algo).
 * Replaces the autograd of model/corr.py:58-60 (bmm + division by sqrt(D)).
 */
size_t corr_build_bwd_ex_workspace(int algo, int B, int D, int NQ, int H, int W);
int corr_build_bwd_ex(int algo, const float *grad_c, const float *fmap1_rows, int NQ,
                      const float *fmap2, int B, int D, int H, int W, float *dfmap1_rows,
                      float *dfmap2, void *workspace, size_t workspace_bytes, void *stream);

/*
 * The backward of one build and all its lookups in three launches (autograd of model/corr.py:
 * 25-27, 45, 58-60 for the whole GRU loop at once; coords carry no gradient, eraft.py:128).
 * coords_rows / grad_out_rows: HOST arrays of T device pointers, the lookups' coords and upstream
 * gradients ([B][2][NQ], [B][levels*K][NQ]), accumulated in this order.
 *   corr_lookup_bwd_multi: the T lookups' input-gradients into grad_pyr, which it OVERWRITES
 *     (zero-initialised inside the kernel: no memset; each workgroup's RMWs stay L2-resident).
 *     Per cell G = ((0 + S_0) + S_1) + ... with S_t lookup t's scatter-order sum: bit-identical to
 *     zeroing grad_pyr and calling corr_lookup_bwd_rows for t = 0..T-1.
 *   corr_pool_fold: the avg_pool2d backward of every level folded into level 0 in place (one pass;
 *     bit-identical to corr_pool_bwd): afterwards grad_pyr[0] = dLoss/dcorr.
 *   corr_backward: both, then the two GEMMs of corr_build_bwd_ex; grad_pyr is scratch (left =
 *     dC in level 0), the outputs dfmap1_rows / dfmap2 as corr_build_bwd_ex.  When the
 *     workgroup's LDS image fits (levels <= 4, T <= 32, BQ = 64 / pow2ceil(2r+3) queries' maps of
 *     every level in 160 KiB: e.g. r = 4 up to 60x80 fmaps), the lookups and the fold run as ONE
 *     kernel whose gradient maps live in LDS and which writes only dC (plus dC's row maxima and
 *     per-workgroup column maxima for the F16X3 packs; BF16X6 needs none); otherwise corr_lookup_bwd_multi +
 *     corr_pool_fold.  At radius 4 the fused kernel sums a window's cells separably (the column's
 *     x-taps first, then the y-taps: the same (tap, corner) terms per cell with the reference's
 *     per-tap weights, rounded in another order — dC within ~1e-7 norm-relative of the staged
 *     path; windows whose taps are not all on a regular grid, e.g. the cold-start integer grid,
 *     by the general form with four slots per tap; a window with a corner outside its
 *     neighbourhood, or in a wave holding a non-finite upstream gradient, by the reference's
 *     sequential scatter, so infinities give the staged path's inf / NaN cells);
 *     algo | CORR_BACKWARD_EXACT_FOLD makes it replay grid_sampler_2d_backward's
 *     per-tap products instead, bit-identical to corr_lookup_bwd_multi + corr_pool_fold (as every
 *     other radius and the non-fused path always are).  Workspace: corr_backward_workspace
 *     (radius sizes the column-maxima partials; the flag does not change it).
 */
#define CORR_BACKWARD_EXACT_FOLD 0x400
int corr_lookup_bwd_multi(const float *const *coords_rows, const float *const *grad_out_rows, int T, int B,
                          int NQ, int H, int W, int levels, int radius, float *const *grad_pyr, void *stream);
int corr_pool_fold(float *const *grad_pyr, int B, int NQ, int H, int W, int levels, void *stream);
size_t corr_backward_workspace(int algo, int B, int D, int NQ, int H, int W, int radius);
int corr_backward(int algo, const float *const *coords_rows, const float *const *grad_out_rows, int T,
                  const float *fmap1_rows, int NQ, const float *fmap2, int B, int D, int H, int W, int levels,
                  int radius, float *const *grad_pyr, float *dfmap1_rows, float *dfmap2, void *workspace,
                  size_t workspace_bytes, void *stream);

/*
 * Warm-start forward splat.  Replaces forward_interpolate_pytorch (utils/image_utils.py:52-83)
 * with grid_sample_values (:10-50): flow [B][2][H][W] -> out [B][2][H][W], every source pixel
 * splatted to its floor / ceil neighbours with bilinear weights, out = sum(z w) / (sum(w) +
 * 1e-15).  Deterministic and bit-identical to the reference's CPU put_(accumulate=True) order
 * (corner-major, source order; an integer coordinate's floor == ceil corner counts twice, as
 * in the reference).  Workspace: corr_forward_splat_workspace(B, H, W) bytes.
 */
size_t corr_forward_splat_workspace(int B, int H, int W);

/*
 * Lookup fused with its consumer, BasicMotionEncoder's cor = relu(convc1(corr))
 * (model/update.py:68,75; a 1x1 convolution L*(2r+1)^2 -> 256): the window lookup of
 * corr_lookup into an on-chip tile, then out[b][o][h][w] = (relu?)(bias[o] +
 * sum_c weight[o][c] * corr[b][c][h][w]) on the bf16 MFMA with CORR_BUILD_BF16X6's exact
 * three-piece split (six products per fp32 product, no scales: no narrower than fp32).  The weight (convc1.weight viewed [256][L*K], fp32) is split once
 * per weight version by corr_lookup_conv_weights into a corr_lookup_conv_weights_bytes() buffer;
 * out [B][256][H][W].  radius 4, levels <= 4 (E-RAFT); CORR_EUNSUPPORTED otherwise.  This call
 * is the forward; corr_lookup_conv_bwd below is its training backward.
 */
size_t corr_lookup_conv_weights_bytes(void);
int corr_lookup_conv_weights(const float *weight, int out_channels, int in_channels, void *packed, void *stream);
int corr_lookup_conv(const float *const *pyr, const float *coords, int B, int H, int W,
                     int levels, int radius, const void *packed_weight, const float *bias, int relu,
                     float *out, void *stream);

/*
 * Training backward of corr_lookup_conv (autograd of update.py:68,75 through corr.py:29-50).
 * grad_out = dL/d out [B][256][H][W]; with relu, g' = grad_out where out > 0 (or out is NaN),
 * else 0 (torch's threshold backward; `out` is the forward's output, unused without relu).
 *   grad_weight [256][levels*K] = sum_{b,n} g'[b][o][n] lookup[b][c][n]    (OVERWRITTEN)
 *   grad_bias   [256]           = sum_{b,n} g'[b][o][n]                    (OVERWRITTEN)
 *   grad_lookup [B][levels*K][H][W] = sum_o weight[o][c] g'[b][o][n]  — the lookup's upstream
 *               gradient, to be passed to corr_backward / corr_lookup_bwd like a plain lookup's
 * Any of the three may be NULL (not computed).  The lookup is recomputed on chip (bit-identical
 * to corr_lookup's values) and never written.  Both products run on the bf16 MFMA with the
 * exact three-piece split of CORR_BUILD_BF16X6 (six products per fp32 product, no scales);
 * dW and the bias sum per-workgroup partials in a fixed order (deterministic).  packed_weight
 * from corr_lookup_conv_weights; workspace of corr_lookup_conv_bwd_workspace(B, H, W, levels)
 * bytes (16-B aligned) when grad_weight or grad_bias is requested.  radius 4, levels <= 4.
 */
size_t corr_lookup_conv_bwd_workspace(int B, int H, int W, int levels);
int corr_lookup_conv_bwd(const float *const *pyr, const float *coords, int B, int H, int W, int levels, int radius,
                         const void *packed_weight, const float *out, int relu, const float *grad_out,
                         float *grad_weight, float *grad_bias, float *grad_lookup, void *workspace,
                         size_t workspace_bytes, void *stream);

/*
 * DSEC event -> voxel grid.  Replaces VoxelGrid.convert (utils/dsec_utils.py:26-64) as the DSEC
 * loader calls it (loader/loader_dsec.py:245-257): events as float32 device arrays x, y, t
 * (t in [0, 1], ascending), p in {0, 1}; out [C][H][W].  Bilinear in x and y, nearest-lower
 * bin in t (the reference's t loop is commented out); the raw grid is bit-identical to the
 * reference run single-threaded (main.py:2-5) — deterministic, no float atomics.  normalize:
 * nonzero cells -> (v - mean) / std (unbiased std; fp64 statistics, tolerance-level).
 * Workspace: corr_voxel_grid_workspace(n_events, C, H, W) bytes.
 */
size_t corr_voxel_grid_workspace(int n_events, int C, int H, int W);
int corr_voxel_grid(const float *x, const float *y, const float *t, const float *p, int n_events,
                    int C, int H, int W, int normalize, float *out, void *workspace,
                    size_t workspace_bytes, void *stream);

/*
 * MVSEC event -> voxel grid.  Replaces EventSequenceToVoxelGrid_Pytorch.__call__
 * (utils/transformers.py:36-126), the representation of loader/loader_mvsec_flow.py:35:
 * events [n_events][4] float64 device rows (t, x, y, p), as the loader's event_sequence.features
 * .astype('float') holds them (t ascending in practice; t_0 = row 0, t_end = the last row);
 * out [C][H][W].  Bilinear in t: t_n = (C-1)(t - t_0)/(t_end - t_0) (fp64), each event adds
 * p(1 - dt) at bin floor(t_n) and p dt at floor(t_n) + 1 (p = 0 -> -1, dt rounded to fp32),
 * at flat index trunc(x) + trunc(y) W + bin H W.  The raw grid is bit-identical to the
 * reference's two index_add_ passes (left then right, event order) — deterministic, no float
 * atomics.  An entry whose flat index falls outside the grid is dropped (the reference raises).
 * normalize: as corr_voxel_grid.  Workspace: corr_voxel_grid_tbilinear_workspace(...) bytes.
 */
size_t corr_voxel_grid_tbilinear_workspace(int n_events, int C, int H, int W);
int corr_voxel_grid_tbilinear(const double *events, int n_events, int C, int H, int W,
                              int normalize, float *out, void *workspace, size_t workspace_bytes,
                              void *stream);

/*
 * Convex upsampling of the 1/8-resolution flow after every GRU iteration.  Replaces
 * ERAFT.upsample_flow (model/eraft.py:75-86): softmax over the 9 taps of mask
 * [N][9*64][h][w], weighted sum of the zero-padded 3x3 neighbourhood of 8*flow [N][2][h][w]
 * -> out [N][2][8h][8w], in one pass (fp32; tolerance-level parity, the reference's
 * reduction order is ATen's).
 */
int corr_convex_upsample(const float *flow, const float *mask, int N, int h, int w, float *out,
                         void *stream);
/*
 * Backward of corr_convex_upsample (autograd of model/eraft.py:75-86 w.r.t. flow and mask):
 * grad_out [N][2][8h][8w] -> dflow [N][2][h][w], dmask [N][576][h][w] (both overwritten).
 * Softmax backward p_k (dv_k - sum p dv) per sub-pixel; dflow gathers 8 * sum p_k G over the
 * sub-pixels and taps that read each coarse pixel.  Workspace: the per-tap partial sums,
 * corr_convex_upsample_bwd_workspace(N, h, w) bytes.  fp32, tolerance-level parity.
 */
size_t corr_convex_upsample_bwd_workspace(int N, int h, int w);
int corr_convex_upsample_bwd(const float *flow, const float *mask, const float *grad_out, int N, int h, int w,
                             float *dflow, float *dmask, void *workspace, size_t workspace_bytes, void *stream);
int corr_forward_splat(const float *flow, int B, int H, int W, float *out, void *workspace,
                       size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* CORR_MI355X_H */
