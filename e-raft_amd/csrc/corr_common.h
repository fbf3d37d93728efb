// Internal definitions shared by the gfx950 correlation kernels (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/corr_mi355x.h"

namespace corr {

// Host-side launch arguments carrying the per-level pointers by value (no device-side
// pointer table to allocate).
struct LevelPtrs {
    float *p[CORR_MAX_LEVELS];
};
struct ConstLevelPtrs {
    const float *p[CORR_MAX_LEVELS];
};

// ---------------------------------------------------------------------------------------
// Pyramid layout (the build's output, the lookups' input).  Every query's level-l map
// (H_l x W_l cells, corr.py:21-27) is stored as tiles of 4 rows x kTileW cells, tiles row-major
// over the map, cells row-major inside a tile:
//     cell (y, x) at ((y >> 2) * TC + x / kTileW) * 4 kTileW + (y & 3) * kTileW + x % kTileW,
//     TC = ceil(W_l / kTileW) tiles per map row, a map = ceil(H_l / 4) * TC * 4 kTileW floats.
// A query's maps are contiguous (level by level, query after query), so a row slab of queries
// is a contiguous range, as before.  The cells past W_l / H_l in the last tile column / row are
// padding: the builds may write anything there and nothing reads them (the lookups zero
// out-of-map cells themselves).  A (2r+2)^2 window then spans a few whole tiles (one 16-B
// tile-row chunk per lane and window row in the gather), where row-major maps gave one 40-B
// segment per window row in a different line (profiles/r05f_kbench_lookup_tiled.txt).  The
// reference layout [B*N, 1, H_l, W_l] is materialised on demand (corr_pyramid_export).
constexpr int kTileW = 4;  // 64-B tiles (profiles/r05i_kbench_*_tw{4,8}.txt: 4 x 8 bands cost the lookups more)
__host__ __device__ inline int map_tiles(int n) { return (n + 3) >> 2; }  // 4-cell groups (tile rows, 16-B chunks)
__host__ __device__ inline int map_tcols(int Wl) { return (Wl + kTileW - 1) / kTileW; }
__host__ __device__ inline size_t map_floats(int Hl, int Wl) {
    return (size_t)map_tiles(Hl) * map_tcols(Wl) * 4 * kTileW;
}
__host__ __device__ inline unsigned map_cell(int y, int x, int TC) {
    return (unsigned)((((y >> 2) * TC + x / kTileW) * 4 + (y & 3)) * kTileW + x % kTileW);
}
// Offset of the 16-B chunk holding cells (y, 4t .. 4t + 3).
__host__ __device__ inline unsigned map_row4(int y, int t, int TC) { return map_cell(y, 4 * t, TC); }

// Sum of a three-piece split product's two accumulators (hi*hi; the five smaller piece products).
// An infinite feature splits as (inf, 0, 0), so the small products hold inf * 0 = NaN where fp32
// gives inf * x = inf; the leading sum already carries fp32's inf / NaN status (inf * 0 and
// opposite infinities reach it as NaN), so an infinite leading sum is the result.
__device__ inline float split_sum(float hi, float lo) { return __builtin_isinf(hi) ? hi : hi + lo; }

// The bf16x6 backward GEMMs' non-finite rule.  C[b][i][j] = sum_k A[b][i][k] Bm[b][j][k] / s runs
// on exact three-piece bf16 splits into ONE accumulator, so an infinite operand element meets
// zero pieces of the other operand (inf * 0 = NaN) and every output it reaches comes out NaN
// where the reference's fp32 matmul gives +-inf (autograd of model/corr.py:58-60).  The split-K
// reduce (and the direct epilogue) therefore recompute exactly the outputs that came out NaN as
// the reference does — dmatmul = dC / sqrt(D) elementwise, then a plain fp32 dot product — so
// NaN stays NaN where fp32 has one (a NaN operand, inf * 0, opposite infinities) and the rest
// become fp32's +-inf.  Finite inputs never reach it (no NaN), so their bits are unchanged.
// K = 0: off (the fp32-operand and f16x3 GEMMs).
struct NanFix {
    const float *A = nullptr, *Bm = nullptr;
    long a_sb = 0, a_sr = 0, b_sb = 0, b_sr = 0, b_sk = 0;
    int NI = 0, NJ = 0, K = 0;
    float s = 1.f;  // sqrt(D): the reference divides dC by it before the matmul
};
// (inlined: a call would give every kernel that holds it a call stack — 336 B of scratch and
// +24 % on the backward GEMMs, +120 % on the reduce when the fixup was a __noinline__ function)
__device__ __forceinline__ float nanfix_dot(const NanFix &f, int b, int i, int j) {
    const float *a = f.A + (size_t)b * f.a_sb + (size_t)i * f.a_sr;
    const float *m = f.Bm + (size_t)b * f.b_sb + (size_t)j * f.b_sr;
    float acc = 0.f;
    for (int k = 0; k < f.K; ++k) acc = fmaf(a[k], m[(size_t)k * f.b_sk] / f.s, acc);
    return acc;
}
// The same for flat output index e of C [B][NI][NJ].  Only the split-K reduces call these (the
// separate reduce kernel and a GEMM's appended tail-reduce workgroups); the bf16x6 GEMMs always
// take the slab path, so no GEMM epilogue carries the fixup.
__device__ __forceinline__ float nanfix_flat(const NanFix &f, size_t e) {
    const size_t per = (size_t)f.NI * f.NJ;
    const size_t r = e % per;
    return nanfix_dot(f, (int)(e / per), (int)(r / f.NJ), (int)(r % f.NJ));
}

// Set the thread-local error and return `code`.
int fail(int code, const char *fmt, ...);
// Map a HIP status to CORR_OK / CORR_EHIP (recording the message).
int hip_status(hipError_t e, const char *what);

// Launch entry points implemented in the .hip translation units (all asynchronous).
// NQ = query pixels per batch item (H*W for the reference shape, rows*W for a row slab);
// H, W = the target map (fmap2) whose pyramid levels are [B*NQ][H>>l][W>>l].
hipError_t launch_build(const float *f1, int NQ, const float *f2, int B, int D, int H, int W,
                        int levels, const LevelPtrs &pyr, hipStream_t s);
hipError_t launch_pool_levels(const LevelPtrs &pyr, int l_from, int levels, long BN, int H,
                              int W, hipStream_t s);
hipError_t launch_lookup(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H,
                         int W, int levels, int radius, float *out, hipStream_t s);
hipError_t launch_lookup_bwd(const float *coords, const float *grad_out, int B, int NQ, int H,
                             int W, int levels, int radius, const LevelPtrs &gpyr, hipStream_t s);
hipError_t launch_pool_bwd(const LevelPtrs &gpyr, long BN, int H, int W, int levels,
                           hipStream_t s);
hipError_t launch_lookup_bwd_multi(const float *const *coords, const float *const *grad_out, int T, int B, int NQ,
                                   int H, int W, int levels, int radius, const LevelPtrs &gpyr, hipStream_t s);
int lookup_bwd_fold_groups(int NQ, int radius);
// Row |max| of two row-major operands [B][rows][cols[t]] (the backward GEMMs' F2 and F1 row
// maxima), computed by extra workgroups appended to a launch's grid; out[t] gets float bits.
struct FoldRowMax {
    const float *x[2];
    unsigned *out[2];
    int cols[2];
    int rows;  // 0: none
};
// exact: regular windows replay grid_sampler_2d_backward's per-tap products bit for bit (else the
// separable closed form at radius 4, corr_backward's default).
hipError_t launch_lookup_bwd_fold(const float *const *coords, const float *const *grad_out, int T, int B, int NQ,
                                  int H, int W, int levels, int radius, float *dc, unsigned *rmax, unsigned *cmax,
                                  float *cpart, hipStream_t s, const FoldRowMax &rm = FoldRowMax{},
                                  bool exact = true);
size_t backward_workspace(int algo, int B, int D, int NQ, int H, int W, int radius);
hipError_t launch_pool_fold(const LevelPtrs &gpyr, int B, int NQ, int H, int W, int levels, void *ws, int D,
                            hipStream_t s);
hipError_t launch_backward(int algo, const float *const *coords, const float *const *grad_out, int T,
                           const float *f1, int NQ, const float *f2, int B, int D, int H, int W, int levels, int radius,
                           const LevelPtrs &gpyr, float *df1, float *df2, void *ws, hipStream_t s);
// The f16-split build (corr_build_split.hip): pack kernel + f16 MFMA kernel, operands in `ws`.
size_t build_split_workspace(int B, int D, int NQ, int H, int W);
bool build_split_supported(int D);
hipError_t launch_build_split(const float *f1, int NQ, const float *f2, int B, int D, int H, int W,
                              int levels, const LevelPtrs &pyr, void *ws, hipStream_t s, int part = 0);
// The bf16 three-piece build (corr_build_bf16.hip): pack kernel + bf16 MFMA kernel.
size_t build_bf16_workspace(int B, int D, int NQ, int H, int W);
hipError_t launch_build_bf16(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, int levels,
                             const LevelPtrs &pyr, void *ws, hipStream_t s, int part = 0);
hipError_t launch_build_bf16_region(const float *f1, int NQ, const float *f2_rows, int y0, int y1, int B, int D,
                                    int H, int W, int levels, const LevelPtrs &pyr, void *ws, bool pack_q,
                                    hipStream_t s);
// Ordered split-K sum + 1/sqrt(D) of [splits][per] partial slabs into C (corr_bwd.hip).
// fix: the bf16x6 GEMMs' NaN recompute (NanFix), or null.
hipError_t launch_splitk_reduce(const float *ws, float *C, int splits, size_t per, float sD, hipStream_t s,
                                bool vec4 = true, const NanFix *fix = nullptr);
size_t build_bwd_split_workspace(int B, int D, int NQ, int H, int W);
hipError_t launch_build_bwd_split(const float *grad_c, const float *f1, int NQ, const float *f2, int B, int D, int H,
                                  int W, float *df1, float *df2, void *ws, hipStream_t s, bool bf);
hipError_t launch_convex_upsample(const float *flow, const float *mask, int N, int h, int w, float *out,
                                  hipStream_t s);
size_t convex_upsample_bwd_workspace(int N, int h, int w);
hipError_t launch_convex_upsample_bwd(const float *flow, const float *mask, const float *dout, int N, int h, int w,
                                      float *dflow, float *dmask, void *ws, hipStream_t s);
size_t lookup_conv_weights_bytes();
hipError_t launch_lookup_conv_weights(const float *w, int O, int C, void *packed, hipStream_t s);
hipError_t launch_lookup_conv(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H, int W,
                              int levels, int radius, const void *packed, const float *bias, int relu, float *out,
                              hipStream_t s);
size_t lookup_conv_bwd_workspace(int B, int NQ, int levels);
hipError_t launch_lookup_conv_bwd(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H, int W,
                                  int levels, int radius, const void *packed, const float *out, int relu,
                                  const float *grad_out, float *dW, float *db, float *dlk, void *ws, hipStream_t s);
size_t splat_workspace(int B, int H, int W);
size_t voxel_workspace(int M, int C, int H, int W);
size_t voxel_tbilinear_workspace(int M, int C, int H, int W);
hipError_t launch_voxel_grid_tbilinear(const double *events, int M, int C, int H, int W, int normalize, float *out,
                                       void *ws, hipStream_t s);
hipError_t launch_voxel_grid(const float *x, const float *y, const float *t, const float *p, int M, int C, int H,
                             int W, int normalize, float *out, void *ws, hipStream_t s);
hipError_t launch_forward_splat(const float *flow, int B, int H, int W, float *out, void *ws, hipStream_t s);
// Tiled pyramid <-> the reference's row-major [BN][H_l][W_l] (corr_lookup.hip).
hipError_t launch_pyramid_export(const ConstLevelPtrs &pyr, long BN, int H, int W, int levels, const LevelPtrs &out,
                                 hipStream_t s);
hipError_t launch_pyramid_import(const ConstLevelPtrs &src, long BN, int H, int W, int levels, const LevelPtrs &pyr,
                                 hipStream_t s);
size_t build_bwd_workspace(int B, int D, int NQ, int H, int W);
hipError_t launch_build_bwd(const float *grad_c, const float *f1, int NQ, const float *f2, int B,
                            int D, int H, int W, float *df1, float *df2, float *ws, hipStream_t s);

// Number of levels the build kernel pools in its epilogue (8x8 target patches).
constexpr int kFusedLevels = 4;

}  // namespace corr
