// corr_bwd_split.hip — the backward GEMMs of the all-pairs product on the f16 MFMA at fp32
// accuracy (the CORR_BUILD_F16X3 scheme of corr_build_split.hip, applied to autograd of
// model/corr.py:58-60):
//
//   dF1[b][d][n] = sum_m F2[b][d][m] * dC[b][n][m] / sqrt(D)    rows d of F2,  rows n of dC  (k = m)
//   dF2[b][d][m] = sum_n F1[b][d][n] * dC[b][n][m] / sqrt(D)    rows d of F1,  cols m of dC  (k = n)
//
// Both are "C = A * B^T" with A and B read along k.  Every operand row r is split as
// x = 2^e_r (hi + lo) in f16 (e_r puts the row's largest |x| in [2^14, 2^15)) WHILE the GEMM
// stages it from the fp32 operand into LDS (split_gemm_f32_kernel: the fragment layout
//   per row and 16-deep chunk: hi(k 0..7), lo(same), hi(k 8..15), lo(same)),
// and accumulates lo_A hi_B + hi_A lo_B + hi_A hi_B on v_mfma_f32_32x32x16_f16 into one fp32
// accumulator (each f16 x f16 product exact in fp32).  The epilogue applies 2^(e_A + e_B); K is
// split over workgroups (partial slabs, summed in split order by splitk_reduce_kernel of
// corr_bwd.hip, which applies 1/sqrt(D)) — deterministic, no atomics.
//
// BF16X6 (BF = true, the default build's backward): every operand element is split EXACTLY into
// three bf16 pieces while staging (split3 of corr_build_common.h: no scales, no row maxima), and
// the six largest piece products go on v_mfma_f32_32x32x16_bf16 — lo.hi + hi.lo + mid.mid +
// mid.hi + hi.mid into a second accumulator, hi.hi into the first, the two added once in the
// epilogue (the build's bf16x6 scheme): no narrower than an fp32 GEMM.
//
// Row maxima (f16x3 only): F1 / F2 from rowmax2_kernel; dC's row and column maxima from the fused backward
// (corr_lookup.hip) or, for a caller-supplied dC, from absmax_kernel (unsigned atomicMax on the
// bits of non-negative floats: exact and order free).  Also here: the pool-backward fold with
// dC's maxima (pool_fold_max_kernel) and the column-maxima reduce of the fused backward.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "corr_build_common.h"

namespace corr {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kBK = 16;  // k per chunk = one MFMA k-step

// Row / column |max| of X[b] (rows x cols, row-major, ld = cols).  Block: 256 threads over
// 256 columns x kRowGroups groups of kRowsPer rows; the column maxima stay in registers over
// all the block's rows.  rmax / cmax: zeroed uint arrays
// (float bits), may be null.
constexpr int kRowsPer = 16, kRowGroups = 1;  // 4 groups measured slower (41 vs 37 us at train)
__global__ __launch_bounds__(256) void absmax_kernel(const float *__restrict__ X, int rows, int cols,
                                                     unsigned *__restrict__ rmax, unsigned *__restrict__ cmax) {
    __shared__ float red[kRowGroups][kRowsPer][4];
    const int b = blockIdx.z;
    const int c = blockIdx.x * 256 + threadIdx.x;
    const float *x = X + (size_t)b * rows * cols;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float cm = 0.f;
#pragma unroll
    for (int g = 0; g < kRowGroups; ++g) {
        const int r0 = (blockIdx.y * kRowGroups + g) * kRowsPer;
        float v[kRowsPer];
#pragma unroll
        for (int i = 0; i < kRowsPer; ++i)
            v[i] = (c < cols && r0 + i < rows) ? fabsf(x[(size_t)(r0 + i) * cols + c]) : 0.f;
#pragma unroll
        for (int i = 0; i < kRowsPer; ++i) cm = fmaxf(cm, v[i]);  // fmaxf drops NaN
        if (rmax) {
#pragma unroll
            for (int i = 0; i < kRowsPer; ++i) {
                float m = v[i];
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
                if (lane == 0) red[g][i][w] = m;
            }
        }
    }
    if (cmax && c < cols && cm > 0.f) atomicMax(&cmax[(size_t)b * cols + c], __float_as_uint(cm));
    if (rmax) {
        __syncthreads();
        if (threadIdx.x < kRowGroups * kRowsPer) {
            const int g = threadIdx.x / kRowsPer, i = threadIdx.x % kRowsPer;
            const int r = (blockIdx.y * kRowGroups + g) * kRowsPer + i;
            const float m = fmaxf(fmaxf(red[g][i][0], red[g][i][1]), fmaxf(red[g][i][2], red[g][i][3]));
            if (r < rows && m > 0.f) atomicMax(&rmax[(size_t)b * rows + r], __float_as_uint(m));
        }
    }
}

// Row |max| of two row-major operands at once (F2 and F1: rows = D features, k = pixels).
// One wave owns a row and walks it with 16-B loads, so the cross-lane reduction runs once per
// row and the result is stored directly (the zeroed-array + atomicMax convention holds: the
// value is the same).  grid.z = 2 B (operand t = z / B, batch b = z % B).
struct RowMaxArgs {
    const float *X[2];
    unsigned *rmax[2];
    int cols[2];
    int rows, B;
};

__global__ __launch_bounds__(256) void rowmax2_kernel(RowMaxArgs a) {
    const int t = blockIdx.z / a.B, b = blockIdx.z % a.B;
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= a.rows) return;  // whole waves
    const int cols = a.cols[t];
    const float *x = a.X[t] + ((size_t)b * a.rows + r) * cols;
    float m = 0.f;
    if ((cols & 3) == 0 && ((uintptr_t)a.X[t] & 15) == 0) {
#pragma unroll 4
        for (int c = lane * 4; c < cols; c += 256) {
            const float4 q = *reinterpret_cast<const float4 *>(x + c);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fmaxf(fabsf(q.z), fabsf(q.w))));
        }
    } else {
#pragma unroll 4
        for (int c = lane; c < cols; c += 64) m = fmaxf(m, fabsf(x[c]));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) a.rmax[t][(size_t)b * a.rows + r] = m > 0.f ? __float_as_uint(m) : 0u;
}

// avg_pool2d backward of the whole pyramid folded into level 0 IN PLACE, with the |max| of every
// row and column of the result (autograd of model/corr.py:25-27; replaces corr_pool_bwd's
// level-by-level passes + absmax_kernel's extra read of dC).  Per level-0 cell (y, x):
//   G'_{L-1} = G_{L-1};  G'_{l}(p_l) = G_l(p_l) + G'_{l+1}(p_{l+1}) * 0.25 where p_{l+1} = p_l / 2
//   lies in the pooled region (y_l < 2 H_{l+1}, x_l < 2 W_{l+1}) — exactly corr_pool_bwd's
//   sequence of fine += coarse * 0.25, recomputed per cell (bit-identical).
// Workgroup: kFoldQ query rows of one batch item x a chunk of columns; thread = kFoldU units of 4
// consecutive level-0 cells (vec: W % 4 == 0 and 16-byte aligned levels -> one float4 of level 0,
// one float2 of level 1 and one value of each coarser level per unit; otherwise per-cell loads).
// Column maxima stay in registers over the rows (one atomicMax per column per workgroup); row
// maxima are wave-reduced into LDS.  rmax is written (this block owns its rows); cmax must be
// zeroed; both hold float bits (atomicMax on non-negative floats is exact).  NaN is dropped as
// fmaxf drops it (absmax_kernel's convention).
constexpr int kFoldQ = 32;
constexpr int kFoldU = 2;
constexpr int kFoldChunk = 256 * 4 * kFoldU;  // level-0 cells per column chunk

struct FoldArgs {
    float *g[CORR_MAX_LEVELS];
    int L, NQ, H, W, vec;
    unsigned *rmax, *cmax;  // [B][NQ], [B][H*W]; may be null
};

// Offset of cell (y, x)'s level-l ancestor in its query map, and the mask of levels l whose
// cell receives from level l + 1.
__device__ __forceinline__ void fold_cell_geom(int y, int x, int H, int W, int L, int (&off)[CORR_MAX_LEVELS],
                                               unsigned &rc) {
    rc = 0;
#pragma unroll
    for (int l = 0; l < CORR_MAX_LEVELS; ++l) {
        const int Hl = H >> l, Wl = W >> l, yl = y >> l, xl = x >> l;
        off[l] = yl * Wl + xl;
        if (l + 1 < L && yl < 2 * (Hl >> 1) && xl < 2 * (Wl >> 1)) rc |= 1u << l;
    }
}

// The fold of one cell from its per-level values, coarsest first (corr_pool_bwd's order).
__device__ __forceinline__ float fold_cell(const float (&v)[CORR_MAX_LEVELS], unsigned rc, int L) {
    float up = 0.f;
    bool have = false;
#pragma unroll
    for (int l = CORR_MAX_LEVELS - 1; l >= 0; --l) {
        if (l >= L) continue;
        float gv = v[l];
        if (have) gv = gv + up * 0.25f;  // fine += coarse * 0.25
        up = gv;
        have = l > 0 && ((rc >> (l - 1)) & 1u);
    }
    return up;
}

template <bool VEC>
__global__ __launch_bounds__(256) void pool_fold_max_kernel(FoldArgs a) {
    __shared__ unsigned rm[kFoldQ];
    const int nqb = (a.NQ + kFoldQ - 1) / kFoldQ;
    const int b = blockIdx.x / nqb, q0 = (blockIdx.x - b * nqb) * kFoldQ;
    const int nq = min(kFoldQ, a.NQ - q0);
    const int H = a.H, W = a.W, N = H * W, L = a.L;
    const int tid = threadIdx.x, lane = tid & 63;
    size_t msz[CORR_MAX_LEVELS];
#pragma unroll
    for (int l = 0; l < CORR_MAX_LEVELS; ++l) msz[l] = (size_t)(H >> l) * (W >> l);
    if (tid < kFoldQ) rm[tid] = 0u;
    __syncthreads();
    for (int m0 = 0; m0 < N; m0 += kFoldChunk) {
        // VEC: a unit's 4 cells share y and every level >= 2 ancestor; W % 4 == 0 so levels 0 and 1
        // always receive in x, and the unit's receive mask is its first cell's.
        int off[kFoldU][CORR_MAX_LEVELS];
        unsigned rc[kFoldU];
        bool live[kFoldU];
#pragma unroll
        for (int u = 0; u < kFoldU; ++u) {
            const int m = m0 + 4 * (tid + 256 * u);
            live[u] = m < N;
            const int y = live[u] ? m / W : 0;
            if (VEC) fold_cell_geom(y, m - y * W, H, W, L, off[u], rc[u]);
        }
        float cm[kFoldU][4];
#pragma unroll
        for (int u = 0; u < kFoldU; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) cm[u][j] = 0.f;
        for (int qq = 0; qq < nq; ++qq) {
            const size_t qrow = (size_t)b * a.NQ + q0 + qq;
            float rmx = 0.f;
#pragma unroll
            for (int u = 0; u < kFoldU; ++u) {
                if (!live[u]) continue;
                const int mu = m0 + 4 * (tid + 256 * u);
                float res[4];
                if (VEC) {
                    float v[4][CORR_MAX_LEVELS];
                    const float4 t0 = *reinterpret_cast<const float4 *>(a.g[0] + qrow * msz[0] + off[u][0]);
                    v[0][0] = t0.x, v[1][0] = t0.y, v[2][0] = t0.z, v[3][0] = t0.w;
                    if (L > 1) {
                        const float2 t1 = *reinterpret_cast<const float2 *>(a.g[1] + qrow * msz[1] + off[u][1]);
                        v[0][1] = v[1][1] = t1.x;
                        v[2][1] = v[3][1] = t1.y;
                    }
#pragma unroll
                    for (int l = 2; l < CORR_MAX_LEVELS; ++l)
                        if (l < L) v[0][l] = v[1][l] = v[2][l] = v[3][l] = a.g[l][qrow * msz[l] + off[u][l]];
#pragma unroll
                    for (int j = 0; j < 4; ++j) res[j] = fold_cell(v[j], rc[u], L);
                    *reinterpret_cast<float4 *>(a.g[0] + qrow * msz[0] + off[u][0]) =
                        make_float4(res[0], res[1], res[2], res[3]);
                } else {
                    int mv = mu;
                    asm volatile("" : "+v"(mv));  // recompute the geometry per row (hoisted it costs 160 VGPRs)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int m = mv + j;
                        res[j] = 0.f;
                        if (m >= N) continue;
                        const int y = m / W;
                        int o[CORR_MAX_LEVELS];
                        unsigned r;
                        fold_cell_geom(y, m - y * W, H, W, L, o, r);
                        float v[CORR_MAX_LEVELS];
#pragma unroll
                        for (int l = 0; l < CORR_MAX_LEVELS; ++l) v[l] = l < L ? a.g[l][qrow * msz[l] + o[l]] : 0.f;
                        res[j] = fold_cell(v, r, L);
                        a.g[0][qrow * msz[0] + m] = res[j];
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float av = fabsf(res[j]);
                    cm[u][j] = fmaxf(cm[u][j], av);
                    rmx = fmaxf(rmx, av);
                }
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) rmx = fmaxf(rmx, __shfl_xor(rmx, o));
            if (lane == 0 && rmx > 0.f) atomicMax(&rm[qq], __float_as_uint(rmx));
        }
        if (a.cmax) {
#pragma unroll
            for (int u = 0; u < kFoldU; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int m = m0 + 4 * (tid + 256 * u) + j;
                    if (m < N && cm[u][j] > 0.f) atomicMax(&a.cmax[(size_t)b * N + m], __float_as_uint(cm[u][j]));
                }
        }
    }
    __syncthreads();
    if (a.rmax && tid < nq) a.rmax[(size_t)b * a.NQ + q0 + tid] = rm[tid];
}

// Column maxima of dC from the fused backward's per-workgroup partials: cmax[b][m] = max over
// groups g of part[b][g][m] (float bits; fmaxf drops NaN as absmax_kernel does).  Block: 64
// columns x 16 slices of the groups (lane = column: coalesced 256-B rows), 8 loads in flight per
// thread, the slices combined through LDS.
constexpr int kCmCols = 64, kCmSlices = 16;

__global__ __launch_bounds__(kCmCols *kCmSlices) void colmax_reduce_kernel(const float *__restrict__ part, int G, int N,
                                                                         unsigned *__restrict__ cmax) {
    __shared__ float red[kCmSlices][kCmCols];
    const int b = blockIdx.y, c = threadIdx.x % kCmCols, sl = threadIdx.x / kCmCols;
    const int m = blockIdx.x * kCmCols + c;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (m < N) {
        const float *p = part + (size_t)b * G * N + m;
        int g = sl;
        for (; g + 7 * kCmSlices < G; g += 8 * kCmSlices)
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] = fmaxf(a[u], p[(size_t)(g + u * kCmSlices) * N]);
        for (; g < G; g += kCmSlices) a[0] = fmaxf(a[0], p[(size_t)g * N]);
    }
#pragma unroll
    for (int u = 1; u < 8; ++u) a[0] = fmaxf(a[0], a[u]);
    red[sl][c] = a[0];
    __syncthreads();
    if (sl == 0 && m < N) {
        float r = red[0][c];
#pragma unroll
        for (int k = 1; k < kCmSlices; ++k) r = fmaxf(r, red[k][c]);
        cmax[(size_t)b * N + m] = __float_as_uint(r);
    }
}

// Exponent of a row from its max (as split_pack_wide_kernel): max * 2^s < 2^15.
__device__ __forceinline__ int split_shift(float mm) {
    int s = 0;
    if (mm > 0.f && mm <= 3.402823466e38f) {
        int E;
        (void)frexpf(mm, &E);
        s = 15 - E;
    }
    return s;
}

// Two elements at once on gfx950's packed converts (v_cvt_pk_f16_f32, v_pk_add_f32).  The inf
// guard of split_pair is needed only in rows whose max is inf (then s = 0): a finite max bounds
// every |y| below 2^15, and a NaN gives NaN either way — so `guard` is per row.
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2(float x0, float x1, int s, bool guard, half2v &hi, half2v &lo) {
    const f32x2v y = f32x2v{ldexpf(x0, s), ldexpf(x1, s)};
    hi = __builtin_convertvector(y, half2v);
    const f32x2v back = __builtin_convertvector(hi, f32x2v);
    lo = __builtin_convertvector(y - back, half2v);
    if (guard) {
        if (__builtin_isinf(y.x)) lo.x = (_Float16)0.f;
        if (__builtin_isinf(y.y)) lo.y = (_Float16)0.f;
    }
}

// The exact three-piece bf16 split of a pair, branch-free (the GEMM's staging runs it on every
// element it reads): hi = bf16_rn of x clamped to +-M (M = 0x7F7F7FFF, the largest float that
// rounds to a finite bf16), mid = bf16_rn(x - hi), lo = x - hi - mid.  Finite x: x - hi is exact
// (same binade, or |x| <= 2^-126 ... ), and so is the last difference, so x = hi + mid + lo bit for
// bit — the same pieces as split3 wherever hi does not overflow; past M, hi = the bf16 maximum
// and the residual carries the rest (split3 truncates there instead).  An infinite element
// splits as (the clamped hi, inf, NaN), so every output it reaches comes out of the MFMAs as NaN
// (one accumulator cannot tell inf * 0 from a real NaN); the split-K reduce then recomputes
// exactly those outputs as the fp32 reference does (NanFix, corr_common.h), which restores
// fp32's +-inf.
__device__ __forceinline__ void split3_bwd(float a, float b, unsigned &hi, unsigned &mid, unsigned &lo) {
    constexpr float M = 3.3961775e38f;  // 0x7F7F7FFF
    float ha, hb, ma, mb, da, db;
    hi = rn_pair(__builtin_amdgcn_fmed3f(a, -M, M), __builtin_amdgcn_fmed3f(b, -M, M), ha, hb);
    const float ra = a - ha, rb = b - hb;
    mid = rn_pair(ra, rb, ma, mb);
    lo = rn_pair(ra - ma, rb - mb, da, db);
}

// ---------------------------------------------------------------------------------------
// The GEMM: C[b][i][j] (+)= sum_k A[b][i][k] B[b][j][k].  4 waves (2 along i x 2 along j),
// each 64 i x 128 j (2 x 4 blocks of 32 x 32), workgroup 128 x 256; K chunks staged through
// LDS double-buffered, the next chunk's global loads in flight during the MFMAs.  On the
// LDS-DMA path with more than 128 rows the workgroup is 8 waves (4 along i), 256 x 256: each
// staged element then feeds twice the MFMAs (split_gemm_f32_kernel's WI = 4).
// ---------------------------------------------------------------------------------------
constexpr int kWI = 2, kWJ = 2, kMI = 2, kNJ = 4;
constexpr int kTI = 32 * kMI * kWI;   // 128
constexpr int kTJ = 32 * kNJ * kWJ;   // 256
constexpr int kNT = 256;
static_assert(kTI == kNT / 2 && kTJ == kNT, "staging: one A row-octet and two B row-octets per thread");

// LDS slot of 16-B unit u (k-octet x hi/lo) of staging row j.  The (j >> 2) & 3 term keeps the
// fragment reads (ds_read_b128: 16-lane groups of rows {0-3, 12-15, 20-27} / {4-11, 16-19,
// 28-31}) on 16 distinct 4-bank groups; XOR-ing 3 into it for odd j >> 1 puts the staging
// writes (ds_write_b128, 8-lane groups) on 8 distinct 4-bank groups as well, both the row-octet
// writes (rows 4k..4k+3 x 2 octets) and the column writes (rows 8k..8k+7) — without it rows 4k
// and 4k + 2 collide (2-way conflicts on every staging write).  Checked exhaustively offline.
__device__ __forceinline__ int swz(int j, int u) { return j * 4 + (u ^ ((j >> 2) & 3) ^ (((j >> 1) & 1) * 3)); }

// The same GEMM reading the fp32 operands and splitting them while staging (no convert
// kernels, no packed copies: the fp32 element is as many bytes as its hi / lo pair).  A rows
// are k-contiguous (F1 / F2 rows); B rows are k-contiguous (dC rows, BCOL = false) or dC
// COLUMNS (BCOL = true: element (j, k) at B[k * b_sk + j]; thread = column, so each of its 16
// loads per chunk is, across the wave, one 256-B run of a dC row).  Row shifts come from the row
// maxima (float bits) exactly as the converts compute them, so every staged unit — and the
// result — is bit-identical to the packed path.  Per chunk (16 k) a thread stages A row
// tid / 2, k-octet tid % 2 (8 values) and 16 B values: BCOL = false rows tid / 2 + 128 u,
// k-octet tid % 2; BCOL = true column tid, all 16 k.
struct FGemmParams {
    const float *A;
    long a_sb, a_sr;
    const float *Bm;
    long b_sb, b_sr, b_sk;
    const unsigned *mxA, *mxB;
    float *C;
    int B, NI, NJ, K, nkc;
    int ti, tj, splits, kc_per;
    float alpha;
    int direct, vec;  // vec: 16-B loads legal (strides / bases / K multiples of 4)
    int nt;           // non-temporal epilogue stores
    // Tail reduce: the previous GEMM's ordered split-K sum (splitk_reduce_vec4_kernel's
    // arithmetic), run by `tail_wgs` extra workgroups appended after the `gemm_wgs` GEMM ones —
    // they land on the CUs the GEMM's grid leaves idle.  tail_wgs = 0: none.
    const float4 *tail_ws;
    float4 *tail_C;
    size_t tail_per4;
    int tail_splits, tail_exact, tail_wgs, gemm_wgs;
    float tail_alpha, tail_s;
    NanFix fix, tail_fix;  // BF: NaN outputs recomputed in fp32 (the tail reduce's GEMM: tail_fix)
};

// The tail reduce's share of workgroup t of p.tail_wgs (bit-identical to the separate reduce).
template <int NT>
__device__ __forceinline__ void gemm_tail_reduce(const FGemmParams &p, int t) {
    for (size_t i = (size_t)t * NT + threadIdx.x; i < p.tail_per4; i += (size_t)p.tail_wgs * NT) {
        float4 acc = p.tail_ws[i];
        for (int k = 1; k < p.tail_splits; ++k) {
            const float4 v = p.tail_ws[(size_t)k * p.tail_per4 + i];
            acc.x = acc.x + v.x, acc.y = acc.y + v.y, acc.z = acc.z + v.z, acc.w = acc.w + v.w;
        }
        if (p.tail_exact)
            acc.x = acc.x * p.tail_alpha, acc.y = acc.y * p.tail_alpha, acc.z = acc.z * p.tail_alpha,
            acc.w = acc.w * p.tail_alpha;
        else
            acc.x = acc.x / p.tail_s, acc.y = acc.y / p.tail_s, acc.z = acc.z / p.tail_s, acc.w = acc.w / p.tail_s;
        if (p.tail_fix.K && __builtin_expect(acc.x != acc.x || acc.y != acc.y || acc.z != acc.z || acc.w != acc.w, 0)) {
            if (acc.x != acc.x) acc.x = nanfix_flat(p.tail_fix, 4 * i);
            if (acc.y != acc.y) acc.y = nanfix_flat(p.tail_fix, 4 * i + 1);
            if (acc.z != acc.z) acc.z = nanfix_flat(p.tail_fix, 4 * i + 2);
            if (acc.w != acc.w) acc.w = nanfix_flat(p.tail_fix, 4 * i + 3);
        }
        p.tail_C[i] = acc;
    }
}

typedef __attribute__((address_space(3))) void gemm_lds_t;

// One LDS-DMA piece: 16 B per lane from g into LDS at lds + 16 * lane (global_load_lds_dwordx4,
// M0 = the wave-uniform LDS byte address); counted in vmcnt like any vector load.
__device__ __forceinline__ void gemm_dma16(const void *g, uint32_t lds) {
    asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds) : "memory");
}

template <int N>
__device__ __forceinline__ void gemm_wait_vm_barrier() {
    static_assert(N == 0 || N == 4 || N == 6, "vmcnt immediates of the DMA ring (pieces per wave per chunk)");
    if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Dynamic LDS of the GEMM: the hi/lo staging (2 stages; DMA: 1), the row exponents, and (DMA)
// a 2-slot ring of raw fp32 chunks (kTI + kTJ rows x 16 k; BCOL: B as 16 k-rows x 256 columns).
// PIPE (DMA path): a 3-slot raw ring, so chunk k + 1 can be split while chunk k's MFMAs run.
// BF: each stage holds (hi, mid) in the hi/lo layout plus a kTJ-row plane of the lo pieces (A
// row i's in unit slot 2o, B row j's in slot 2o + 1), and there are no row exponents.
// BF + PIPE: two staging stages and a 2-slot ring (chunk k + 1 split into the other stage while
// chunk k's fragments are read and multiplied): 160 KiB at the 256-row tile.
template <bool DMA, int WI = kWI, bool PIPE = false, bool BF = false>
constexpr int gemm_stages() { return DMA && !(PIPE && BF) ? 1 : 2; }
template <bool DMA, int WI = kWI, bool PIPE = false, bool BF = false>
constexpr int gemm_lds_bytes() {
    constexpr int rows = 32 * kMI * WI + kTJ;
    return gemm_stages<DMA, WI, PIPE, BF>() * (rows + (BF ? kTJ : 0)) * 4 * (int)sizeof(u32x4) +
           (BF ? 0 : rows * (int)sizeof(int)) + (DMA ? (PIPE && !BF ? 3 : 2) * rows * kBK * (int)sizeof(float) : 0);
}

// DMA = true: the raw fp32 chunks arrive by LDS-DMA two chunks ahead (no register staging, so a
// chunk's loads have two MFMA phases to land); each chunk is then split LDS -> registers -> the
// hi/lo staging (the same split and layout as the register path, so the same bits).  Needs 16-B
// aligned operands, K % 16 == 0 and (BCOL) NJ % 4 == 0.
// lo = f16(y - f32(h)) of an element pair in two VOP3P instructions: v_fma_mix{lo,hi}_f16 take
// h as f16 and y as f32, and y - h is exact in f32 (h is y rounded to 11 bits), so the one
// rounding to f16 gives the same bits as converting h back, subtracting and converting.
__device__ __forceinline__ unsigned split_lo_mix(unsigned h2, float y0, float y1) {
    unsigned lo;
    asm volatile("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(h2), "v"(y0));
    asm volatile("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(h2), "v"(y1));
    return lo;
}

template <bool BCOL, bool DMA = false, int WI = kWI, bool PIPE = false, bool BF = false>
__global__ __launch_bounds__(64 * WI * kWJ, 2) void split_gemm_f32_kernel(FGemmParams p) {
    // WI = 4 (DMA path only): 8 waves, a 256 x 256 tile (each wave still 64 x 128), so every
    // staged element feeds twice the MFMAs
    static_assert(WI == kWI || (WI == 4 && DMA), "the wide tile exists on the DMA path only");
    constexpr int TI = 32 * kMI * WI, NT = 64 * WI * kWJ, ROWS = TI + kTJ;
    constexpr int UB = 2 * kTJ / NT;      // B row-octets per thread (BCOL = false)
    constexpr int KO = 2 * kTJ / NT;      // B k-octets per thread (BCOL = true; column tid % kTJ)
    constexpr int NW = NT / 64, PB = 16 / NW;  // waves; B DMA pieces per wave and chunk
    constexpr int STG = (ROWS + (BF ? kTJ : 0)) * 4;  // u32x4 units per staging stage
    static_assert(TI == NT / 2, "one A row-octet per thread");
    static_assert(TI <= kTJ, "the BF lo plane holds kTJ rows");
    extern __shared__ __attribute__((aligned(16))) u32x4 gemm_smem[];
    u32x4 *lds = gemm_smem;
    int *lex = reinterpret_cast<int *>(gemm_smem + gemm_stages<DMA, WI, PIPE, BF>() * STG);
    float *raw = reinterpret_cast<float *>(lex + (BF ? 0 : ROWS));
    if ((int)blockIdx.x >= p.gemm_wgs) {  // appended tail-reduce workgroups
        gemm_tail_reduce<NT>(p, (int)blockIdx.x - p.gemm_wgs);
        return;
    }
    int id = xcd_swizzle(blockIdx.x, p.gemm_wgs);
    const int tj = id % p.tj;
    id /= p.tj;
    const int ti = id % p.ti;
    id /= p.ti;
    const int split = id % p.splits;
    const int b = id / p.splits;
    const int i0 = ti * TI, j0 = tj * kTJ;
    const int kc0 = split * p.kc_per, kc1 = min(p.nkc, kc0 + p.kc_per);

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wv = tid >> 6, wi = wv / kWJ, wj = wv % kWJ;

    if constexpr (!BF) {
        for (int row = tid; row < ROWS; row += NT) {
            const unsigned m = row < TI ? p.mxA[(size_t)b * p.NI + min(i0 + row, p.NI - 1)]
                                         : p.mxB[(size_t)b * p.NJ + min(j0 + row - TI, p.NJ - 1)];
            lex[row] = -split_shift(__uint_as_float(m));
        }
        __syncthreads();
    }

    // staging tasks
    const int arow = tid >> 1, aoct = tid & 1;
    const float *ap = p.A + (size_t)b * p.a_sb + (size_t)min(i0 + arow, p.NI - 1) * p.a_sr + aoct * 8;
    const int sa = BF ? 0 : -lex[arow];
    auto row_inf = [&](const unsigned *mx, int row, int n) {
        return !BF && __uint_as_float(mx[(size_t)b * n + min(row, n - 1)]) > 3.402823466e38f;
    };
    const bool ga = row_inf(p.mxA, i0 + arow, p.NI);
    const float *bp[2];
    int sb[4];
    bool gb[4];
    int brow[2];
    const int bcol = tid % kTJ, boct0 = (tid / kTJ) * KO;  // BCOL: column, first k-octet
    if (!BCOL) {
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            brow[u] = (tid >> 1) + (NT / 2) * u;
            bp[u] = p.Bm + (size_t)b * p.b_sb + (size_t)min(j0 + brow[u], p.NJ - 1) * p.b_sr + aoct * 8;
            sb[u] = BF ? 0 : -lex[TI + brow[u]];
            gb[u] = row_inf(p.mxB, j0 + brow[u], p.NJ);
        }
    } else {
        bp[0] = p.Bm + (size_t)b * p.b_sb;  // + n * b_sk + j
        sb[0] = BF ? 0 : -lex[TI + bcol];
        gb[0] = row_inf(p.mxB, j0 + bcol, p.NJ);
    }
    const bool vec = p.vec;
    // Fast staging (wave-uniform): no staged row has an inf max and every shift has a normal
    // 2^s (s <= 127; s >= -113 always), so x * 2^s — one v_pk_mul_f32 per element pair — is
    // exactly ldexp(x, s) and the inf guard is dead.  Otherwise the exact split2 path.
    bool slow_t = ga || sa > 127;
    if (!BCOL) {
#pragma unroll
        for (int u = 0; u < UB; ++u) slow_t = slow_t || gb[u] || sb[u] > 127;
    } else {
        slow_t = slow_t || gb[0] || sb[0] > 127;
    }
    const bool fast = __builtin_amdgcn_ballot_w64(slow_t) == 0;
    auto pow2f = [](int e) { return __uint_as_float((unsigned)(e + 127) << 23); };  // 2^e, normal e
    const float fa = pow2f(fast ? sa : 0);
    float fb[2];
    fb[0] = pow2f(fast ? sb[0] : 0);
    fb[1] = (BCOL || UB < 2) ? 1.0f : pow2f(fast ? sb[1] : 0);
    // BCOL: two register sets — chunk c is loaded two iterations before its MFMAs (one iteration
    // before it is staged into LDS), so a load has two MFMA phases to arrive
    float ra0[8], rb0[16], ra1[8], rb1[16];
    auto load_chunk = [&](int kc, float (&ra)[8], float (&rb)[16]) {
        const int k0 = kc * kBK;
        const int ka = k0 + aoct * 8;  // this thread's A octet
        if (vec && ka + 8 <= p.K) {
            const float4 x0 = *reinterpret_cast<const float4 *>(ap + k0);
            const float4 x1 = *reinterpret_cast<const float4 *>(ap + k0 + 4);
            ra[0] = x0.x, ra[1] = x0.y, ra[2] = x0.z, ra[3] = x0.w;
            ra[4] = x1.x, ra[5] = x1.y, ra[6] = x1.z, ra[7] = x1.w;
        } else {
#pragma unroll
            for (int t = 0; t < 8; ++t) ra[t] = ka + t < p.K ? ap[k0 + t] : 0.f;
        }
        if (!BCOL) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (vec && ka + 8 <= p.K) {
                    const float4 x0 = *reinterpret_cast<const float4 *>(bp[u] + k0);
                    const float4 x1 = *reinterpret_cast<const float4 *>(bp[u] + k0 + 4);
                    rb[8 * u + 0] = x0.x, rb[8 * u + 1] = x0.y, rb[8 * u + 2] = x0.z, rb[8 * u + 3] = x0.w;
                    rb[8 * u + 4] = x1.x, rb[8 * u + 5] = x1.y, rb[8 * u + 6] = x1.z, rb[8 * u + 7] = x1.w;
                } else {
#pragma unroll
                    for (int t = 0; t < 8; ++t) rb[8 * u + t] = ka + t < p.K ? bp[u][k0 + t] : 0.f;
                }
            }
        } else {
            // column j0 + tid (lanes = consecutive columns: every load is a 256-B row run)
            const int jc = min(j0 + tid, p.NJ - 1);  // clamped columns feed discarded outputs
            const float *q = bp[0] + (size_t)k0 * p.b_sk + jc;
#pragma unroll
            for (int t = 0; t < 16; ++t) rb[t] = k0 + t < p.K ? q[(size_t)t * p.b_sk] : 0.f;
        }
    };
    using FM0 = std::integral_constant<int, 0>;
    // FM: 0 = the runtime `fast` choice, 1 = fast split only, 2 = exact split2 only (the pipelined
    // loop runs one branch-free copy per case, so its MFMAs can be scheduled among the split)
    auto store_chunk = [&](int st, const float (&ra)[8], const float (&rb)[16], auto fm_tag) {
        constexpr int FM = decltype(fm_tag)::value;
        u32x4 *S = lds + (size_t)st * STG;
        if constexpr (BF) {
            // (hi, mid) into the hi/lo layout's two slots, lo into the lo plane: A rows in slot 2o,
            // B rows in slot 2o + 1 (the same bank pattern as the hi / lo writes of those rows)
            u32x4 *S1 = S + ROWS * 4;
            auto split8 = [&](const float *v, u32x4 &hi, u32x4 &mid, u32x4 &lo) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    unsigned h_, m_, l_;
                    split3_bwd(v[2 * t], v[2 * t + 1], h_, m_, l_);
                    hi[t] = h_, mid[t] = m_, lo[t] = l_;
                }
            };
            {
                u32x4 hi, mid, lo;
                split8(ra, hi, mid, lo);
                S[swz(arow, 2 * aoct)] = hi;
                S[swz(arow, 2 * aoct + 1)] = mid;
                S1[swz(arow, 2 * aoct)] = lo;
            }
            if (!BCOL) {
#pragma unroll
                for (int u = 0; u < UB; ++u) {
                    u32x4 hi, mid, lo;
                    split8(rb + 8 * u, hi, mid, lo);
                    S[swz(TI + brow[u], 2 * aoct)] = hi;
                    S[swz(TI + brow[u], 2 * aoct + 1)] = mid;
                    S1[swz(brow[u], 2 * aoct + 1)] = lo;
                }
            } else {
#pragma unroll
                for (int o = 0; o < KO; ++o) {
                    u32x4 hi, mid, lo;
                    split8(rb + 8 * o, hi, mid, lo);
                    S[swz(TI + bcol, 2 * (boct0 + o))] = hi;
                    S[swz(TI + bcol, 2 * (boct0 + o) + 1)] = mid;
                    S1[swz(bcol, 2 * (boct0 + o) + 1)] = lo;
                }
            }
            return;
        }
        auto split8 = [&](const float *v, int sh, bool guard, float f, u32x4 &hi, u32x4 &lo) {
            half2v h[4], l[4];
            if (FM == 1 || (FM == 0 && fast)) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const f32x2v y = f32x2v{v[2 * t], v[2 * t + 1]} * f32x2v{f, f};
                    h[t] = __builtin_convertvector(y, half2v);
                    l[t] = __builtin_bit_cast(half2v, split_lo_mix(__builtin_bit_cast(unsigned, h[t]), y[0], y[1]));
                }
            } else {
#pragma unroll
                for (int t = 0; t < 4; ++t) split2(v[2 * t], v[2 * t + 1], sh, guard, h[t], l[t]);
            }
            hi = u32x4{__builtin_bit_cast(unsigned, h[0]), __builtin_bit_cast(unsigned, h[1]),
                       __builtin_bit_cast(unsigned, h[2]), __builtin_bit_cast(unsigned, h[3])};
            lo = u32x4{__builtin_bit_cast(unsigned, l[0]), __builtin_bit_cast(unsigned, l[1]),
                       __builtin_bit_cast(unsigned, l[2]), __builtin_bit_cast(unsigned, l[3])};
        };
        {
            u32x4 hi, lo;
            split8(ra, sa, ga, fa, hi, lo);
            S[swz(arow, 2 * aoct)] = hi;
            S[swz(arow, 2 * aoct + 1)] = lo;
        }
        if (!BCOL) {
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                u32x4 hi, lo;
                split8(rb + 8 * u, sb[u], gb[u], fb[u], hi, lo);
                S[swz(TI + brow[u], 2 * aoct)] = hi;
                S[swz(TI + brow[u], 2 * aoct + 1)] = lo;
            }
        } else {
#pragma unroll
            for (int o = 0; o < KO; ++o) {  // this thread's k-octets of its column
                u32x4 hi, lo;
                split8(rb + 8 * o, sb[0], gb[0], fb[0], hi, lo);
                S[swz(TI + bcol, 2 * (boct0 + o))] = hi;
                S[swz(TI + bcol, 2 * (boct0 + o) + 1)] = lo;
            }
        }
    };

    f32x16 acc[kMI][kNJ];
#pragma unroll
    for (int m = 0; m < kMI; ++m)
#pragma unroll
        for (int n = 0; n < kNJ; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

    const int arow0 = wi * (32 * kMI) + l32, brow0 = TI + wj * (32 * kNJ) + l32;
    // One chunk's fragments (the staged pieces of this wave's rows); m* only for BF.
    struct Frags {
        u32x4 ah[kMI], am[kMI], al[kMI], bh[kNJ], bm[kNJ], bl[kNJ];
    };
    auto frags = [&](int st, Frags &f) __attribute__((always_inline)) {
        const u32x4 *S = lds + (size_t)st * STG;
#pragma unroll
        for (int m = 0; m < kMI; ++m) {
            f.ah[m] = S[swz(arow0 + 32 * m, 2 * h)];
            if (BF) f.am[m] = S[swz(arow0 + 32 * m, 2 * h + 1)], f.al[m] = S[ROWS * 4 + swz(arow0 + 32 * m, 2 * h)];
            else f.al[m] = S[swz(arow0 + 32 * m, 2 * h + 1)];
        }
#pragma unroll
        for (int n = 0; n < kNJ; ++n) {
            f.bh[n] = S[swz(brow0 + 32 * n, 2 * h)];
            if (BF) f.bm[n] = S[swz(brow0 + 32 * n, 2 * h + 1)], f.bl[n] = S[ROWS * 4 + swz(brow0 - TI + 32 * n, 2 * h + 1)];
            else f.bl[n] = S[swz(brow0 + 32 * n, 2 * h + 1)];
        }
    };
    auto mfmas = [&](const Frags &f) __attribute__((always_inline)) {
        if constexpr (BF) {
            auto mm = [](u32x4 a, u32x4 b, f32x16 c) {
                return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8g, a),
                                                               __builtin_bit_cast(bf16x8g, b), c, 0, 0, 0);
            };
            // smallest first: lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi (one accumulator: the
            // register budget of two waves per SIMD holds one 64 x 128 set)
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.al[m], f.bh[n], acc[m][n]);
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.ah[m], f.bl[n], acc[m][n]);
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.am[m], f.bm[n], acc[m][n]);
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.am[m], f.bh[n], acc[m][n]);
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.ah[m], f.bm[n], acc[m][n]);
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.ah[m], f.bh[n], acc[m][n]);
        } else {
            auto mm = [](u32x4 a, u32x4 b, f32x16 c) {
                return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b),
                                                              c, 0, 0, 0);
            };
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.al[m], f.bh[n], acc[m][n]);
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.ah[m], f.bl[n], acc[m][n]);
#pragma unroll
            for (int m = 0; m < kMI; ++m)
#pragma unroll
                for (int n = 0; n < kNJ; ++n) acc[m][n] = mm(f.ah[m], f.bh[n], acc[m][n]);
        }
    };
    auto mfma_chunk = [&](int st) {
        Frags f;
        frags(st, f);
        mfmas(f);
    };
    if constexpr (DMA) {
        const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
        const uint32_t raw_base = (uint32_t)(uintptr_t)(gemm_lds_t *)raw;
        // this wave's pieces of a chunk: A rows 16 (2w + q) + lane / 4, 16-B piece lane % 4;
        // B rows 16 (4w + q) + lane / 4 (BCOL: k-row 4w + q, columns 4 lane .. 4 lane + 3)
        const float *asrc[2], *bsrc[4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int row = 16 * (2 * w + q) + (lane >> 2);
            asrc[q] = p.A + (size_t)b * p.a_sb + (size_t)min(i0 + row, p.NI - 1) * p.a_sr + (lane & 3) * 4;
        }
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            if (!BCOL) {
                const int row = 16 * (PB * w + q) + (lane >> 2);
                bsrc[q] = p.Bm + (size_t)b * p.b_sb + (size_t)min(j0 + row, p.NJ - 1) * p.b_sr + (lane & 3) * 4;
            } else {
                bsrc[q] = p.Bm + (size_t)b * p.b_sb + (size_t)(PB * w + q) * p.b_sk + min(j0 + 4 * lane, p.NJ - 4);
            }
        }
        auto issue = [&](int kc, int slot) __attribute__((always_inline)) {
            const uint32_t base = raw_base + slot * (ROWS * kBK) * 4;
            const size_t ka = (size_t)kc * kBK, kb = BCOL ? (size_t)kc * kBK * p.b_sk : ka;
#pragma unroll
            for (int q = 0; q < 2; ++q) gemm_dma16(asrc[q] + ka, base + (2 * w + q) * 1024);
#pragma unroll
            for (int q = 0; q < PB; ++q) gemm_dma16(bsrc[q] + kb, base + TI * kBK * 4 + (PB * w + q) * 1024);
        };
        auto read_raw = [&](int slot) __attribute__((always_inline)) {
            const float *R = raw + slot * (ROWS * kBK);
            const float4 *ar = reinterpret_cast<const float4 *>(R + arow * kBK + aoct * 8);
            const float4 x0 = ar[0], x1 = ar[1];
            ra0[0] = x0.x, ra0[1] = x0.y, ra0[2] = x0.z, ra0[3] = x0.w;
            ra0[4] = x1.x, ra0[5] = x1.y, ra0[6] = x1.z, ra0[7] = x1.w;
            const float *RB = R + TI * kBK;
            if (!BCOL) {
#pragma unroll
                for (int u = 0; u < UB; ++u) {
                    const float4 *br = reinterpret_cast<const float4 *>(RB + brow[u] * kBK + aoct * 8);
                    const float4 y0 = br[0], y1 = br[1];
                    rb0[8 * u + 0] = y0.x, rb0[8 * u + 1] = y0.y, rb0[8 * u + 2] = y0.z, rb0[8 * u + 3] = y0.w;
                    rb0[8 * u + 4] = y1.x, rb0[8 * u + 5] = y1.y, rb0[8 * u + 6] = y1.z, rb0[8 * u + 7] = y1.w;
                }
            } else {
#pragma unroll
                for (int t = 0; t < 8 * KO; ++t) rb0[t] = RB[(8 * boct0 + t) * kTJ + bcol];
            }
        };
        if constexpr (PIPE && BF) {
            // Chunk c: ring slot (c - kc0) & 1, staged into stage (c - kc0) & 1.  Iteration kc:
            // one barrier (chunk kc + 1 landed; every wave done with iteration kc - 1, so stage
            // st ^ 1 and ring slot st are free), chunk kc + 2's DMA into slot st, then one region
            // holding chunk kc's fragment reads and MFMAs together with chunk kc + 1's split into
            // stage st ^ 1.  Same splits, same MFMA order: the same bits as the other plans.
            constexpr int G = 2 + PB;
            if (kc0 < kc1) issue(kc0, 0);
            if (kc0 + 1 < kc1) issue(kc0 + 1, 1);
            if (kc0 < kc1) {
                if (kc0 + 1 < kc1) wait_vmcnt_barrier<G>();
                else wait_vmcnt_barrier<0>();
                read_raw(0);
                store_chunk(0, ra0, rb0, FM0{});
            }
            int kc = kc0;
            for (; kc + 1 < kc1; ++kc) {
                const int st = (kc - kc0) & 1;
                wait_vmcnt_barrier<0>();
                if (kc + 2 < kc1) issue(kc + 2, st);
                Frags f;
                frags(st, f);
                read_raw(st ^ 1);
                store_chunk(st ^ 1, ra0, rb0, FM0{});
                mfmas(f);
            }
            if (kc < kc1) {  // the last chunk
                __syncthreads();
                mfma_chunk((kc - kc0) & 1);
            }
        } else if constexpr (!PIPE) {
            if (kc0 < kc1) issue(kc0, 0);
            if (kc0 + 1 < kc1) issue(kc0 + 1, 1);
            for (int kc = kc0; kc < kc1; ++kc) {
                const int slot = (kc - kc0) & 1;
                if (kc + 1 < kc1) gemm_wait_vm_barrier<2 + PB>();  // chunk kc landed (every wave's pieces)
                else gemm_wait_vm_barrier<0>();
                read_raw(slot);
                store_chunk(0, ra0, rb0, FM0{});
                __syncthreads();  // staging complete, ring slot read
                if (kc + 2 < kc1) issue(kc + 2, slot);
                mfma_chunk(0);
            }
        } else {
            // Chunk c's raw fp32 pieces go to ring slot (c - kc0) % 3, issued three chunks ahead.
            // Iteration kc: read chunk kc's fragments from the staging into registers; barrier
            // (every wave has read them, chunk kc + 1's pieces have landed); then chunk kc + 1's
            // split into the staging and chunk kc's MFMAs (from registers) in one region, so the
            // split's VALU and LDS stores overlap the MFMA pipe within each wave; barrier; issue
            // chunk kc + 4 into the freed slot.  Same splits, same MFMA order: the same bits.
            constexpr int G = 2 + PB;  // DMA pieces per wave and chunk
            auto wait_groups = [&](int n) __attribute__((always_inline)) {  // <= n chunks still in flight
                if (n >= 2) wait_vmcnt_barrier<2 * G>();
                else if (n == 1) wait_vmcnt_barrier<G>();
                else wait_vmcnt_barrier<0>();
            };
            for (int c = 0; c < 3; ++c)
                if (kc0 + c < kc1) issue(kc0 + c, c);
            if (kc0 < kc1) {
                wait_groups(min(kc1, kc0 + 3) - kc0 - 1);
                read_raw(0);
                store_chunk(0, ra0, rb0, FM0{});
                __syncthreads();
                if (kc0 + 3 < kc1) issue(kc0 + 3, 0);
            }
            // every iteration but the last: chunk kc + 1 is split (branch-free, one copy per split
            // mode) in the same region as chunk kc's MFMAs
            auto body = [&](auto fm_tag) __attribute__((always_inline)) {
                for (int kc = kc0; kc + 1 < kc1; ++kc) {
                    Frags f;
                    frags(0, f);
                    wait_groups(min(kc1, kc + 4) - kc - 2);  // chunk kc + 1 landed; fragments read
                    read_raw((kc + 1 - kc0) % 3);
                    store_chunk(0, ra0, rb0, fm_tag);
                    mfmas(f);
                    __syncthreads();  // chunk kc + 1 staged; its ring slot read by every wave
                    if (kc + 4 < kc1) issue(kc + 4, (kc + 1 - kc0) % 3);
                }
            };
            if (BF || fast) body(std::integral_constant<int, 1>{});
            else body(std::integral_constant<int, 2>{});
            if (kc0 < kc1) mfma_chunk(0);  // the last chunk
        }
    } else if constexpr (!BCOL || BF) {  // row operands (and BF): one set (two would spill at 256 VGPRs)
        if (kc0 < kc1) {
            load_chunk(kc0, ra0, rb0);
            store_chunk(0, ra0, rb0, FM0{});
        }
        __syncthreads();
        for (int kc = kc0; kc < kc1; ++kc) {
            const int st = (kc - kc0) & 1;
            if (kc + 1 < kc1) load_chunk(kc + 1, ra0, rb0);
            mfma_chunk(st);
            if (kc + 1 < kc1) store_chunk(st ^ 1, ra0, rb0, FM0{});
            __syncthreads();
        }
    } else {
    if (kc0 < kc1) {
        load_chunk(kc0, ra0, rb0);
        if (kc0 + 1 < kc1) load_chunk(kc0 + 1, ra1, rb1);
        store_chunk(0, ra0, rb0, FM0{});
    }
    __syncthreads();
    for (int kc = kc0; kc < kc1; kc += 2) {
        // even step: chunk kc in stage 0, chunk kc + 1 in set 1, chunk kc + 2 -> set 0
        if (kc + 2 < kc1) load_chunk(kc + 2, ra0, rb0);
        mfma_chunk(0);
        if (kc + 1 < kc1) store_chunk(1, ra1, rb1, FM0{});
        __syncthreads();
        if (kc + 1 >= kc1) break;
        // odd step: chunk kc + 1 in stage 1, chunk kc + 2 in set 0, chunk kc + 3 -> set 1
        if (kc + 3 < kc1) load_chunk(kc + 3, ra1, rb1);
        mfma_chunk(1);
        if (kc + 2 < kc1) store_chunk(0, ra0, rb0, FM0{});
        __syncthreads();
    }
    }

    const size_t slab = (size_t)p.B * p.NI * p.NJ;
    float *C = p.C + (p.direct ? 0 : (size_t)split * slab) + (size_t)b * p.NI * p.NJ;
#pragma unroll
    for (int n = 0; n < kNJ; ++n) {
        const int jl = wj * (32 * kNJ) + 32 * n + l32;
        const int j = j0 + jl;
        const int ej = BF ? 0 : lex[TI + jl];
#pragma unroll
        for (int m = 0; m < kMI; ++m) {
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int il = wi * (32 * kMI) + 32 * m + (g & 3) + 8 * (g >> 2) + 4 * h;
                const int i = i0 + il;
                float x = BF ? acc[m][n][g] : ldexpf(acc[m][n][g], lex[il] + ej);
                if (p.direct) x = x * p.alpha;
                if (i < p.NI && j < p.NJ) {
                    if (p.nt) __builtin_nontemporal_store(x, &C[(size_t)i * p.NJ + j]);
                    else C[(size_t)i * p.NJ + j] = x;
                }
            }
        }
    }
}

// Split-K so that tiles x splits fills ONE wave of workgroup slots (MI355X: 256 CUs x 2
// resident GEMM workgroups = 512) without spilling into a second, partly empty wave: at the
// train shape 112 tiles -> 4 splits, 448 workgroups (measured 377 us for the whole backward vs
// 436 us with 5 splits = 560 workgroups, 401 us with 3).
constexpr long kGemmSlots = 512;

// Plan knobs of the backward GEMMs.  The library always runs the defaults; tools/kbench_gemm.hip
// passes others for its A/B runs (no global state).
struct GemmTune {
    int splits = 0;          // split-K count override (0 = plan_split_k's plan)
    bool dma = true;         // LDS-DMA operand ring when the shape allows
    bool wide = true;        // 256 x 256 tiles of 8 waves on the DMA path when NI > 128
    bool reduce_vec4 = true; // the 16-B split-K reduce when aligned
    bool pipe = true;        // wide DMA path: split chunk k + 1 under chunk k's MFMAs (3-slot ring)
    bool nt = true;          // non-temporal epilogue (slab / direct output) stores: ~1 us per GEMM, same bits
};

int plan_split_k(int NI, int NJ, int nkc, int batch, const GemmTune &t = GemmTune{}) {
    if (t.splits > 0) return t.splits;
    const long tiles = (long)((NI + kTI - 1) / kTI) * ((NJ + kTJ - 1) / kTJ) * batch;
    long splits = std::max(1L, kGemmSlots / tiles);
    splits = std::min<long>(splits, std::max(1, nkc / 8));  // >= 128 k per split
    return (int)std::max(1L, splits);
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct BwdWs {
    unsigned *mxA, *mxB, *mxC, *mxA2;  // row max of F2, of dC rows, column max of dC, row max of F1
    unsigned *mx0;                     // start of the four (contiguous, zeroed once per call)
    size_t mx_bytes;
    float *slab, *slab2;               // split-K partial sums of dF1 and dF2
};

size_t slab_floats(int B, int D, int NQ, int N, const GemmTune &t);

// The maxima (B rows up to max(N, NQ)), then the split-K slabs of dF1 and of dF2.
BwdWs carve(void *ws, int B, int D, int NQ, int N) {
    const size_t R = std::max(NQ, N);
    char *w = (char *)ws;
    BwdWs r;
    r.mx0 = r.mxA = (unsigned *)w;
    w += al256((size_t)B * D * 4);
    r.mxB = (unsigned *)w;
    w += al256((size_t)B * R * 4);
    r.mxC = (unsigned *)w;
    w += al256((size_t)B * R * 4);
    r.mxA2 = (unsigned *)w;
    w += al256((size_t)B * D * 4);
    r.mx_bytes = (size_t)(w - (char *)r.mx0);
    r.slab = (float *)w;
    r.slab2 = (float *)(w + al256(slab_floats(B, D, NQ, N, GemmTune{}) * sizeof(float)));
    return r;
}

size_t slab_floats(int B, int D, int NQ, int N, const GemmTune &t) {
    const int K1 = (N + kBK - 1) / kBK, K2 = (NQ + kBK - 1) / kBK;
    const size_t s1 = (size_t)plan_split_k(D, NQ, K1, B, t) * B * D * NQ;
    const size_t s2 = (size_t)plan_split_k(D, N, K2, B, t) * B * D * N;
    return std::max(s1, s2);
}

// rmax / cmax must be zeroed by the caller (one memset covers every maximum of a call).
hipError_t absmax(const float *X, int B, int rows, int cols, unsigned *rmax, unsigned *cmax, hipStream_t s) {
    constexpr int RB = kRowsPer * kRowGroups;
    hipLaunchKernelGGL(absmax_kernel, dim3((cols + 255) / 256, (rows + RB - 1) / RB, B), dim3(256), 0, s, X, rows,
                       cols, rmax, cmax);
    return hipGetLastError();
}

// Row maxima of X0 [B][rows][cols0] and X1 [B][rows][cols1] in one launch.
hipError_t rowmax2(const float *X0, int cols0, unsigned *rmax0, const float *X1, int cols1, unsigned *rmax1, int B,
                   int rows, hipStream_t s) {
    RowMaxArgs a{{X0, X1}, {rmax0, rmax1}, {cols0, cols1}, rows, B};
    hipLaunchKernelGGL(rowmax2_kernel, dim3((rows + 3) / 4, 1, 2 * B), dim3(256), 0, s, a);
    return hipGetLastError();
}


}  // namespace

size_t bwd_split_workspace_tuned(int B, int D, int NQ, int H, int W, const GemmTune &t) {
    const int N = H * W;
    const size_t R = std::max(NQ, N);
    return 2 * al256((size_t)B * D * 4) + 2 * al256((size_t)B * R * 4) +
           al256(slab_floats(B, D, NQ, N, GemmTune{}) * sizeof(float)) + slab_floats(B, D, NQ, N, t) * sizeof(float);
}

size_t build_bwd_split_workspace(int B, int D, int NQ, int H, int W) {
    return bwd_split_workspace_tuned(B, D, NQ, H, W, GemmTune{});
}

// The GEMMs once dC's row maxima (w.mxB) and column maxima (w.mxC) are in the workspace (f16x3;
// bf: the exact bf16x6 split, no maxima read).
// C[b] (NI x NJ) = A[b] B[b]^T / sqrt(D) straight from the fp32 operands (split while staging).
// A GEMM's split-K sum not launched yet: the next GEMM runs it as appended tail workgroups
// (vec4 layout only: per % 4 == 0, 16-B aligned slab and C).
struct PendingReduce {
    const float *ws = nullptr;
    float *C = nullptr;
    int splits = 0;
    size_t per = 0;
    float sD = 1.f;
    NanFix fix;
};

// CU count of the current device, looked up once per device (a process may drive parts with
// different counts: the tail-reduce plan depends on it).
inline int device_cus() {
    static std::atomic<int> n[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::atomic<int> &slot = n[dev & 63];
    int v = slot.load(std::memory_order_relaxed);
    if (v == 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        slot.store(v, std::memory_order_relaxed);
    }
    return v;
}

// defer: if non-null and the sum is vec4-able, it is returned there instead of launched; tail: a
// previous GEMM's deferred sum, run by workgroups appended to this GEMM's grid (on the CUs its
// tiles leave idle) — the same bits as the separate reduce either way.
template <bool BCOL>
hipError_t gemm_f32(const float *A, long a_sb, long a_sr, const float *Bm, long b_sb, long b_sr, long b_sk,
                    const unsigned *mxA, const unsigned *mxB, int B, int NI, int NJ, int K, float sD, float *C,
                    float *slab, hipStream_t s, const GemmTune &t = GemmTune{}, bool bf = false,
                    PendingReduce *defer = nullptr, const PendingReduce *tail = nullptr) {
    FGemmParams p{};
    p.A = A, p.a_sb = a_sb, p.a_sr = a_sr;
    p.Bm = Bm, p.b_sb = b_sb, p.b_sr = b_sr, p.b_sk = b_sk;
    p.mxA = mxA, p.mxB = mxB;
    p.B = B, p.NI = NI, p.NJ = NJ, p.K = K;
    p.nkc = (K + kBK - 1) / kBK;
    p.ti = (NI + kTI - 1) / kTI;
    p.tj = (NJ + kTJ - 1) / kTJ;
    p.splits = plan_split_k(NI, NJ, p.nkc, B, t);
    p.kc_per = (p.nkc + p.splits - 1) / p.splits;
    p.splits = (p.nkc + p.kc_per - 1) / p.kc_per;
    const bool exact = is_pow2(sD);
    p.alpha = 1.0f / sD;
    // bf16x6: always the slab path, so that the reduce applies the non-finite rule (NanFix)
    p.direct = p.splits == 1 && exact && !bf;
    p.C = p.direct ? C : slab;
    p.nt = t.nt ? 1 : 0;
    auto al16 = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
    p.vec = al16(A) && al16(Bm) && a_sb % 4 == 0 && a_sr % 4 == 0 && b_sb % 4 == 0 &&
            (BCOL ? b_sk % 4 == 0 : b_sr % 4 == 0);
    if (bf) {  // the bf16x6 non-finite rule: NaN outputs recomputed as fp32 computes them
        p.fix.A = A, p.fix.Bm = Bm, p.fix.a_sb = a_sb, p.fix.a_sr = a_sr;
        p.fix.b_sb = b_sb, p.fix.b_sr = b_sr, p.fix.b_sk = b_sk;
        p.fix.NI = NI, p.fix.NJ = NJ, p.fix.K = K, p.fix.s = sD;
    }
    const bool dma = t.dma && p.vec && K % kBK == 0 && (!BCOL || NJ % 4 == 0);
    // 256-row tiles when there are more than 128 rows (D = 256): every staged element feeds twice
    // the MFMAs, a third less split work per MFMA (train: dF1 73 -> 67, dF2 75 -> 67 us)
    const bool wide = dma && t.wide && NI > 32 * kMI * kWI;
    hipError_t e;
    auto go1 = [&](auto dma_tag, auto wi_tag, auto pipe_tag, auto bf_tag) {
        constexpr bool D = decltype(dma_tag)::value;
        constexpr int WI = decltype(wi_tag)::value;
        constexpr bool P = decltype(pipe_tag)::value;
        constexpr bool BF = decltype(bf_tag)::value;
        FGemmParams q = p;
        q.ti = (NI + 32 * kMI * WI - 1) / (32 * kMI * WI);
        const long grid = (long)q.ti * q.tj * q.splits * B;
        q.gemm_wgs = (int)grid;
        long tail_wgs = 0;
        // resident workgroups per CU: LDS-bound (160 KiB) and wave-bound (32 waves per CU)
        constexpr int lds = gemm_lds_bytes<D, WI, P, BF>();
        constexpr int per_cu = std::min(163840 / lds, 32 / (WI * kWJ));
        const long slots = (long)device_cus() * per_cu;
        if (tail && tail->ws && grid + 16 > slots) {
            // no idle slots in the first round: the sum runs as its own launch, before this GEMM
            hipError_t e3 = launch_splitk_reduce(tail->ws, tail->C, tail->splits, tail->per, tail->sD, s, true,
                                                 &tail->fix);
            if (e3 != hipSuccess) return e3;
        } else if (tail && tail->ws) {
            tail_wgs = slots - grid;
            q.tail_ws = reinterpret_cast<const float4 *>(tail->ws);
            q.tail_C = reinterpret_cast<float4 *>(tail->C);
            q.tail_per4 = tail->per / 4;
            q.tail_splits = tail->splits;
            q.tail_exact = is_pow2(tail->sD) ? 1 : 0;
            q.tail_alpha = 1.0f / tail->sD;
            q.tail_s = tail->sD;
            q.tail_wgs = (int)tail_wgs;
            q.tail_fix = tail->fix;
        }
        static std::atomic<unsigned long long> done{0};
        hipError_t e2 = ensure_lds_limit((const void *)split_gemm_f32_kernel<BCOL, D, WI, P, BF>,
                                         gemm_lds_bytes<D, WI, P, BF>(), done);
        if (e2 != hipSuccess) return e2;
        hipLaunchKernelGGL((split_gemm_f32_kernel<BCOL, D, WI, P, BF>), dim3((unsigned)(grid + tail_wgs)),
                           dim3(64 * WI * kWJ), (gemm_lds_bytes<D, WI, P, BF>()), s, q);
        return hipSuccess;
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    using W2 = std::integral_constant<int, kWI>;
    using W4 = std::integral_constant<int, 4>;
    auto go = [&](auto dma_tag, auto wi_tag, auto pipe_tag) {
        return bf ? go1(dma_tag, wi_tag, pipe_tag, T_{}) : go1(dma_tag, wi_tag, pipe_tag, F_{});
    };
    e = wide ? (t.pipe ? go(T_{}, W4{}, T_{}) : go(T_{}, W4{}, F_{})) : dma ? go(T_{}, W2{}, F_{})
                                                                           : go(F_{}, W2{}, F_{});
    if (e != hipSuccess) return e;
    e = hipGetLastError();
    if (e != hipSuccess || p.direct) return e;
    const size_t per = (size_t)B * NI * NJ;
    if (defer && t.reduce_vec4 && per % 4 == 0 && al16(slab) && al16(C)) {
        defer->ws = slab, defer->C = C, defer->splits = p.splits, defer->per = per, defer->sD = sD;
        defer->fix = p.fix;
        return hipSuccess;
    }
    return launch_splitk_reduce(slab, C, p.splits, per, sD, s, t.reduce_vec4, &p.fix);
}

// rowmax_done: F2's and F1's row maxima are already in w.mxA / w.mxA2 (computed by the fold
// launch's appended workgroups).  bf: the bf16x6 GEMMs (no maxima at all).
hipError_t bwd_split_gemms(const float *grad_c, const float *f1, int NQ, const float *f2, int B, int D, int H, int W,
                           float *df1, float *df2, const BwdWs &w, hipStream_t s, bool rowmax_done = false,
                           bool bf = false) {
    const int N = H * W;
    const float sD = std::sqrt((float)D);
    hipError_t e;
#define CK_(x)                          \
    if ((e = (x)) != hipSuccess) return e;
    if (!rowmax_done && !bf) CK_(rowmax2(f2, N, w.mxA, f1, NQ, w.mxA2, B, D, s));
    // dF1 = F2 . dC^T : A = F2 rows d (k = m), B = dC rows n (k = m)
    // (its split-K sum deferred: dF2's grid carries it on the CUs its tiles leave idle)
    PendingReduce pend;
    CK_(gemm_f32<false>(f2, (long)D * N, N, grad_c, (long)NQ * N, N, 1, w.mxA, w.mxB, B, D, NQ, N, sD, df1, w.slab, s,
                        GemmTune{}, bf, &pend));
    // dF2 = F1 . dC : A = F1 rows d (k = n), B = dC columns m (k = n); its own slabs
    CK_(gemm_f32<true>(f1, (long)D * NQ, NQ, grad_c, (long)NQ * N, 1, N, w.mxA2, w.mxC, B, D, N, NQ, sD, df2, w.slab2,
                       s, GemmTune{}, bf, nullptr, &pend));
#undef CK_
    return hipSuccess;
}

// grad_c [B][NQ][N]; f1 [B][D][NQ]; f2 [B][D][N].  bf: the bf16x6 GEMMs (no maxima pass).
hipError_t launch_build_bwd_split(const float *grad_c, const float *f1, int NQ, const float *f2, int B, int D, int H,
                                  int W, float *df1, float *df2, void *ws, hipStream_t s, bool bf) {
    const int N = H * W;
    const BwdWs w = carve(ws, B, D, NQ, N);
    if (bf) return bwd_split_gemms(grad_c, f1, NQ, f2, B, D, H, W, df1, df2, w, s, true, true);
    hipError_t e = hipMemsetAsync(w.mx0, 0, w.mx_bytes, s);
    if (e == hipSuccess) e = absmax(grad_c, B, NQ, N, w.mxB, w.mxC, s);  // one pass: dC row and column maxima
    if (e != hipSuccess) return e;
    return bwd_split_gemms(grad_c, f1, NQ, f2, B, D, H, W, df1, df2, w, s);
}

// corr_backward's workspace: the backward GEMMs' plus, for F16X3, the fused path's per-workgroup
// column maxima ([B][groups][H*W] floats, 256-B aligned after the GEMM workspace).
size_t backward_workspace(int algo, int B, int D, int NQ, int H, int W, int radius) {
    if (algo == CORR_BUILD_FP32) return build_bwd_workspace(B, D, NQ, H, W);
    if (algo == CORR_BUILD_BF16X6) return build_bwd_split_workspace(B, D, NQ, H, W);
    if (algo != CORR_BUILD_F16X3) return (size_t)-1;
    const size_t base = (build_bwd_split_workspace(B, D, NQ, H, W) + 255) / 256 * 256;
    return base + (size_t)B * std::max(1, lookup_bwd_fold_groups(NQ, radius)) * H * W * sizeof(float);
}

// The pool-backward fold of a gradient pyramid into level 0 (in place); with `ws` (an F16X3
// backward workspace) its row / column maxima land where bwd_split_gemms reads them.
hipError_t launch_pool_fold(const LevelPtrs &gpyr, int B, int NQ, int H, int W, int levels, void *ws, int D,
                            hipStream_t s) {
    FoldArgs a{};
    for (int l = 0; l < levels; ++l) a.g[l] = gpyr.p[l];
    a.L = levels, a.NQ = NQ, a.H = H, a.W = W;
    a.vec = W % 4 == 0 && ((uintptr_t)gpyr.p[0] & 15) == 0 && (levels < 2 || ((uintptr_t)gpyr.p[1] & 7) == 0);
    if (ws) {
        const BwdWs w = carve(ws, B, D, NQ, H * W);
        hipError_t e = hipMemsetAsync(w.mx0, 0, w.mx_bytes, s);
        if (e != hipSuccess) return e;
        a.rmax = w.mxB, a.cmax = w.mxC;
    }
    const int nqb = (NQ + kFoldQ - 1) / kFoldQ;
    if (a.vec)
        hipLaunchKernelGGL(pool_fold_max_kernel<true>, dim3((unsigned)(nqb * B)), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(pool_fold_max_kernel<false>, dim3((unsigned)(nqb * B)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// The whole backward of one build and its T lookups (corr_backward): multi-lookup gradient
// assembly into gpyr (overwritten), the fold with dC's maxima, then the two GEMMs.
hipError_t launch_backward(int algo, const float *const *coords, const float *const *grad_out, int T,
                           const float *f1, int NQ, const float *f2, int B, int D, int H, int W, int levels, int radius,
                           const LevelPtrs &gpyr, float *df1, float *df2, void *ws, hipStream_t s) {
    const bool exact = (algo & CORR_BACKWARD_EXACT_FOLD) != 0;
    algo &= ~CORR_BACKWARD_EXACT_FOLD;
    hipError_t e;
    {  // fused: all lookups + the fold in one launch, dC and its row maxima straight out of LDS,
       // the column maxima as per-workgroup partials reduced by colmax_reduce_kernel
        unsigned *rmax = nullptr, *cmax = nullptr;
        float *cpart = nullptr;
        BwdWs w{};
        const int N = H * W, G = lookup_bwd_fold_groups(NQ, radius);
        if (algo == CORR_BUILD_F16X3) {
            // no memset: every maximum is stored whole — dC's row maxima by the fold kernel, its
            // column maxima by colmax_reduce_kernel, F1's and F2's by rowmax2_kernel (the
            // fallback below zeroes them for pool_fold_max_kernel's atomics itself)
            w = carve(ws, B, D, NQ, N);
            rmax = w.mxB, cmax = w.mxC;
            cpart = reinterpret_cast<float *>(static_cast<char *>(ws) +
                                              (build_bwd_split_workspace(B, D, NQ, H, W) + 255) / 256 * 256);
        }
        FoldRowMax rm{};
        if (algo == CORR_BUILD_F16X3) {  // F2's and F1's row maxima in the fold launch's tail
            rm.x[0] = f2, rm.x[1] = f1;
            rm.out[0] = w.mxA, rm.out[1] = w.mxA2;
            rm.cols[0] = N, rm.cols[1] = NQ;
            rm.rows = D;
        }
        e = launch_lookup_bwd_fold(coords, grad_out, T, B, NQ, H, W, levels, radius, gpyr.p[0], rmax, cmax, cpart, s,
                                   rm, exact);
        if (e == hipSuccess) {
            if (algo == CORR_BUILD_BF16X6)
                return bwd_split_gemms(gpyr.p[0], f1, NQ, f2, B, D, H, W, df1, df2, carve(ws, B, D, NQ, N), s, true,
                                       true);
            if (algo == CORR_BUILD_F16X3) {
                hipLaunchKernelGGL(colmax_reduce_kernel, dim3((unsigned)((N + kCmCols - 1) / kCmCols), (unsigned)B),
                                   dim3(kCmCols * kCmSlices), 0, s, cpart, G, N, cmax);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                return bwd_split_gemms(gpyr.p[0], f1, NQ, f2, B, D, H, W, df1, df2, w, s, true);
            }
            return launch_build_bwd(gpyr.p[0], f1, NQ, f2, B, D, H, W, df1, df2, (float *)ws, s);
        }
        if (e != hipErrorNotSupported) return e;
        (void)hipGetLastError();
    }
    e = launch_lookup_bwd_multi(coords, grad_out, T, B, NQ, H, W, levels, radius, gpyr, s);
    if (e != hipSuccess) return e;
    if (algo == CORR_BUILD_BF16X6) {
        e = launch_pool_fold(gpyr, B, NQ, H, W, levels, nullptr, D, s);
        if (e != hipSuccess) return e;
        return bwd_split_gemms(gpyr.p[0], f1, NQ, f2, B, D, H, W, df1, df2, carve(ws, B, D, NQ, H * W), s, true, true);
    }
    if (algo == CORR_BUILD_F16X3) {
        e = launch_pool_fold(gpyr, B, NQ, H, W, levels, ws, D, s);
        if (e != hipSuccess) return e;
        return bwd_split_gemms(gpyr.p[0], f1, NQ, f2, B, D, H, W, df1, df2, carve(ws, B, D, NQ, H * W), s);
    }
    e = launch_pool_fold(gpyr, B, NQ, H, W, levels, nullptr, D, s);
    if (e != hipSuccess) return e;
    return launch_build_bwd(gpyr.p[0], f1, NQ, f2, B, D, H, W, df1, df2, (float *)ws, s);
}

}  // namespace corr
