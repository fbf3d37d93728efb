// build_split_r01.hip — ROUND-1 f16x3 build (kept for A/B timing in tools/kbench_build.hip only;
// not part of libcorr_mi355x.so).  32x32x16 MFMA, queries as MFMA rows, LDS-staged epilogue.
// Namespace corr::r01 so that it links beside the product kernels.
//
// Replaces the same reference code as corr_build.hip — CorrBlock.corr (model/corr.py:52-60:
// matmul(F1^T, F2) / sqrt(D)) and the pyramid loop of CorrBlock.__init__ (model/corr.py:21-27)
// — but runs the contraction on the f16 MFMA, which gfx950 issues 16x faster than its fp32 MFMA.
//
// Operands.  Every fp32 feature x of pixel n is rewritten as
//     x = 2^e_n * (hi + lo) + O(2^-22 |x|),   hi = f16(x * 2^-e_n),  lo = f16(x * 2^-e_n - hi)
// with a per-pixel power-of-two e_n that puts the pixel's largest |x| in [2^14, 2^15): neither
// half overflows, and the f16 subnormal floor lies 2^-38 below the pixel's largest value.  A dot
// product is then three f16 MFMAs into ONE fp32 accumulator,
//     acc += lo_q * hi_t;   acc += hi_q * lo_t;   acc += hi_q * hi_t,
// whose f16 x f16 products are exact in fp32; what is dropped (lo*lo, the lo rounding) is
// <= 2^-22 relative per term — the size of fp32 accumulation rounding itself.  The epilogue
// multiplies by 2^(e_q + e_t) (exact) and by 1/sqrt(D) as the fp32 build does.  Measured: the
// split build differs from the exact-fp32 MFMA build by ~1e-6 of max|C| (tools/kbench_split.hip);
// both are checked against the reference within the north_star's 1e-4.
//
// Tile.  A = queries (MFMA rows), B = targets (MFMA columns), so every lane owns ONE target
// pixel of a 32-pixel block and the 16 accumulator registers hold 16 queries.  A target block
// is 2 rows x 16 columns of the map, interleaved lane = 2*col + row: one accumulator register
// stored as is writes 64-byte runs of 16 consecutive pixels (4 runs per instruction, no
// shuffles), and every 2x2 average-pool window sits inside one lane quad, so the pyramid is
// built in registers with DPP adds (levels 2 and 3 with row shifts by 4 and 8 lanes).  A wave
// owns 32*MQ queries x an 8x16 target patch (4 blocks); a workgroup WQ x WT waves, the patch
// 8*WT rows tall.  K = D is staged through LDS in 16-deep chunks (one MFMA k-step), double
// buffered, the global loads of chunk c+1 in flight while chunk c feeds the MFMAs.
//
// Packed operand layout (split_pack_kernel -> corr_build_split_kernel), chunk-major so that a
// workgroup's chunk of consecutive pixels is one contiguous run:
//   pk[b][kc][n][4 x 16 B]  kc = 0..KP/16-1; the four 16-B units are hi(k = 16kc..+7),
//                           lo(same), hi(k = 16kc+8..+15), lo(same)  (8 f16 each)
//   ex[b][n] = e_n (int32).  KP = D rounded up to 16 (zero padding).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "../../e-raft_amd/csrc/corr_build_common.h"

namespace corr {
namespace r01 {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs

constexpr int kSplitBK = 16;  // k per chunk (= per MFMA k-step); 64 B per pixel per chunk

inline int split_kp(int D) { return (D + kSplitBK - 1) / kSplitBK * kSplitBK; }

// ---------------------------------------------------------------------------------------
// Operand pack.  One workgroup per TP pixels of one tensor (blockIdx.z: 0 = fmap1, 1 = fmap2):
// the [D][TP] block is read once (coalesced rows) into LDS as [TP][KP + 4], the per-pixel
// max |x| is reduced, and each thread writes one 16-B unit, consecutive threads covering a
// chunk plane's consecutive pixels (fully coalesced stores).
// ---------------------------------------------------------------------------------------
struct PackArgs {
    const float *f[2];
    u32x4 *pk[2];
    int *ex[2];
    int np[2];
    int D, KP, TP;
};

__global__ __launch_bounds__(256) void split_pack_kernel(PackArgs a) {
    extern __shared__ __attribute__((aligned(16))) float pack_lds[];
    const int z = blockIdx.z, b = blockIdx.y, tid = threadIdx.x;
    const int NP = a.np[z], D = a.D, KP = a.KP, TP = a.TP, RS = KP + 4;
    const int n0 = blockIdx.x * TP;
    if (n0 >= NP) return;  // the grid covers the larger of the two tensors
    float *tile = pack_lds;           // [TP][RS]
    float *red = pack_lds + TP * RS;  // [256] partial maxima, then [TP] shifts
    const float *src = a.f[z] + (size_t)b * D * NP;
    const int G = 256 / TP, p = tid % TP, g = tid / TP;
    const int n = min(n0 + p, NP - 1);  // clamped: unconditional loads
    float m = 0.f;
#pragma unroll 4
    for (int d = g; d < D; d += G) {
        const float v = src[(size_t)d * NP + n];
        tile[p * RS + d] = v;
        m = fmaxf(m, fabsf(v));
    }
    for (int d = D + g; d < KP; d += G) tile[p * RS + d] = 0.f;
    red[tid] = m;
    __syncthreads();
    if (tid < TP) {
        float mm = 0.f;
        for (int k = 0; k < G; ++k) mm = fmaxf(mm, red[k * TP + tid]);
        int s = 0;
        if (mm > 0.f && mm <= 3.402823466e38f) {
            int E;
            (void)frexpf(mm, &E);  // mm < 2^E
            s = 15 - E;            // mm * 2^s < 2^15: neither half overflows
        }
        if (n0 + tid < NP) a.ex[z][(size_t)b * NP + n0 + tid] = -s;
        red[256 + tid] = __int_as_float(s);
    }
    __syncthreads();
    const int nkc = KP / kSplitBK, units = TP * 4;  // 16-B units per chunk plane of this block
    const int valid = min(TP, NP - n0);
    for (int it = tid; it < nkc * units; it += 256) {
        const int kc = it / units, r = it - kc * units;
        const int px = r >> 2, u = r & 3;  // u: (k-octet u >> 1, lo = u & 1)
        if (px >= valid) continue;
        const int s = __float_as_int(red[256 + px]);
        const float *x = &tile[px * RS + kc * 16 + (u >> 1) * 8];
        const float4 u0 = *reinterpret_cast<const float4 *>(x);
        const float4 u1 = *reinterpret_cast<const float4 *>(x + 4);
        const float xs[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
        half8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float y = ldexpf(xs[j], s);
            const _Float16 hi = (_Float16)y;
            o[j] = (u & 1) ? (__builtin_isinf(y) ? (_Float16)0.f : (_Float16)(y - (float)hi)) : hi;
        }
        a.pk[z][(((size_t)b * nkc + kc) * NP + n0 + px) * 4 + u] = __builtin_bit_cast(u32x4, o);
    }
}

// Register-resident pack (the default for D <= 512): 16 pixels per workgroup of 4 waves, lane
// = 4 * pixel + unit, so every store instruction of a wave writes 16 consecutive pixels' four
// 16-B units — one contiguous 1 KiB run of a chunk plane.  Wave w holds the chunks
// kc = w, w + 4, ... : the lane loads the 8 features of its unit's k-octet (the hi and lo lanes
// of an octet load the same addresses; the coalescer merges them), all loads issued before the
// first use.  The per-pixel max is reduced over the quad with a DPP swap and over the 4 waves
// through LDS.  Same arithmetic as split_pack_kernel, element for element (bit-identical packs).
constexpr int kPackTP = 16, kPackW = 4;

template <int CPT>
__global__ __launch_bounds__(64 * kPackW) void split_pack_reg_kernel(PackArgs a) {
    __shared__ float red[kPackW][kPackTP];
    const int z = blockIdx.z, b = blockIdx.y, tid = threadIdx.x;
    const int NP = a.np[z], D = a.D, nkc = a.KP / kSplitBK;
    const int n0 = blockIdx.x * kPackTP;
    if (n0 >= NP) return;  // the grid covers the larger of the two tensors (uniform exit)
    const int lane = tid & 63, w = tid >> 6;
    const int p = lane >> 2, u = lane & 3;  // u: (k-octet u >> 1, lo = u & 1)
    const int n = min(n0 + p, NP - 1);      // clamped: unconditional loads
    const float *src = a.f[z] + (size_t)b * D * NP + n;
    float v[CPT][8];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int kc = w + kPackW * c;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int d = kc * kSplitBK + (u >> 1) * 8 + j;
            v[c][j] = (kc < nkc && d < D) ? src[(size_t)d * NP] : 0.f;
        }
    }
    float m = 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[c][j]));
    m = fmaxf(m, __shfl_xor(m, 2));  // the other k-octet of the pixel's chunks
    if (u == 0) red[w][p] = m;
    __syncthreads();
    float mm = 0.f;
#pragma unroll
    for (int k = 0; k < kPackW; ++k) mm = fmaxf(mm, red[k][p]);
    int s = 0;
    if (mm > 0.f && mm <= 3.402823466e38f) {
        int E;
        (void)frexpf(mm, &E);  // mm < 2^E
        s = 15 - E;            // mm * 2^s < 2^15: neither half overflows
    }
    const bool live = n0 + p < NP;
    if (w == 0 && u == 0 && live) a.ex[z][(size_t)b * NP + n0 + p] = -s;
    if (!live) return;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int kc = w + kPackW * c;
        if (kc >= nkc) break;
        half8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float y = ldexpf(v[c][j], s);
            const _Float16 hi = (_Float16)y;
            o[j] = (u & 1) ? (__builtin_isinf(y) ? (_Float16)0.f : (_Float16)(y - (float)hi)) : hi;
        }
        a.pk[z][(((size_t)b * nkc + kc) * NP + n0 + p) * 4 + u] = __builtin_bit_cast(u32x4, o);
    }
}

// Pixel-lane pack: lane = pixel, 64 consecutive pixels per workgroup of NW waves, wave w holding
// the chunks kc = w, w + NW, ... .  Every load instruction reads one feature of 64 consecutive
// pixels (256 contiguous bytes; the register pack's read 2 x 64 B), and a lane writes its
// pixel's whole 64-B chunk record as four 16-B stores that together cover the wave's 4 KiB run.
// The per-pixel max is reduced over the NW waves through LDS.  Same arithmetic as
// split_pack_kernel, element for element (bit-identical packs).
template <int NW, int CPT>
__global__ __launch_bounds__(64 * NW) void split_pack_px_kernel(PackArgs a) {
    __shared__ float red[NW][64];
    const int z = blockIdx.z, b = blockIdx.y, tid = threadIdx.x;
    const int NP = a.np[z], D = a.D, nkc = a.KP / kSplitBK;
    const int n0 = blockIdx.x * 64;
    if (n0 >= NP) return;  // the grid covers the larger of the two tensors (uniform exit)
    const int lane = tid & 63, w = tid >> 6;
    const int n = min(n0 + lane, NP - 1);  // clamped: unconditional loads
    const float *src = a.f[z] + (size_t)b * D * NP + n;
    float v[CPT][16];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int kc = w + NW * c;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int d = kc * kSplitBK + j;
            v[c][j] = (kc < nkc && d < D) ? src[(size_t)d * NP] : 0.f;
        }
    }
    float m = 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int j = 0; j < 16; ++j) m = fmaxf(m, fabsf(v[c][j]));
    red[w][lane] = m;
    __syncthreads();
    float mm = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) mm = fmaxf(mm, red[k][lane]);
    int s = 0;
    if (mm > 0.f && mm <= 3.402823466e38f) {
        int E;
        (void)frexpf(mm, &E);  // mm < 2^E
        s = 15 - E;            // mm * 2^s < 2^15: neither half overflows
    }
    const bool live = n0 + lane < NP;
    if (w == 0 && live) a.ex[z][(size_t)b * NP + n0 + lane] = -s;
    if (!live) return;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int kc = w + NW * c;
        if (kc >= nkc) break;
        u32x4 *dst = a.pk[z] + (((size_t)b * nkc + kc) * NP + n0 + lane) * 4;
#pragma unroll
        for (int oct = 0; oct < 2; ++oct) {
            half8 hi8, lo8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float y = ldexpf(v[c][oct * 8 + j], s);
                const _Float16 hi = (_Float16)y;
                hi8[j] = hi;
                lo8[j] = __builtin_isinf(y) ? (_Float16)0.f : (_Float16)(y - (float)hi);
            }
            dst[2 * oct] = __builtin_bit_cast(u32x4, hi8);
            dst[2 * oct + 1] = __builtin_bit_cast(u32x4, lo8);
        }
    }
}

// Chunks per wave of the register pack for this KP, 0 = use the LDS pack.
inline int split_pack_cpt(int KP) {
    const int nkc = KP / kSplitBK;
    const int cpt = (nkc + kPackW - 1) / kPackW;
    return cpt <= 8 ? cpt : 0;
}

// Pixels per pack workgroup for this KP (LDS: TP*(KP+4)*4 + (256+TP)*4 <= 160 KiB); 0 = too large.
inline int split_pack_tp(int KP) {
    for (int tp = 32; tp >= 4; tp >>= 1)
        if ((size_t)tp * (KP + 4) * 4 + (256 + tp) * 4 <= 160 * 1024) return tp;
    return 0;
}

// ---------------------------------------------------------------------------------------
// The MFMA build.
// ---------------------------------------------------------------------------------------
template <int WQ_, int WT_, int MQ_, int OCC_>
struct SplitCfg {
    static constexpr int WQ = WQ_, WT = WT_, MQ = MQ_, OCC = OCC_;
    static constexpr int NT = 64 * WQ * WT;
    static constexpr int BQ = 32 * MQ * WQ;       // queries per tile
    static constexpr int PH = 8 * WT;             // target patch rows (x 16 columns)
    static constexpr int BT = 128 * WT;           // targets per tile
    static constexpr int ROWS = BQ + BT;          // LDS rows (pixels) per stage, 64 B each
    static constexpr int RPP = NT / 4;            // rows staged per pass (4 threads x 16 B)
    static constexpr int LPT = ROWS / RPP;        // 16-B loads per thread per chunk
    static constexpr size_t LDS_OPS = 2ull * ROWS * 64;
    static constexpr size_t LDS_EPI = (size_t)(NT / 64) * 13568;  // per-wave epilogue staging (kEpiBytes)
    static constexpr size_t LDS_MAIN = LDS_OPS > LDS_EPI ? LDS_OPS : LDS_EPI;
    static constexpr size_t LDS = LDS_MAIN + (size_t)ROWS * 4;  // + exponents
    static_assert(ROWS % RPP == 0, "staging must tile the chunk");
};

using SplitDefault = SplitCfg<2, 2, 2, 2>;

struct SplitParams {
    const u32x4 *pk1, *pk2;  // packed queries / targets
    const int *ex1, *ex2;
    float *lvl[kFusedLevels];
    int B, H, W, N, NQ, nkc, nlev;
    int nq, npx, npy;        // query blocks, patch columns (16 px), patch rows (8*WT px)
    int eshift;              // log2(1/sqrt(D)) when that is exact, else 0
    int exact;               // 1/sqrt(D) is a power of two, folded into the exponent
    int vec0, vec1;          // !VEC: store width of levels 0 / 1 (store_run4_mode: 2, 1 or 0)
    float inv_s;             // 1/sqrt(D) otherwise (multiplied: within tolerance, not bitwise)
};

// LDS image of a stage: row j (pixel) = 4 x 16-B units, unit u stored at u ^ ((j >> 2) & 3):
// each 16-lane ds_read_b128 group of a 32x32x16 fragment read then hits 16 distinct 16-B bank
// groups, and the row stores (8 lanes = 2 rows) 8 distinct ones.
__device__ __forceinline__ int swz(int j, int u) { return j * 4 + (u ^ ((j >> 2) & 3)); }

// Grouped tile order (L2 reuse): per batch item, query blocks in groups of kGroupQ; inside a
// group the query block runs fastest, then the target patch.  The tiles one XCD has in flight
// (consecutive, see xcd_swizzle) cover ~kGroupQ query blocks x a few target patches.
constexpr int kGroupQ = 8;

struct TileCoord {
    int px, py, qb, b;
};

__device__ __forceinline__ TileCoord tile_coord(const SplitParams &p, int tile) {
    const int np = p.npx * p.npy, per_b = p.nq * np;
    TileCoord t;
    t.b = tile / per_b;
    const int r = tile - t.b * per_b;
    const int g = r / (kGroupQ * np);
    const int gm = min(kGroupQ, p.nq - g * kGroupQ);
    const int r2 = r - g * kGroupQ * np;
    const int tp = r2 / gm;
    t.qb = g * kGroupQ + (r2 - tp * gm);
    t.px = tp % p.npx;
    t.py = tp / p.npx;
    return t;
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
constexpr int kQuadSwap1 = 0xB1;  // quad_perm [1,0,3,2]: lane 4k reads 4k+1
constexpr int kRowShl4 = 0x104;   // lane i reads i+4 (same 16-lane row)
constexpr int kRowShl8 = 0x108;   // lane i reads i+8

// ((a + b) + c) + d for the 2x2 window whose a sits in this lane (the reference's order).
template <int CB, int CC, int CD>
__device__ __forceinline__ float pool_sum(float ab, float cd) {
    float t = ab + dpp<CB>(ab);
    t = t + dpp<CC>(cd);
    return t + dpp<CD>(cd);
}

// Store n = 1, 2 or 4 consecutive values of one map row at columns [X, X + n), clipped to the row
// width Wl.  VEC: the launch guarantees aligned, fully in-map runs whenever X < Wl.
template <int NV, bool VEC>
__device__ __forceinline__ void store_run(float *row, int X, int Wl, const float *v) {
    if constexpr (VEC) {
        if (X < Wl) {
            if constexpr (NV == 4) *reinterpret_cast<float4 *>(row + X) = make_float4(v[0], v[1], v[2], v[3]);
            else if constexpr (NV == 2) *reinterpret_cast<float2 *>(row + X) = make_float2(v[0], v[1]);
            else row[X] = v[0];
        }
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (X + k < Wl) row[X + k] = v[k];
    }
}

// Run of 4 at column X (a multiple of 4) with a store width picked per launch: mode 2 = one
// 16-B store (W % 4 == 0), 1 = two 8-B stores (W even), 0 = element stores.  Uniform per level.
__device__ __forceinline__ void store_run4_mode(float *row, int X, int Wl, const float *v, int mode) {
    if (mode == 2) {
        store_run<4, true>(row, X, Wl, v);
    } else if (mode == 1) {
        if (X < Wl) *reinterpret_cast<float2 *>(row + X) = make_float2(v[0], v[1]);
        if (X + 2 < Wl) *reinterpret_cast<float2 *>(row + X + 2) = make_float2(v[2], v[3]);
    } else {
        store_run<4, false>(row, X, Wl, v);
    }
}

// Per-wave LDS staging of the epilogue (floats): L0 [32 q][4 rows][16 cols] (half of the 8x16
// patch at a time), L1 [32][4][8], L2 [32][2][4], L3 [32][2].
constexpr int kEpiL0 = 32 * 4 * 16, kEpiL1 = 32 * 4 * 8, kEpiL2 = 32 * 2 * 4, kEpiL3 = 32 * 2;
constexpr size_t kEpiBytes = (size_t)(kEpiL0 + kEpiL1 + kEpiL2 + kEpiL3) * 4;

// Epilogue.  (1) In the MFMA layout: exponents back and 1/sqrt(D) (one ldexp; a multiply by
// 1/sqrt(D) when that is not a power of two), then the 32 queries x 4 rows x 16 columns of half
// the patch go to this wave's LDS region.  (2) Drain: lane L reads 16 B = 4 consecutive pixels
// of (query, row) = (u >> 4, (u >> 2) & 3) for u = 64 it + L and stores them; the rows of a
// 2x2 pooling window then sit 4 lanes apart, so level 1 is two DPP-fused add chains per float4,
// level 2 pairs level-1 rows 8 lanes apart, level 3 pairs level-2 columns in adjacent lanes
// across the two halves — every pooled value is produced once, in the reference's
// ((a + b) + c) + d order, and staged for 16-B row-run stores.
// MFMA layout: lane l32 = 2c + r of block tt holds target (Y0 + 2tt + r, X0 + c); register g
// holds query (g & 3) + 8 (g >> 2) + 4h of the 32-query block.
template <class Cfg, bool VEC>
__device__ __forceinline__ void split_epilogue(const SplitParams &p, f32x16 (&acc)[Cfg::MQ][4], const TileCoord &tc,
                                               const int *lds_ex, float *epi, const int wq, const int wt,
                                               const int h, const int l32) {
    constexpr int BQ = Cfg::BQ, MQ = Cfg::MQ;
    const int b = tc.b, q0 = tc.qb * BQ;
    const int NQ = p.NQ, W = p.W, H = p.H, N = p.N;
    const int lane = h * 32 + l32;
    const int trow0 = BQ + wt * 128 + l32;
    const int Y0 = (tc.py * Cfg::WT + wt) * 8, X0 = tc.px * 16;
    const int c = l32 >> 1, rr = l32 & 1;
    const int H1 = H >> 1, W1 = W >> 1, H2 = H >> 2, W2 = W >> 2, H3 = H >> 3, W3 = W >> 3;
    const int nlev = p.nlev;
    float *R0 = epi, *R1 = epi + kEpiL0, *R2 = R1 + kEpiL1, *R3 = R2 + kEpiL2;
    int et[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) et[t] = lds_ex[trow0 + 32 * t] + p.eshift;
    // this lane's drain coordinates (fixed over iterations except the query)
    const int dc4 = lane & 3, drow = (lane >> 2) & 3;
#pragma unroll
    for (int i = 0; i < MQ; ++i) {
        const int qb0 = wq * (32 * MQ) + i * 32;  // block's first query (tile-local)
        // ---- scale in place ----
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int eq = lds_ex[qb0 + (g & 3) + 8 * (g >> 2) + 4 * h];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                float x = ldexpf(acc[i][t][g], eq + et[t]);
                if (!p.exact) x = x * p.inv_s;
                acc[i][t][g] = x;
            }
        }
        float l2keep[8];
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            // stage rows 4 half .. 4 half + 3 (blocks tt = 2 half, 2 half + 1)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int ql = (g & 3) + 8 * (g >> 2) + 4 * h;
                R0[ql * 64 + rr * 16 + c] = acc[i][2 * half][g];
                R0[ql * 64 + (2 + rr) * 16 + c] = acc[i][2 * half + 1][g];
            }
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int ql = it * 4 + (lane >> 4);
                const float4 v4 = reinterpret_cast<const float4 *>(R0)[it * 64 + lane];
                const int q = q0 + qb0 + ql;
                const size_t qrow = (size_t)b * NQ + q;
                const bool qok = q < NQ;
                {
                    const int Y = Y0 + 4 * half + drow;
                    const float e4[4] = {v4.x, v4.y, v4.z, v4.w};
                    if (nlev > 0 && qok && Y < H) {
                        float *row = p.lvl[0] + qrow * N + (size_t)Y * W;
                        if constexpr (VEC) store_run<4, true>(row, X0 + 4 * dc4, W, e4);
                        else store_run4_mode(row, X0 + 4 * dc4, W, e4, p.vec0);
                    }
                }
                // level 1 at lanes with an even row: columns 2 dc4, 2 dc4 + 1 of L1 row 2 half + drow / 2
                float s0 = v4.x + v4.y;
                s0 = s0 + dpp<kRowShl4>(v4.x);
                s0 = s0 + dpp<kRowShl4>(v4.y);
                float s1 = v4.z + v4.w;
                s1 = s1 + dpp<kRowShl4>(v4.z);
                s1 = s1 + dpp<kRowShl4>(v4.w);
                const float a0 = s0 * 0.25f, a1 = s1 * 0.25f;
                if ((drow & 1) == 0)
                    *reinterpret_cast<float2 *>(&R1[ql * 32 + (2 * half + (drow >> 1)) * 8 + 2 * dc4]) = make_float2(a0, a1);
                // level 2 at lanes with row 0: column dc4 of L2 row `half`
                float s2 = a0 + a1;
                s2 = s2 + dpp<kRowShl8>(a0);
                s2 = s2 + dpp<kRowShl8>(a1);
                const float a2 = s2 * 0.25f;
                if (drow == 0) R2[ql * 8 + half * 4 + dc4] = a2;
                if (half == 0) {
                    l2keep[it] = a2;
                } else {
                    // level 3 at lanes with row 0 and an even column: column dc4 / 2
                    float s3 = l2keep[it] + dpp<kQuadSwap1>(l2keep[it]);
                    s3 = s3 + a2;
                    s3 = s3 + dpp<kQuadSwap1>(a2);
                    if (drow == 0 && (dc4 & 1) == 0) R3[ql * 2 + (dc4 >> 1)] = s3 * 0.25f;
                }
            }
        }
        // ---- drain L1 (4 x 16 B per lane), L2 (16 B), L3 (8 B) ----
        if (nlev > 1) {
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int u = it * 64 + lane, ql = u >> 3, row = (u >> 1) & 3, c4 = u & 1;
                const float4 v4 = reinterpret_cast<const float4 *>(R1)[u];
                const float e4[4] = {v4.x, v4.y, v4.z, v4.w};
                const int q = q0 + qb0 + ql, Y = (Y0 >> 1) + row;
                if (q < NQ && Y < H1) {
                    float *row1 = p.lvl[1] + ((size_t)b * NQ + q) * (size_t)(H1 * W1) + (size_t)Y * W1;
                    if constexpr (VEC) store_run<4, true>(row1, (X0 >> 1) + 4 * c4, W1, e4);
                    else store_run4_mode(row1, (X0 >> 1) + 4 * c4, W1, e4, p.vec1);
                }
            }
        }
        if (nlev > 2) {
            const int ql = lane >> 1, row = lane & 1;
            const float4 v4 = reinterpret_cast<const float4 *>(R2)[lane];
            const float e4[4] = {v4.x, v4.y, v4.z, v4.w};
            const int q = q0 + qb0 + ql, Y = (Y0 >> 2) + row;
            if (q < NQ && Y < H2)
                store_run<4, VEC>(p.lvl[2] + ((size_t)b * NQ + q) * (size_t)(H2 * W2) + (size_t)Y * W2, X0 >> 2, W2, e4);
        }
        if (nlev > 3 && lane < 32) {
            const float2 v2 = reinterpret_cast<const float2 *>(R3)[lane];
            const float e2[2] = {v2.x, v2.y};
            const int q = q0 + qb0 + lane, Y = Y0 >> 3;
            if (q < NQ && Y < H3)
                store_run<2, VEC>(p.lvl[3] + ((size_t)b * NQ + q) * (size_t)(H3 * W3) + (size_t)Y * W3, X0 >> 3, W3, e2);
        }
    }
}

template <class Cfg, bool VEC>
__global__ __launch_bounds__(Cfg::NT, Cfg::OCC) void corr_build_split_kernel(SplitParams p) {
    constexpr int BQ = Cfg::BQ, MQ = Cfg::MQ, ROWS = Cfg::ROWS, RPP = Cfg::RPP, LPT = Cfg::LPT;
    extern __shared__ __attribute__((aligned(16))) u32x4 smem_split[];
    static_assert(Cfg::LDS_EPI == (Cfg::NT / 64) * kEpiBytes, "epilogue staging size");
    int *lds_ex = reinterpret_cast<int *>(reinterpret_cast<char *>(smem_split) + Cfg::LDS_MAIN);

    const TileCoord tc = tile_coord(p, xcd_swizzle(blockIdx.x, gridDim.x));
    const int b = tc.b, q0 = tc.qb * BQ;
    const int NQ = p.NQ, W = p.W, H = p.H, N = p.N;
    const int tid = threadIdx.x;
    const int lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wv = tid >> 6, wq = wv / Cfg::WT, wt = wv % Cfg::WT;

    // staging: thread -> unit (tid & 3) of rows (tid >> 2) + RPP*i.  Rows outside the map load
    // a clamped in-map pixel: they feed only outputs the epilogue discards, and unconditional
    // loads keep a chunk's loads in flight together.
    const int unit = tid & 3, r0 = tid >> 2;
    auto row_pixel = [&](int j, const u32x4 *&base, const int *&ebase) {
        if (j < BQ) {
            const int q = min(q0 + j, NQ - 1);
            base = p.pk1 + ((size_t)b * p.nkc * NQ + q) * 4;
            ebase = p.ex1 + (size_t)b * NQ + q;
        } else {
            const int t = j - BQ;  // wave-row wt2 = t >> 7, block tt = (t >> 5) & 3, lane l = t & 31
            const int Y = min((tc.py * Cfg::WT + (t >> 7)) * 8 + ((t >> 5) & 3) * 2 + (t & 1), H - 1);
            const int X = min(tc.px * 16 + ((t & 31) >> 1), W - 1);
            base = p.pk2 + ((size_t)b * p.nkc * N + (size_t)Y * W + X) * 4;
            ebase = p.ex2 + (size_t)b * N + (size_t)Y * W + X;
        }
    };
    static_assert(BQ % RPP == 0, "query rows fill whole staging passes");
    constexpr int LQ = BQ / RPP;  // passes i < LQ stage query rows, the rest target rows
    const u32x4 *src[LPT];
    const size_t plane1 = (size_t)NQ * 4, plane2 = (size_t)N * 4;  // u32x4 per chunk plane
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
        const int *eb;
        row_pixel(r0 + RPP * i, src[i], eb);
        src[i] += unit;
    }
    // exponents of the tile's rows -> LDS (read after the first barrier)
    for (int j = tid; j < ROWS; j += Cfg::NT) {
        const u32x4 *bb;
        const int *eb;
        row_pixel(j, bb, eb);
        lds_ex[j] = *eb;
    }

    u32x4 rg[LPT];
    auto load_chunk = [&](int kc) {
#pragma unroll
        for (int i = 0; i < LPT; ++i) rg[i] = src[i][kc * (i < LQ ? plane1 : plane2)];
    };
    auto store_chunk = [&](int st) {
        u32x4 *S = smem_split + (size_t)st * ROWS * 4;
#pragma unroll
        for (int i = 0; i < LPT; ++i) S[swz(r0 + RPP * i, unit)] = rg[i];
    };

    f32x16 acc[MQ][4];
#pragma unroll
    for (int i = 0; i < MQ; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int qrow0 = wq * (32 * MQ) + l32;  // LDS row of this lane's query fragment (mq = 0)
    const int trow0 = BQ + wt * 128 + l32;   // ... of its target fragment (tt = 0)
    load_chunk(0);
    store_chunk(0);
    __syncthreads();
    for (int kc = 0; kc < p.nkc; ++kc) {
        const int st = kc & 1;
        if (kc + 1 < p.nkc) load_chunk(kc + 1);
        const u32x4 *S = smem_split + (size_t)st * ROWS * 4;
        half8 qh[MQ], ql[MQ], th[4], tl[4];
#pragma unroll
        for (int i = 0; i < MQ; ++i) {
            qh[i] = __builtin_bit_cast(half8, S[swz(qrow0 + 32 * i, 2 * h)]);
            ql[i] = __builtin_bit_cast(half8, S[swz(qrow0 + 32 * i, 2 * h + 1)]);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            th[t] = __builtin_bit_cast(half8, S[swz(trow0 + 32 * t, 2 * h)]);
            tl[t] = __builtin_bit_cast(half8, S[swz(trow0 + 32 * t, 2 * h + 1)]);
        }
#pragma unroll
        for (int i = 0; i < MQ; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ql[i], th[t], acc[i][t], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MQ; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qh[i], tl[t], acc[i][t], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MQ; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qh[i], th[t], acc[i][t], 0, 0, 0);
        if (kc + 1 < p.nkc) store_chunk(st ^ 1);
        __syncthreads();
    }

    // (the loop's last barrier: every wave is done with the stages the epilogue reuses)
    float *epi = reinterpret_cast<float *>(reinterpret_cast<char *>(smem_split) + (size_t)wv * kEpiBytes);
    split_epilogue<Cfg, VEC>(p, acc, tc, lds_ex, epi, wq, wt, h, l32);
}

// Ring variant: LDS-DMA (global_load_lds_dwordx4) into a STAGES-deep ring of chunk buffers, the
// loads running STAGES-1 chunks ahead of the MFMAs with no staging registers.  A chunk buffer
// is filled lane-linearly (1 KiB = 16 rows per wave-instruction); the unit swizzle is applied on
// the global source address.  Synchronisation per chunk: wait for this wave's DMAs of the chunk
// (counted vmcnt), raw s_barrier (every wave's DMAs landed; every wave done with the buffer the
// next DMA overwrites), issue the DMA of chunk kc+STAGES-1, then read + MFMA.
typedef __attribute__((address_space(3))) void lds_void_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else static_assert(N == 0, "add the vmcnt immediate");
}

template <class Cfg, int STAGES, bool VEC>
__global__ __launch_bounds__(Cfg::NT, 1) void corr_build_split_ring_kernel(SplitParams p) {
    constexpr int BQ = Cfg::BQ, MQ = Cfg::MQ, ROWS = Cfg::ROWS, NW = Cfg::NT / 64;
    static_assert(ROWS % (16 * NW) == 0, "whole 16-row DMA pieces per wave");
    constexpr int PPW = ROWS / 16 / NW;  // DMA pieces (wave-instructions) per wave per chunk
    constexpr size_t STAGE = (size_t)ROWS * 64;
    constexpr size_t MAIN = STAGES * STAGE > NW * kEpiBytes ? STAGES * STAGE : NW * kEpiBytes;
    extern __shared__ __attribute__((aligned(16))) u32x4 smem_ring[];
    int *lds_ex = reinterpret_cast<int *>(reinterpret_cast<char *>(smem_ring) + MAIN);

    const TileCoord tc = tile_coord(p, xcd_swizzle(blockIdx.x, gridDim.x));
    const int b = tc.b, q0 = tc.qb * BQ;
    const int NQ = p.NQ, W = p.W, H = p.H, N = p.N;
    const int tid = threadIdx.x;
    const int lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wv = tid >> 6, wq = wv / Cfg::WT, wt = wv % Cfg::WT;

    auto row_src = [&](int j, const int *&ebase) -> const u32x4 * {
        if (j < BQ) {
            const int q = min(q0 + j, NQ - 1);
            ebase = p.ex1 + (size_t)b * NQ + q;
            return p.pk1 + ((size_t)b * p.nkc * NQ + q) * 4;
        }
        const int t = j - BQ;
        const int Y = min((tc.py * Cfg::WT + (t >> 7)) * 8 + ((t >> 5) & 3) * 2 + (t & 1), H - 1);
        const int X = min(tc.px * 16 + ((t & 31) >> 1), W - 1);
        ebase = p.ex2 + (size_t)b * N + (size_t)Y * W + X;
        return p.pk2 + ((size_t)b * p.nkc * N + (size_t)Y * W + X) * 4;
    };
    // per piece: this lane's source (row (16*piece + lane/4), logical unit of its phys slot)
    const u32x4 *src[PPW];
    size_t plane[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int piece = wv + NW * i;
        const int j = piece * 16 + (lane >> 2);
        const int *eb;
        src[i] = row_src(j, eb) + ((lane & 3) ^ ((j >> 2) & 3));
        plane[i] = j < BQ ? (size_t)NQ * 4 : (size_t)N * 4;
    }
    for (int j = tid; j < ROWS; j += Cfg::NT) {
        const int *eb;
        (void)row_src(j, eb);
        lds_ex[j] = *eb;
    }
    auto issue = [&](int kc) {
        char *base = reinterpret_cast<char *>(smem_ring) + (size_t)(kc % STAGES) * STAGE;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int piece = wv + NW * i;
            __builtin_amdgcn_global_load_lds((const void *)(src[i] + (size_t)kc * plane[i]),
                                             (lds_void_t *)(base + piece * 1024), 16, 0, 0);
        }
    };

    f32x16 acc[MQ][4];
#pragma unroll
    for (int i = 0; i < MQ; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nkc = p.nkc;
    // the exponent loads above must land before any DMA is counted against vmcnt
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < STAGES - 1; ++k)
        if (k < nkc) issue(k);

    const int qrow0 = wq * (32 * MQ) + l32;
    const int trow0 = BQ + wt * 128 + l32;
    for (int kc = 0; kc < nkc; ++kc) {
        // this wave's DMAs of chunk kc are done once at most (chunks issued after kc) x PPW remain
        const int ahead = min(STAGES - 2, nkc - 1 - kc);
        if (ahead >= 2) wait_vmcnt<2 * PPW>();
        else if (ahead == 1) wait_vmcnt<PPW>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (kc + STAGES - 1 < nkc) issue(kc + STAGES - 1);
        const u32x4 *S = smem_ring + (size_t)(kc % STAGES) * ROWS * 4;
        half8 qh[MQ], ql[MQ], th[4], tl[4];
#pragma unroll
        for (int i = 0; i < MQ; ++i) {
            qh[i] = __builtin_bit_cast(half8, S[swz(qrow0 + 32 * i, 2 * h)]);
            ql[i] = __builtin_bit_cast(half8, S[swz(qrow0 + 32 * i, 2 * h + 1)]);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            th[t] = __builtin_bit_cast(half8, S[swz(trow0 + 32 * t, 2 * h)]);
            tl[t] = __builtin_bit_cast(half8, S[swz(trow0 + 32 * t, 2 * h + 1)]);
        }
#pragma unroll
        for (int i = 0; i < MQ; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ql[i], th[t], acc[i][t], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MQ; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qh[i], tl[t], acc[i][t], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MQ; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qh[i], th[t], acc[i][t], 0, 0, 0);
    }
    __syncthreads();  // every wave done with the ring before the epilogue reuses it
    float *epi = reinterpret_cast<float *>(reinterpret_cast<char *>(smem_ring) + (size_t)wv * kEpiBytes);
    split_epilogue<Cfg, VEC>(p, acc, tc, lds_ex, epi, wq, wt, h, l32);
}

// ---------------------------------------------------------------------------------------
// Host side.
// ---------------------------------------------------------------------------------------
namespace {
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct SplitWs {
    u32x4 *pk1, *pk2;
    int *ex1, *ex2;
};

SplitWs split_ws(void *ws, int B, int D, int NQ, int H, int W) {
    const size_t KP = split_kp(D), N = (size_t)H * W;
    char *w = (char *)ws;
    SplitWs r;
    r.pk1 = (u32x4 *)w;
    w += align256((size_t)B * NQ * KP * 4);
    r.pk2 = (u32x4 *)w;
    w += align256((size_t)B * N * KP * 4);
    r.ex1 = (int *)w;
    w += align256((size_t)B * NQ * 4);
    r.ex2 = (int *)w;
    return r;
}
}  // namespace

// Vector (16-B / 8-B) stores in every fused level: W % 16 == 0 keeps each level's row runs
// aligned and never straddling the right edge; level bases must be 16-B aligned.
// Store width of one level's runs of 4 (columns X = 4k; row offsets are multiples of Wl).
int split_store_mode(int Wl, const float *base) {
    if (Wl % 4 == 0 && (uintptr_t)base % 16 == 0) return 2;
    if (Wl % 2 == 0 && (uintptr_t)base % 8 == 0) return 1;
    return 0;
}

bool split_vec_ok(int W, const LevelPtrs &pyr, int nlev) {
    if (W % 16) return false;
    for (int l = 0; l < nlev; ++l)
        if ((uintptr_t)pyr.p[l] % 16) return false;
    return true;
}

// Workspace: pk1 [B][KP/16][NQ][64 B] | pk2 [B][KP/16][N][64 B] | ex1 [B*NQ] | ex2 [B*N] int32.
size_t build_split_workspace(int B, int D, int NQ, int H, int W) {
    const size_t KP = split_kp(D), N = (size_t)H * W;
    return align256((size_t)B * NQ * KP * 4) + align256((size_t)B * N * KP * 4) + align256((size_t)B * NQ * 4) +
           align256((size_t)B * N * 4);
}

bool build_split_supported(int D) { return split_pack_tp(split_kp(D)) > 0; }

// Pixel-lane pack with NW waves per workgroup (kbench variants; D <= 16 * NW * 4).
template <int NW>
hipError_t launch_split_pack_px(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, void *ws,
                                hipStream_t s) {
    const SplitWs w = split_ws(ws, B, D, NQ, H, W);
    PackArgs a{};
    a.f[0] = f1, a.f[1] = f2;
    a.pk[0] = w.pk1, a.pk[1] = w.pk2;
    a.ex[0] = w.ex1, a.ex[1] = w.ex2;
    a.np[0] = NQ, a.np[1] = H * W;
    a.D = D;
    a.KP = split_kp(D);
    const int np = std::max(NQ, H * W);
    const int cpt = (a.KP / kSplitBK + NW - 1) / NW;
    const dim3 grid((np + 63) / 64, B, 2), blk(64 * NW);
    switch (cpt) {
        case 1: hipLaunchKernelGGL((split_pack_px_kernel<NW, 1>), grid, blk, 0, s, a); break;
        case 2: hipLaunchKernelGGL((split_pack_px_kernel<NW, 2>), grid, blk, 0, s, a); break;
        case 3: hipLaunchKernelGGL((split_pack_px_kernel<NW, 3>), grid, blk, 0, s, a); break;
        case 4: hipLaunchKernelGGL((split_pack_px_kernel<NW, 4>), grid, blk, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// lds_pack: force the LDS-tiled pack (any D; the register pack covers D <= 512).
hipError_t launch_split_pack(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, void *ws,
                             hipStream_t s, bool lds_pack = false) {
    const SplitWs w = split_ws(ws, B, D, NQ, H, W);
    PackArgs a{};
    a.f[0] = f1, a.f[1] = f2;
    a.pk[0] = w.pk1, a.pk[1] = w.pk2;
    a.ex[0] = w.ex1, a.ex[1] = w.ex2;
    a.np[0] = NQ, a.np[1] = H * W;
    a.D = D;
    a.KP = split_kp(D);
    const int np = std::max(NQ, H * W);
    if (!lds_pack) {
        const dim3 grid((np + kPackTP - 1) / kPackTP, B, 2);
        const dim3 blk(64 * kPackW);
        switch (split_pack_cpt(a.KP)) {
#define CORR_PACK_CASE(c) \
    case c: hipLaunchKernelGGL(split_pack_reg_kernel<c>, grid, blk, 0, s, a); return hipGetLastError();
            CORR_PACK_CASE(1) CORR_PACK_CASE(2) CORR_PACK_CASE(3) CORR_PACK_CASE(4)
            CORR_PACK_CASE(5) CORR_PACK_CASE(6) CORR_PACK_CASE(7) CORR_PACK_CASE(8)
#undef CORR_PACK_CASE
            default: break;
        }
    }
    a.TP = split_pack_tp(a.KP);
    if (!a.TP) return hipErrorInvalidValue;
    const size_t lds = (size_t)a.TP * (a.KP + 4) * 4 + (256 + a.TP) * 4;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void *)split_pack_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(split_pack_kernel, dim3((np + a.TP - 1) / a.TP, B, 2), dim3(256), lds, s, a);
    return hipGetLastError();
}

// The MFMA part (operands already packed in ws).  levels == 0: the MFMAs only (measurement).
template <class Cfg>
hipError_t launch_split_mfma_cfg(int NQ, int B, int D, int H, int W, int levels, const LevelPtrs &pyr, void *ws,
                                 hipStream_t s) {
    const SplitWs w = split_ws(ws, B, D, NQ, H, W);
    SplitParams p{};
    p.pk1 = w.pk1, p.pk2 = w.pk2, p.ex1 = w.ex1, p.ex2 = w.ex2;
    p.B = B;
    p.H = H;
    p.W = W;
    p.N = H * W;
    p.NQ = NQ;
    p.nkc = split_kp(D) / kSplitBK;
    p.nlev = std::min(levels, kFusedLevels);
    for (int l = 0; l < kFusedLevels; ++l) p.lvl[l] = l < p.nlev ? pyr.p[l] : nullptr;
    p.nq = (NQ + Cfg::BQ - 1) / Cfg::BQ;
    p.npx = (W + 15) / 16;
    p.npy = (H + Cfg::PH - 1) / Cfg::PH;
    const float sD = std::sqrt((float)D);
    p.inv_s = 1.0f / sD;
    p.exact = is_pow2(sD);
    p.eshift = 0;
    if (p.exact) {
        int e;
        std::frexp(p.inv_s, &e);
        p.eshift = e - 1;  // 1/s = 2^(e-1)
    }
    const long tiles = (long)p.nq * p.npx * p.npy * B;
    if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
    const bool vec = split_vec_ok(W, pyr, p.nlev);
    p.vec0 = p.nlev > 0 ? split_store_mode(W, pyr.p[0]) : 0;
    p.vec1 = p.nlev > 1 ? split_store_mode(W >> 1, pyr.p[1]) : 0;
    static bool attr_set[2] = {false, false};
    if (!attr_set[vec]) {
        hipError_t e = hipFuncSetAttribute(vec ? (const void *)corr_build_split_kernel<Cfg, true>
                                               : (const void *)corr_build_split_kernel<Cfg, false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
        if (e != hipSuccess) return e;
        attr_set[vec] = true;
    }
    if (levels == 0) {  // measurement: no stores (the kernel still runs its epilogue arithmetic)
        p.nlev = 0;
    }
    if (vec)
        hipLaunchKernelGGL((corr_build_split_kernel<Cfg, true>), dim3((unsigned)tiles), dim3(Cfg::NT), Cfg::LDS, s, p);
    else
        hipLaunchKernelGGL((corr_build_split_kernel<Cfg, false>), dim3((unsigned)tiles), dim3(Cfg::NT), Cfg::LDS, s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (levels > kFusedLevels) return launch_pool_levels(pyr, kFusedLevels, levels, (long)B * NQ, H, W, s);
    return hipSuccess;
}

template <class Cfg, int STAGES>
hipError_t launch_split_ring_cfg(int NQ, int B, int D, int H, int W, int levels, const LevelPtrs &pyr, void *ws,
                                 hipStream_t s) {
    const SplitWs w = split_ws(ws, B, D, NQ, H, W);
    SplitParams p{};
    p.pk1 = w.pk1, p.pk2 = w.pk2, p.ex1 = w.ex1, p.ex2 = w.ex2;
    p.B = B;
    p.H = H;
    p.W = W;
    p.N = H * W;
    p.NQ = NQ;
    p.nkc = split_kp(D) / kSplitBK;
    p.nlev = std::min(levels, kFusedLevels);
    for (int l = 0; l < kFusedLevels; ++l) p.lvl[l] = l < p.nlev ? pyr.p[l] : nullptr;
    p.nq = (NQ + Cfg::BQ - 1) / Cfg::BQ;
    p.npx = (W + 15) / 16;
    p.npy = (H + Cfg::PH - 1) / Cfg::PH;
    const float sD = std::sqrt((float)D);
    p.inv_s = 1.0f / sD;
    p.exact = is_pow2(sD);
    p.eshift = 0;
    if (p.exact) {
        int e;
        std::frexp(p.inv_s, &e);
        p.eshift = e - 1;
    }
    const long tiles = (long)p.nq * p.npx * p.npy * B;
    if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
    const size_t lds = std::max(STAGES * (size_t)Cfg::ROWS * 64, (size_t)(Cfg::NT / 64) * kEpiBytes) +
                       (size_t)Cfg::ROWS * 4;
    const bool vec = split_vec_ok(W, pyr, p.nlev);
    p.vec0 = p.nlev > 0 ? split_store_mode(W, pyr.p[0]) : 0;
    p.vec1 = p.nlev > 1 ? split_store_mode(W >> 1, pyr.p[1]) : 0;
    static bool attr_set[2] = {false, false};
    if (!attr_set[vec]) {
        hipError_t e = hipFuncSetAttribute(vec ? (const void *)corr_build_split_ring_kernel<Cfg, STAGES, true>
                                               : (const void *)corr_build_split_ring_kernel<Cfg, STAGES, false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set[vec] = true;
    }
    if (vec)
        hipLaunchKernelGGL((corr_build_split_ring_kernel<Cfg, STAGES, true>), dim3((unsigned)tiles), dim3(Cfg::NT), lds,
                           s, p);
    else
        hipLaunchKernelGGL((corr_build_split_ring_kernel<Cfg, STAGES, false>), dim3((unsigned)tiles), dim3(Cfg::NT), lds,
                           s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (levels > kFusedLevels) return launch_pool_levels(pyr, kFusedLevels, levels, (long)B * NQ, H, W, s);
    return hipSuccess;
}

template <class Cfg>
hipError_t launch_build_split_cfg(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, int levels,
                                  const LevelPtrs &pyr, void *ws, hipStream_t s) {
    hipError_t e = launch_split_pack(f1, NQ, f2, B, D, H, W, ws, s);
    if (e != hipSuccess) return e;
    return launch_split_mfma_cfg<Cfg>(NQ, B, D, H, W, levels, pyr, ws, s);
}

// Tile geometry per shape.  The candidates compute identical bits (every output sums the same
// chunk sequence through the same three MFMAs and the same epilogue; only the workgroup shape
// differs), so the choice is free.  Every wave owns a 64-query x 128-target tile in all three,
// so the padded work — and the rounds of waves over the chip — is proportional to the wave
// count; take the configuration with the fewest, ties to 4x1, then 2x2.  Measured
// (profiles/r01j_kbench_split.txt, r01k_tile_ab.txt): DSEC 60x80 all tie -> 4x1 (bench 6504
// vs 6418 frame-pairs/s for 2x2); train 36x48 B8 4x1 (67 vs 69 us); MVSEC 36x44 B16 2x1.
// CORR_SPLIT_TILE=0|1|2 forces 2x2 | 4x1 | 2x1 (tests: all three must agree bit for bit).
using SplitTall = SplitCfg<4, 1, 2, 2>;
using SplitSmall = SplitCfg<2, 1, 2, 2>;

template <class Cfg>
long split_waves(int NQ, int B, int H, int W) {
    return (long)((NQ + Cfg::BQ - 1) / Cfg::BQ) * ((W + 15) / 16) * ((H + Cfg::PH - 1) / Cfg::PH) * B * (Cfg::NT / 64);
}

int split_tile_choice(int NQ, int B, int H, int W) {
    if (const char *e = std::getenv("CORR_SPLIT_TILE")) {
        const int v = std::atoi(e);
        if (v >= 0 && v <= 2) return v;
    }
    const long w[3] = {split_waves<SplitDefault>(NQ, B, H, W), split_waves<SplitTall>(NQ, B, H, W),
                       split_waves<SplitSmall>(NQ, B, H, W)};
    int pick = 1;  // ties: 4x1 first (DSEC, 3 interleaved A/B runs: 72.3 vs 73.9 us for 2x2)
    for (int k : {0, 2})
        if (w[k] < w[pick]) pick = k;
    return pick;
}

hipError_t launch_build_split(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, int levels,
                              const LevelPtrs &pyr, void *ws, hipStream_t s) {
    switch (split_tile_choice(NQ, B, H, W)) {
        case 1: return launch_build_split_cfg<SplitTall>(f1, NQ, f2, B, D, H, W, levels, pyr, ws, s);
        case 2: return launch_build_split_cfg<SplitSmall>(f1, NQ, f2, B, D, H, W, levels, pyr, ws, s);
        default: return launch_build_split_cfg<SplitDefault>(f1, NQ, f2, B, D, H, W, levels, pyr, ws, s);
    }
}

}  // namespace r01
}  // namespace corr
