// corr_lookup.hip — (2r+1)^2 bilinear window lookup and its input-gradient on gfx950.
//
// Forward replaces CorrBlock.__call__ (model/corr.py:29-50) + bilinear_sampler
// (model/utils.py:7-21, F.grid_sample(align_corners=True), zero padding).  The ~12 ATen ops
// per level, the per-call CPU->GPU offset copies (corr.py:37-39), the cat and the
// permute().contiguous() (corr.py:49-50) become ONE launch that writes the NCHW output
// directly.
//
// Work layout: a workgroup owns QB (32; 16 on small maps) consecutive query pixels of one batch
// item at one pyramid level; thread (q, i) is query q's window column i (the x-tap;
// corr.py:37-43: the slow window index moves x).
//   1. thread (q, i): tap i of query q on both axes, rounded exactly as the reference does
//      (x/2^l + (i - r) -> 2X/(W_l-1) - 1 -> ((x'+1)/2)(W_l-1); one fp32 rounding per op),
//      its floor and the two 1-D weights; y-taps -> LDS, the thread keeps its x-tap;
//   2. every query's (S+2)^2 neighbourhood (anchored at the floor of its tap 0, zero outside
//      the map) is gathered from the TILED map (corr_common.h) into LDS, one 16-B tile row per
//      lane — all of a thread's loads issued before any LDS store, so the gather costs one
//      memory round trip;
//   3. thread (q, i) produces the S outputs (i, j = 0..S-1): 4 corner reads from LDS, fmaf in
//      the order nw, ne, sw, se (bit-identical to ATen's CPU grid_sampler_2d), stores to
//      out[b][l*K + i*S + j][n] — consecutive n per wave, fully coalesced.
// Tap floors are monotone in the tap index, so one check of the first and last tap proves
// that every corner lies inside the neighbourhood.  A workgroup where that fails for some
// query (only possible for |coordinates| near 2^20) takes a uniform slow path that reads such
// corners from global memory — keeping global loads out of the common loop (a load there
// makes every iteration wait on vmcnt, i.e. on the previous iteration's stores).
//
// Backward (autograd of utils.py:15 w.r.t. the pyramid; coords are detached at
// eraft.py:128): with regular taps (floor of tap t = anchor + t on both axes — the common
// case) each neighbourhood cell receives exactly the <= 4 (tap, corner) contributions
//   se(cx-1, cy-1), ne(cx-1, cy), sw(cx, cy-1), nw(cx, cy)
// and is computed as a GATHER, summed in the reference's scatter order (taps row-major,
// corners nw, ne, sw, se), then added once to the gradient pyramid.  A query's cells belong
// to its own map only, so there are no atomics and results are deterministic.  Irregular
// workgroups fall back to a sequential per-query scatter in the same order.
#include <cmath>
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "corr_build_common.h"
#include "corr_common.h"
#include "corr_div.h"

namespace corr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Sentinel anchor for NaN / huge coordinates: every window cell is outside the map.
constexpr int kFarAnchor = -(1 << 28);

struct Axis {
    float f;   // floor(ix) as float (may be NaN / huge)
    float lo;  // (f + 1) - ix  : weight of corner f
    float hi;  // ix - f        : weight of corner f + 1
};

// rden = recip_rn(size - 1), hoisted by the callers (per level)
__device__ __forceinline__ Axis tap_axis(float c, float inv_scale, int t, int r, int size, float rden) {
    // corr.py:41  centroid = coords / 2**l   (exact: power-of-two scale)
    // corr.py:43  + delta (integer offsets from linspace(-r, r, 2r+1))
    // utils.py:11 2*x/(W-1) - 1 ; grid_sample unnormalise ((x'+1)/2)*(W-1)
    // The division is correctly rounded (corr_div.h: the same bits as __fdiv_rn in 3 VALU)
    const float cl = c * inv_scale;
    const float X = cl + (float)(t - r);
    const float den = (float)(size - 1);
    const float xn = __fsub_rn(div_rn(2.0f * X, den, rden), 1.0f);
    const float ix = __fmul_rn(__fmul_rn(__fadd_rn(xn, 1.0f), 0.5f), den);
    Axis a;
    a.f = floorf(ix);
    a.hi = __fsub_rn(ix, a.f);
    a.lo = __fsub_rn(__fadd_rn(a.f, 1.0f), ix);
    return a;
}

__device__ __forceinline__ int anchor_of(float f) {
    return (f >= -1048576.0f && f <= 1048576.0f) ? (int)f : kFarAnchor;
}

__device__ __forceinline__ bool in_map(float xf, float yf, int Wl, int Hl) {
    return xf >= 0.0f && xf < (float)Wl && yf >= 0.0f && yf < (float)Hl;
}

// True when every in-map corner of the query's taps lies inside its (S+2)^2 neighbourhood.
template <int S>
__device__ __forceinline__ bool window_covers(float fx0, float fxl, float fy0, float fyl) {
    if (anchor_of(fx0) == kFarAnchor || anchor_of(fy0) == kFarAnchor) return true;
    return (fxl - fx0) <= (float)S && (fyl - fy0) <= (float)S;
}

template <int S, int QB>
struct LookupSmem {
    static constexpr int WIN = S + 2;
    static constexpr int NTC = (WIN + 6) / 4;  // tile columns that hold WIN cells at any offset
    // Window row of query q: cell cx (column anchor + cx) at win[q * WQ + cy * WW + 3 + cx].  A
    // gather lane stores its tile row's 4 cells at columns 4 tc - (anchor & 3) + 3 + c, i.e.
    // without predicates: cells left or right of the window land in the 3 + (4 NTC - WIN) spare
    // columns of the row.  Odd query stride: lane = query reads are conflict-free.
    static constexpr int WW = 4 * NTC + 3;
    static constexpr int WQ = (WIN * WW) | 1;
    float win[QB * WQ];
    float ty[3][S][QB];
    float fx[2][QB];  // floor of x-tap 0 and S-1
    int ax[QB], ay[QB];
    int flags;
};

// Forward gather from the tiled maps (corr_common.h): one wave per query at a time, lane =
// (window row rr, tile column tc): one 16-B load of the tile row holding cells (anchor_y + rr,
// 4 (anchor_x / 4 + tc) .. + 3), zero outside the map; then four LDS stores realigned to the
// window (unconditional: out-of-window cells go to the row's spare columns).  All of a thread's
// loads are issued before any LDS store, so the gather costs one memory round trip.  The
// query map bases are wave-uniform: qb is moved to a scalar register, so the 64-bit base
// arithmetic is scalar.  TIGHT: only the rows / 16-B chunks the query's taps can touch (anchor ..
// floor(last tap) + 1 on each axis: floors are monotone in the tap index) are loaded — a regular
// window is 10 x 10 of the 11 x 11 neighbourhood; uncovered and far queries load all of it.  The
// cells not loaded are written as zeros and never read.  NOLOAD: ablation (tools/kbench_lookup.hip).
template <int S, int QB, int NT, bool NOLOAD = false, bool TIGHT = false>
__device__ __forceinline__ void gather_window_tiled(LookupSmem<S, QB> &sm, const float *P, size_t qbase,
                                                    unsigned mapsz, int n0, int N, int Wl, int Hl, int tid) {
    using SM = LookupSmem<S, QB>;
    constexpr int WIN = SM::WIN, NTC = SM::NTC, WW = SM::WW, WQ = SM::WQ;
    constexpr int LPQ = NTC * WIN;           // lanes per query
    constexpr int EPL = (LPQ + 63) / 64;     // loads per lane and query
    constexpr int NW = NT / 64;
    constexpr int QPW = (QB + NW - 1) / NW;  // queries per wave
    static_assert(QPW <= 64, "one lane per query of the wave");
    const unsigned TW = (unsigned)map_tiles(Wl);  // 16-B chunks per map row
    const int TC = map_tcols(Wl);                  // tiles per map row
    const int lane = tid & 63;
    int rr[EPL], tc[EPL];
#pragma unroll
    for (int v = 0; v < EPL; ++v) {
        const int e = lane + 64 * v;
        rr[v] = e / NTC;
        tc[v] = e - rr[v] * NTC;
    }
    // The query a wave handles at step k is wave-uniform: all of the wave's anchors are read from
    // LDS at once (lane k holds query k's) and moved to scalar registers with readlane.
    const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    const unsigned qb = __builtin_amdgcn_readfirstlane((unsigned)qbase);
    int myX = kFarAnchor, myY = kFarAnchor, myE = WIN | (WIN << 8);
    {
        const int qq = wu + NW * lane;
        if (lane < QPW && qq < QB && n0 + qq < N) {
            myX = sm.ax[qq];
            myY = sm.ay[qq];
            if (TIGHT && myX != kFarAnchor && myY != kFarAnchor) {
                const float fx0 = sm.fx[0][qq], fxl = sm.fx[1][qq], fy0 = sm.ty[0][0][qq], fyl = sm.ty[0][S - 1][qq];
                if (window_covers<S>(fx0, fxl, fy0, fyl)) myE = ((int)(fxl - fx0) + 2) | (((int)(fyl - fy0) + 2) << 8);
            }
        }
    }
    f32x4 vals[QPW][EPL];
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
        const int qq = wu + NW * k;
        const int X0 = __builtin_amdgcn_readlane(myX, k);
        const int Y0 = __builtin_amdgcn_readlane(myY, k);
        const float *Pq = P + (size_t)(qb + (unsigned)qq) * mapsz;
        int nx = WIN, ny = WIN;
        if (TIGHT) {
            const int E = __builtin_amdgcn_readlane(myE, k);
            nx = (E & 255) + (X0 & 3), ny = E >> 8;  // chunk columns start at X0 & ~3
        }
#pragma unroll
        for (int v = 0; v < EPL; ++v) {
            const unsigned T = (unsigned)((X0 >> 2) + tc[v]), Y = (unsigned)(Y0 + rr[v]);
            const bool need = !TIGHT || (rr[v] < ny && 4 * tc[v] < nx);
            const bool ok = (lane + 64 * v < LPQ) && need && T < TW && Y < (unsigned)Hl;
            vals[k][v] = (ok && !NOLOAD) ? *reinterpret_cast<const f32x4 *>(Pq + map_row4((int)Y, (int)T, TC))
                                         : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    const bool ragged = (Wl & 3) != 0;  // the last tile column holds cells past W_l: zero them
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
        const int qq = wu + NW * k;
        const int X0 = __builtin_amdgcn_readlane(myX, k);
        if (qq >= QB) continue;
#pragma unroll
        for (int v = 0; v < EPL; ++v) {
            if (lane + 64 * v < LPQ) {
                f32x4 x = vals[k][v];
                if (ragged) {
                    const int xb = ((X0 >> 2) + tc[v]) * 4;
#pragma unroll
                    for (int c = 0; c < 4; ++c) x[c] = xb + c < Wl ? x[c] : 0.0f;
                }
                float *row = &sm.win[qq * WQ + rr[v] * WW + 4 * tc[v] + 3 - (X0 & 3)];
#pragma unroll
                for (int c = 0; c < 4; ++c) row[c] = x[c];
            }
        }
    }
}

constexpr int lookup_threads(int S, int QB) { return (QB * S + 63) / 64 * 64; }

// ABL: diagnostic ablations for tools/kbench_lookup.hip only (0 in the library): bit 0 = no
// neighbourhood loads, bit 1 = no output stores, bit 2 = no coords load, bit 3 = plain (L2-cached)
// output stores instead of the non-temporal ones (lookup_kernel).
// One pyramid level of one block of QB queries (NT threads): the whole lookup of
// lookup_kernel below.  emit(j, acc) receives output tap (i, j) of this thread's window column
// i = tid / QB for query q = tid % QB (called only for live queries).  Shared by lookup_kernel
// (global NCHW stores), lookup_conv_kernel (LDS tile feeding the fused 1x1 convolution) and
// lookup_conv_bwd_dw_kernel.  The lookup of one block with its coords already loaded (cxv, cyv:
// this thread's query; 0 for threads without one).
template <int S, int QB, int NT, int ABL, class Emit, bool TIGHT = false>
__device__ __forceinline__ void lookup_block_v(LookupSmem<S, QB> &sm, const float *__restrict__ P, float cxv,
                                               float cyv, int b, int n0, int N, int H, int W, int l, int tid,
                                               Emit emit) {
    constexpr int R = (S - 1) / 2;
    using SM = LookupSmem<S, QB>;
    constexpr int WIN = SM::WIN, WW = SM::WW, WQ = SM::WQ;
    const int Hl = H >> l, Wl = W >> l;
    const float inv_scale = 1.0f / (float)(1 << l);
    const unsigned mapsz = (unsigned)map_floats(Hl, Wl);
    const int TC = map_tcols(Wl);
    const size_t qbase = (size_t)b * N + n0;

    const int q = tid % QB;
    const int i = tid / QB;  // this thread's x-tap (window column); i >= S: gather only
    const bool act = i < S;
    const int n = n0 + q;
    const bool qok = act && n < N;

    // ---- 1. taps ----
    if (tid == 0) sm.flags = 0;
    const Axis tx = tap_axis(cxv, inv_scale, i, R, Wl, recip_rn((float)(Wl - 1)));
    const Axis ty = tap_axis(cyv, inv_scale, i, R, Hl, recip_rn((float)(Hl - 1)));
    if (act) {
        sm.ty[0][i][q] = ty.f;
        sm.ty[1][i][q] = ty.lo;
        sm.ty[2][i][q] = ty.hi;
        if (i == 0) {
            sm.ax[q] = anchor_of(tx.f);
            sm.ay[q] = anchor_of(ty.f);
            sm.fx[0][q] = tx.f;
        }
        if (i == S - 1) sm.fx[1][q] = tx.f;
    }
    __syncthreads();
    // Workgroup-uniform mode: bit 0 = some corner lies outside its neighbourhood (slow path),
    // bit 1 = some query's taps are not regular (floor(tap t) != floor(tap 0) + t).
    if (act) {
        const int ax0 = sm.ax[q], ay0 = sm.ay[q];
        const bool far = ax0 == kFarAnchor || ay0 == kFarAnchor;
        const bool covers = window_covers<S>(sm.fx[0][q], sm.fx[1][q], sm.ty[0][0][q], sm.ty[0][S - 1][q]);
        const bool reg = far || (tx.f == (float)(ax0 + i) && ty.f == (float)(ay0 + i));
        const int f = (covers ? 0 : 1) | (reg ? 0 : 2);
        if (f) atomicOr(&sm.flags, f);
    }

    // ---- 2. neighbourhoods -> LDS ----
    gather_window_tiled<S, QB, NT, (ABL & 1) != 0, TIGHT>(sm, P, qbase, mapsz, n0, N, Wl, Hl, tid);
    __syncthreads();
    const int mode = sm.flags;
    if (!act) return;

    // ---- 3. outputs (i, 0..S-1) of query q ----
    const int ax = sm.ax[q], ay = sm.ay[q];
    const float *wq = &sm.win[q * WQ + 3];
    const float x0 = tx.f, ex = tx.lo, wx = tx.hi;
    if (mode == 0) {
        // regular taps: tap (i, j) has corners at neighbourhood column i, i+1 and rows j, j+1,
        // so the S+1 rows of the column pair are read once and shared by consecutive taps
        // (far queries read an all-zero neighbourhood: their taps have no in-map corner).
        const float *col = wq + i;
        float c0[S + 1], c1[S + 1];
#pragma unroll
        for (int j = 0; j <= S; ++j) {
            c0[j] = col[j * WW];
            c1[j] = col[j * WW + 1];
        }
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const float ey = sm.ty[1][j][q], ny = sm.ty[2][j][q];
            float acc = __fmul_rn(c0[j], __fmul_rn(ey, ex));
            acc = __builtin_fmaf(c1[j], __fmul_rn(ey, wx), acc);
            acc = __builtin_fmaf(c0[j + 1], __fmul_rn(ny, ex), acc);
            acc = __builtin_fmaf(c1[j + 1], __fmul_rn(ny, wx), acc);
            if (qok && (!(ABL & 2) || acc == 1234.5f)) emit(j, acc);
        }
    } else if (!(mode & 1)) {
        // every corner is inside the neighbourhood (cells outside the map hold 0)
        const bool far = (ax == kFarAnchor) || (ay == kFarAnchor);
        const int cx = far ? 0 : (int)x0 - ax;
        const float *col = wq + cx;
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const float y0 = sm.ty[0][j][q], ey = sm.ty[1][j][q], ny = sm.ty[2][j][q];
            const int cy = far ? 0 : (int)y0 - ay;
            const float *c = col + cy * WW;
            float acc = __fmul_rn(c[0], __fmul_rn(ey, ex));
            acc = __builtin_fmaf(c[1], __fmul_rn(ey, wx), acc);
            acc = __builtin_fmaf(c[WW], __fmul_rn(ny, ex), acc);
            acc = __builtin_fmaf(c[WW + 1], __fmul_rn(ny, wx), acc);
            if (qok) emit(j, acc);
        }
    } else {
        const float *Pq = P + (qbase + q) * mapsz;
        auto fetch = [&](float xf, float yf) -> float {
            if (!in_map(xf, yf, Wl, Hl)) return 0.0f;
            const int xi = (int)xf, yi = (int)yf;
            const unsigned ux = (unsigned)(xi - ax), uy = (unsigned)(yi - ay);
            if (ux < (unsigned)WIN && uy < (unsigned)WIN) return wq[uy * WW + ux];
            return Pq[map_cell(yi, xi, TC)];
        };
        const float x1 = __fadd_rn(x0, 1.0f);
        for (int j = 0; j < S; ++j) {
            const float y0 = sm.ty[0][j][q], ey = sm.ty[1][j][q], ny = sm.ty[2][j][q];
            const float y1 = __fadd_rn(y0, 1.0f);
            float acc = __fmul_rn(fetch(x0, y0), __fmul_rn(ey, ex));
            acc = __builtin_fmaf(fetch(x1, y0), __fmul_rn(ey, wx), acc);
            acc = __builtin_fmaf(fetch(x0, y1), __fmul_rn(ny, ex), acc);
            acc = __builtin_fmaf(fetch(x1, y1), __fmul_rn(ny, wx), acc);
            if (qok) emit(j, acc);
        }
    }
}

template <int S, int QB, int NT, int ABL, bool TIGHT = false, class Emit>
__device__ __forceinline__ void lookup_block(LookupSmem<S, QB> &sm, const float *__restrict__ P,
                                             const float *__restrict__ coords, int b, int n0, int N,
                                             int H, int W, int l, int tid, Emit emit) {
    const int n = n0 + tid % QB;
    const bool qok = tid / QB < S && n < N;
    const float cxv = (ABL & 4) ? (float)(n % W) : qok ? coords[((size_t)b * 2 + 0) * N + n] : 0.0f;
    const float cyv = (ABL & 4) ? (float)(n / W) : qok ? coords[((size_t)b * 2 + 1) * N + n] : 0.0f;
    lookup_block_v<S, QB, NT, ABL, Emit, TIGHT>(sm, P, cxv, cyv, b, n0, N, H, W, l, tid, emit);
}

template <int S, int QB, int ABL = 0, bool TIGHT = false>
__global__ __launch_bounds__(lookup_threads(S, QB)) void lookup_kernel(
    ConstLevelPtrs pyr, const float *__restrict__ coords, int B, int NQ, int H, int W, int L,
    float *__restrict__ out) {
    constexpr int K = S * S, NT = lookup_threads(S, QB);
    __shared__ LookupSmem<S, QB> sm;
    const int N = NQ;  // query pixels per batch item (H*W, or a row slab of it)
    const int nqb = (N + QB - 1) / QB;
    const int b = __builtin_amdgcn_readfirstlane(blockIdx.x / nqb);
    const int n0 = __builtin_amdgcn_readfirstlane((blockIdx.x - b * nqb) * QB);
    const int l = blockIdx.y;
    const int i = threadIdx.x / QB, n = n0 + threadIdx.x % QB;
    float *o = out + (((size_t)b * L + l) * K + (size_t)i * S) * N + n;
    lookup_block<S, QB, NT, ABL, TIGHT>(sm, pyr.p[l], coords, b, n0, N, H, W, l, (int)threadIdx.x, [&](int j, float acc) {
        // non-temporal: the output streams past L2 (nothing in this kernel re-reads it), so the
        // kernel's end has no dirty lines of it to write back (DSEC 5.8 -> 5.4 us, train 12.2 ->
        // 11.4 us, same bits; profiles/r04q_kbench_lookup_nt.txt)
        if constexpr ((ABL & 8) != 0) o[(size_t)j * N] = acc;
        else __builtin_nontemporal_store(acc, &o[(size_t)j * N]);
    });
}

// Lookup fused with the consumer's 1x1 convolution (BasicMotionEncoder.convc1, update.py:68,75:
// cor = relu(convc1(corr)), L*K = 324 -> 256 channels), on the bf16 MFMA with the build's exact
// three-piece split (x = hi + mid + lo, six products per fp32 product, smallest first: no
// narrower than fp32, no scales).  A workgroup owns 32 queries: two groups of 5 waves look them
// up, two levels at a time (lookup_block, bit-identical values), into an LDS tile ct[L*K][32];
// the tile is split into bf16 pieces [piece][q][k] (aliasing the lookup staging); 8 waves then
// multiply by the pre-split weight (corr_lookup_conv_weights: W's pieces in the 16x16x32 MFMA
// A-fragment order, streamed from L2 one K step ahead) into two accumulators (hi*hi; the rest)
// and write relu(acc + acs + bias) as [B][O][NQ].  The 324-channel lookup output never reaches
// HBM.  r = 4, L <= 4, O = 256.
constexpr int kLcQB = 32, kLcO = 256, kLcKC = 11, kLcKP = 32 * kLcKC /* 352 >= 4*81 */, kLcXS = kLcKP / 2 + 4;
constexpr int kLcGT = lookup_threads(9, kLcQB), kLcNT = 2 * kLcGT;
constexpr size_t kLcFwdU = (size_t)(kLcO / 16) * kLcKC * 3 * 64;  // u32x4 of the forward W pack

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf16(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                  0, 0, 0);
}

// weight [O][C] fp32 -> W's pieces [O/16][kLcKC][hi, mid, lo][64 lanes]: lane = 16 kg + r holds
// W[16 ob + r][32 kc + 8 kg + j], j < 8 (zero past C).  One block of 64 lanes per (ob, kc).
__global__ __launch_bounds__(64) void lookup_conv_weights_kernel(const float *__restrict__ w, int C,
                                                                 u32x4 *__restrict__ frag) {
    const int kc = blockIdx.x, ob = blockIdx.y, lane = threadIdx.x;
    const int o = 16 * ob + (lane & 15), k0 = 32 * kc + 8 * (lane >> 4);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = k0 + j < C ? w[(size_t)o * C + k0 + j] : 0.f;
    unsigned h[4], m[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split3(v[2 * j], v[2 * j + 1], h[j], m[j], lo[j]);
    u32x4 *dst = frag + (((size_t)ob * kLcKC + kc) * 3) * 64 + lane;
    dst[0] = u32x4{h[0], h[1], h[2], h[3]};
    dst[64] = u32x4{m[0], m[1], m[2], m[3]};
    dst[128] = u32x4{lo[0], lo[1], lo[2], lo[3]};
}

struct LcSmem {
    union {
        LookupSmem<9, kLcQB> lk[2];         // lookups
        unsigned x[3][kLcQB][kLcXS];        // the tile's pieces [piece][q][k pair] (after the lookups)
    } u;
    float ct[4 * 81][kLcQB];
};

__global__ __launch_bounds__(kLcNT) void lookup_conv_kernel(ConstLevelPtrs pyr, const float *__restrict__ coords,
                                                             int B, int NQ, int H, int W, int L,
                                                             const u32x4 *__restrict__ frag,
                                                             const float *__restrict__ bias, int relu,
                                                             float *__restrict__ out) {
    constexpr int S = 9, K = S * S, QB = kLcQB;
    __shared__ LcSmem sm;
    const int N = NQ;
    const int nqb = (N + QB - 1) / QB;
    const int b = blockIdx.x / nqb;
    const int n0 = (blockIdx.x - b * nqb) * QB;
    const int tid = threadIdx.x;
    const int g = tid / kLcGT, ltid = tid - g * kLcGT;
    const int KC = L * K;
    // ---- lookups: levels 2p + g of pass p (groups beyond L repeat the last level, discarded) ----
#pragma unroll 1
    for (int p = 0; p < 2; ++p) {
        const int l = 2 * p + g, lc = l < L ? l : L - 1;
        const int i = ltid / QB, q = ltid % QB;
        lookup_block<S, QB, kLcGT, 0>(sm.u.lk[g], pyr.p[lc], coords, b, n0, N, H, W, lc, ltid,
                                      [&](int j, float acc) {
                                          if (l < L) sm.ct[l * K + i * S + j][q] = acc;
                                      });
        __syncthreads();
    }
    // ---- pieces x[piece][q][k pair] (zero beyond L*K) ----
    for (int idx = tid; idx < QB * (kLcKP / 2); idx += kLcNT) {
        const int kp = idx / QB, q = idx - kp * QB, k = 2 * kp;
        const float y0 = k < KC ? sm.ct[k][q] : 0.f, y1 = k + 1 < KC ? sm.ct[k + 1][q] : 0.f;
        unsigned h, m, lo;
        split3(y0, y1, h, m, lo);
        sm.u.x[0][q][kp] = h;
        sm.u.x[1][q][kp] = m;
        sm.u.x[2][q][kp] = lo;
    }
    __syncthreads();
    // ---- 256 x 32 x 352 GEMM: wave w < 8 owns output channels [32 w, 32 w + 32) ----
    const int lane = tid & 63, w = tid >> 6;
    if (w >= 8) return;
    const int fr = lane & 15, fk = 4 * (lane >> 4);  // B fragment: query fr, k pairs fk .. fk + 3
    f32x4 acc[2][2], acs[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[a][c] = acs[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 wa[2][2][3];  // [buffer][o-tile][piece]
    auto load_a = [&](int buf, int kc) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const size_t base = (((size_t)(2 * w + t) * kLcKC + kc) * 3) * 64 + lane;
#pragma unroll
            for (int p = 0; p < 3; ++p) wa[buf][t][p] = frag[base + 64 * p];
        }
    };
    load_a(0, 0);
#pragma unroll
    for (int kc = 0; kc < kLcKC; ++kc) {
        const int cur = kc & 1;
        if (kc + 1 < kLcKC) load_a(cur ^ 1, kc + 1);
        u32x4 xb[2][3];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                xb[c][p] = *reinterpret_cast<const u32x4 *>(&sm.u.x[p][16 * c + fr][16 * kc + fk]);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const u32x4 wh = wa[cur][t][0], wm = wa[cur][t][1], wl = wa[cur][t][2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                acs[t][c] = mfma_bf16(wl, xb[c][0], acs[t][c]);
                acs[t][c] = mfma_bf16(wh, xb[c][2], acs[t][c]);
                acs[t][c] = mfma_bf16(wm, xb[c][1], acs[t][c]);
                acs[t][c] = mfma_bf16(wm, xb[c][0], acs[t][c]);
                acs[t][c] = mfma_bf16(wh, xb[c][1], acs[t][c]);
                acc[t][c] = mfma_bf16(wh, xb[c][0], acc[t][c]);
            }
        }
    }
    // ---- epilogue: C[row = o][col = q] = acc[4 (lane >> 4) + r][lane & 15] ----
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int q = 16 * c + fr, n = n0 + q;
        if (n >= N) continue;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = 32 * w + 16 * t + 4 * (lane >> 4) + r;
                float v = split_sum(acc[t][c][r], acs[t][c][r]) + bias[o];
                if (relu && v < 0.0f) v = 0.0f;  // torch.relu: a NaN stays a NaN (fmaxf would drop it)
                __builtin_nontemporal_store(v, &out[((size_t)b * kLcO + o) * N + n]);  // streams past L2
            }
    }
}

// ---------------------------------------------------------------------------------------
// Training backward of the fused lookup + convc1 (autograd of update.py:68,75 through
// corr.py:29-50).  With g' = dL/dout under ReLU's threshold backward (out <= 0 -> 0; a NaN
// output passes its gradient, as torch's):
//   d bias[o]     = sum_{b,n} g'[b][o][n]
//   d W[o][c]     = sum_{b,n} g'[b][o][n] lk[b][c][n]    lk = the lookup, RECOMPUTED on chip
//   d lk[b][c][n] = sum_o W[o][c] g'[b][o][n]           the lookup's upstream gradient, which
//                                                       corr_backward's fold consumes
// on the bf16 MFMA with the build's exact three-piece split (x = hi + mid + lo, six products
// per fp32 product, smallest first: no narrower than fp32, no scales).  Workgroup = (query
// range r, level l), 8 waves; per 32-query block of the range:
//   1. wave w loads g' rows o in [32 w, 32 w + 32) straight into its dW A fragments;
//   2. the level-l lookup of the 32 queries (lookup_block: the forward's values bit for bit)
//      into ct[81][32] — the 324-channel lookup never reaches HBM;
//   3. split ct -> lkB[piece][c][q] (dW's B operand) and the A fragments -> gB[piece][q][o]
//      (d lk's B operand);
//   4. d W: wave w's 2 x 6 tiles (o-tiles 2w, 2w+1 x the level's 81 channels padded to 96) add
//      the block's six-product sum (its one 32-deep K step) to fp32 registers;
//   5. d lk: wave w < 6 owns channel tile w, A = the pre-split W^T pieces (L2-resident
//      weight pack), K = 256 in 8 steps, two accumulators (hi*hi; the rest) summed at the end.
// The dW tiles stay in registers across the range; each workgroup writes one partial, and
// lookup_conv_bwd_reduce sums the R partials in range order (deterministic, no atomics).  The
// L workgroups of one range sit 8 block ids apart, i.e. on one XCD, where they share g' in L2.
constexpr int kCbQB = 32, kCbNT = 512, kCbCT = 6 /* 96 >= 81 */, kCbKS = kLcO / 32, kCbGS = kLcO + 8;
constexpr size_t kCbWtU = (size_t)4 * kCbCT * kCbKS * 3 * 64;  // u32x4 of the W^T pack
// dW kernel: waves per SIMD it is compiled for.  2 = one 8-wave workgroup per CU with the dW
// tiles, the prefetched next block and the lookup all in registers (~200 VGPRs); 4 (<= 128
// VGPRs, two workgroups per CU) spills and measured slower.
constexpr int kCbDwWaves = 2;

// W [256][C] -> W^T pieces [level][channel tile][K step][hi, mid, lo][64 lanes] in the 16x16x32
// A-fragment order: lane = 16 kg + c16 holds W[32 ks + 8 kg + j][81 l + 16 ct + c16], j < 8.
__global__ __launch_bounds__(64) void lookup_conv_wt_kernel(const float *__restrict__ w, int C,
                                                            u32x4 *__restrict__ wt) {
    const int ks = blockIdx.x, ct = blockIdx.y, l = blockIdx.z, lane = threadIdx.x;
    const int c = 16 * ct + (lane & 15), cg = 81 * l + c, o0 = 32 * ks + 8 * (lane >> 4);
    const bool ok = c < 81 && cg < C;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ok ? w[(size_t)(o0 + j) * C + cg] : 0.f;
    unsigned h[4], m[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split3(v[2 * j], v[2 * j + 1], h[j], m[j], lo[j]);
    u32x4 *dst = wt + (((size_t)l * kCbCT + ct) * kCbKS + ks) * 3 * 64 + lane;
    dst[0] = u32x4{h[0], h[1], h[2], h[3]};
    dst[64] = u32x4{m[0], m[1], m[2], m[3]};
    dst[128] = u32x4{lo[0], lo[1], lo[2], lo[3]};
}

struct CbArgs {
    ConstLevelPtrs pyr;
    const float *coords, *g, *out;
    const u32x4 *wt;
    float *dlk;    // [B][C][NQ] or null
    float *part;   // [R][256][C] dW partials, or null (no dW)
    float *bpart;  // [R][256] bias partials, or null
    int B, NQ, H, W, L, C, relu, R, nqb;
};

// g and the forward output at this lane's 16 fragment positions (t = 0, 1): o = o0 + 16 t + r16,
// q = 8 kg + j of the block at n0 (g = 0 past N); gprime() applies ReLU's threshold backward.
struct GRaw {
    float g[2][8], o[2][8];
};

__device__ __forceinline__ void load_graw(const CbArgs &a, int b, int n0, int o0, int r16, int kg, bool vec, GRaw &x) {
    const int N = a.NQ;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const size_t row = ((size_t)b * kLcO + o0 + 16 * t + r16) * N + n0 + 8 * kg;
        if (vec) {
            const float4 g0 = *reinterpret_cast<const float4 *>(a.g + row);
            const float4 g1 = *reinterpret_cast<const float4 *>(a.g + row + 4);
            x.g[t][0] = g0.x, x.g[t][1] = g0.y, x.g[t][2] = g0.z, x.g[t][3] = g0.w;
            x.g[t][4] = g1.x, x.g[t][5] = g1.y, x.g[t][6] = g1.z, x.g[t][7] = g1.w;
            if (a.relu) {
                const float4 o0v = *reinterpret_cast<const float4 *>(a.out + row);
                const float4 o1v = *reinterpret_cast<const float4 *>(a.out + row + 4);
                x.o[t][0] = o0v.x, x.o[t][1] = o0v.y, x.o[t][2] = o0v.z, x.o[t][3] = o0v.w;
                x.o[t][4] = o1v.x, x.o[t][5] = o1v.y, x.o[t][6] = o1v.z, x.o[t][7] = o1v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const bool in = n0 + 8 * kg + j < N;
                x.g[t][j] = in ? a.g[row + j] : 0.f;
                x.o[t][j] = (in && a.relu) ? a.out[row + j] : 1.f;
            }
        }
    }
}

__device__ __forceinline__ void gprime(const CbArgs &a, const GRaw &x, float (&v)[2][8]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[t][j] = (a.relu && x.o[t][j] <= 0.f) ? 0.f : x.g[t][j];
}

// Lane pair (o, o ^ 1) trades halves of a packed bf16 pair along q: the even lane returns row q
// = 2j's (o, o + 1) pair, the odd lane row 2j + 1's (DPP quad_perm [1, 0, 3, 2] + v_perm).
__device__ __forceinline__ unsigned pair_transpose(unsigned own, bool odd) {
    const unsigned other = (unsigned)__builtin_amdgcn_mov_dpp((int)own, 0xB1, 0xF, 0xF, false);
    return odd ? __builtin_amdgcn_perm(own, other, 0x07060302u) : __builtin_amdgcn_perm(other, own, 0x05040100u);
}

// ---- d lk = W^T g' (and nothing else): one workgroup per 32-query block, all levels ----
// Wave w stages g' rows o in [32 w, 32 w + 32) of the block as bf16 pieces gB[piece][q][o pair]
// (lane pairs transpose, one dword store per piece and pair of queries); then wave w owns
// channel tiles w, w + 8, w + 16 of the 4 levels x 6 tiles (A = the pre-split W^T pieces, L2),
// K = 256 in 8 steps, two accumulators (hi*hi; the rest) summed at the end.
__global__ __launch_bounds__(kCbNT) void lookup_conv_bwd_dlk_kernel(CbArgs a) {
    __shared__ unsigned gB[3][kCbQB][kCbGS / 2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, kg = lane >> 4;
    const int N = a.NQ;
    const int blk = blockIdx.x;
    const int b = blk / a.nqb, n0 = (blk - b * a.nqb) * kCbQB;
    const bool vec = (N & 3) == 0 && n0 + kCbQB <= N;
    {
        GRaw x;
        load_graw(a, b, n0, 32 * w, r16, kg, vec, x);
        float v[2][8];
        gprime(a, x, v);
        const bool odd = r16 & 1;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int col = 16 * w + 8 * t + (r16 >> 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                unsigned h, m, lo;
                split3(v[t][2 * j], v[t][2 * j + 1], h, m, lo);
                const int q = 8 * kg + 2 * j + (odd ? 1 : 0);
                gB[0][q][col] = pair_transpose(h, odd);
                gB[1][q][col] = pair_transpose(m, odd);
                gB[2][q][col] = pair_transpose(lo, odd);
            }
        }
    }
    __syncthreads();
    constexpr int PS = kCbQB * (kCbGS / 2);  // piece stride (dwords)
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
        const int ct = w + 8 * k, l = ct / kCbCT, cl = ct - l * kCbCT;
        if (l >= a.L) break;
        // two partial sums per query tile (hi*hi + lo*hi + hi*lo; mid*mid + mid*hi + hi*mid) and
        // two query tiles: four independent MFMA chains.  W^T pieces (L2) run kPf steps ahead.
        f32x4 acc[2], acs[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = acs[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const u32x4 *wp = a.wt + (size_t)ct * kCbKS * 3 * 64 + lane;
        constexpr int kPf = 4;
        u32x4 wq[kPf][3];
#pragma unroll
        for (int k2 = 0; k2 < kPf; ++k2)
#pragma unroll
            for (int p = 0; p < 3; ++p) wq[k2][p] = wp[(3 * k2 + p) * 64];
#pragma unroll
        for (int ks = 0; ks < kCbKS; ++ks) {
            const u32x4 wh = wq[ks % kPf][0], wm = wq[ks % kPf][1], wl = wq[ks % kPf][2];
            if (ks + kPf < kCbKS) {
#pragma unroll
                for (int p = 0; p < 3; ++p) wq[ks % kPf][p] = wp[(3 * (ks + kPf) + p) * 64];
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const unsigned *gq = &gB[0][16 * t + r16][16 * ks + 4 * kg];
                const u32x4 gh = *reinterpret_cast<const u32x4 *>(gq);
                const u32x4 gm = *reinterpret_cast<const u32x4 *>(gq + PS);
                const u32x4 gl = *reinterpret_cast<const u32x4 *>(gq + 2 * PS);
                acs[t] = mfma_bf16(wl, gh, acs[t]);
                acc[t] = mfma_bf16(wm, gm, acc[t]);
                acs[t] = mfma_bf16(wh, gl, acs[t]);
                acc[t] = mfma_bf16(wm, gh, acc[t]);
                acs[t] = mfma_bf16(wh, gh, acs[t]);
                acc[t] = mfma_bf16(wh, gm, acc[t]);
            }
        }
        // C[row = channel 16 cl + 4 kg + i of level l][col = query 16 t + r16]
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = n0 + 16 * t + r16;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = 16 * cl + 4 * kg + i;
                if (c < 81 && n < N)  // non-temporal, as the lookup's output
                    __builtin_nontemporal_store(acc[t][i] + acs[t][i], &a.dlk[((size_t)b * a.C + 81 * l + c) * N + n]);
            }
        }
    }
}

// ---- dW (and d bias): workgroup (query range r, level l), dW tiles in registers across it ----
struct CbSmem {
    LookupSmem<9, kCbQB> lk;                      // the lookup's staging
    float ct[81][kCbQB];                          // the lookup of the block
    unsigned lkB[3][kCbCT * 16][kCbQB / 2 + 4];   // its pieces [piece][c][q pair] (+4: no conflicts)
};

__global__ __launch_bounds__(kCbNT, kCbDwWaves) void lookup_conv_bwd_dw_kernel(CbArgs a) {
    constexpr int S = 9;
    __shared__ CbSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, kg = lane >> 4;
    const int bid = blockIdx.x, grp = bid >> 3;
    const int l = grp % a.L, r = (grp / a.L) * 8 + (bid & 7);
    const int N = a.NQ, NB = a.B * a.nqb;
    const int blk0 = (int)((long long)r * NB / a.R), blk1 = (int)((long long)(r + 1) * NB / a.R);
    const bool do_dw = a.part != nullptr, do_b = a.bpart != nullptr && l == 0;
    if (!do_dw && !do_b) return;
    const bool nvec = (N & 3) == 0;
    f32x4 mW[2][kCbCT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < kCbCT; ++c) mW[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    float mb[2] = {0.f, 0.f};
    // The next block's coords (this thread's query of the lookup) and g / out (its A-fragment
    // positions) are loaded one block ahead, during this block's lookup and MFMAs.
    const int q = tid % kCbQB;
    const bool coord_thread = tid / kCbQB < S;
    float pcx = 0.f, pcy = 0.f;
    GRaw nx;
    auto prefetch_coords = [&](int blk) {
        const int b = blk / a.nqb, n0 = (blk - b * a.nqb) * kCbQB;
        if (do_dw && coord_thread && n0 + q < N) {
            pcx = a.coords[((size_t)b * 2 + 0) * N + n0 + q];
            pcy = a.coords[((size_t)b * 2 + 1) * N + n0 + q];
        }
    };
    auto prefetch_g = [&](int blk) {
        const int b = blk / a.nqb, n0 = (blk - b * a.nqb) * kCbQB;
        load_graw(a, b, n0, 32 * w, r16, kg, nvec && n0 + kCbQB <= N, nx);
    };
    if (blk0 < blk1) {
        prefetch_coords(blk0);
        prefetch_g(blk0);
    }
#pragma unroll 1
    for (int blk = blk0; blk < blk1; ++blk) {
        const int b = blk / a.nqb, n0 = (blk - b * a.nqb) * kCbQB;
        const bool more = blk + 1 < blk1;
        const float cxv = pcx, cyv = pcy;
        if (more) prefetch_coords(blk + 1);
        // ---- 1. the level-l lookup of the block -> ct (bit-identical to corr_lookup) ----
        if (do_dw)
            lookup_block_v<S, kCbQB, kCbNT, 0>(sm.lk, a.pyr.p[l], cxv, cyv, b, n0, N, a.H, a.W, l, tid,
                                               [&](int j, float acc) { sm.ct[(tid / kCbQB) * S + j][q] = acc; });
        float v[2][8];
        gprime(a, nx, v);
        // ---- 2. bias: this lane's g' column sums ----
        if (do_b) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                float s = v[t][0];
#pragma unroll
                for (int j = 1; j < 8; ++j) s += v[t][j];
                mb[t] += s;
            }
        }
        if (!do_dw) {
            if (more) prefetch_g(blk + 1);
            continue;
        }
        __syncthreads();  // ct complete
        // ---- 3. ct -> lkB pieces; g' -> A fragments (registers) ----
        for (int idx = tid; idx < kCbCT * 16 * (kCbQB / 2); idx += kCbNT) {
            const int c = idx / (kCbQB / 2), qp = idx - c * (kCbQB / 2), q = 2 * qp;
            float x0 = 0.f, x1 = 0.f;
            if (c < 81) {
                if (n0 + q < N) x0 = sm.ct[c][q];
                if (n0 + q + 1 < N) x1 = sm.ct[c][q + 1];
            }
            unsigned h, m, lo;
            split3(x0, x1, h, m, lo);
            sm.lkB[0][c][qp] = h;
            sm.lkB[1][c][qp] = m;
            sm.lkB[2][c][qp] = lo;
        }
        u32x4 ah[2], am[2], al[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            unsigned h[4], m[4], lo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) split3(v[t][2 * j], v[t][2 * j + 1], h[j], m[j], lo[j]);
            ah[t] = u32x4{h[0], h[1], h[2], h[3]};
            am[t] = u32x4{m[0], m[1], m[2], m[3]};
            al[t] = u32x4{lo[0], lo[1], lo[2], lo[3]};
        }
        if (more) prefetch_g(blk + 1);  // in flight during the MFMAs and the next lookup
        __syncthreads();  // lkB complete (the next block's lookup rewrites ct / lkB only after
                          // its own barriers, which every wave reaches after these MFMAs)
        // ---- 4. dW += g'(block) lk(block)^T: A = g' rows (registers), B = lk rows (lkB) ----
#pragma unroll
        for (int c = 0; c < kCbCT; ++c) {
            const u32x4 bh = *reinterpret_cast<const u32x4 *>(&sm.lkB[0][16 * c + r16][4 * kg]);
            const u32x4 bm = *reinterpret_cast<const u32x4 *>(&sm.lkB[1][16 * c + r16][4 * kg]);
            const u32x4 bl = *reinterpret_cast<const u32x4 *>(&sm.lkB[2][16 * c + r16][4 * kg]);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                f32x4 s = mfma_bf16(al[t], bh, f32x4{0.f, 0.f, 0.f, 0.f});
                s = mfma_bf16(ah[t], bl, s);
                s = mfma_bf16(am[t], bm, s);
                s = mfma_bf16(am[t], bh, s);
                s = mfma_bf16(ah[t], bm, s);
                s = mfma_bf16(ah[t], bh, s);
                mW[t][c] += s;
            }
        }
    }
    // ---- partials: C[row = o][col = channel] ----
    if (do_dw) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int c = 0; c < kCbCT; ++c) {
                const int ch = 16 * c + r16;
                if (ch >= 81) continue;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int o = 32 * w + 16 * t + 4 * kg + i;
                    a.part[((size_t)r * kLcO + o) * a.C + 81 * l + ch] = mW[t][c][i];
                }
            }
    }
    if (do_b) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            float s = mb[t];  // this lane's 8-query column sums; then the 4 column groups in order
            const float s1 = __shfl_xor(s, 16), s2 = __shfl_xor(s, 32), s3 = __shfl_xor(s, 48);
            if (kg == 0) a.bpart[(size_t)r * kLcO + 32 * w + 16 * t + r16] = ((s + s1) + s2) + s3;
        }
    }
}

// dW[o][c] = sum_r part[r][o][c], d bias[o] = sum_r bpart[r][o], r in order (loads 8 deep).
__global__ __launch_bounds__(256) void lookup_conv_bwd_reduce_kernel(const float *__restrict__ part,
                                                                     const float *__restrict__ bpart, int R, int C,
                                                                     float *__restrict__ dW, float *__restrict__ db) {
    const int i = blockIdx.x * 256 + threadIdx.x, n = kLcO * C;
    const float *src;
    size_t stride;
    float *dst;
    if (i < n) {
        src = part + i, stride = (size_t)n, dst = dW ? dW + i : nullptr;
    } else if (i < n + kLcO) {
        src = bpart + (i - n), stride = kLcO, dst = db ? db + (i - n) : nullptr;
    } else {
        return;
    }
    if (!dst) return;
    float s = 0.f;
    int r = 0;
    for (; r + 8 <= R; r += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = src[(size_t)(r + k) * stride];
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; r < R; ++r) s += src[(size_t)r * stride];
    *dst = s;
}

template <int S, int BQ>
struct LookupBwdSmem {
    static constexpr int WIN = S + 2;
    static constexpr int WSTR = (WIN * WIN) | 1;  // odd stride: lane = query writes conflict-free
    float g[S * S][BQ];   // upstream gradient tile
    float tx[3][S][BQ];   // floor, lo, hi per x-tap
    float ty[3][S][BQ];
    int ax[BQ], ay[BQ];
    float win[BQ * WSTR];  // per-query neighbourhood sums (cell (cy, cx) at cy * WIN + cx)
};

constexpr int lookup_bwd_threads(int S, int BQ) { return (BQ * (S + 2) + 63) / 64 * 64; }
constexpr int kBwdQB = 64;  // queries per workgroup (32: 4 workgroups per CU but 10% slower, measured)

// Backward, three phases (BQ queries; thread (q, t) = (tid % BQ, tid / BQ), t < S + 2):
//   1. thread (q, t < S): tap t of query q on both axes + the gradient row of x-tap t -> LDS;
//   2. q = query, t = neighbourhood COLUMN cx: every cell (cx, cy) of the column sums its
//      contributions in the reference's scatter order (x-tap i outer, y-tap j inner; one
//      corner per (i, j)) — reads conflict-free (query-fastest LDS rows), sums -> win;
//   3. lane = consecutive cells of one query: coalesced read-modify-write of the gradient
//      pyramid, G = G + sum (one RMW per cell, no atomics: the cells are the query's own).
// Regular workgroups (floor(tap t) = floor(tap 0) + t on both axes) use the closed form — cell
// (cx, cy) of the (S+1)^2 block gets se(cx-1, cy-1), ne(cx-1, cy), sw(cx, cy-1), nw(cx, cy) —
// with all of a column's taps in registers.  Other workgroups find each column's / row's taps
// as the contiguous ranges {i : floor_i - anchor in {c - 1, c}} (floors are monotone in the
// tap index), which reduces to the same four terms, in the same order, for regular taps.
// Workgroups where some corner falls outside the (S+2)^2 neighbourhood (|coords| near 2^20)
// take the sequential per-query scatter (wave 0, lane = query) of the previous design.
// T lookups' (coords, upstream gradient) pairs of one build, processed in order by one launch
// (corr_lookup_bwd_multi / corr_backward): zero = the workgroup first zeroes its queries' maps of
// its level, so the gradient pyramid needs no separate memset and every lookup's RMW hits cells
// this workgroup wrote moments before (L2-resident).  The single-lookup entry is T = 1, zero = 0.
constexpr int kMaxLookups = 32;
struct BwdLookups {
    const float *coords[kMaxLookups];
    const float *grad[kMaxLookups];
    int T, zero;
};

template <int S, int BQ>
__global__ __launch_bounds__(lookup_bwd_threads(S, BQ)) void lookup_bwd_kernel(BwdLookups lk, int B, int NQ, int H,
                                                                           int W, int L, LevelPtrs gpyr) {
    constexpr int R = (S - 1) / 2, K = S * S, NT = lookup_bwd_threads(S, BQ);
    using SM = LookupBwdSmem<S, BQ>;
    constexpr int WIN = SM::WIN, WS = WIN * WIN, WSTR = SM::WSTR;
    constexpr int C = S + 1;  // cells per axis reached by regular taps
    __shared__ SM sm;

    const int N = NQ;  // query pixels per batch item (H*W, or a row slab of it)
    const int nqb = (N + BQ - 1) / BQ;
    const int b = blockIdx.x / nqb;
    const int n0 = (blockIdx.x - b * nqb) * BQ;
    const int l = blockIdx.y;
    const int Hl = H >> l, Wl = W >> l;
    const float inv_scale = 1.0f / (float)(1 << l);
    float *G = gpyr.p[l];
    const size_t mapsz = (size_t)Hl * Wl;
    const size_t qbase = (size_t)b * N + n0;

    const int tid = threadIdx.x;
    const int q = tid % BQ;
    const int t = tid / BQ;  // tap in phase 1, neighbourhood column in phase 2
    const int n = n0 + q;
    const bool qok = n < N;

    if (lk.zero) {  // this workgroup's query maps of level l (contiguous), before the first lookup
        const size_t cells = (size_t)min(BQ, N - n0) * mapsz;
        float *Z = G + qbase * mapsz;
        for (size_t i = tid; i < cells; i += NT) Z[i] = 0.0f;
        __syncthreads();
    }
    const float rdx = recip_rn((float)(Wl - 1)), rdy = recip_rn((float)(Hl - 1));
    for (int lt = 0; lt < lk.T; ++lt) {
    // constant-index selects (s_cselect): a dynamic index into the by-value table would copy it
    // to scratch
    const float *__restrict__ coords = lk.coords[0];
    const float *__restrict__ grad_out = lk.grad[0];
#pragma unroll
    for (int k = 1; k < kMaxLookups; ++k)
        if (k == lt) {
            coords = lk.coords[k];
            grad_out = lk.grad[k];
        }

    // ---- 1. taps and the upstream gradient tile ----
    Axis a{}, c{};
    if (t < S) {
        const float cxv = qok ? coords[((size_t)b * 2 + 0) * N + n] : 0.0f;
        const float cyv = qok ? coords[((size_t)b * 2 + 1) * N + n] : 0.0f;
        a = tap_axis(cxv, inv_scale, t, R, Wl, rdx);
        c = tap_axis(cyv, inv_scale, t, R, Hl, rdy);
        const float *g = grad_out + (((size_t)b * L + l) * K + (size_t)t * S) * N + n;
        float v[S];
#pragma unroll
        for (int u = 0; u < S; ++u) v[u] = qok ? g[(size_t)u * N] : 0.0f;
        sm.tx[0][t][q] = a.f;
        sm.tx[1][t][q] = a.lo;
        sm.tx[2][t][q] = a.hi;
        sm.ty[0][t][q] = c.f;
        sm.ty[1][t][q] = c.lo;
        sm.ty[2][t][q] = c.hi;
        if (t == 0) {
            sm.ax[q] = anchor_of(a.f);
            sm.ay[q] = anchor_of(c.f);
        }
#pragma unroll
        for (int u = 0; u < S; ++u) sm.g[t * S + u][q] = v[u];
    }
    __syncthreads();
    const float fx0 = sm.tx[0][0][q], fy0 = sm.ty[0][0][q];
    const bool far = anchor_of(fx0) == kFarAnchor || anchor_of(fy0) == kFarAnchor;
    const bool reg = t >= S || far || (a.f - fx0 == (float)t && c.f - fy0 == (float)t);
    const bool cov = t > 0 || window_covers<S>(fx0, sm.tx[0][S - 1][q], fy0, sm.ty[0][S - 1][q]);
    const int irregular = __syncthreads_or(!reg);
    const int uncovered = __syncthreads_or(!cov);

    if (!uncovered) {
        float *wq = &sm.win[q * WSTR];
        const int cx = t;
        if (!irregular) {
            // ---- 2a. closed form: column cx of the (S+1)^2 block ----
            if (cx < C && !far) {
                float wlo = 0.f, whi = 0.f;  // x weights: lo of tap cx, hi of tap cx - 1
                if (cx < S) wlo = sm.tx[1][cx][q];
                if (cx >= 1) whi = sm.tx[2][cx - 1][q];
                float ylo[S], yhi[S], gp[S], gc[S];
#pragma unroll
                for (int j = 0; j < S; ++j) {
                    ylo[j] = sm.ty[1][j][q];
                    yhi[j] = sm.ty[2][j][q];
                    gp[j] = cx >= 1 ? sm.g[(cx - 1) * S + j][q] : 0.f;
                    gc[j] = cx < S ? sm.g[cx * S + j][q] : 0.f;
                }
#pragma unroll
                for (int cy = 0; cy < C; ++cy) {
                    float s = 0.0f;
                    if (cx >= 1 && cy >= 1) s = s + __fmul_rn(gp[cy - 1], __fmul_rn(yhi[cy - 1], whi));  // se
                    if (cx >= 1 && cy < S) s = s + __fmul_rn(gp[cy], __fmul_rn(ylo[cy], whi));           // ne
                    if (cx < S && cy >= 1) s = s + __fmul_rn(gc[cy - 1], __fmul_rn(yhi[cy - 1], wlo));   // sw
                    if (cx < S && cy < S) s = s + __fmul_rn(gc[cy], __fmul_rn(ylo[cy], wlo));            // nw
                    wq[cy * WIN + cx] = s;
                }
            }
        } else if (!far && cx < WIN) {
            // ---- 2b. general taps: contiguous hit ranges per column / row ----
            float dy[S];
#pragma unroll
            for (int j = 0; j < S; ++j) dy[j] = sm.ty[0][j][q] - fy0;
            int i0 = 0, i1 = 0;
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const float d = sm.tx[0][i][q] - fx0;
                i0 += d < (float)(cx - 1);
                i1 += d <= (float)cx;
            }
#pragma unroll
            for (int cy = 0; cy < WIN; ++cy) {
                int j0 = 0, j1 = 0;
#pragma unroll
                for (int j = 0; j < S; ++j) {
                    j0 += dy[j] < (float)(cy - 1);
                    j1 += dy[j] <= (float)cy;
                }
                float s = 0.0f;
                for (int i = i0; i < i1; ++i) {
                    const float wx = (sm.tx[0][i][q] - fx0 == (float)cx) ? sm.tx[1][i][q] : sm.tx[2][i][q];
                    for (int j = j0; j < j1; ++j) {
                        const float wy = (sm.ty[0][j][q] - fy0 == (float)cy) ? sm.ty[1][j][q] : sm.ty[2][j][q];
                        s = s + __fmul_rn(sm.g[i * S + j][q], __fmul_rn(wy, wx));
                    }
                }
                wq[cy * WIN + cx] = s;
            }
        }
        __syncthreads();
        // ---- 3. coalesced read-modify-write of the query's cells ----
        int tidv = tid;
        asm volatile("" : "+v"(tidv));  // opaque per lookup: keeps the cell-index math out of the
                                        // loop preheader (hoisted, it held ~120 VGPRs and spilled)
        auto rmw = [&](auto cc_tag) {
            constexpr int CC = decltype(cc_tag)::value;
            constexpr int CELLS = BQ * CC * CC;
            constexpr int PER = (CELLS + NT - 1) / NT;
            float sum[PER], old[PER];
            size_t dst[PER];
            bool live[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int item = tidv + NT * u;
                const int qq = item / (CC * CC);
                const int e = item - qq * (CC * CC);
                const int cy = e / CC, cx2 = e - cy * CC;
                const int X = sm.ax[qq] + cx2, Y = sm.ay[qq] + cy;
                live[u] = item < CELLS && n0 + qq < N && X >= 0 && X < Wl && Y >= 0 && Y < Hl;
                sum[u] = live[u] ? sm.win[qq * WSTR + cy * WIN + cx2] : 0.0f;
                dst[u] = live[u] ? (qbase + qq) * mapsz + (size_t)Y * Wl + X : 0;
                old[u] = live[u] ? G[dst[u]] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < PER; ++u)
                if (live[u]) G[dst[u]] = old[u] + sum[u];
        };
        if (!irregular)
            rmw(std::integral_constant<int, C>{});
        else
            rmw(std::integral_constant<int, WIN>{});
        __syncthreads();  // the next lookup reuses the LDS and re-reads these cells
        continue;
    }

    // ---- 2c. uncovered workgroup: sequential per-query scatter (wave 0, lane = query) ----
    for (int g = tid; g < BQ * WSTR; g += NT) sm.win[g] = 0.0f;
    __syncthreads();
    if (t == 0 && qok) {
        const int ax = sm.ax[q], ay = sm.ay[q];
        float *wq = &sm.win[q * WSTR];
        float *Gq = G + (qbase + q) * mapsz;
        auto scatter = [&](float xf, float yf, float v) {
            if (!in_map(xf, yf, Wl, Hl)) return;
            const int xi = (int)xf, yi = (int)yf;
            const unsigned ux = (unsigned)(xi - ax), uy = (unsigned)(yi - ay);
            if (ux < (unsigned)WIN && uy < (unsigned)WIN)
                wq[uy * WIN + ux] += v;
            else
                Gq[(size_t)yi * Wl + xi] += v;  // outside the neighbourhood: disjoint cells
        };
        for (int ii = 0; ii < S; ++ii) {
            const float x0 = sm.tx[0][ii][q], x1 = __fadd_rn(x0, 1.0f);
            const float ex = sm.tx[1][ii][q], wx = sm.tx[2][ii][q];
            for (int j = 0; j < S; ++j) {
                const float gv = sm.g[ii * S + j][q];
                const float y0 = sm.ty[0][j][q], y1 = __fadd_rn(y0, 1.0f);
                const float ey = sm.ty[1][j][q], ny = sm.ty[2][j][q];
                scatter(x0, y0, __fmul_rn(gv, __fmul_rn(ey, ex)));
                scatter(x1, y0, __fmul_rn(gv, __fmul_rn(ey, wx)));
                scatter(x0, y1, __fmul_rn(gv, __fmul_rn(ny, ex)));
                scatter(x1, y1, __fmul_rn(gv, __fmul_rn(ny, wx)));
            }
        }
    }
    __syncthreads();
    for (int g = tid; g < BQ * WS; g += NT) {
        const int qq = g / WS;
        const int e = g - qq * WS;
        if (n0 + qq >= N) continue;
        const int ry = e / WIN, rx = e - ry * WIN;
        const int Y = sm.ay[qq] + ry, X = sm.ax[qq] + rx;
        if (X >= 0 && X < Wl && Y >= 0 && Y < Hl) {
            float *d = G + (qbase + qq) * mapsz + (size_t)Y * Wl + X;
            *d = *d + sm.win[qq * WSTR + e];
        }
    }
    __syncthreads();
    }  // lookups
}

// ---------------------------------------------------------------------------------------------
// Fused backward of one build's T lookups + the avg-pool backward (corr_backward's fast path).
// A workgroup owns BQ query pixels and ALL (<= 4) levels of their gradient maps, resident in LDS
// for the whole launch: zeroed, then every lookup's window sums are added in lookup order (the
// same per-cell values as lookup_bwd_kernel: s = the cell's contributions of one lookup in the
// reference's scatter order, then M = M + s), then the maps are folded coarse-to-fine into
// level 0 (pool_fold_max_kernel's per-cell recurrence) and ONLY dC = level 0 is written, with
// its row maxima (written) and column maxima (atomicMax).  The coarse levels never reach HBM and
// no cell is read-modify-written in HBM: traffic = the upstream gradients + coords + dC.
// Wave w = level w; lane = (query q, neighbourhood column cx) with SLOTS = pow2 >= S + 2 lanes
// per query, so BQ = 64 / SLOTS queries (4 at r = 4).  A wave touches only its own level's maps
// and staging, so the lookup loop has NO workgroup barrier: each wave streams through the T
// lookups on its own (the next lookup's loads in flight), and the workgroup meets once, before
// the fold.  Per lookup: lanes cx < S compute tap cx of both axes; the closed form takes the
// group's other taps by DPP (row_newbcast for the y-taps and the anchors, row_shr for x-tap
// cx - 1 and its gradients), so a regular lookup touches LDS only for its cells.  Lane cx then
// produces its column's cells — closed form (regular taps), contiguous hit ranges (irregular;
// separable: the general separable form), or, when a corner leaves the (S+2)^2 neighbourhood,
// lookup_bwd_kernel's sequential scatter into a zeroed window scratch (the exact kernel reads
// every tap and gradient for these from the wave's LDS staging, written only when some group of
// the wave needs it; the separable kernel has no staging and shuffles them) — and adds them to
// the map (out-of-map cells: clamped into guard rows, or a per-lane dump slot).
constexpr int kFusedLv = 4;  // level slots (= waves) per workgroup

// median of three (v_med3_i32: clang does not form it from min / max with runtime bounds)
__device__ __forceinline__ int med3_i32(int x, int lo, int hi) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

// A byte address past any workgroup's LDS allocation (<= 160 KiB) even after a map's worth of rows
// is subtracted: DS reads there return 0, DS writes are dropped.
constexpr int kLdsOob = 1 << 20;

constexpr int fused_slots(int S) { return S + 2 <= 4 ? 4 : S + 2 <= 8 ? 8 : S + 2 <= 16 ? 16 : 32; }

struct FusedOut {
    float *dc;              // [B * NQ][H * W]
    unsigned *rmax, *cmax;  // [B][NQ] (written), [B][H * W] (atomicMax; zeroed by the caller); may be null
    float *cpart;           // [B][groups][H * W]: per-workgroup column maxima instead of cmax atomics
    int B, NQ, H, W, L;
    int moff[kFusedLv], msz[kFusedLv];  // LDS float offset of level l's maps, cells per map
    int qstr[kFusedLv];                 // LDS floats between two queries' maps (bank-staggered)
    int aux;                            // LDS float offset of the per-wave staging
    int nfold;                          // fold workgroups; blocks past them compute rm
    int rm_rows_per_wave;
    FoldRowMax rm;
};

// Row |max| work of the blocks appended to the fold grid (rowmax2_kernel's per-row reduction:
// a wave walks each of its rows with 16-B loads, one cross-lane reduction per row).  They sit
// at the end of the grid, so they run in the fold's last, partly empty round of workgroups.
__device__ __forceinline__ void fold_rowmax_block(const FusedOut &o, int blk, int waves) {
    const FoldRowMax &a = o.rm;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int per_op = o.B * a.rows;  // rows of one operand, over the batch
    for (int k = 0; k < o.rm_rows_per_wave; ++k) {
        const int g = (blk * waves + wv) * o.rm_rows_per_wave + k;
        if (g >= 2 * per_op) return;  // whole waves
        const int t = g / per_op, br = g - t * per_op;
        const int cols = a.cols[t];
        const float *x = a.x[t] + (size_t)br * cols;
        float m = 0.f;
        if ((cols & 3) == 0 && ((uintptr_t)a.x[t] & 15) == 0) {
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
        for (int sh = 32; sh >= 1; sh >>= 1) m = fmaxf(m, __shfl_xor(m, sh));
        if (lane == 0) a.out[t][br] = m > 0.f ? __float_as_uint(m) : 0u;
    }
}

// Per-wave staging (floats): taps TX/TY [3][S][BQ], gradients [K][BQ], anchors [2][BQ], dump
// slots [64].
template <int S>
struct FusedStage {
    static constexpr int SLOTS = fused_slots(S), BQ = 64 / SLOTS, K = S * S, WIN = S + 2;
    static constexpr int TX = 0, TY = TX + 3 * S * BQ, GG = TY + 3 * S * BQ, AX = GG + K * BQ, AY = AX + BQ,
                         DUMP = AY + BQ, SIZE = DUMP + 64;
};

// The separable fold with one DPP row per (query, level) group keeps no per-wave staging in LDS:
// its irregular windows take the general separable form and its rare windows (corners outside
// the neighbourhood, taps more than one cell off, non-finite gradients) the sequential scatter,
// which reads the group's taps and gradients by lane shuffles (ds_bpermute: no LDS allocated).
template <int S, bool SEP>
constexpr bool fold_no_staging() { return SEP && FusedStage<S>::SLOTS == 16; }

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2).  Renumber them so
// every XCD gets a contiguous range: neighbouring query groups — which share the 128-B lines of
// the upstream gradients and coords — then read those lines through one L2 instead of eight.
// A bijection on [0, n) for any n.
__device__ __forceinline__ int xcd_contiguous(int bid, int n) {
    constexpr int kXcd = 8;
    const int q = n / kXcd, r = n % kXcd;
    const int x = bid % kXcd, k = bid / kXcd;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// x of the previous lane of a SLOTS-lane group, 0 for the group's first lane (cx = 0).  Groups of
// <= 16 lanes sit inside one DPP row: row_shr:1 (bound_ctrl: lane 0 of a row reads 0); larger
// groups use a bpermute.
template <int SLOTS>
__device__ __forceinline__ float lane_prev(float x, int cx) {
    if constexpr (SLOTS == 16) {  // the group is the DPP row: its lane 0 (cx = 0) reads the 0
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xF, 0xF, true));
    } else if constexpr (SLOTS < 16) {
        const int y = __builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xF, 0xF, true);
        return cx == 0 ? 0.f : __int_as_float(y);
    } else {
        const float y = __shfl_up(x, 1, 64);
        return cx == 0 ? 0.f : y;
    }
}

// Lane J of this lane's SLOTS-lane group.  Groups of 16 lanes are DPP rows: row_newbcast:J (one
// VALU move, no LDS); other group sizes use a bpermute.
template <int SLOTS, int J>
__device__ __forceinline__ float group_lane(float x, int lane) {
    if constexpr (SLOTS == 16) {  // every lane is written: no old value to initialise
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x150 + J, 0xF, 0xF, false));
    } else {
        return __shfl(x, (lane & ~(SLOTS - 1)) + J, 64);
    }
}

template <int SLOTS, int N, int J = 0>
__device__ __forceinline__ void group_lanes(float x, int lane, float (&out)[N]) {
    if constexpr (J < N) {
        out[J] = group_lane<SLOTS, J>(x, lane);
        group_lanes<SLOTS, N, J + 1>(x, lane, out);
    }
}

// Orders this wave's LDS traffic (LDS executes one wave's operations in issue order; the asm
// also keeps the compiler from moving LDS accesses across it).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// The lookup table (the kernel's FIRST argument) in VGPRs: lane i holds lookup i's two pointers,
// read once from the kernarg segment by a vector load; lookup t's are then two pairs of
// v_readlane.  Indexing the by-value copy with a runtime t makes the compiler either spill the
// table to scratch or emit a 32-way branch tree, and a scalar load per lookup would make every
// lookup wait for lgkmcnt(0) — i.e. also for the previous lookup's LDS writes — before its loads.
struct LaneTable {
    uint32_t c_lo, c_hi, g_lo, g_hi;
    __device__ __forceinline__ explicit LaneTable(int lane) {
        typedef const BwdLookups __attribute__((address_space(4))) *KPtr;
        const KPtr kp = (KPtr)__builtin_amdgcn_kernarg_segment_ptr();
        const int i = min(lane, kMaxLookups - 1);
        const uint64_t c = (uint64_t)kp->coords[i], g = (uint64_t)kp->grad[i];
        c_lo = (uint32_t)c, c_hi = (uint32_t)(c >> 32), g_lo = (uint32_t)g, g_hi = (uint32_t)(g >> 32);
    }
    __device__ __forceinline__ void get(int t, const float *&c, const float *&g) const {
        // (readlane returns int: widen through uint32_t, or a low word >= 2^31 sign-extends)
        c = reinterpret_cast<const float *>(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(c_hi, t) << 32) |
                                            (uint64_t)(uint32_t)__builtin_amdgcn_readlane(c_lo, t));
        g = reinterpret_cast<const float *>(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(g_hi, t) << 32) |
                                            (uint64_t)(uint32_t)__builtin_amdgcn_readlane(g_lo, t));
    }
};

// PROBE (measurement builds only, tools/kbench_bwd.hip; the library uses 0): bit 0 = no lookup
// loop, bit 1 = no fold (no dC / maxima), bit 2 = no LDS zero-init (wrong results, timing only),
// bit 3 = plain (L2-cached) dC stores instead of the non-temporal ones, bit 4 = wait for the
// lookup's LDS writes at the end of each lookup (round 5's s_waitcnt).  (Moving the closed form's
// y-tap broadcasts, or its previous-column gradients, from DPP to ds_bpermute — LDS pipe
// instead of VALU — was measured and dropped: T = 12 79 -> 88 / 83 us,
// profiles/r06f_kbench_bwd_lean.txt; so was an L2 warm-up of lookup t + 3's gradient lines, one
// dword per row by the first workgroup of each 32-query line group: 145 -> 144 us with the
// gradients evicted before the launch, 79 -> 114 us warm, profiles/r06i_kbench_bwd_l2warm.txt.)
// SEP: regular windows by the separable closed form (corr_backward's default); false replays
// grid_sampler_2d_backward's per-tap products bit for bit (CORR_BACKWARD_EXACT_FOLD).
// (Several query groups per workgroup — 8 or 16 queries, so that the groups' waves would share
// L1 fills of the upstream-gradient lines — were measured and dropped: L2 requests unchanged,
// T = 12 92 -> 101 / 164 us, profiles/r05zi_kbench_bwd_groups_dropped.txt.)
// LEAN: the fold phase for the common case — 4 levels, no maxima (the bf16x6 backward),
// W % 4 == 0 and 16-B aligned dC — with the level values shared across a thread's 4 cells read
// once and no maxima arithmetic (the generic fold recomputed the coarse chain per cell and took
// |max| of every value: ~45 % of the fold phase's VALU).  The same per-cell sums in the same
// order (bit-identical).
template <int S, int PROBE = 0, bool SEP = false, bool LEAN = false>
__global__ __launch_bounds__(64 * kFusedLv) void lookup_bwd_fold_kernel(BwdLookups lk, FusedOut o) {
    using ST = FusedStage<S>;
    constexpr int R = (S - 1) / 2, K = S * S, C = S + 1, WIN = ST::WIN;
    constexpr int SLOTS = ST::SLOTS, BQ = ST::BQ, WQ = BQ, NT = 64 * kFusedLv;
    constexpr bool NOST = fold_no_staging<S, SEP>();
    extern __shared__ float fsm[];

    if ((int)blockIdx.x >= o.nfold) {  // appended row-maxima blocks (uniform per workgroup)
        fold_rowmax_block(o, (int)blockIdx.x - o.nfold, kFusedLv);
        return;
    }
    const int NQ = o.NQ, H = o.H, W = o.W, L = o.L, N = H * W;
    const int nqb = (NQ + WQ - 1) / WQ;
    const int blk = xcd_contiguous(blockIdx.x, o.nfold);
    const int b = blk / nqb, n0 = (blk - b * nqb) * WQ;
    const int tid = threadIdx.x, lane = tid & 63;
    const int l = tid >> 6;  // wave = level
    const int q = lane / SLOTS, cx = lane - q * SLOTS;
    const bool act = l < L;
    const int n = n0 + q;
    const bool qok = n < NQ;
    const int lc = act ? l : 0;
    const int Hl = H >> lc, Wl = W >> lc;
    const float inv_scale = 1.0f / (float)(1 << lc);
    const float rdx = recip_rn((float)(Wl - 1)), rdy = recip_rn((float)(Hl - 1));
    float *st = fsm + o.aux + lc * ST::SIZE;  // this wave's staging
    const int mbase = o.moff[lc] + q * o.qstr[lc];
    // fsm's LDS byte address (0 unless the kernel gains static LDS) and an LDS float at an
    // absolute byte address
    const int lds_base = (int)(uintptr_t)(__attribute__((address_space(3))) float *)fsm;
    auto lds_at = [](unsigned a) { return (__attribute__((address_space(3))) float *)(uintptr_t)a; };
    const int dump = o.aux + lc * ST::SIZE + ST::DUMP + lane;
    auto tx = [&](int c, int t) -> float & { return st[ST::TX + (c * S + t) * BQ + q]; };
    auto ty = [&](int c, int t) -> float & { return st[ST::TY + (c * S + t) * BQ + q]; };
    auto gg = [&](int k) -> float & { return st[ST::GG + k * BQ + q]; };
    unsigned *RM = reinterpret_cast<unsigned *>(fsm + o.aux + (NOST ? 0 : kFusedLv * ST::SIZE));  // [WQ]

    // the next lookup's coords and upstream gradients are loaded one lookup ahead (registers),
    // by buffer loads over batch item b's slice: every lane loads, and the lanes that own no
    // (tap, query) point past the slice, so the range check returns their zeros (no branch
    // around the loads, no select at use, 32-bit offsets).  The gradients are loaded in the
    // transposed lane order (lane 4 cx + q holds x-tap cx of query q), so the 4 lanes of a quad
    // read one 16-B run (the BQ queries' values of one row): one cache access per quad instead
    // of one per lane — the vector memory pipe (TA / TD ~85 % busy) bounded the lookup loop
    // (profiles/r05zg_fold_pmc.txt) — and one ds_bpermute per value restores lane order.
    const bool loader = act && cx < S && qok;
    const int cxl = min(cx, S - 1);
    constexpr uint32_t kOob = 0x80000000u;
    const uint32_t coff = loader ? (uint32_t)n * 4u : kOob;
    constexpr bool kQuadLoads = SLOTS == 16 && BQ == 4;
    const int lq = kQuadLoads ? ((lane & 3) ^ ((lane >> 5) << 1)) : q, lx = kQuadLoads ? (lane >> 2) : cx;
    const bool gloader = act && lx < S && n0 + lq < NQ;
    const uint32_t goff = gloader ? (uint32_t)(((lc * K + lx * S) * NQ + n0 + lq) * 4) : kOob;
    // ds_bpermute byte address of this lane's loader (lane 4 cx + (q ^ 2 [cx >= 8]))
    const int gsrc = kQuadLoads ? 4 * (4 * cx + (q ^ ((cx >> 3) << 1))) : 0;
    float pcx, pcy, pv[S];
    const LaneTable table(lane);
    auto prefetch = [&](int t) {
        const float *coords, *grad_out;
        table.get(t, coords, grad_out);
        const auto rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(coords + (size_t)b * 2 * NQ), 0,
                                                          2 * NQ * 4, 0x00020000);
        const auto rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(grad_out + (size_t)b * L * K * NQ), 0,
                                                          L * K * NQ * 4, 0x00020000);
        pcx = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, coff, 0, 0));
        pcy = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, coff, NQ * 4, 0));
#pragma unroll
        for (int u = 0; u < S; ++u)
            pv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, goff, u * NQ * 4, 0));
    };
    if (act) prefetch(0);  // issued before the LDS zeroing, so its latency hides behind it
    if (!(PROBE & 4))
        // every map of the workgroup, 16 B per store (o.aux is a multiple of 4 floats)
        for (int i = 4 * tid; i < o.aux; i += 4 * NT) *reinterpret_cast<float4 *>(fsm + i) = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < WQ) RM[tid] = 0u;
    __syncthreads();

    for (int t = 0; !(PROBE & 1) && act && t < lk.T; ++t) {  // absent levels (l >= L) only join the fold
        // ---- 1. tap cx of both axes; the group's taps reach the other lanes by DPP ----
        const float cxv = pcx, cyv = pcy;  // 0 for the lanes without a (tap, query)
        float v[S];
#pragma unroll
        for (int u = 0; u < S; ++u)
            v[u] = kQuadLoads ? __int_as_float(__builtin_amdgcn_ds_bpermute(gsrc, __float_as_int(pv[u]))) : pv[u];
        prefetch(min(t + 1, lk.T - 1));
        const Axis a = tap_axis(cxv, inv_scale, cxl, R, Wl, rdx);
        const Axis c = tap_axis(cyv, inv_scale, cxl, R, Hl, rdy);
        // ---- 2. the (query, level) group's form, decided per group ----
        const float fx0 = group_lane<SLOTS, 0>(a.f, lane), fy0 = group_lane<SLOTS, 0>(c.f, lane);
        const bool bad = cx < S && !(a.f - fx0 == (float)cx && c.f - fy0 == (float)cx);
        const unsigned long long gmask = (SLOTS == 64 ? ~0ull : ((1ull << SLOTS) - 1)) << (q * SLOTS);
        const bool irregular = (__ballot(bad) & gmask) != 0;
        const int ax = anchor_of(fx0), ay = anchor_of(fy0);
        const bool far = ax == kFarAnchor || ay == kFarAnchor;
        const bool unc = qok && !window_covers<S>(fx0, group_lane<SLOTS, S - 1>(a.f, lane), fy0,
                                                  group_lane<SLOTS, S - 1>(c.f, lane));
        // irregular groups take the range form (exact) — or, without staging (NOST), the general
        // separable form below, unless a tap's floor is more than one cell off its regular place
        // (only near |coordinates| ~ 2^20) or some upstream gradient of the wave is not finite
        // (that form multiplies every candidate tap, so a zero weight would turn an infinite
        // gradient into a NaN the reference does not have): those groups, like the groups whose
        // corners leave the neighbourhood, take the sequential scatter (seq)
        bool rangef = irregular, seq = unc;
        if constexpr (NOST) {
            rangef = false;
            if (__ballot(irregular)) {
                const bool odd = cx < S && !(fabsf(a.f - fx0 - (float)cx) <= 1.f && fabsf(c.f - fy0 - (float)cx) <= 1.f);
                bool nonfin = false;
#pragma unroll
                for (int u = 0; u < S; ++u) nonfin |= !__builtin_isfinite(v[u]);
                seq = unc || (irregular && qok && !far &&
                              (__ballot(nonfin) != 0 || (__ballot(odd && qok && !far) & gmask) != 0));
            }
        } else if (__ballot(rangef || unc)) {
            // the range form and the sequential scatter read any tap and any tap's gradients from
            // the wave's staging: written only when some group of the wave takes one of those paths
            if (cx < S) {
                tx(0, cx) = a.f, tx(1, cx) = a.lo, tx(2, cx) = a.hi;
                ty(0, cx) = c.f, ty(1, cx) = c.lo, ty(2, cx) = c.hi;
#pragma unroll
                for (int u = 0; u < S; ++u) gg(cx * S + u) = v[u];
            }
            wave_lds_sync();
        }
        const int X = ax + cx;
        const bool colok = qok && !seq && !far && cx < WIN && X >= 0 && X < Wl;
        // cell (cx, cy) of the window -> its map address, or the lane's dump slot when the cell
        // is outside the map / the column is not this lane's to write
        const int ayv = colok ? ay : -(1 << 30);
        const int rowbase = mbase + ay * Wl + X;
        auto cell_at = [&](int cy) { return (unsigned)(ayv + cy) < (unsigned)Hl ? rowbase + cy * Wl : dump; };
        // adds the column's NC cells sv[cy] (rows ay + cy) to the map.  Byte addresses: row ay + cy
        // clamped to [-1, Hl] — rows -1 and Hl of every map are guard rows (fused_lds_bytes), so
        // the window's cells above / below the map land in a guard row nothing reads — and a column
        // that is not this lane's to write starts past the workgroup's LDS allocation, where DS
        // reads return 0 and DS writes are dropped.  Clamping the ADDRESS of row ay + cy between
        // those of rows -1 and H_l is the same (addresses grow with the row), so a cell costs one
        // add and one v_med3.
        auto add_column = [&]<int NC>(const float (&sv)[NC]) {
            const bool mine = colok && cx < NC;
            // absolute LDS byte addresses (fsm's own offset folded into cb once: the accesses
            // then take the clamped address as is, no add per cell)
            const int cb = lds_base + (mine ? 4 * (mbase + X) : kLdsOob);
            const int s4 = 4 * Wl;
            const int gtop = cb - s4, gbot = cb + Hl * s4;
            // rows past [-NC, H_l] clamp like those bounds (and keep s4 * ay in range)
            int ra = cb + s4 * (mine ? min(max(ay, -NC), Hl) : 0);
            float old[NC];
            unsigned at[NC];
#pragma unroll
            for (int cy = 0; cy < NC; ++cy, ra += s4) at[cy] = (unsigned)med3_i32(ra, gtop, gbot);
#pragma unroll
            for (int cy = 0; cy < NC; ++cy) old[cy] = *lds_at(at[cy]);  // all reads, then all writes
#pragma unroll
            for (int cy = 0; cy < NC; ++cy) *lds_at(at[cy]) = old[cy] + sv[cy];
        };
        if (!irregular) {
            // closed form.  Absent terms (window edges) carry zero weights and gradients: adding
            // +-0 to a sum that started at +0 leaves it unchanged, so every cell sums its 4 terms
            // in the reference's order (se, ne, sw, nw) with the same bits.  Arrays are indexed
            // by y-tap j + 1 with zero sentinels at j = -1 and j = S, and two cells (cy, cy + 1)
            // go through each packed-fp32 instruction (v_pk_mul_f32 / v_pk_add_f32, IEEE per lane).
            // x-tap cx is this lane's own, x-tap cx - 1 the previous lane's; y-tap j is lane j's.
            const float wlo = cx < S ? a.lo : 0.f;
            const float hprev = lane_prev<SLOTS>(a.hi, cx);
            const float whi = cx >= 1 && cx <= S ? hprev : 0.f;
            float ylo_[S], yhi_[S];
            group_lanes<SLOTS, S>(c.lo, lane, ylo_);
            group_lanes<SLOTS, S>(c.hi, lane, yhi_);
            auto yv = [&](int cc, int j) { return j >= 0 && j < S ? (cc == 1 ? ylo_[j] : yhi_[j]) : 0.f; };
            // the gradients of x-tap cx are this lane's own loads (v: zero for cx >= S and for
            // absent queries), those of x-tap cx - 1 the previous lane's (lane_prev: zero at cx = 0)
            float gpr[S];
#pragma unroll
            for (int j = 0; j < S; ++j) gpr[j] = lane_prev<SLOTS>(v[j], cx);
            auto gpv = [&](int j) { return j >= 0 && j < S ? gpr[j] : 0.f; };
            auto gcv = [&](int j) { return j >= 0 && j < S ? v[j] : 0.f; };
            const f32x2 WH = f32x2{whi, whi}, WL = f32x2{wlo, wlo};
            float sv[C + 1];
            if constexpr (SEP) {
                // separable (the default): the column's two x-taps first, hx[j] = g(cx - 1, j) whi +
                // g(cx, j) wlo for each y-tap j, then the y-taps, cell cy = hx[cy - 1] yhi[cy - 1] +
                // hx[cy] ylo[cy] — the same four (tap, corner) terms with the same per-tap weights,
                // rounded in another order (~1e-7 relative; tests/test_gpu_parity.py), for ~30
                // instead of ~70 VALU per lane
                float hx[S];
#pragma unroll
                for (int j = 0; j + 1 < S; j += 2) {
                    const f32x2 h = __builtin_elementwise_fma(f32x2{v[j], v[j + 1]}, WL, f32x2{gpr[j], gpr[j + 1]} * WH);
                    hx[j] = h.x, hx[j + 1] = h.y;
                }
                if constexpr ((S & 1) != 0) hx[S - 1] = __builtin_fmaf(v[S - 1], wlo, gpr[S - 1] * whi);
#pragma unroll
                for (int cy = 0; cy < C; ++cy) {
                    const float up = cy >= 1 ? hx[cy - 1] * yhi_[cy - 1] : 0.f;
                    sv[cy] = cy < S ? __builtin_fmaf(hx[cy], ylo_[cy], up) : up;
                }
            } else
#pragma unroll
            for (int cy = 0; cy < C; cy += 2) {  // cells cy, cy + 1; se / sw use y-tap cy - 1, ne / nw cy
                const f32x2 yhi = f32x2{yv(2, cy - 1), yv(2, cy)}, ylo = f32x2{yv(1, cy), yv(1, cy + 1)};
                const f32x2 gpm = f32x2{gpv(cy - 1), gpv(cy)}, gp0 = f32x2{gpv(cy), gpv(cy + 1)};
                const f32x2 gcm = f32x2{gcv(cy - 1), gcv(cy)}, gc0 = f32x2{gcv(cy), gcv(cy + 1)};
                // se first.  The reference's cell starts at +0 (0 + se): starting at se differs
                // only when every term is -0, giving -0 instead of +0 — and the map value it is
                // added to is never -0 (it starts at +0 and no round-to-nearest sum of it is -0),
                // so old + sv is the same bits either way.
                f32x2 acc = gpm * (yhi * WH);
                acc = acc + gp0 * (ylo * WH);                    // ne
                acc = acc + gcm * (yhi * WL);                    // sw
                acc = acc + gc0 * (ylo * WL);                    // nw
                sv[cy] = acc.x;
                sv[cy + 1] = acc.y;
            }
            add_column(reinterpret_cast<const float (&)[C]>(sv));
        } else if (!rangef) {
            if constexpr (SEP && SLOTS == 16) {
                // general separable form (irregular windows: taps of a query whose floors are not all
                // anchor + t, e.g. the cold-start integer grid, where rounding leaves some taps a hair
                // below their integer).  Tap t's floor is anchor + t + e_t with e_t in {-1, 0, 1}, so it
                // reaches cells t - 1 .. t + 2 of the neighbourhood: slot k in {-1, 0, 1, 2} weighs
                // lo at k = e_t, hi at k = e_t + 1, 0 elsewhere.  Column cx gathers x-taps cx, cx - 1,
                // cx - 2, cx + 1 (DPP row shifts: the 16-lane group is the DPP row, lanes outside it
                // read 0), then row cy gathers y-taps cy, cy - 1, cy - 2, cy + 1 (broadcast weights).
                // Non-reached slots multiply a finite gradient by 0 (seq takes the waves with non-finite ones).
                const bool tv = cx < S;
                auto slots = [&](float e, float lo, float hi, float &wm1, float &w0, float &w1, float &w2) {
                    const bool m = e == -1.f, z = e == 0.f, p = e == 1.f;  // e = 2: no tap
                    wm1 = m ? lo : 0.f;
                    w0 = m ? hi : (z ? lo : 0.f);
                    w1 = z ? hi : (p ? lo : 0.f);
                    w2 = p ? hi : 0.f;
                };
                float xm1, x0, x1, x2, ym1, y0, y1, y2;
                slots(tv ? a.f - fx0 - (float)cx : 2.f, a.lo, a.hi, xm1, x0, x1, x2);
                slots(tv ? c.f - fy0 - (float)cx : 2.f, c.lo, c.hi, ym1, y0, y1, y2);
                auto shr1 = [](float x) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xF, 0xF, true)); };
                auto shr2 = [](float x) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x112, 0xF, 0xF, true)); };
                auto shl1 = [](float x) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x101, 0xF, 0xF, true)); };
                const float wp1 = shr1(x1), wp2 = shr2(x2), wn1 = shl1(xm1);
                float hx[S];
#pragma unroll
                for (int j = 0; j < S; ++j)
                    hx[j] = __builtin_fmaf(v[j], x0, __builtin_fmaf(shr1(v[j]), wp1, __builtin_fmaf(shr2(v[j]), wp2, shl1(v[j]) * wn1)));
                float Ym1[S], Y0[S], Y1[S], Y2[S];
                group_lanes<SLOTS, S>(ym1, lane, Ym1);
                group_lanes<SLOTS, S>(y0, lane, Y0);
                group_lanes<SLOTS, S>(y1, lane, Y1);
                group_lanes<SLOTS, S>(y2, lane, Y2);
                float sv[WIN];
#pragma unroll
                for (int cy = 0; cy < WIN; ++cy) {
                    float acc = cy < S ? hx[cy] * Y0[cy] : 0.f;
                    if (cy >= 1 && cy - 1 < S) acc = __builtin_fmaf(hx[cy - 1], Y1[cy - 1], acc);
                    if (cy >= 2 && cy - 2 < S) acc = __builtin_fmaf(hx[cy - 2], Y2[cy - 2], acc);
                    if (cy + 1 < S) acc = __builtin_fmaf(hx[cy + 1], Ym1[cy + 1], acc);
                    sv[cy] = acc;
                }
                add_column(sv);
            }
        } else if constexpr (!NOST) {
            float dy[S];
#pragma unroll
            for (int j = 0; j < S; ++j) dy[j] = ty(0, j) - fy0;
            int i0 = 0, i1 = 0;
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const float d = tx(0, i) - fx0;
                i0 += d < (float)(cx - 1);
                i1 += d <= (float)cx;
            }
            for (int cy = 0; cy < WIN; ++cy) {
                int j0 = 0, j1 = 0;
#pragma unroll
                for (int j = 0; j < S; ++j) {
                    j0 += dy[j] < (float)(cy - 1);
                    j1 += dy[j] <= (float)cy;
                }
                float sv = 0.0f;
                if (colok)
                    for (int i = i0; i < i1; ++i) {
                        const float wx = (tx(0, i) - fx0 == (float)cx) ? tx(1, i) : tx(2, i);
                        for (int j = j0; j < j1; ++j) {
                            const float wy = (ty(0, j) - fy0 == (float)cy) ? ty(1, j) : ty(2, j);
                            sv = sv + __fmul_rn(gg(i * S + j), __fmul_rn(wy, wx));
                        }
                    }
                const int at = cell_at(cy);
                fsm[at] = fsm[at] + sv;
            }
        }
        // ---- 2c. groups whose corners leave the neighbourhood (and, NOST, the rare irregular
        // ones): sequential scatter ----
        // The group's in-map window cells are saved to registers and zeroed, so they serve as the
        // zeroed window scratch; afterwards cell = saved + scatter sum (lookup_bwd_kernel's order).
        if (__ballot(seq)) {
            float *Mq = fsm + mbase;
            const bool mine = seq && cx < WIN && X >= 0 && X < Wl;
            float keep[WIN];
#pragma unroll
            for (int ry = 0; ry < WIN; ++ry) {
                const int Y = ay + ry;
                keep[ry] = 0.f;
                if (mine && Y >= 0 && Y < Hl) {
                    keep[ry] = Mq[Y * Wl + X];
                    Mq[Y * Wl + X] = 0.0f;
                }
            }
            wave_lds_sync();
            auto scatter = [&](float xf, float yf, float val) {
                if (!in_map(xf, yf, Wl, Hl)) return;
                Mq[(int)yf * Wl + (int)xf] += val;  // window cells: the zeroed scratch
            };
            if constexpr (NOST) {
                // the group's taps and gradients by lane shuffles (all lanes take part; lane 0 of
                // each sequential group scatters)
                const int g0 = lane & ~(SLOTS - 1);
                for (int ii = 0; ii < S; ++ii) {
                    const float x0 = __shfl(a.f, g0 + ii, 64), ex = __shfl(a.lo, g0 + ii, 64);
                    const float wx = __shfl(a.hi, g0 + ii, 64), x1 = __fadd_rn(x0, 1.0f);
#pragma unroll
                    for (int j = 0; j < S; ++j) {
                        const float gv = __shfl(v[j], g0 + ii, 64);
                        const float y0 = __shfl(c.f, g0 + j, 64), ey = __shfl(c.lo, g0 + j, 64);
                        const float ny = __shfl(c.hi, g0 + j, 64), y1 = __fadd_rn(y0, 1.0f);
                        if (seq && cx == 0) {
                            scatter(x0, y0, __fmul_rn(gv, __fmul_rn(ey, ex)));
                            scatter(x1, y0, __fmul_rn(gv, __fmul_rn(ey, wx)));
                            scatter(x0, y1, __fmul_rn(gv, __fmul_rn(ny, ex)));
                            scatter(x1, y1, __fmul_rn(gv, __fmul_rn(ny, wx)));
                        }
                    }
                }
            } else if (seq && cx == 0) {
                for (int ii = 0; ii < S; ++ii) {
                    const float x0 = tx(0, ii), x1 = __fadd_rn(x0, 1.0f);
                    const float ex = tx(1, ii), wx = tx(2, ii);
                    for (int j = 0; j < S; ++j) {
                        const float gv = gg(ii * S + j);
                        const float y0 = ty(0, j), y1 = __fadd_rn(y0, 1.0f);
                        const float ey = ty(1, j), ny = ty(2, j);
                        scatter(x0, y0, __fmul_rn(gv, __fmul_rn(ey, ex)));
                        scatter(x1, y0, __fmul_rn(gv, __fmul_rn(ey, wx)));
                        scatter(x0, y1, __fmul_rn(gv, __fmul_rn(ny, ex)));
                        scatter(x1, y1, __fmul_rn(gv, __fmul_rn(ny, wx)));
                    }
                }
            }
            wave_lds_sync();
#pragma unroll
            for (int ry = 0; ry < WIN; ++ry) {
                const int Y = ay + ry;
                if (mine && Y >= 0 && Y < Hl) Mq[Y * Wl + X] = keep[ry] + Mq[Y * Wl + X];
            }
        }
        // the next lookup rewrites the staging: a compiler barrier keeps this lookup's LDS accesses
        // before the next one's (one wave's DS operations execute in issue order, so no wait is
        // needed: the map writes drain while the next lookup's taps are computed)
        if constexpr ((PROBE & 16) != 0) wave_lds_sync();
        else asm volatile("" ::: "memory");
    }
    __syncthreads();

    if constexpr ((PROBE & 2) != 0) return;
    // ---- 3. fold into level 0, write dC with its row / column maxima ----
    if constexpr (LEAN) {
        // 4 consecutive level-0 cells of one row per thread (x % 4 == 0): they share one level-2
        // and one level-3 cell and two level-1 cells, so the coarse chain is folded once per
        // shared cell — g2 = c2 + c3 / 4, g1 = c1 + g2 / 4, g0 = c0 + g1 / 4, each "+ coarse *
        // 0.25" only where the finer cell lies in the coarser level's pooled region (corr_pool_bwd)
        const int W1 = W >> 1, W2 = W >> 2, W3 = W >> 3;
        const int PH0 = 2 * (H >> 1), PH1 = 2 * (H >> 2), PH2 = 2 * (H >> 3);  // pooled rows of levels 0..2
        const int PW1 = 2 * (W1 >> 1), PW2 = 2 * (W2 >> 1);                      // pooled columns of levels 1, 2
        const f32x4 *F4 = reinterpret_cast<const f32x4 *>(fsm);
        const f32x2 *F2 = reinterpret_cast<const f32x2 *>(fsm);
        for (int u = tid; u < N / 4; u += NT) {
            const int m = 4 * u, y = m / W, x = m - y * W;
            const int y1 = y >> 1, y2 = y >> 2, y3 = y >> 3, x1 = x >> 1, x2 = x >> 2, x3 = x >> 3;
            // pooled-region flags: level-0 rows (columns always: W even), level-1 cells x1, x1 + 1,
            // the level-2 cell
            const bool p0 = y < PH0;
            const bool p1a = y1 < PH1 && x1 < PW1, p1b = y1 < PH1 && x1 + 1 < PW1;
            const bool p2 = y2 < PH2 && x2 < PW2;
            const int o0 = (o.moff[0] + y * W + x) >> 2, o1 = (o.moff[1] + y1 * W1 + x1) >> 1;
            const int o2 = o.moff[2] + y2 * W2 + x2, o3 = o.moff[3] + y3 * W3 + x3;
#pragma unroll
            for (int k = 0; k < WQ; ++k) {
                if (n0 + k >= NQ) continue;
                const f32x4 c0 = F4[o0 + ((k * o.qstr[0]) >> 2)];
                const f32x2 c1 = F2[o1 + ((k * o.qstr[1]) >> 1)];
                const float c2 = fsm[o2 + k * o.qstr[2]], c3 = fsm[o3 + k * o.qstr[3]];
                const float g2 = p2 ? c2 + c3 * 0.25f : c2;
                const float g1a = p1a ? c1.x + g2 * 0.25f : c1.x, g1b = p1b ? c1.y + g2 * 0.25f : c1.y;
                f32x4 r;
                r.x = p0 ? c0.x + g1a * 0.25f : c0.x;
                r.y = p0 ? c0.y + g1a * 0.25f : c0.y;
                r.z = p0 ? c0.z + g1b * 0.25f : c0.z;
                r.w = p0 ? c0.w + g1b * 0.25f : c0.w;
                f32x4 *dst = reinterpret_cast<f32x4 *>(o.dc + ((size_t)b * NQ + n0 + k) * N + m);
                if constexpr ((PROBE & 8) != 0) *dst = r;
                else __builtin_nontemporal_store(r, dst);
            }
        }
        return;
    }
    float rq[WQ];
#pragma unroll
    for (int k = 0; k < WQ; ++k) rq[k] = 0.f;
    if (W % 4 == 0 && ((uintptr_t)o.dc & 15) == 0 && ((uintptr_t)o.cpart & 15) == 0) {
        // 4 consecutive cells of one row per thread: one 16-B LDS read of level 0, one 8-B read of
        // level 1 (W/2 even, so its 2 cells are 8-B aligned), one value of each coarser level
        // (shared by the 4 cells), one 16-B store of dC
        for (int u = tid; u < N / 4; u += NT) {
            const int m = 4 * u, y = m / W, x = m - y * W;
            int off[kFusedLv];
            unsigned rc = 0;
#pragma unroll
            for (int v = 0; v < kFusedLv; ++v) {
                const int Hv = H >> v, Wv = W >> v, yv = y >> v, xv = x >> v;
                off[v] = o.moff[v < L ? v : 0] + yv * Wv + xv;
                if (v + 1 < L && yv < 2 * (Hv >> 1) && xv < 2 * (Wv >> 1)) rc |= 1u << v;
            }
            float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < WQ; ++k) {
                if (n0 + k >= NQ) continue;
                float lv[kFusedLv][4];
                const float4 t0 = *reinterpret_cast<const float4 *>(fsm + off[0] + k * o.qstr[0]);
                lv[0][0] = t0.x, lv[0][1] = t0.y, lv[0][2] = t0.z, lv[0][3] = t0.w;
                if (L > 1) {
                    const float2 t1 = *reinterpret_cast<const float2 *>(fsm + off[1] + k * o.qstr[1]);
                    lv[1][0] = lv[1][1] = t1.x;
                    lv[1][2] = lv[1][3] = t1.y;
                }
#pragma unroll
                for (int v = 2; v < kFusedLv; ++v)
                    if (v < L) lv[v][0] = lv[v][1] = lv[v][2] = lv[v][3] = fsm[off[v] + k * o.qstr[v]];
                float res[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float up = 0.f;
                    bool have = false;
#pragma unroll
                    for (int v = kFusedLv - 1; v >= 0; --v) {
                        if (v >= L) continue;
                        float gv = lv[v][j];
                        if (have) gv = gv + up * 0.25f;  // fine += coarse * 0.25 (corr_pool_bwd order)
                        up = gv;
                        have = v > 0 && ((rc >> (v - 1)) & 1u);
                    }
                    res[j] = up;
                    const float av = fabsf(up);
                    cm[j] = fmaxf(cm[j], av);
                    rq[k] = fmaxf(rq[k], av);
                }
                // dC streams past the caches (non-temporal): same bits; in back-to-back launches of
                // this kernel alone the upstream gradients then stay cache-resident (T = 12: 153 ->
                // 135 us, profiles/r04q_kbench_bwd_nt.txt); in the training step, where the forward
                // runs in between, neutral (corr_backward 336-337 us)
                f32x4 *dst = reinterpret_cast<f32x4 *>(o.dc + ((size_t)b * NQ + n0 + k) * N + m);
                if constexpr ((PROBE & 8) != 0) *dst = f32x4{res[0], res[1], res[2], res[3]};
                else __builtin_nontemporal_store(f32x4{res[0], res[1], res[2], res[3]}, dst);
            }
            if (o.cpart)
                *reinterpret_cast<float4 *>(o.cpart + ((size_t)b * nqb + (blk - b * nqb)) * N + m) =
                    make_float4(cm[0], cm[1], cm[2], cm[3]);
            else if (o.cmax)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (cm[j] > 0.f) atomicMax(&o.cmax[(size_t)b * N + m + j], __float_as_uint(cm[j]));
        }
    } else {
        for (int m = tid; m < N; m += NT) {
            const int y = m / W, x = m - y * W;
            float cm = 0.f;
            int off[kFusedLv];
            unsigned rc = 0;
#pragma unroll
            for (int v = 0; v < kFusedLv; ++v) {
                const int Hv = H >> v, Wv = W >> v, yv = y >> v, xv = x >> v;
                off[v] = o.moff[v < L ? v : 0] + yv * Wv + xv;
                if (v + 1 < L && yv < 2 * (Hv >> 1) && xv < 2 * (Wv >> 1)) rc |= 1u << v;
            }
#pragma unroll
            for (int k = 0; k < WQ; ++k) {
                if (n0 + k >= NQ) continue;
                float up = 0.f;
                bool have = false;
#pragma unroll
                for (int v = kFusedLv - 1; v >= 0; --v) {
                    if (v >= L) continue;
                    float gv = fsm[off[v] + k * o.qstr[v]];
                    if (have) gv = gv + up * 0.25f;
                    up = gv;
                    have = v > 0 && ((rc >> (v - 1)) & 1u);
                }
                if constexpr ((PROBE & 8) != 0) o.dc[((size_t)b * NQ + n0 + k) * N + m] = up;
                else __builtin_nontemporal_store(up, &o.dc[((size_t)b * NQ + n0 + k) * N + m]);
                const float av = fabsf(up);
                cm = fmaxf(cm, av);
                rq[k] = fmaxf(rq[k], av);
            }
            if (o.cpart)
                o.cpart[((size_t)b * nqb + (blk - b * nqb)) * N + m] = cm;
            else if (o.cmax && cm > 0.f)
                atomicMax(&o.cmax[(size_t)b * N + m], __float_as_uint(cm));
        }
    }
#pragma unroll
    for (int k = 0; k < WQ; ++k) {
        float r = rq[k];
#pragma unroll
        for (int sh = 32; sh >= 1; sh >>= 1) r = fmaxf(r, __shfl_xor(r, sh));
        if (lane == 0 && r > 0.f) atomicMax(&RM[k], __float_as_uint(r));
    }
    __syncthreads();
    if (o.rmax && tid < WQ && n0 + tid < NQ) o.rmax[(size_t)b * NQ + n0 + tid] = RM[tid];
}

// avg_pool2d backward, one level: fine[q][y][x] += coarse[q][y/2][x/2] * 0.25 on the pooled
// region (y < 2*Hc, x < 2*Wc); floor-dropped rows / cols receive nothing.
// Idx: 32-bit cell index whenever the level fits (no 64-bit divisions).
template <typename Idx>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const float *__restrict__ coarse,
                                                       float *__restrict__ fine, long BN, int Hf,
                                                       int Wf) {
    const int Hc = Hf >> 1, Wc = Wf >> 1;
    const int Hr = 2 * Hc, Wr = 2 * Wc;
    const Idx per = (Idx)Hr * Wr;
    const Idx total = (Idx)BN * per;
    for (Idx i = (Idx)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (Idx)gridDim.x * blockDim.x) {
        const size_t qq = i / per;
        const int rem = (int)(i - (Idx)qq * per);
        const int y = rem / Wr, x = rem - y * Wr;
        float *d = fine + qq * Hf * Wf + (size_t)y * Wf + x;
        *d = *d + coarse[qq * Hc * Wc + (size_t)(y >> 1) * Wc + (x >> 1)] * 0.25f;
    }
}

template <int S, int QB>
hipError_t launch_lookup_qb(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H, int W, int L,
                            float *out, hipStream_t s) {
    // TIGHT (only the window rows / 16-B chunks the query's taps touch) pays once the grid is
    // bandwidth-bound, >= 18,000 queries; below that its extents arithmetic sits on the latency
    // chain (same bits; profiles/r05m_kbench_lookup.txt: 1280x960 16.8 -> 16.1 us, B12 36x48
    // 15.9 -> 15.5, MVSEC 36x44 B16 18.6 -> 18.5; DSEC 5.6 -> 6.1, train B8 10.4 -> 10.6)
    const int nqb = (NQ + QB - 1) / QB;
    if ((long)B * NQ >= 18000)
        hipLaunchKernelGGL((lookup_kernel<S, QB, 0, true>), dim3(nqb * B, L), dim3(lookup_threads(S, QB)), 0, s,
                           pyr, coords, B, NQ, H, W, L, out);
    else
        hipLaunchKernelGGL((lookup_kernel<S, QB>), dim3(nqb * B, L), dim3(lookup_threads(S, QB)), 0, s, pyr, coords,
                           B, NQ, H, W, L, out);
    return hipGetLastError();
}

template <int S>
hipError_t launch_lookup_s(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H,
                           int W, int L, float *out, hipStream_t s) {
    // queries per workgroup: 32; 16 for r = 4 on maps of <= 2048 cells with >= 20,000 queries in
    // all, where the smaller workgroups pack the CUs better over several rounds (same bits;
    // tools/kbench_lookup with the non-temporal output stores, profiles/r04t_kbench_lookup_qb2.txt:
    // QB 16 / 32 = MVSEC 36x44 B16 19.0 / 19.6 us, B12 36x48 16.1 / 16.1; train B8 12.0 / 11.7,
    // MVSEC crop 32x32 B16 12.3 / 11.3, DSEC 5.5 / 5.4, 1280x960 22.6 / 22.1; with the tiled
    // pyramid, profiles/r05m_kbench_lookup.txt: MVSEC 18.6 / 19.2, B12 15.9 / 15.7, train 10.3 / 10.2)
    if (S == 9 && H * W <= 2048 && (long)B * NQ >= 20000) return launch_lookup_qb<S, 16>(pyr, coords, B, NQ, H, W, L, out, s);
    return launch_lookup_qb<S, 32>(pyr, coords, B, NQ, H, W, L, out, s);
}

template <int S>
hipError_t launch_lookup_bwd_s(const BwdLookups &lk, int B, int NQ, int H, int W, int L, const LevelPtrs &gpyr,
                               hipStream_t s) {
    const int nqb = (NQ + kBwdQB - 1) / kBwdQB;
    hipLaunchKernelGGL((lookup_bwd_kernel<S, kBwdQB>), dim3(nqb * B, L), dim3(lookup_bwd_threads(S, kBwdQB)), 0, s,
                       lk, B, NQ, H, W, L, gpyr);
    return hipGetLastError();
}

hipError_t launch_lookup_bwd_lk(const BwdLookups &lk, int B, int NQ, int H, int W, int levels, int radius,
                                const LevelPtrs &gpyr, hipStream_t s) {
    switch (radius) {
        case 0: return launch_lookup_bwd_s<1>(lk, B, NQ, H, W, levels, gpyr, s);
        case 1: return launch_lookup_bwd_s<3>(lk, B, NQ, H, W, levels, gpyr, s);
        case 2: return launch_lookup_bwd_s<5>(lk, B, NQ, H, W, levels, gpyr, s);
        case 3: return launch_lookup_bwd_s<7>(lk, B, NQ, H, W, levels, gpyr, s);
        case 4: return launch_lookup_bwd_s<9>(lk, B, NQ, H, W, levels, gpyr, s);
        case 5: return launch_lookup_bwd_s<11>(lk, B, NQ, H, W, levels, gpyr, s);
        case 6: return launch_lookup_bwd_s<13>(lk, B, NQ, H, W, levels, gpyr, s);
        case 7: return launch_lookup_bwd_s<15>(lk, B, NQ, H, W, levels, gpyr, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_lookup(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H,
                         int W, int levels, int radius, float *out, hipStream_t s) {
    switch (radius) {
        case 0: return launch_lookup_s<1>(pyr, coords, B, NQ, H, W, levels, out, s);
        case 1: return launch_lookup_s<3>(pyr, coords, B, NQ, H, W, levels, out, s);
        case 2: return launch_lookup_s<5>(pyr, coords, B, NQ, H, W, levels, out, s);
        case 3: return launch_lookup_s<7>(pyr, coords, B, NQ, H, W, levels, out, s);
        case 4: return launch_lookup_s<9>(pyr, coords, B, NQ, H, W, levels, out, s);
        case 5: return launch_lookup_s<11>(pyr, coords, B, NQ, H, W, levels, out, s);
        case 6: return launch_lookup_s<13>(pyr, coords, B, NQ, H, W, levels, out, s);
        case 7: return launch_lookup_s<15>(pyr, coords, B, NQ, H, W, levels, out, s);
        default: return hipErrorInvalidValue;
    }
}

// Packed weight buffer: the forward's W pieces (kLcFwdU u32x4), then the backward's W^T pieces
// (kCbWtU u32x4).
constexpr size_t kLcWtOff = kLcFwdU * sizeof(u32x4);

size_t lookup_conv_weights_bytes() { return kLcWtOff + kCbWtU * sizeof(u32x4); }

hipError_t launch_lookup_conv_weights(const float *w, int O, int C, void *packed, hipStream_t s) {
    if (O != kLcO || C < 1 || C > kLcKP) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lookup_conv_weights_kernel, dim3(kLcKC, kLcO / 16), dim3(64), 0, s, w, C,
                       static_cast<u32x4 *>(packed));
    hipLaunchKernelGGL(lookup_conv_wt_kernel, dim3(kCbKS, kCbCT, 4), dim3(64), 0, s, w, C,
                       reinterpret_cast<u32x4 *>(static_cast<char *>(packed) + kLcWtOff));
    return hipGetLastError();
}

namespace {
// Query ranges of the dW kernel: >= ~4 blocks per workgroup (each writes a 256 x C partial),
// at most the workgroups that are resident at once (256 CUs x kCbDwWaves / 2 over the levels).
int conv_bwd_ranges(int B, int NQ) {
    const int nb = B * ((NQ + kCbQB - 1) / kCbQB);
    const int r = (nb / 4 + 7) / 8 * 8;
    return std::max(8, std::min(64 * kCbDwWaves / 2, r));
}
}  // namespace

size_t lookup_conv_bwd_workspace(int B, int NQ, int levels) {
    (void)levels;
    const int R = conv_bwd_ranges(B, NQ);
    return (size_t)R * kLcO * (4 * 81 + 1) * sizeof(float);
}

hipError_t launch_lookup_conv_bwd(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H, int W,
                                  int levels, int radius, const void *packed, const float *out, int relu,
                                  const float *grad_out, float *dW, float *db, float *dlk, void *ws, hipStream_t s) {
    if (radius != 4 || levels < 1 || levels > 4) return hipErrorInvalidValue;
    if (!dW && !db && !dlk) return hipSuccess;
    CbArgs a{};
    a.pyr = pyr;
    a.coords = coords;
    a.g = grad_out;
    a.out = out;
    a.wt = reinterpret_cast<const u32x4 *>(static_cast<const char *>(packed) + kLcWtOff);
    a.dlk = dlk;
    a.B = B, a.NQ = NQ, a.H = H, a.W = W, a.L = levels, a.C = levels * 81, a.relu = relu;
    a.R = conv_bwd_ranges(B, NQ);
    a.nqb = (NQ + kCbQB - 1) / kCbQB;
    float *part = static_cast<float *>(ws);
    a.part = dW ? part : nullptr;
    a.bpart = db ? part + (size_t)a.R * kLcO * a.C : nullptr;
    if (dlk) hipLaunchKernelGGL(lookup_conv_bwd_dlk_kernel, dim3(B * a.nqb), dim3(kCbNT), 0, s, a);
    if (dW || db) hipLaunchKernelGGL(lookup_conv_bwd_dw_kernel, dim3(a.R * levels), dim3(kCbNT), 0, s, a);
    if (dW || db) {
        const int n = kLcO * a.C + kLcO;
        hipLaunchKernelGGL(lookup_conv_bwd_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a.part, a.bpart, a.R,
                           a.C, dW, db);
    }
    return hipGetLastError();
}

hipError_t launch_lookup_conv(const ConstLevelPtrs &pyr, const float *coords, int B, int NQ, int H, int W,
                              int levels, int radius, const void *packed, const float *bias, int relu, float *out,
                              hipStream_t s) {
    if (radius != 4 || levels < 1 || levels > 4) return hipErrorInvalidValue;  // E-RAFT: r = 4, L <= 4
    const u32x4 *frag = static_cast<const u32x4 *>(packed);
    const int nqb = (NQ + kLcQB - 1) / kLcQB;
    hipLaunchKernelGGL(lookup_conv_kernel, dim3(nqb * B), dim3(kLcNT), 0, s, pyr, coords, B, NQ, H, W, levels, frag,
                       bias, relu, out);
    return hipGetLastError();
}

hipError_t launch_lookup_bwd(const float *coords, const float *grad_out, int B, int NQ, int H,
                             int W, int levels, int radius, const LevelPtrs &gpyr, hipStream_t s) {
    BwdLookups lk{};
    lk.coords[0] = coords;
    lk.grad[0] = grad_out;
    lk.T = 1;
    lk.zero = 0;
    return launch_lookup_bwd_lk(lk, B, NQ, H, W, levels, radius, gpyr, s);
}

// T lookups in order into a gradient pyramid that this call OVERWRITES (zero-initialised by the
// kernel itself); more than kMaxLookups lookups go in chunks (the later chunks accumulate).
hipError_t launch_lookup_bwd_multi(const float *const *coords, const float *const *grad_out, int T, int B, int NQ,
                                   int H, int W, int levels, int radius, const LevelPtrs &gpyr, hipStream_t s) {
    for (int t0 = 0; t0 < T || t0 == 0; t0 += kMaxLookups) {
        BwdLookups lk{};
        lk.T = std::min(kMaxLookups, T - t0);
        lk.zero = t0 == 0;
        for (int k = 0; k < lk.T; ++k) {
            lk.coords[k] = coords[t0 + k];
            lk.grad[k] = grad_out[t0 + k];
        }
        hipError_t e = launch_lookup_bwd_lk(lk, B, NQ, H, W, levels, radius, gpyr, s);
        if (e != hipSuccess) return e;
        if (T == 0) break;
    }
    return hipSuccess;
}

hipError_t launch_pool_bwd(const LevelPtrs &gpyr, long BN, int H, int W, int levels,
                           hipStream_t s) {
    for (int l = levels - 1; l >= 1; --l) {
        const int Hf = H >> (l - 1), Wf = W >> (l - 1);
        const size_t total = (size_t)BN * (2 * (Hf >> 1)) * (2 * (Wf >> 1));
        if (total == 0) continue;
        const int grid = (int)((total + 255) / 256 < 32768 ? (total + 255) / 256 : 32768);
        if (total + (size_t)grid * 256 < (1ull << 32))
            hipLaunchKernelGGL(pool_bwd_kernel<unsigned>, dim3(grid), dim3(256), 0, s, gpyr.p[l], gpyr.p[l - 1],
                               BN, Hf, Wf);
        else
            hipLaunchKernelGGL(pool_bwd_kernel<size_t>, dim3(grid), dim3(256), 0, s, gpyr.p[l], gpyr.p[l - 1],
                               BN, Hf, Wf);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// corr_backward's fused path: hipErrorNotSupported when the workgroup's LDS image (BQ queries'
// maps at every level + per-wave staging) exceeds 160 KiB, or levels > 4, or T > kMaxLookups —
// the caller then takes the staged path.
namespace {
template <int S, bool SEP = false>
size_t fused_lds_bytes(int H, int W, int levels, FusedOut *o) {
    using ST = FusedStage<S>;
    // query stride = map cells plus one guard row, rounded up to an ODD multiple of 64 / BQ
    // floats: the BQ queries' maps then start in BQ different LDS banks (q * stride mod 64), so a
    // wave's read-modify-writes of neighbouring queries' windows (whose anchors differ by about
    // one pixel) do not collide.  Every map has a guard row above (row -1) and below (row H_l),
    // which the closed form's clamped rows write (one row may serve as one map's row H_l and the
    // next map's row -1); a level's region is a leading guard row and BQ query strides, rounded
    // to 4 floats (16-B zeroing; the fold's 16-B / 8-B reads of levels 0 / 1).  The per-wave
    // staging follows unless the kernel has none (fold_no_staging).
    size_t maps = 0;
    const int stag = 64 / ST::BQ;
    for (int l = 0; l < kFusedLv; ++l) {
        const int Hl = H >> l, Wl = W >> l;
        const int msz = l < levels ? Hl * Wl : 0;
        int qs = 0;
        if (msz) {
            qs = ((Hl + 1) * Wl + stag - 1) / stag * stag;
            if (ST::BQ > 1 && ((qs / stag) & 1) == 0) qs += stag;
        }
        if (o) o->moff[l] = (int)maps + (msz ? Wl : 0), o->msz[l] = msz, o->qstr[l] = qs;
        if (msz) maps += ((size_t)Wl + (size_t)ST::BQ * qs + 3) / 4 * 4;
    }
    if (o) o->aux = (int)maps;
    return (maps + (fold_no_staging<S, SEP>() ? 0 : (size_t)kFusedLv * ST::SIZE) + ST::BQ) * 4;
}

template <int S, bool SEP = false>
hipError_t launch_fused_s(const BwdLookups &lk, FusedOut o, hipStream_t s) {
    const size_t bytes = fused_lds_bytes<S, SEP>(o.H, o.W, o.L, &o);
    // the dynamic-LDS limit is raised once per device to the largest image this path accepts
    // (not to this call's size: a later, larger shape must not run against a smaller limit),
    // capped at what the device offers per workgroup
    int dev = 0, dev_max = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&dev_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
    if (e != hipSuccess) return e;
    const int limit = std::min(160 * 1024, dev_max);
    if (bytes > (size_t)limit) return hipErrorNotSupported;
    // the lean fold (no maxima, 4 levels, 16-B rows of dC): the bf16x6 backward at radius 4
    const bool lean = S == 9 && !o.rmax && !o.cmax && !o.cpart && o.L == kFusedLv && o.W % 4 == 0 &&
                      ((uintptr_t)o.dc & 15) == 0;
    const void *fn = lean ? (const void *)lookup_bwd_fold_kernel<S, 0, SEP, S == 9>
                          : (const void *)lookup_bwd_fold_kernel<S, 0, SEP>;
    static std::atomic<unsigned long long> done[2];
    e = ensure_lds_limit(fn, limit, done[lean]);
    if (e != hipSuccess) return e;
    constexpr int WQ = FusedStage<S>::BQ, WAVES = kFusedLv;
    const int nqb = (o.NQ + WQ - 1) / WQ;
    o.nfold = nqb * o.B;
    // row-maxima blocks: at most half a round of workgroup slots (the fold's tail), >= 1 row per wave
    int extra = 0;
    if (o.rm.rows > 0) {
        const long rows = 2L * o.B * o.rm.rows;
        const long cap = std::max(1L, (long)(256 * std::max<size_t>(1, 160 * 1024 / bytes)) / 2);
        o.rm_rows_per_wave = (int)std::max(1L, (rows + cap * WAVES - 1) / (cap * WAVES));
        extra = (int)((rows + (long)o.rm_rows_per_wave * WAVES - 1) / ((long)o.rm_rows_per_wave * WAVES));
    }
    if (lean)
        hipLaunchKernelGGL((lookup_bwd_fold_kernel<S, 0, SEP, S == 9>), dim3((unsigned)(o.nfold + extra)),
                           dim3(64 * WAVES), bytes, s, lk, o);
    else
        hipLaunchKernelGGL((lookup_bwd_fold_kernel<S, 0, SEP>), dim3((unsigned)(o.nfold + extra)), dim3(64 * WAVES),
                           bytes, s, lk, o);
    return hipGetLastError();
}
}  // namespace

int lookup_bwd_fold_groups(int NQ, int radius) {
    if (radius < 0 || radius > 7) return 0;
    const int bq = 64 / fused_slots(2 * radius + 1);
    return (NQ + bq - 1) / bq;
}

hipError_t launch_lookup_bwd_fold(const float *const *coords, const float *const *grad_out, int T, int B, int NQ,
                                  int H, int W, int levels, int radius, float *dc, unsigned *rmax, unsigned *cmax,
                                  float *cpart, hipStream_t s, const FoldRowMax &rm, bool exact) {
    if (T < 1 || T > kMaxLookups || levels < 1 || levels > kFusedLv) return hipErrorNotSupported;
    BwdLookups lk{};
    lk.T = T;
    for (int k = 0; k < T; ++k) {
        lk.coords[k] = coords[k];
        lk.grad[k] = grad_out[k];
    }
    FusedOut o{};
    o.dc = dc, o.rmax = rmax, o.cmax = cmax, o.cpart = cpart;
    o.B = B, o.NQ = NQ, o.H = H, o.W = W, o.L = levels;
    o.rm = rm;
    switch (radius) {
        case 0: return launch_fused_s<1>(lk, o, s);
        case 1: return launch_fused_s<3>(lk, o, s);
        case 2: return launch_fused_s<5>(lk, o, s);
        case 3: return launch_fused_s<7>(lk, o, s);
        // the separable closed form is instantiated for E-RAFT's radius only
        case 4: return exact ? launch_fused_s<9, false>(lk, o, s) : launch_fused_s<9, true>(lk, o, s);
        case 5: return launch_fused_s<11>(lk, o, s);
        case 6: return launch_fused_s<13>(lk, o, s);
        case 7: return launch_fused_s<15>(lk, o, s);
        default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------------------------------
// Tiled pyramid (corr_common.h) <-> the reference's row-major [BN][H_l][W_l]: EXPORT
// materialises corr_pyramid's view (corr.py:16,24,27,36 read it as [B*N, 1, H_l, W_l]); IMPORT
// installs a pyramid given in that layout (padding cells zeroed).  One thread per 16-B tile row.
// ---------------------------------------------------------------------------------------
namespace {
template <bool EXPORT>
__global__ __launch_bounds__(256) void pyramid_layout_kernel(const float *__restrict__ src, float *__restrict__ dst,
                                                             long BN, int Hl, int Wl) {
    const int TC = map_tcols(Wl);
    const long per = (long)map_floats(Hl, Wl) / 4;  // 16-B chunks per map
    const long total = BN * per;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long n = i / per;
        const int rem = (int)(i - n * per);
        const int t = rem / kTileW, cq = rem % kTileW;  // tile, chunk in the tile (kTileW / 4 per row)
        const int Y = 4 * (t / TC) + cq / (kTileW / 4), X = kTileW * (t % TC) + 4 * (cq % (kTileW / 4));
        const size_t row = ((size_t)n * Hl + Y) * Wl;
        if (EXPORT) {
            if (Y >= Hl) continue;
            const f32x4 v = reinterpret_cast<const f32x4 *>(src)[i];
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (X + c < Wl) dst[row + X + c] = v[c];
        } else {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (Y < Hl && X + c < Wl) v[c] = src[row + X + c];
            reinterpret_cast<f32x4 *>(dst)[i] = v;
        }
    }
}

template <bool EXPORT>
hipError_t launch_pyramid_layout(const ConstLevelPtrs &src, long BN, int H, int W, int levels, const LevelPtrs &dst,
                                 hipStream_t s) {
    for (int l = 0; l < levels; ++l) {
        const int Hl = H >> l, Wl = W >> l;
        const long rows = BN * (long)(map_floats(Hl, Wl) / 4);
        const int grid = (int)std::min<long>((rows + 255) / 256, 8192);
        hipLaunchKernelGGL((pyramid_layout_kernel<EXPORT>), dim3(grid), dim3(256), 0, s, src.p[l], dst.p[l], BN, Hl,
                           Wl);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
}  // namespace

hipError_t launch_pyramid_export(const ConstLevelPtrs &pyr, long BN, int H, int W, int levels, const LevelPtrs &out,
                                 hipStream_t s) {
    return launch_pyramid_layout<true>(pyr, BN, H, W, levels, out, s);
}

hipError_t launch_pyramid_import(const ConstLevelPtrs &src, long BN, int H, int W, int levels, const LevelPtrs &pyr,
                                 hipStream_t s) {
    return launch_pyramid_layout<false>(src, BN, H, W, levels, pyr, s);
}

}  // namespace corr

