// corr_lookup.hip — (2r+1)^2 bilinear window lookup and its input-gradient on gfx950.
//
// Forward replaces CorrBlock.__call__ (model/corr.py:29-50) + bilinear_sampler
// (model/utils.py:7-21, F.grid_sample(align_corners=True), zero padding).  The ~12 ATen ops
// per level, the per-call CPU->GPU offset copies (corr.py:37-39), the cat and the
// permute().contiguous() (corr.py:49-50) become ONE launch that writes the NCHW output
// directly.
//
// Layout of the work: a workgroup owns 64 consecutive query pixels of one batch item at one
// pyramid level.
//   1. per query and axis: the 2r+1 tap coordinates, exactly as the reference rounds them
//      (x/2^l + (t - r) -> 2X/(W_l-1) - 1 -> ((x'+1)/2)(W_l-1); fp32, one rounding per op),
//      their floor and the two 1-D weights -> LDS;
//   2. the (2r+3)^2 neighbourhood of every query (anchored at its first tap's floor, zero
//      outside the map) is gathered from HBM with lanes running along the rows -> LDS;
//   3. lane = query, 4 waves split the taps: 4 corner reads from LDS, fmaf in the order
//      nw, ne, sw, se (bit-identical to ATen's CPU grid_sampler_2d) and a coalesced store of
//      out[b][l*K + tap][n] for 64 consecutive n.
// A corner that lands outside the LDS neighbourhood (only possible under large-magnitude
// rounding) is read from global memory instead, so semantics never depend on the window.
//
// Backward (autograd of utils.py:15 w.r.t. the pyramid; coords are detached at
// eraft.py:128): one wave per 64 queries x level; each lane scatters its query's taps into a
// zeroed LDS neighbourhood in a fixed order (taps row-major, corners nw, ne, sw, se), then
// the neighbourhood is added to the gradient pyramid.  A query's contributions never leave
// its own map, so no atomics are needed and results are deterministic.
#include <cmath>

#include "corr_common.h"

namespace corr {
namespace {

constexpr int kQB = 64;  // queries per workgroup

// Sentinel anchor for NaN / huge coordinates: every window cell is outside the map.
constexpr int kFarAnchor = -(1 << 28);

struct Axis {
    float f;   // floor(ix) as float (may be NaN / huge)
    float lo;  // (f + 1) - ix  : weight of corner f
    float hi;  // ix - f        : weight of corner f + 1
};

__device__ __forceinline__ Axis tap_axis(float c, float inv_scale, int t, int r, int size) {
    // corr.py:41  centroid = coords / 2**l   (exact: power-of-two scale)
    // corr.py:43  + delta (integer offsets from linspace(-r, r, 2r+1))
    // utils.py:11 2*x/(W-1) - 1 ; grid_sample unnormalise ((x'+1)/2)*(W-1)
    const float cl = c * inv_scale;
    const float X = cl + (float)(t - r);
    const float den = (float)(size - 1);
    const float xn = __fsub_rn(__fdiv_rn(2.0f * X, den), 1.0f);
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

template <int S>
struct LookupSmem {
    static constexpr int WIN = S + 2;
    static constexpr int WS = WIN * WIN;
    static constexpr int WSTR = WS | 1;  // odd stride: conflict-free lane = query reads
    float win[kQB * WSTR];
    float tx[3][S][kQB];
    float ty[3][S][kQB];
    int ax[kQB], ay[kQB];
};

template <int S>
__global__ __launch_bounds__(256) void lookup_kernel(ConstLevelPtrs pyr, const float *__restrict__ coords,
                                                     int B, int H, int W, int L,
                                                     float *__restrict__ out) {
    constexpr int R = (S - 1) / 2, K = S * S;
    using SM = LookupSmem<S>;
    constexpr int WIN = SM::WIN, WS = SM::WS, WSTR = SM::WSTR;
    __shared__ SM sm;

    const int N = H * W;
    const int nqb = (N + kQB - 1) / kQB;
    const int b = blockIdx.x / nqb;
    const int n0 = (blockIdx.x - b * nqb) * kQB;
    const int l = blockIdx.y;
    const int Hl = H >> l, Wl = W >> l;
    const float inv_scale = 1.0f / (float)(1 << l);
    const float *P = pyr.p[l];
    const size_t mapsz = (size_t)Hl * Wl;

    const int tid = threadIdx.x;
    const int q = tid & (kQB - 1);
    const int role = tid >> 6;  // 0,1: x taps; 2,3: y taps
    const int n = n0 + q;
    const bool qok = n < N;

    // ---- 1. tap coordinates ----
    {
        const int axis = role >> 1;
        const float c = qok ? coords[((size_t)b * 2 + axis) * N + n] : 0.0f;
        const int size = axis ? Hl : Wl;
        constexpr int half = (S + 1) / 2;
        const int t0 = (role & 1) ? half : 0, t1 = (role & 1) ? S : half;
        for (int t = t0; t < t1; ++t) {
            const Axis a = tap_axis(c, inv_scale, t, R, size);
            if (axis == 0) {
                sm.tx[0][t][q] = a.f;
                sm.tx[1][t][q] = a.lo;
                sm.tx[2][t][q] = a.hi;
                if (t == 0) sm.ax[q] = anchor_of(a.f);
            } else {
                sm.ty[0][t][q] = a.f;
                sm.ty[1][t][q] = a.lo;
                sm.ty[2][t][q] = a.hi;
                if (t == 0) sm.ay[q] = anchor_of(a.f);
            }
        }
    }
    __syncthreads();

    // ---- 2. gather every query's neighbourhood (zero outside the map) ----
    const size_t qbase = (size_t)b * N + n0;
    for (int g = tid; g < kQB * WS; g += 256) {
        const int qq = g / WS;
        const int e = g - qq * WS;
        const int ry = e / WIN, rx = e - ry * WIN;
        float v = 0.0f;
        if (n0 + qq < N) {
            const int Y = sm.ay[qq] + ry, X = sm.ax[qq] + rx;
            if (X >= 0 && X < Wl && Y >= 0 && Y < Hl) v = P[(qbase + qq) * mapsz + (size_t)Y * Wl + X];
        }
        sm.win[qq * WSTR + e] = v;
    }
    __syncthreads();

    // ---- 3. lane = query; the 4 waves split the K taps ----
    const int ax = sm.ax[q], ay = sm.ay[q];
    const float *wq = &sm.win[q * WSTR];
    const float *Pq = P + (qbase + q) * mapsz;
    auto fetch = [&](float xf, float yf) -> float {
        if (!in_map(xf, yf, Wl, Hl)) return 0.0f;
        const int xi = (int)xf, yi = (int)yf;
        const unsigned cx = (unsigned)(xi - ax), cy = (unsigned)(yi - ay);
        if (cx < (unsigned)WIN && cy < (unsigned)WIN) return wq[cy * WIN + cx];
        return Pq[(size_t)yi * Wl + xi];
    };
    constexpr int KP = (K + 3) / 4;
    const int k0 = role * KP, k1 = (k0 + KP < K) ? k0 + KP : K;
    float *o = out + ((size_t)b * L + l) * K * N + n;
    for (int k = k0; k < k1; ++k) {
        const int i = k / S, j = k - (k / S) * S;
        const float x0 = sm.tx[0][i][q], ex = sm.tx[1][i][q], wx = sm.tx[2][i][q];
        const float y0 = sm.ty[0][j][q], ey = sm.ty[1][j][q], ny = sm.ty[2][j][q];
        const float x1 = __fadd_rn(x0, 1.0f), y1 = __fadd_rn(y0, 1.0f);
        const float vnw = fetch(x0, y0), vne = fetch(x1, y0);
        const float vsw = fetch(x0, y1), vse = fetch(x1, y1);
        float acc = __fmul_rn(vnw, __fmul_rn(ey, ex));
        acc = __builtin_fmaf(vne, __fmul_rn(ey, wx), acc);
        acc = __builtin_fmaf(vsw, __fmul_rn(ny, ex), acc);
        acc = __builtin_fmaf(vse, __fmul_rn(ny, wx), acc);
        if (qok) o[(size_t)k * N] = acc;
    }
}

template <int S>
struct LookupBwdSmem {
    static constexpr int WIN = S + 2;
    static constexpr int WS = WIN * WIN;
    static constexpr int WSTR = WS | 1;
    float win[kQB * WSTR];
    int ax[kQB], ay[kQB];
};

template <int S>
__global__ __launch_bounds__(64) void lookup_bwd_kernel(const float *__restrict__ coords,
                                                        const float *__restrict__ grad_out, int B,
                                                        int H, int W, int L, LevelPtrs gpyr) {
    constexpr int R = (S - 1) / 2, K = S * S;
    using SM = LookupBwdSmem<S>;
    constexpr int WIN = SM::WIN, WS = SM::WS, WSTR = SM::WSTR;
    __shared__ SM sm;

    const int N = H * W;
    const int nqb = (N + kQB - 1) / kQB;
    const int b = blockIdx.x / nqb;
    const int n0 = (blockIdx.x - b * nqb) * kQB;
    const int l = blockIdx.y;
    const int Hl = H >> l, Wl = W >> l;
    const float inv_scale = 1.0f / (float)(1 << l);
    float *G = gpyr.p[l];
    const size_t mapsz = (size_t)Hl * Wl;
    const size_t qbase = (size_t)b * N + n0;

    const int q = threadIdx.x;
    const int n = n0 + q;
    const bool qok = n < N;
    const float cx = qok ? coords[((size_t)b * 2 + 0) * N + n] : 0.0f;
    const float cy = qok ? coords[((size_t)b * 2 + 1) * N + n] : 0.0f;

    Axis tx[S], ty[S];
#pragma unroll
    for (int t = 0; t < S; ++t) {
        tx[t] = tap_axis(cx, inv_scale, t, R, Wl);
        ty[t] = tap_axis(cy, inv_scale, t, R, Hl);
    }
    const int ax = anchor_of(tx[0].f), ay = anchor_of(ty[0].f);
    sm.ax[q] = ax;
    sm.ay[q] = ay;
    for (int g = q; g < kQB * WSTR; g += 64) sm.win[g] = 0.0f;
    __syncthreads();

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
    if (qok) {
        const float *g = grad_out + ((size_t)b * L + l) * K * N + n;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const float x0 = tx[i].f, x1 = __fadd_rn(tx[i].f, 1.0f);
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const float gv = g[(size_t)(i * S + j) * N];
                const float y0 = ty[j].f, y1 = __fadd_rn(ty[j].f, 1.0f);
                scatter(x0, y0, __fmul_rn(gv, __fmul_rn(ty[j].lo, tx[i].lo)));
                scatter(x1, y0, __fmul_rn(gv, __fmul_rn(ty[j].lo, tx[i].hi)));
                scatter(x0, y1, __fmul_rn(gv, __fmul_rn(ty[j].hi, tx[i].lo)));
                scatter(x1, y1, __fmul_rn(gv, __fmul_rn(ty[j].hi, tx[i].hi)));
            }
        }
    }
    __syncthreads();

    // add the neighbourhoods to the gradient pyramid (lanes along window rows)
    for (int g = q; g < kQB * WS; g += 64) {
        const int qq = g / WS;
        const int e = g - qq * WS;
        if (n0 + qq >= N) continue;
        const int ry = e / WIN, rx = e - ry * WIN;
        const int Y = sm.ay[qq] + ry, X = sm.ax[qq] + rx;
        if (X >= 0 && X < Wl && Y >= 0 && Y < Hl) {
            float *dst = G + (qbase + qq) * mapsz + (size_t)Y * Wl + X;
            *dst = *dst + sm.win[qq * WSTR + e];
        }
    }
}

// avg_pool2d backward, one level: fine[q][y][x] += coarse[q][y/2][x/2] * 0.25 on the pooled
// region (y < 2*Hc, x < 2*Wc); floor-dropped rows / cols receive nothing.
__global__ __launch_bounds__(256) void pool_bwd_kernel(const float *__restrict__ coarse,
                                                       float *__restrict__ fine, long BN, int Hf,
                                                       int Wf) {
    const int Hc = Hf >> 1, Wc = Wf >> 1;
    const int Hr = 2 * Hc, Wr = 2 * Wc;
    const size_t per = (size_t)Hr * Wr;
    const size_t total = (size_t)BN * per;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const size_t qq = i / per;
        const int rem = (int)(i - qq * per);
        const int y = rem / Wr, x = rem - y * Wr;
        float *d = fine + qq * Hf * Wf + (size_t)y * Wf + x;
        *d = *d + coarse[qq * Hc * Wc + (size_t)(y >> 1) * Wc + (x >> 1)] * 0.25f;
    }
}

template <int S>
hipError_t launch_lookup_s(const ConstLevelPtrs &pyr, const float *coords, int B, int H, int W,
                           int L, float *out, hipStream_t s) {
    const int nqb = (H * W + kQB - 1) / kQB;
    hipLaunchKernelGGL(lookup_kernel<S>, dim3(nqb * B, L), dim3(256), 0, s, pyr, coords, B, H, W,
                       L, out);
    return hipGetLastError();
}

template <int S>
hipError_t launch_lookup_bwd_s(const float *coords, const float *grad_out, int B, int H, int W,
                               int L, const LevelPtrs &gpyr, hipStream_t s) {
    const int nqb = (H * W + kQB - 1) / kQB;
    hipLaunchKernelGGL(lookup_bwd_kernel<S>, dim3(nqb * B, L), dim3(64), 0, s, coords, grad_out,
                       B, H, W, L, gpyr);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_lookup(const ConstLevelPtrs &pyr, const float *coords, int B, int H, int W,
                         int levels, int radius, float *out, hipStream_t s) {
    switch (radius) {
        case 0: return launch_lookup_s<1>(pyr, coords, B, H, W, levels, out, s);
        case 1: return launch_lookup_s<3>(pyr, coords, B, H, W, levels, out, s);
        case 2: return launch_lookup_s<5>(pyr, coords, B, H, W, levels, out, s);
        case 3: return launch_lookup_s<7>(pyr, coords, B, H, W, levels, out, s);
        case 4: return launch_lookup_s<9>(pyr, coords, B, H, W, levels, out, s);
        case 5: return launch_lookup_s<11>(pyr, coords, B, H, W, levels, out, s);
        case 6: return launch_lookup_s<13>(pyr, coords, B, H, W, levels, out, s);
        case 7: return launch_lookup_s<15>(pyr, coords, B, H, W, levels, out, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_lookup_bwd(const float *coords, const float *grad_out, int B, int H, int W,
                             int levels, int radius, const LevelPtrs &gpyr, hipStream_t s) {
    switch (radius) {
        case 0: return launch_lookup_bwd_s<1>(coords, grad_out, B, H, W, levels, gpyr, s);
        case 1: return launch_lookup_bwd_s<3>(coords, grad_out, B, H, W, levels, gpyr, s);
        case 2: return launch_lookup_bwd_s<5>(coords, grad_out, B, H, W, levels, gpyr, s);
        case 3: return launch_lookup_bwd_s<7>(coords, grad_out, B, H, W, levels, gpyr, s);
        case 4: return launch_lookup_bwd_s<9>(coords, grad_out, B, H, W, levels, gpyr, s);
        case 5: return launch_lookup_bwd_s<11>(coords, grad_out, B, H, W, levels, gpyr, s);
        case 6: return launch_lookup_bwd_s<13>(coords, grad_out, B, H, W, levels, gpyr, s);
        case 7: return launch_lookup_bwd_s<15>(coords, grad_out, B, H, W, levels, gpyr, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_pool_bwd(const LevelPtrs &gpyr, long BN, int H, int W, int levels,
                           hipStream_t s) {
    for (int l = levels - 1; l >= 1; --l) {
        const int Hf = H >> (l - 1), Wf = W >> (l - 1);
        const size_t total = (size_t)BN * (2 * (Hf >> 1)) * (2 * (Wf >> 1));
        if (total == 0) continue;
        const int grid = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
        hipLaunchKernelGGL(pool_bwd_kernel, dim3(grid), dim3(256), 0, s, gpyr.p[l], gpyr.p[l - 1], BN,
                           Hf, Wf);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace corr
