// corr_upsample.hip — E-RAFT's convex upsampling of the 1/8-resolution flow, run after every
// GRU iteration (model/eraft.py:75-86 upsample_flow, called at :142):
//
//   mask  [N, 9*8*8, h, w] -> softmax over the 9 taps (dim 2 of view(N, 1, 9, 8, 8, h, w))
//   up    = unfold(8 * flow, 3x3, padding 1)            [N, 2, 9, 1, 1, h, w]
//   out[n, c, 8y + i, 8x + j] = sum_k softmax_k(mask[n, 64k + 8i + j, y, x]) * up[n, c, k, y, x]
//
// The reference runs softmax, unfold, a broadcast multiply, a sum and a permute+reshape copy
// (six launches, the 576-channel mask read twice and a 9x-expanded product materialised).
// Here one thread per output sub-pixel (n, y, i, x, j), j fastest: consecutive threads write
// consecutive floats of an output row; each thread reads its 9 mask logits once, the 3x3
// flow neighbourhood from L1/L2, and writes both flow channels.  fp32 throughout; the sum over
// taps runs in tap order k = 0..8 (the reference's reduction order is ATen's, so parity is
// tolerance-based: tests/test_gpu_parity.py).
#include <algorithm>
#include <cmath>

#include "corr_common.h"

namespace corr {
namespace {

__global__ __launch_bounds__(256) void convex_upsample_kernel(const float *__restrict__ flow,
                                                              const float *__restrict__ mask, int N, int h,
                                                              int w, float *__restrict__ out) {
    const size_t total = (size_t)N * h * 8 * w * 8;
    const size_t plane = (size_t)h * w;
    for (size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (size_t)gridDim.x * blockDim.x) {
        const int j = (int)(id & 7);
        size_t r = id >> 3;
        const int x = (int)(r % w);
        r /= w;
        const int i = (int)(r & 7);
        r >>= 3;
        const int y = (int)(r % h);
        const int n = (int)(r / h);
        const float *m = mask + ((size_t)n * 576 + 8 * i + j) * plane + (size_t)y * w + x;
        float lg[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) lg[k] = m[(size_t)k * 64 * plane];
        float mx = lg[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) mx = fmaxf(mx, lg[k]);
        float e[9], s = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            e[k] = expf(lg[k] - mx);
            s += e[k];
        }
        const float *f0 = flow + (size_t)n * 2 * plane, *f1 = f0 + plane;
        float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
            const bool in = yy >= 0 && yy < h && xx >= 0 && xx < w;
            const size_t o = in ? (size_t)yy * w + xx : 0;
            const float p = e[k] / s;
            const float u0 = in ? 8.0f * f0[o] : 0.0f, u1 = in ? 8.0f * f1[o] : 0.0f;
            a0 += p * u0;
            a1 += p * u1;
        }
        const size_t W8 = (size_t)8 * w, H8 = (size_t)8 * h;
        const size_t o = ((size_t)n * 2 * H8 + 8 * y + i) * W8 + 8 * x + j;
        out[o] = a0;
        out[o + H8 * W8] = a1;
    }
}

// Backward of the above (autograd of eraft.py:75-86 w.r.t. flow and mask), in two passes.
//   p_k = softmax_k(mask[n, 64k + 8i + j, y, x]),  G_c = dout[n, c, 8y + i, 8x + j]
//   u_kc = 8 flow[n, c, y + dy_k, x + dx_k] (0 outside),  dv_k = G_0 u_k0 + G_1 u_k1
//   dmask[n, 64k + 8i + j, y, x] = p_k (dv_k - sum_k' p_k' dv_k')        (softmax backward)
//   dflow[n, c, y', x'] = 8 sum over (y, x, k) with (y + dy_k, x + dx_k) = (y', x') of
//                         S_kc(y, x),  S_kc(y, x) = sum_{i,j} p_k G_c
// Pass 1: a workgroup = 8 waves over 64 consecutive coarse pixels x of one row y; wave w owns
// sub-pixel row i = w, lane = x, and walks j = 0..7 (mask logits and dmask coalesced along x);
// each lane keeps its 18 partial S in registers and the 8 waves add theirs through LDS (in
// wave order i = 0..7), then S goes to the workspace [n][2][9][h][w].  Pass 2: dflow by
// gathering the 9 S planes at the shifted positions, tap order k = 0..8.
constexpr int kUpWaves = 8;

__global__ __launch_bounds__(64 * kUpWaves) void convex_upsample_bwd_kernel(const float *__restrict__ flow,
                                                                         const float *__restrict__ mask,
                                                                         const float *__restrict__ dout, int h,
                                                                         int w, float *__restrict__ dmask,
                                                                         float *__restrict__ S) {
    __shared__ float red[kUpWaves][18][64];
    const int nxb = (w + 63) / 64;
    const int xb = blockIdx.x % nxb, y = (blockIdx.x / nxb) % h, n = blockIdx.x / (nxb * h);
    const int lane = threadIdx.x & 63, i = threadIdx.x >> 6;
    const int x = xb * 64 + lane;
    const bool ok = x < w;
    const int xc = ok ? x : w - 1;
    const size_t plane = (size_t)h * w;
    const float *f0 = flow + (size_t)n * 2 * plane, *f1 = f0 + plane;
    float u0[9], u1[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int yy = y + k / 3 - 1, xx = xc + k % 3 - 1;
        const bool in = yy >= 0 && yy < h && xx >= 0 && xx < w;
        const size_t o = in ? (size_t)yy * w + xx : 0;
        u0[k] = in ? 8.0f * f0[o] : 0.0f;
        u1[k] = in ? 8.0f * f1[o] : 0.0f;
    }
    float s0[9], s1[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) s0[k] = s1[k] = 0.0f;
    const size_t W8 = (size_t)8 * w, H8 = (size_t)8 * h;
    for (int j = 0; j < 8; ++j) {
        const size_t mo = ((size_t)n * 576 + 8 * i + j) * plane + (size_t)y * w + xc;
        float lg[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) lg[k] = mask[mo + (size_t)k * 64 * plane];
        float mx = lg[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) mx = fmaxf(mx, lg[k]);
        float e[9], sum = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            e[k] = expf(lg[k] - mx);
            sum += e[k];
        }
        const size_t go = ((size_t)n * 2 * H8 + 8 * y + i) * W8 + 8 * (size_t)xc + j;
        const float g0 = ok ? dout[go] : 0.0f, g1 = ok ? dout[go + H8 * W8] : 0.0f;
        float p[9], dv[9], pdv = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            p[k] = e[k] / sum;
            dv[k] = g0 * u0[k] + g1 * u1[k];
            pdv += p[k] * dv[k];
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            if (ok) dmask[mo + (size_t)k * 64 * plane] = p[k] * (dv[k] - pdv);
            s0[k] += p[k] * g0;
            s1[k] += p[k] * g1;
        }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        red[i][k][lane] = s0[k];
        red[i][9 + k][lane] = s1[k];
    }
    __syncthreads();
    // 18 planes x 64 lanes, summed over the 8 waves in order; wave t reduces planes t, t + 8, ...
    for (int q = i; q < 18; q += kUpWaves) {
        float a = 0.0f;
#pragma unroll
        for (int v = 0; v < kUpWaves; ++v) a += red[v][q][lane];
        const int c = q / 9, k = q - 9 * c;
        if (ok) S[(((size_t)n * 2 + c) * 9 + k) * plane + (size_t)y * w + x] = a;
    }
}

__global__ __launch_bounds__(256) void convex_upsample_bwd_flow_kernel(const float *__restrict__ S, int N, int h,
                                                                       int w, float *__restrict__ dflow) {
    const size_t plane = (size_t)h * w, total = (size_t)N * 2 * plane;
    for (size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (size_t)gridDim.x * blockDim.x) {
        const size_t nc = id / plane;
        const int r = (int)(id - nc * plane), yp = r / w, xp = r - yp * w;
        const float *Sc = S + nc * 9 * plane;
        float a = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int yy = yp - (k / 3 - 1), xx = xp - (k % 3 - 1);  // the coarse pixel whose tap k is (yp, xp)
            if (yy >= 0 && yy < h && xx >= 0 && xx < w) a += Sc[(size_t)k * plane + (size_t)yy * w + xx];
        }
        dflow[id] = 8.0f * a;
    }
}

}  // namespace

size_t convex_upsample_bwd_workspace(int N, int h, int w) { return (size_t)N * 2 * 9 * h * w * sizeof(float); }

hipError_t launch_convex_upsample_bwd(const float *flow, const float *mask, const float *dout, int N, int h, int w,
                                      float *dflow, float *dmask, void *ws, hipStream_t s) {
    if ((size_t)N * h * w == 0) return hipSuccess;
    float *S = static_cast<float *>(ws);
    const unsigned blocks = (unsigned)((size_t)N * h * ((w + 63) / 64));
    hipLaunchKernelGGL(convex_upsample_bwd_kernel, dim3(blocks), dim3(64 * kUpWaves), 0, s, flow, mask, dout, h, w,
                       dmask, S);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t total = (size_t)N * 2 * h * w;
    const int grid = (int)std::min<size_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(convex_upsample_bwd_flow_kernel, dim3(grid), dim3(256), 0, s, S, N, h, w, dflow);
    return hipGetLastError();
}

hipError_t launch_convex_upsample(const float *flow, const float *mask, int N, int h, int w, float *out,
                                  hipStream_t s) {
    const size_t total = (size_t)N * h * 8 * w * 8;
    if (total == 0) return hipSuccess;
    const size_t blocks = (total + 255) / 256;
    const int grid = (int)(blocks < 65536 ? blocks : 65536);
    hipLaunchKernelGGL(convex_upsample_kernel, dim3(grid), dim3(256), 0, s, flow, mask, N, h, w, out);
    return hipGetLastError();
}

}  // namespace corr
