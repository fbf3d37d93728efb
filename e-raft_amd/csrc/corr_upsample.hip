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

}  // namespace

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
