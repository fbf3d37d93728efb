// corr_splat.hip — the warm-start forward splat between consecutive frame pairs
// (utils/image_utils.py:52-83 forward_interpolate_pytorch + :10-50 grid_sample_values; called
// by the warm-start evaluation, test.py:209, to seed flow_init of the next pair).
//
// Every source pixel p moves to (x, y) = (x0 + dx, y0 + dy) and is splatted onto its four
// floor / ceil neighbours with weight w = (1 - |x - x_v|)(1 - |y - y_v|); each target t keeps
// sum(z w) and sum(w) and the result is their ratio (+1e-15).  The reference accumulates with
// put_(accumulate=True): on CPU a sequential pass per corner (x floor / ceil outer, y floor /
// ceil inner) in source order, so every target's sums are ordered by e = corner * N + p.  A
// scatter with float atomics would be order-nondeterministic; instead:
//   1. splat_count_kernel: thread per (corner, source) entry e: count entries per target;
//   2. splat_scan_kernel:  one workgroup per batch item: exclusive scan of the counts;
//   3. splat_fill_kernel:  each entry drops its index e into its target's bucket;
//   4. splat_gather_kernel: thread per target: visits its bucket in ascending e (buckets are
//      a few entries; selection by "smallest e above the last one") and sums in exactly the
//      reference's order — bit-identical results, no float atomics.
#include <cmath>

#include "corr_common.h"

namespace corr {
namespace {

struct SplatEntry {
    float w;
    int t;  // target index, -1 when out of bounds
};

// Entry e = corner * N + p of one batch item (corner: bit 1 = x ceil, bit 0 = y ceil).
__device__ __forceinline__ SplatEntry splat_entry(const float *dx, const float *dy, int e, int N, int H, int W) {
    const int corner = e / N, p = e - corner * N;
    const float x = (float)(p % W) + dx[p], y = (float)(p / W) + dy[p];
    const float xv = (corner & 2) ? ceilf(x) : floorf(x);
    const float yv = (corner & 1) ? ceilf(y) : floorf(y);
    SplatEntry r;
    r.w = __fmul_rn(__fsub_rn(1.0f, fabsf(__fsub_rn(x, xv))), __fsub_rn(1.0f, fabsf(__fsub_rn(y, yv))));
    const bool in = xv < (float)W && xv >= 0.0f && yv < (float)H && yv >= 0.0f;
    r.t = in ? (int)__fadd_rn(xv, __fmul_rn((float)W, yv)) : -1;
    return r;
}

__global__ __launch_bounds__(256) void splat_count_kernel(const float *__restrict__ flow, int H, int W,
                                                          int *__restrict__ cnt) {
    const int N = H * W, b = blockIdx.y;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= 4 * N) return;
    const float *dx = flow + (size_t)b * 2 * N, *dy = dx + N;
    const SplatEntry s = splat_entry(dx, dy, e, N, H, W);
    if (s.t >= 0) atomicAdd(&cnt[(size_t)b * N + s.t], 1);
}

// Exclusive scan of cnt[b][0..N) -> off[b][...], one 1024-thread workgroup per batch item.
__global__ __launch_bounds__(1024) void splat_scan_kernel(const int *__restrict__ cnt, int N, int *__restrict__ off) {
    __shared__ int part[1024];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int per = (N + 1023) / 1024;
    const int lo = min(N, tid * per), hi = min(N, lo + per);
    const int *c = cnt + (size_t)b * N;
    int s = 0;
    for (int i = lo; i < hi; ++i) s += c[i];
    part[tid] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan of the partials
        const int v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int run = tid ? part[tid - 1] : 0;
    int *o = off + (size_t)b * N;
    for (int i = lo; i < hi; ++i) {
        o[i] = run;
        run += c[i];
    }
}

__global__ __launch_bounds__(256) void splat_fill_kernel(const float *__restrict__ flow, int H, int W,
                                                         const int *__restrict__ off, int *__restrict__ fill,
                                                         int *__restrict__ ent) {
    const int N = H * W, b = blockIdx.y;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= 4 * N) return;
    const float *dx = flow + (size_t)b * 2 * N, *dy = dx + N;
    const SplatEntry s = splat_entry(dx, dy, e, N, H, W);
    if (s.t < 0) return;
    const size_t t = (size_t)b * N + s.t;
    ent[(size_t)b * 4 * N + off[t] + atomicAdd(&fill[t], 1)] = e;  // slot order is free: sorted below
}

__global__ __launch_bounds__(256) void splat_gather_kernel(const float *__restrict__ flow, int H, int W,
                                                           const int *__restrict__ cnt, const int *__restrict__ off,
                                                           const int *__restrict__ ent, float *__restrict__ out) {
    const int N = H * W, b = blockIdx.y;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= N) return;
    const float *dx = flow + (size_t)b * 2 * N, *dy = dx + N;
    const int k = cnt[(size_t)b * N + t];
    const int *bucket = ent + (size_t)b * 4 * N + off[(size_t)b * N + t];
    float v0 = 0.0f, v1 = 0.0f, acc = 0.0f;
    int last = -1;
    for (int i = 0; i < k; ++i) {
        int e = 0x7fffffff;
        for (int j = 0; j < k; ++j) {  // next entry in the reference's order
            const int c = bucket[j];
            if (c > last && c < e) e = c;
        }
        last = e;
        const int p = e % N;
        const SplatEntry s = splat_entry(dx, dy, e, N, H, W);
        v0 = __fadd_rn(v0, __fmul_rn(dx[p], s.w));
        v1 = __fadd_rn(v1, __fmul_rn(dy[p], s.w));
        acc = __fadd_rn(acc, s.w);
    }
    const float den = __fadd_rn(acc, 1e-15f);
    out[(size_t)b * 2 * N + t] = __fdiv_rn(v0, den);
    out[((size_t)b * 2 + 1) * N + t] = __fdiv_rn(v1, den);
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// cnt [B*N] | off [B*N] | fill [B*N] | ent [B*4N] (int32)
size_t splat_workspace(int B, int H, int W) {
    const size_t BN = (size_t)B * H * W;
    return 3 * al256(BN * 4) + al256(4 * BN * 4);
}

hipError_t launch_forward_splat(const float *flow, int B, int H, int W, float *out, void *ws, hipStream_t s) {
    const size_t BN = (size_t)B * H * W;
    const int N = H * W;
    char *w = (char *)ws;
    int *cnt = (int *)w, *off = (int *)(w + al256(BN * 4)), *fill = (int *)(w + 2 * al256(BN * 4));
    int *ent = (int *)(w + 3 * al256(BN * 4));
    hipError_t e = hipMemsetAsync(cnt, 0, BN * 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(fill, 0, BN * 4, s);
    if (e != hipSuccess) return e;
    const dim3 ge((4 * N + 255) / 256, B), gt((N + 255) / 256, B);
    hipLaunchKernelGGL(splat_count_kernel, ge, dim3(256), 0, s, flow, H, W, cnt);
    hipLaunchKernelGGL(splat_scan_kernel, dim3(B), dim3(1024), 0, s, cnt, N, off);
    hipLaunchKernelGGL(splat_fill_kernel, ge, dim3(256), 0, s, flow, H, W, off, fill, ent);
    hipLaunchKernelGGL(splat_gather_kernel, gt, dim3(256), 0, s, flow, H, W, cnt, off, ent, out);
    return hipGetLastError();
}

}  // namespace corr
