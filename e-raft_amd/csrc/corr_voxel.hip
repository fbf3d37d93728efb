// corr_voxel.hip — the DSEC event -> voxel-grid representation, the producer of every frame
// pair's network input (utils/dsec_utils.py:26-64 VoxelGrid.convert, called by
// loader/loader_dsec.py:245-257 on the host CPU in the reference).
//
// Each event e (float32 x, y, t in [0, 1], p in {0, 1}) votes into C temporal bins:
//   t_n = ((C-1)(t - t_0)) / (t_{M-1} - t_0); corners (x_l, y_l) in {x0, x0+1} x {y0, y0+1}
//   (x0 = trunc x), t_l = trunc t_n; weight ((2p-1)(1-|x_l-x|))(1-|y_l-y|))(1-|t_l-t_n|);
//   in-bounds corners accumulate at H*W*t_l + W*y_l + x_l.
// The reference accumulates with put_(accumulate=True) — single-threaded (main.py:2-5 pins one
// thread) that is a sequential pass per corner in event order.  As in corr_splat.hip the
// accumulation is made deterministic and order-exact without float atomics: count entries per
// cell, scan, bucket the entry indices, then each cell sums its bucket in ascending entry
// order (entry = corner * M + event).  Buckets here can be long (many events on one pixel), so
// a bucket is sorted in place first (insertion sort; typical sizes are a few to tens).
// Optional normalisation (:54-62) over the nonzero cells: count, sum and sum of squared
// deviations in fp64 (fixed partitions over 512 workgroups + ordered tree: deterministic), then
// v = (v - mean) / std in fp32 (std unbiased; v - mean when std is not > 0).
//
// The MVSEC representation (utils/transformers.py:18-126 EventSequenceToVoxelGrid_Pytorch, fed by
// loader/loader_mvsec_flow.py:35) runs through the same count / scan / bucket / ordered-sum
// pipeline with a different entry source (VoxTArgs): events [M][4] float64 (t, x, y, p) as
// the loader hands them over (.astype('float'), :46); each event makes two entries, "left"
// (bin floor(t_n), weight p (1 - dt)) and "right" (bin floor(t_n) + 1, weight p dt) with
// t_n = ((C-1) (t - t_0)) / (t_{M-1} - t_0) in fp64 and dt rounded to fp32 (:77-89).  The
// reference adds them with two index_add_ passes (:99-112), each sequential in event order on
// CPU, so entry = side * M + event reproduces its per-cell order exactly.
#include <cmath>

#include "corr_common.h"

namespace corr {
namespace {

struct VoxEntry {
    float w;
    int cell;  // -1: out of bounds
};

// DSEC (dsec_utils.py:26-64): four xy corners per event, entry = corner * M + event.
struct VoxArgs {
    const float *x, *y, *t, *p;
    int M, C, H, W;
    static constexpr int kSides = 4;
    __device__ __forceinline__ VoxEntry entry(int e) const;
};

// MVSEC (transformers.py:36-126): two temporal sides per event, entry = side * M + event.
struct VoxTArgs {
    const double *ev;  // [M][4]: t, x, y, p
    int M, C, H, W;
    static constexpr int kSides = 2;
    __device__ __forceinline__ VoxEntry entry(int e) const;
};

__device__ __forceinline__ VoxEntry VoxArgs::entry(int e) const {
    const VoxArgs &a = *this;
    const int corner = e / a.M, i = e - corner * a.M;
    const float t0 = a.t[0], dt = __fsub_rn(a.t[a.M - 1], t0);
    const float tn = __fdiv_rn(__fmul_rn((float)(a.C - 1), __fsub_rn(a.t[i], t0)), dt);
    const float xf = a.x[i], yf = a.y[i];
    const int xl = (int)xf + (corner >> 1), yl = (int)yf + (corner & 1), tl = (int)tn;
    VoxEntry r;
    const bool in = xl < a.W && xl >= 0 && yl < a.H && yl >= 0 && tl >= 0 && tl < a.C;
    r.cell = in ? (tl * a.H + yl) * a.W + xl : -1;
    const float value = __fsub_rn(__fmul_rn(2.0f, a.p[i]), 1.0f);
    float w = __fmul_rn(value, __fsub_rn(1.0f, fabsf(__fsub_rn((float)xl, xf))));
    w = __fmul_rn(w, __fsub_rn(1.0f, fabsf(__fsub_rn((float)yl, yf))));
    r.w = __fmul_rn(w, __fsub_rn(1.0f, fabsf(__fsub_rn((float)tl, tn))));
    return r;
}

// transformers.py:66-112, op for op: t_n in fp64 (:77, (C-1) * (t - t0) first, then / deltaT,
// deltaT = 1 when the stamps are equal :74-75); tis = floor(t_n), dts = t_n - tis (fp64) then
// rounded to fp32 (:85-89); pols = fp32(p), 0 -> -1 (:81-82); x, y truncated to int64 (:79-80).
// left: valid for 0 <= tis < C; right: bin tis + 1, valid for 0 <= tis and tis + 1 < C
// (:91-92, :106-107).  The flat index x + y W + bin W H is the reference's (:100-101); one
// outside [0, C H W) makes index_add_ raise in the reference and is dropped here.
__device__ __forceinline__ VoxEntry VoxTArgs::entry(int e) const {
    const int side = e >= M ? 1 : 0, i = e - side * M;
    const double t0 = ev[0];
    double dT = __dsub_rn(ev[(size_t)(M - 1) * 4], t0);
    if (dT == 0.0) dT = 1.0;
    const double *q = ev + (size_t)i * 4;
    const double ts = __ddiv_rn(__dmul_rn((double)(C - 1), __dsub_rn(q[0], t0)), dT);
    const double tis = floor(ts);
    const float dts = (float)__dsub_rn(ts, tis);
    float pol = (float)q[3];
    if (pol == 0.0f) pol = -1.0f;
    VoxEntry r;
    r.w = side ? __fmul_rn(pol, dts) : __fmul_rn(pol, __fsub_rn(1.0f, dts));
    r.cell = -1;
    const double bin = __dadd_rn(tis, (double)side);
    const double lim = 2147483648.0;  // |x|, |y| < 2^31: the int64 index below cannot overflow
    if (tis >= 0.0 && bin < (double)C && fabs(q[1]) < lim && fabs(q[2]) < lim) {
        const long long xs = (long long)q[1], ys = (long long)q[2], HW = (long long)H * W;
        const long long cell = xs + ys * W + (long long)bin * HW;
        if (cell >= 0 && cell < HW * C) r.cell = (int)cell;
    }
    return r;
}

template <class A>
__global__ __launch_bounds__(256) void vox_count_kernel(A a, int *__restrict__ cnt) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= A::kSides * a.M) return;
    const VoxEntry v = a.entry(e);
    if (v.cell >= 0) atomicAdd(&cnt[v.cell], 1);
}

// Exclusive scan of n counts: tiles of kTile cells (1024 threads x 8 consecutive cells);
// (1) tile sums, (2) one workgroup scans the tile sums, (3) each tile scans itself from its
// offset.  Integer sums: any order is exact.
constexpr int kTile = 8192;

__global__ __launch_bounds__(1024) void vox_tile_sum_kernel(const int *__restrict__ cnt, int n, int *__restrict__ tsum) {
    __shared__ int red[1024];
    const int base = blockIdx.x * kTile, tid = threadIdx.x;
    int s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = base + j * 1024 + tid;
        s += i < n ? cnt[i] : 0;
    }
    red[tid] = s;
    __syncthreads();
    for (int d = 512; d >= 1; d >>= 1) {
        if (tid < d) red[tid] += red[tid + d];
        __syncthreads();
    }
    if (tid == 0) tsum[blockIdx.x] = red[0];
}

// Exclusive scan of n (small) values in one workgroup.
__global__ __launch_bounds__(1024) void vox_scan_small_kernel(int *__restrict__ v, int n) {
    __shared__ int part[1024];
    const int tid = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int lo = min(n, tid * per), hi = min(n, lo + per);
    int s = 0;
    for (int i = lo; i < hi; ++i) s += v[i];
    part[tid] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int x = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    int run = tid ? part[tid - 1] : 0;
    for (int i = lo; i < hi; ++i) {
        const int c = v[i];
        v[i] = run;
        run += c;
    }
}

__global__ __launch_bounds__(1024) void vox_tile_scan_kernel(const int *__restrict__ cnt, int n,
                                                             const int *__restrict__ toff, int *__restrict__ off) {
    __shared__ int part[1024];
    const int tid = threadIdx.x, base = blockIdx.x * kTile + tid * 8;
    int c[8], s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        c[j] = base + j < n ? cnt[base + j] : 0;
        s += c[j];
    }
    part[tid] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int x = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    int run = toff[blockIdx.x] + (tid ? part[tid - 1] : 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (base + j < n) off[base + j] = run;
        run += c[j];
    }
}

template <class A>
__global__ __launch_bounds__(256) void vox_fill_kernel(A a, const int *__restrict__ off, int *__restrict__ fill,
                                                       int *__restrict__ ent) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= A::kSides * a.M) return;
    const VoxEntry v = a.entry(e);
    if (v.cell >= 0) ent[off[v.cell] + atomicAdd(&fill[v.cell], 1)] = e;
}

// One thread per cell: sort its bucket (ascending entry index = the reference's order), sum.
template <class A>
__global__ __launch_bounds__(256) void vox_gather_kernel(A a, const int *__restrict__ cnt,
                                                         const int *__restrict__ off, int *__restrict__ ent,
                                                         float *__restrict__ out) {
    const int n = a.C * a.H * a.W;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= n) return;
    const int k = cnt[c];
    int *b = ent + off[c];
    for (int i = 1; i < k; ++i) {  // insertion sort, in place (the bucket is this thread's)
        const int v = b[i];
        int j = i - 1;
        while (j >= 0 && b[j] > v) {
            b[j + 1] = b[j];
            --j;
        }
        b[j + 1] = v;
    }
    float s = 0.0f;
    for (int i = 0; i < k; ++i) s = __fadd_rn(s, a.entry(b[i]).w);
    out[c] = s;
}

// Normalisation statistics over the nonzero cells, fp64, deterministic: kStatBlocks
// workgroups reduce fixed grid-stride partitions (tree in LDS), one workgroup folds the
// partials in block order.  pass 0: count and sum -> mean; pass 1: squared deviations -> std.
// st: [0] mean, [1] std (fp32), [2] count; part: kStatBlocks x {sum, count}.
constexpr int kStatBlocks = 512;

__global__ __launch_bounds__(256) void vox_stat_partial_kernel(const float *__restrict__ v, int n, int pass,
                                                               const float *__restrict__ st,
                                                               double *__restrict__ part) {
    __shared__ double rs[256];
    __shared__ double rc[256];
    const int tid = threadIdx.x;
    const double mean64 = pass ? part[2 * kStatBlocks] : 0.0;  // pass 1: the fp64 mean
    (void)st;
    double s = 0.0, c = 0.0;
    for (int i = blockIdx.x * 256 + tid; i < n; i += kStatBlocks * 256) {
        const float x = v[i];
        if (x != 0.0f) {
            if (pass) {
                const double d = (double)x - mean64;
                s += d * d;
            } else {
                s += x;
                c += 1.0;
            }
        }
    }
    rs[tid] = s;
    rc[tid] = c;
    __syncthreads();
    for (int d = 128; d >= 1; d >>= 1) {
        if (tid < d) {
            rs[tid] += rs[tid + d];
            rc[tid] += rc[tid + d];
        }
        __syncthreads();
    }
    if (tid == 0) {
        part[2 * blockIdx.x] = rs[0];
        if (!pass) part[2 * blockIdx.x + 1] = rc[0];
    }
}

__global__ __launch_bounds__(kStatBlocks) void vox_stat_final_kernel(double *__restrict__ part, int pass,
                                                                     float *__restrict__ st) {
    __shared__ double rs[kStatBlocks];
    __shared__ double rc[kStatBlocks];
    const int tid = threadIdx.x;
    rs[tid] = part[2 * tid];
    rc[tid] = part[2 * tid + 1];
    __syncthreads();
    for (int d = kStatBlocks / 2; d >= 1; d >>= 1) {
        if (tid < d) {
            rs[tid] += rs[tid + d];
            if (!pass) rc[tid] += rc[tid + d];
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (!pass) {
            const double cnt = rc[0];
            const double mean = cnt > 0 ? rs[0] / cnt : 0.0;
            part[2 * kStatBlocks] = mean;      // fp64 mean for pass 1
            part[2 * kStatBlocks + 1] = cnt;
            st[0] = (float)mean;
            st[2] = (float)cnt;
        } else {
            const double cnt = part[2 * kStatBlocks + 1];
            st[1] = cnt > 1 ? (float)sqrt(rs[0] / (cnt - 1)) : __int_as_float(0x7fc00000);
        }
    }
}

__global__ __launch_bounds__(256) void vox_normalize_kernel(float *__restrict__ v, int n, const float *__restrict__ st) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = v[i];
    if (x == 0.0f) return;
    const float mean = st[0], sd = st[1];
    v[i] = sd > 0.0f ? __fdiv_rn(__fsub_rn(x, mean), sd) : __fsub_rn(x, mean);
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// cnt [CHW] | off [CHW] | fill [CHW] | ent [entries] | tile sums | stats [4] float | partials (fp64)
size_t voxel_ws_entries(size_t entries, int C, int H, int W) {
    const size_t n = (size_t)C * H * W, tiles = (n + kTile - 1) / kTile;
    return 3 * al256(n * 4) + al256(entries * 4) + al256(tiles * 4) + 256 +
           al256((2 * kStatBlocks + 2) * sizeof(double));
}

template <class A>
hipError_t launch_voxel(const A &a, int normalize, float *out, void *ws, hipStream_t s) {
    const int C = a.C, H = a.H, W = a.W, M = a.M;
    const size_t n = (size_t)C * H * W, entries = (size_t)A::kSides * M;
    char *w = (char *)ws;
    int *cnt = (int *)w, *off = (int *)(w + al256(n * 4)), *fill = (int *)(w + 2 * al256(n * 4));
    int *ent = (int *)(w + 3 * al256(n * 4));
    const size_t tiles = (n + kTile - 1) / kTile;
    int *tsum = (int *)(w + 3 * al256(n * 4) + al256(entries * 4));
    float *st = (float *)((char *)tsum + al256(tiles * 4));
    double *part = (double *)((char *)st + 256);
    hipError_t e = hipMemsetAsync(cnt, 0, n * 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(fill, 0, n * 4, s);
    if (e != hipSuccess) return e;
    const unsigned ge = (unsigned)((entries + 255) / 256), gc = (unsigned)((n + 255) / 256);
    if (M > 0) {
        hipLaunchKernelGGL(vox_count_kernel<A>, dim3(ge), dim3(256), 0, s, a, cnt);
        hipLaunchKernelGGL(vox_tile_sum_kernel, dim3((unsigned)tiles), dim3(1024), 0, s, cnt, (int)n, tsum);
        hipLaunchKernelGGL(vox_scan_small_kernel, dim3(1), dim3(1024), 0, s, tsum, (int)tiles);
        hipLaunchKernelGGL(vox_tile_scan_kernel, dim3((unsigned)tiles), dim3(1024), 0, s, cnt, (int)n, tsum, off);
        hipLaunchKernelGGL(vox_fill_kernel<A>, dim3(ge), dim3(256), 0, s, a, off, fill, ent);
    } else {
        e = hipMemsetAsync(off, 0, n * 4, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(vox_gather_kernel<A>, dim3(gc), dim3(256), 0, s, a, cnt, off, ent, out);
    if (normalize) {
        for (int pass = 0; pass < 2; ++pass) {
            hipLaunchKernelGGL(vox_stat_partial_kernel, dim3(kStatBlocks), dim3(256), 0, s, out, (int)n, pass, st, part);
            hipLaunchKernelGGL(vox_stat_final_kernel, dim3(1), dim3(kStatBlocks), 0, s, part, pass, st);
        }
        hipLaunchKernelGGL(vox_normalize_kernel, dim3(gc), dim3(256), 0, s, out, (int)n, st);
    }
    return hipGetLastError();
}

}  // namespace

size_t voxel_workspace(int M, int C, int H, int W) { return voxel_ws_entries((size_t)VoxArgs::kSides * M, C, H, W); }

size_t voxel_tbilinear_workspace(int M, int C, int H, int W) {
    return voxel_ws_entries((size_t)VoxTArgs::kSides * M, C, H, W);
}

hipError_t launch_voxel_grid(const float *x, const float *y, const float *t, const float *p, int M, int C, int H,
                             int W, int normalize, float *out, void *ws, hipStream_t s) {
    return launch_voxel(VoxArgs{x, y, t, p, M, C, H, W}, normalize, out, ws, s);
}

hipError_t launch_voxel_grid_tbilinear(const double *events, int M, int C, int H, int W, int normalize, float *out,
                                       void *ws, hipStream_t s) {
    return launch_voxel(VoxTArgs{events, M, C, H, W}, normalize, out, ws, s);
}

}  // namespace corr
