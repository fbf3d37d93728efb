// corr_bwd.hip — backward of the all-pairs product (autograd of model/corr.py:58-60).
//
//   dF1[b][d][n] = sum_m dC[b][n][m] * F2[b][d][m] / sqrt(D)     (M = D, N = queries,  K = targets)
//   dF2[b][d][m] = sum_n F1[b][d][n] * dC[b][n][m] / sqrt(D)     (M = D, N = targets,  K = queries)
//
// Both are fp32 GEMMs with a long K (= H*W) and a small output (D x H*W), so the kernel
// splits K over workgroups to fill 256 CUs; each split writes a partial slab and a second
// pass sums the slabs in split order (deterministic, no atomics) and applies 1/sqrt(D).
// Tiles: 128 (d) x 128 (pixels) per 4-wave workgroup, K staged through LDS in 32-deep
// chunks, v_mfma_f32_32x32x2_f32 (exact fp32), A = rows d, B = pixel columns.
#include <algorithm>
#include <cmath>

#include "corr_common.h"

namespace corr {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBM = 128, kBN = 128, kBK = 32, kThreads = 256;
constexpr int kLds = 129;  // padded LDS row (floats): transposed scalar fills are conflict-free
constexpr int kTargetWG = 512;

struct GemmParams {
    const float *A;  // A(m, k) = A[m * lda + k]        (k-contiguous: F1 / F2 rows)
    const float *Bm; // B(k, n) = B_KC ? B[n*ldb + k] : B[k*ldb + n]
    float *C;        // C(m, n) = C[m * ldc + n]  (or a split slab)
    int M, Nn, K;
    long lda, ldb, ldc;
    long sA, sB, sC;  // batch strides
    int batch, splits, kchunk;
    float alpha;
    int direct;       // splits == 1: scale and write C directly
};

template <bool B_KC>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmParams p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *As = smem;                    // [2][kBK][kLds]
    float *Bs = smem + 2 * kBK * kLds;   // [2][kBK][kLds]

    const int tm = (p.M + kBM - 1) / kBM, tn = (p.Nn + kBN - 1) / kBN;
    int id = blockIdx.x;
    const int nt = id % tn;
    id /= tn;
    const int mt = id % tm;
    id /= tm;
    const int split = id % p.splits;
    const int b = id / p.splits;
    const int m0 = mt * kBM, n0 = nt * kBN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);

    const float *A = p.A + (size_t)b * p.sA;
    const float *Bm = p.Bm + (size_t)b * p.sB;

    const int tid = threadIdx.x;
    const int lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wv = tid >> 6, wm = wv >> 1, wn = wv & 1;

    // k-contiguous tile loader: rows r = (tid >> 3) + 32*i, k = 4*(tid & 7) .. +3
    const int kr_row = tid >> 3, kr_k = (tid & 7) * 4;
    // n-contiguous tile loader: k = (tid >> 5) + 8*i, n = 4*(tid & 31) .. +3
    const int nr_k = tid >> 5, nr_n = (tid & 31) * 4;

    float ra[4][4], rb[4][4];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + kr_row + 32 * i;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = k0 + kr_k + e;
                ra[i][e] = (m < p.M && k < kend) ? A[(size_t)m * p.lda + k] : 0.f;
            }
            if (B_KC) {
                const int n = n0 + kr_row + 32 * i;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = k0 + kr_k + e;
                    rb[i][e] = (n < p.Nn && k < kend) ? Bm[(size_t)n * p.ldb + k] : 0.f;
                }
            } else {
                const int k = k0 + nr_k + 8 * i;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int n = n0 + nr_n + e;
                    rb[i][e] = (n < p.Nn && k < kend) ? Bm[(size_t)k * p.ldb + n] : 0.f;
                }
            }
        }
    };
    auto store = [&](int st) {
        float *as = As + st * kBK * kLds;
        float *bs = Bs + st * kBK * kLds;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                as[(kr_k + e) * kLds + kr_row + 32 * i] = ra[i][e];
                if (B_KC)
                    bs[(kr_k + e) * kLds + kr_row + 32 * i] = rb[i][e];
                else
                    bs[(nr_k + 8 * i) * kLds + nr_n + e] = rb[i][e];
            }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nchunks = (kend - kbeg + kBK - 1) / kBK;
    if (nchunks > 0) {
        load(kbeg);
        store(0);
    }
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int st = c & 1;
        if (c + 1 < nchunks) load(kbeg + (c + 1) * kBK);
        const float *as = As + st * kBK * kLds;
        const float *bs = Bs + st * kBK * kLds;
#pragma unroll
        for (int s = 0; s < kBK / 2; ++s) {
            const int k = 2 * s + h;
            const float a0 = as[k * kLds + wm * 64 + l32];
            const float a1 = as[k * kLds + wm * 64 + 32 + l32];
            const float b0 = bs[k * kLds + wn * 64 + l32];
            const float b1 = bs[k * kLds + wn * 64 + 32 + l32];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (c + 1 < nchunks) store(st ^ 1);
        __syncthreads();
    }

    // C/D map: col (n) = l32, row (m) = (r&3) + 8*(r>>2) + 4h
    float *C = p.direct ? p.C + (size_t)b * p.sC
                        : p.C + ((size_t)split * p.batch + b) * (size_t)p.M * p.Nn;
    const long ldc = p.direct ? p.ldc : p.Nn;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 64 + j * 32 + l32;
            if (n >= p.Nn) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < p.M) {
                    const float v = acc[i][j][r];
                    C[(size_t)m * ldc + n] = p.direct ? v * p.alpha : v;
                }
            }
        }
}

// Sum split-K slabs in split order, scale, write C[b][m][n] (ldc = Nn, batch stride sC).
// fix.K > 0: outputs that come out NaN are recomputed in fp32 (NanFix, corr_common.h).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float *__restrict__ ws,
                                                            float *__restrict__ C, int splits,
                                                            size_t per_split, float alpha,
                                                            int exact_mul, float s, NanFix fix) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < per_split;
         i += (size_t)gridDim.x * blockDim.x) {
        float acc = ws[i];
        for (int k = 1; k < splits; ++k) acc = acc + ws[(size_t)k * per_split + i];
        acc = exact_mul ? acc * alpha : acc / s;
        if (fix.K && __builtin_expect(acc != acc, 0)) acc = nanfix_flat(fix, i);
        C[i] = acc;
    }
}

// The same sum, 16 B per lane (per_split % 4 == 0, 16-B aligned slabs and C): the split-K slabs
// of one float4 are loaded together, each element summed in split order as above.
__global__ __launch_bounds__(256) void splitk_reduce_vec4_kernel(const float4 *__restrict__ ws,
                                                                 float4 *__restrict__ C, int splits,
                                                                 size_t per4, float alpha, int exact_mul,
                                                                 float s, NanFix fix) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < per4;
         i += (size_t)gridDim.x * blockDim.x) {
        float4 acc = ws[i];
        for (int k = 1; k < splits; ++k) {
            const float4 v = ws[(size_t)k * per4 + i];
            acc.x = acc.x + v.x, acc.y = acc.y + v.y, acc.z = acc.z + v.z, acc.w = acc.w + v.w;
        }
        if (exact_mul)
            acc.x = acc.x * alpha, acc.y = acc.y * alpha, acc.z = acc.z * alpha, acc.w = acc.w * alpha;
        else
            acc.x = acc.x / s, acc.y = acc.y / s, acc.z = acc.z / s, acc.w = acc.w / s;
        if (fix.K && __builtin_expect(acc.x != acc.x || acc.y != acc.y || acc.z != acc.z || acc.w != acc.w, 0)) {
            if (acc.x != acc.x) acc.x = nanfix_flat(fix, 4 * i);
            if (acc.y != acc.y) acc.y = nanfix_flat(fix, 4 * i + 1);
            if (acc.z != acc.z) acc.z = nanfix_flat(fix, 4 * i + 2);
            if (acc.w != acc.w) acc.w = nanfix_flat(fix, 4 * i + 3);
        }
        C[i] = acc;
    }
}

int plan_splits(int M, int Nn, int K, int batch) {
    const long tiles = (long)((M + kBM - 1) / kBM) * ((Nn + kBN - 1) / kBN) * batch;
    long splits = (kTargetWG + tiles - 1) / tiles;
    const long max_splits = std::max(1, K / 256);  // keep >= 256 k per split
    splits = std::min(splits, max_splits);
    return (int)std::max(1L, splits);
}

bool is_pow2(float s) {
    int e;
    return std::frexp(s, &e) == 0.5f;
}

hipError_t run_gemm(bool b_kcontig, const float *A, const float *Bm, float *C, int M, int Nn, int K,
                    int batch, long lda, long ldb, long ldc, long sA, long sB, long sC, float s,
                    float *ws, hipStream_t stream) {
    GemmParams p{};
    p.A = A;
    p.Bm = Bm;
    p.M = M;
    p.Nn = Nn;
    p.K = K;
    p.lda = lda;
    p.ldb = ldb;
    p.ldc = ldc;
    p.sA = sA;
    p.sB = sB;
    p.sC = sC;
    p.batch = batch;
    p.splits = plan_splits(M, Nn, K, batch);
    const int kchunk = ((K + p.splits - 1) / p.splits + kBK - 1) / kBK * kBK;
    p.kchunk = kchunk;
    p.splits = (K + kchunk - 1) / kchunk;
    const bool exact = is_pow2(s);
    p.alpha = 1.0f / s;
    p.direct = (p.splits == 1) && exact;
    p.C = p.direct ? C : ws;
    const long tiles = (long)((M + kBM - 1) / kBM) * ((Nn + kBN - 1) / kBN) * batch * p.splits;
    const size_t lds = 2 * 2 * kBK * kLds * sizeof(float);
    if (b_kcontig)
        hipLaunchKernelGGL(gemm_kernel<true>, dim3((unsigned)tiles), dim3(kThreads), lds, stream, p);
    else
        hipLaunchKernelGGL(gemm_kernel<false>, dim3((unsigned)tiles), dim3(kThreads), lds, stream, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || p.direct) return e;
    // slabs are [split][batch][M][Nn]; C is [batch] x sC with rows of Nn (ldc == Nn here)
    const size_t per = (size_t)batch * M * Nn;
    const int grid = (int)std::min<size_t>((per + 255) / 256, 8192);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, stream, ws, C, p.splits, per,
                       p.alpha, exact ? 1 : 0, s, NanFix{});
    return hipGetLastError();
}

}  // namespace

// Ordered split-K sum + 1/sqrt(D) for corr_bwd_split.hip's slabs ([split][per] floats).
// vec4 = false: the scalar reduce (tools/kbench_gemm.hip A/B).
hipError_t launch_splitk_reduce(const float *ws, float *C, int splits, size_t per, float sD, hipStream_t s, bool vec4,
                                const NanFix *fix) {
    const NanFix f = fix ? *fix : NanFix{};
    if (per % 4 == 0 && ((uintptr_t)ws & 15) == 0 && ((uintptr_t)C & 15) == 0 && vec4) {
        const size_t per4 = per / 4;
        const int grid = (int)std::min<size_t>((per4 + 255) / 256, 8192);
        hipLaunchKernelGGL(splitk_reduce_vec4_kernel, dim3(grid), dim3(256), 0, s, (const float4 *)ws, (float4 *)C,
                           splits, per4, 1.0f / sD, is_pow2(sD) ? 1 : 0, sD, f);
        return hipGetLastError();
    }
    const int grid = (int)std::min<size_t>((per + 255) / 256, 8192);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, s, ws, C, splits, per, 1.0f / sD,
                       is_pow2(sD) ? 1 : 0, sD, f);
    return hipGetLastError();
}

size_t build_bwd_workspace(int B, int D, int NQ, int H, int W) {
    const int N = H * W;
    // every GEMM goes through the slab path when sqrt(D) is not a power of two
    const size_t s1 = (size_t)plan_splits(D, NQ, N, B) * B * D * NQ;  // dF1
    const size_t s2 = (size_t)plan_splits(D, N, NQ, B) * B * D * N;   // dF2
    return std::max(s1, s2) * sizeof(float);
}

hipError_t launch_build_bwd(const float *grad_c, const float *f1, int NQ, const float *f2, int B,
                            int D, int H, int W, float *df1, float *df2, float *ws, hipStream_t s) {
    const int N = H * W;  // targets; grad_c is [B*NQ][N]
    const float sc = std::sqrt((float)D);
    const long DN = (long)D * N, DQ = (long)D * NQ, QN = (long)NQ * N;
    // dF1[d][n] = sum_m F2[d][m] * dC[n][m]      A = F2 (k-contig), B(k=m, n) = dC[n*N + m]
    hipError_t e = run_gemm(true, f2, grad_c, df1, D, NQ, N, B, N, N, NQ, DN, QN, DQ, sc, ws, s);
    if (e != hipSuccess) return e;
    // dF2[d][m] = sum_n F1[d][n] * dC[n][m]      A = F1 (k-contig), B(k=n, m) = dC[n*N + m]
    return run_gemm(false, f1, grad_c, df2, D, N, NQ, B, NQ, N, N, DQ, QN, DN, sc, ws, s);
}

}  // namespace corr
