// kbench_div.hip — exhaustive check of the reciprocal-and-correct division the lookup's tap
// arithmetic can use in place of __fdiv_rn (corr_lookup.hip tap_axis: 2x / (size - 1)):
//   y = RN(1 / d) (once per level), q = RN(a y), r = fma(-q, d, a) (exact), q' = fma(r, y, q)
// (Markstein's correction), with y from v_rcp_f32 and one Newton step (recip_rn).  First every
// d = 1 .. 2^20 checks recip_rn(d) == __fdiv_rn(1, d); then for every float bit pattern a and
// every d = 1 .. DMAX, q' - 1 is compared bit for bit with __fdiv_rn(a, d) - 1 (the tap
// arithmetic's use) and q' with __fdiv_rn(a, d) wherever that is normal (any NaN equals any NaN;
// a subnormal quotient may differ in its last bits, a zero in its sign); mismatches are counted
// per d and the first few printed.  Run on the GPU:
//   tools/_build/kbench_div [DMAX]
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/_build/kbench_div tools/kbench_div.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

#include "../e-raft_amd/csrc/corr_div.h"

__global__ void check_recip(int n, unsigned *bad, unsigned *first) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (d > n) return;
    const float df = (float)d;
    if (__float_as_uint(corr::recip_rn(df)) != __float_as_uint(__fdiv_rn(1.0f, df))) {
        atomicAdd(bad, 1u);
        atomicMin(first, (unsigned)d);
    }
}

__device__ __forceinline__ float div_corrected(float a, float d, float y) {
    return corr::div_rn(a, d, y);
}

// grid-stride over all 2^32 patterns for one d per blockIdx.y; per-d mismatch count and the
// first mismatching pattern (vector atomics on global memory)
__global__ __launch_bounds__(256) void check(int d0, unsigned long long *cnt, unsigned *first) {
    const int d = d0 + (int)blockIdx.y;
    const float df = (float)d;
    const float y = corr::recip_rn(df);
    unsigned long long bad = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32);
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const float a = __uint_as_float((unsigned)i);
        const float ref = __fdiv_rn(a, df), got = div_corrected(a, df, y);
        // the tap arithmetic's use: q - 1 (bit for bit), and q itself wherever |q| >= 2^-126
        const float rx = __fsub_rn(ref, 1.0f), gx = __fsub_rn(got, 1.0f);
        const bool same_x = (rx != rx && gx != gx) || __float_as_uint(rx) == __float_as_uint(gx);
        const bool same_q = (ref != ref && got != got) || __float_as_uint(ref) == __float_as_uint(got) ||
                            __builtin_fabsf(ref) < 1.17549435e-38f;
        if (!same_x || !same_q) {
            ++bad;
            atomicMin(&first[blockIdx.y], (unsigned)i);
        }
    }
    if (bad) atomicAdd(&cnt[blockIdx.y], bad);
}

int main(int argc, char **argv) {
    const int dmax = argc > 1 ? atoi(argv[1]) : 4096;
    const int chunk = 64;
    unsigned long long *cnt;
    unsigned *first;
    CK(hipMalloc(&cnt, chunk * sizeof(unsigned long long)));
    CK(hipMalloc(&first, chunk * sizeof(unsigned)));
    {
        unsigned *rb;
        CK(hipMalloc(&rb, 8));
        CK(hipMemset(rb, 0, 4));
        CK(hipMemset(rb + 1, 0xff, 4));
        const int n = 1 << 20;
        hipLaunchKernelGGL(check_recip, dim3(n / 256), dim3(256), 0, 0, n, rb, rb + 1);
        unsigned h[2];
        CK(hipMemcpy(h, rb, 8, hipMemcpyDeviceToHost));
        printf("recip_rn vs __fdiv_rn(1, d), d = 1 .. %d: %u mismatches (first d %u)\n", n, h[0], h[0] ? h[1] : 0u);
        fflush(stdout);
        if (h[0]) return 1;
    }
    unsigned long long total = 0;
    int dbad = 0;
    for (int d0 = 1; d0 <= dmax; d0 += chunk) {
        const int n = d0 + chunk - 1 <= dmax ? chunk : dmax - d0 + 1;
        CK(hipMemset(cnt, 0, chunk * sizeof(unsigned long long)));
        CK(hipMemset(first, 0xff, chunk * sizeof(unsigned)));
        hipLaunchKernelGGL(check, dim3(4096, n), dim3(256), 0, 0, d0, cnt, first);
        CK(hipGetLastError());
        std::vector<unsigned long long> c(chunk);
        std::vector<unsigned> f(chunk);
        CK(hipMemcpy(c.data(), cnt, chunk * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        CK(hipMemcpy(f.data(), first, chunk * sizeof(unsigned), hipMemcpyDeviceToHost));
        for (int k = 0; k < n; ++k) {
            if (!c[k]) continue;
            total += c[k];
            if (dbad++ < 20) {
                unsigned u = f[k];
                float a;
                memcpy(&a, &u, 4);
                printf("d=%d mismatches %llu first a=%a (0x%08x)\n", d0 + k, c[k], a, u);
            }
        }
        printf("d %d..%d done, mismatches so far %llu\n", d0, d0 + n - 1, total);
        fflush(stdout);
    }
    printf("TOTAL d=1..%d: %llu mismatches over %d divisors\n", dmax, total, dbad);
    return total != 0;
}
