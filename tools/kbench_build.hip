// kbench_build.hip — A/B timing of corr_build tile geometries in ONE process (variance
// correlated across variants, cdna_hip_programming.md §5.4 rule 24), on random data.
// Every variant must be bit-identical to the default (same k-order) — checked on device.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o kbench_build tools/kbench_build.hip
//   ./kbench_build [reps]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "../e-raft_amd/csrc/corr_build.hip"

using namespace corr;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void fill(float *p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = ((x >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
    }
}

__global__ void count_diff(const float *a, const float *b, size_t n, unsigned long long *cnt) {
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c += (__float_as_uint(a[i]) != __float_as_uint(b[i]));
    if (c) atomicAdd(cnt, c);
}

struct Shape {
    const char *name;
    int B, D, H, W;
};

struct Bufs {
    float *f1, *f2, *ref, *out;
    size_t pyr_elems;
    size_t off[4];
};

static LevelPtrs levels_of(float *base, const Bufs &b) {
    LevelPtrs lp{};
    for (int l = 0; l < 4; ++l) lp.p[l] = base + b.off[l];
    return lp;
}

template <class Cfg>
static void run(const char *name, const Shape &sh, Bufs &b, int reps, bool is_ref) {
    const double flops = 2.0 * sh.B * (double)sh.H * sh.W * sh.H * sh.W * sh.D;
    float *dst = is_ref ? b.ref : b.out;
    LevelPtrs lp = levels_of(dst, b);
    for (int i = 0; i < 3; ++i) CK(launch_build_cfg<Cfg>(b.f1, sh.H * sh.W, b.f2, sh.B, sh.D, sh.H, sh.W, 4, lp, 0));
    CK(hipDeviceSynchronize());
    std::vector<hipEvent_t> ev(2 * reps);
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(ev[2 * i], 0));
        CK(launch_build_cfg<Cfg>(b.f1, sh.H * sh.W, b.f2, sh.B, sh.D, sh.H, sh.W, 4, lp, 0));
        CK(hipEventRecord(ev[2 * i + 1], 0));
    }
    CK(hipDeviceSynchronize());
    std::vector<float> ms(reps);
    for (int i = 0; i < reps; ++i) CK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
    for (auto &e : ev) CK(hipEventDestroy(e));
    std::sort(ms.begin(), ms.end());
    unsigned long long diff = 0;
    if (!is_ref) {
        unsigned long long *d;
        CK(hipMalloc(&d, sizeof(*d)));
        CK(hipMemset(d, 0, sizeof(*d)));
        hipLaunchKernelGGL(count_diff, dim3(2048), dim3(256), 0, 0, b.ref, b.out, b.pyr_elems, d);
        CK(hipMemcpy(&diff, d, sizeof(diff), hipMemcpyDeviceToHost));
        CK(hipFree(d));
    }
    const float med = ms[reps / 2], best = ms[0];
    printf("%-10s %-28s threads %4d LDS %6zu  median %8.2f us  best %8.2f us  %6.1f TF/s  diff %llu\n",
           sh.name, name, Cfg::NT, Cfg::LDS, med * 1e3, best * 1e3, flops / (med * 1e-3) / 1e12, diff);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    std::vector<Shape> shapes = {{"dsec", 1, 256, 60, 80},
                                 {"mvsec-pad", 16, 256, 36, 44},
                                 {"train", 8, 256, 36, 48},
                                 {"1280x960", 1, 256, 120, 160}};
    for (const Shape &sh : shapes) {
        const size_t N = (size_t)sh.H * sh.W, BN = (size_t)sh.B * N;
        Bufs b{};
        size_t tot = 0;
        for (int l = 0; l < 4; ++l) {
            b.off[l] = tot;
            tot += (BN * (sh.H >> l) * (sh.W >> l) + 3) / 4 * 4;
        }
        b.pyr_elems = tot;
        const size_t fe = (size_t)sh.B * sh.D * N;
        CK(hipMalloc(&b.f1, fe * 4));
        CK(hipMalloc(&b.f2, fe * 4));
        CK(hipMalloc(&b.ref, tot * 4));
        CK(hipMalloc(&b.out, tot * 4));
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, b.f1, fe, 1u);
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, b.f2, fe, 2u);
        CK(hipMemset(b.ref, 0, tot * 4));
        CK(hipMemset(b.out, 0, tot * 4));
        run<BuildCfg<2, 2, 2, 32, 2>>("ref  2x2 QT2 BK32", sh, b, reps, true);
        run<BuildCfg<2, 2, 2, 16, 3>>("D    2x2 QT2 BK16 o3", sh, b, reps, false);
        run<BuildCfg<2, 2, 2, 16, 4>>("D4   2x2 QT2 BK16 o4", sh, b, reps, false);
        run<BuildCfg<2, 2, 2, 8, 4>>("D8   2x2 QT2 BK8 o4", sh, b, reps, false);
        run<BuildCfg<2, 2, 1, 16, 4>>("J16  2x2 QT1 BK16 o4", sh, b, reps, false);
        run<BuildCfg<2, 2, 2, 16, 3, true>>("P    2x2 QT2 BK16 o3 PF", sh, b, reps, false);
        run<BuildCfg<2, 2, 2, 16, 4, true>>("P4   2x2 QT2 BK16 o4 PF", sh, b, reps, false);
        run<BuildCfg<2, 2, 2, 32, 2, true>>("P32  2x2 QT2 BK32 o2 PF", sh, b, reps, false);
        run<BuildCfg<2, 2, 2, 8, 4, true>>("P8   2x2 QT2 BK8 o4 PF", sh, b, reps, false);
        run<BuildCfg<2, 2, 4, 16, 2, true>>("PQ4  2x2 QT4 BK16 o2 PF", sh, b, reps, false);
        run<BuildCfg<4, 1, 2, 16, 4, true>>("PE   4x1 QT2 BK16 o4 PF", sh, b, reps, false);
        CK(hipFree(b.f1));
        CK(hipFree(b.f2));
        CK(hipFree(b.ref));
        CK(hipFree(b.out));
    }
    return 0;
}
