// kbench_build.hip — A/B timing of corr_build tile geometries in ONE process, variants
// interleaved round-robin (cdna_hip_programming.md §5.4 rule 24: cross-process / cross-device
// variance otherwise dominates), random data.  Every variant must be bit-identical to the
// first (same k-order) — checked on device.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o kbench_build tools/kbench_build.hip
//   ./kbench_build [rounds]
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../e-raft_amd/csrc/corr_build.hip"

using namespace corr;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
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

struct Variant {
    std::string name;
    std::function<hipError_t(float *)> launch;  // writes the pyramid rooted at the argument
    std::vector<float> us;
};

template <class Cfg>
static Variant make(const char *name, const Shape &sh, const float *f1, const float *f2, const size_t *off) {
    Variant v;
    char buf[128];
    snprintf(buf, sizeof buf, "%-26s thr %4d LDS %6zu", name, Cfg::NT, Cfg::LDS);
    v.name = buf;
    v.launch = [=](float *base) {
        LevelPtrs lp{};
        for (int l = 0; l < 4; ++l) lp.p[l] = base + off[l];
        return launch_build_cfg<Cfg>(f1, sh.H * sh.W, f2, sh.B, sh.D, sh.H, sh.W, 4, lp, 0);
    };
    return v;
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 20;
    constexpr int PER = 4;  // launches per timing sample
    std::vector<Shape> shapes = {{"dsec", 1, 256, 60, 80},
                                 {"mvsec-pad", 16, 256, 36, 44},
                                 {"train", 8, 256, 36, 48},
                                 {"1280x960", 1, 256, 120, 160}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Shape &sh : shapes) {
        const size_t N = (size_t)sh.H * sh.W, BN = (size_t)sh.B * N;
        static size_t off[4];
        size_t tot = 0;
        for (int l = 0; l < 4; ++l) {
            off[l] = tot;
            tot += (BN * (sh.H >> l) * (sh.W >> l) + 3) / 4 * 4;
        }
        const size_t fe = (size_t)sh.B * sh.D * N;
        float *f1, *f2, *ref, *out;
        CK(hipMalloc(&f1, fe * 4));
        CK(hipMalloc(&f2, fe * 4));
        CK(hipMalloc(&ref, tot * 4));
        CK(hipMalloc(&out, tot * 4));
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f1, fe, 1u);
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f2, fe, 2u);
        std::vector<Variant> vs;
        vs.push_back(make<BuildCfg<2, 2, 2, 32, 2, false, false>>("v0  BK32 o2 noPF noSKIP", sh, f1, f2, off));
        vs.push_back(make<BuildCfg<2, 2, 2, 8, 4, true, false>>("P8  BK8 o4 PF noSKIP", sh, f1, f2, off));
        vs.push_back(make<BuildCfg<2, 2, 2, 8, 4, true, true>>("P8S BK8 o4 PF SKIP", sh, f1, f2, off));
        vs.push_back(make<BuildCfg<2, 2, 2, 16, 4, true, true>>("P16S BK16 o4 PF SKIP", sh, f1, f2, off));
        vs.push_back(make<BuildCfg<2, 2, 1, 16, 5, true, true>>("J16S QT1 BK16 o5 PF SKIP", sh, f1, f2, off));
        vs.push_back(make<BuildCfg<4, 2, 2, 16, 2, true, true>>("H16S 8w BK16 o2 PF SKIP", sh, f1, f2, off));
        vs.push_back(make<BuildCfg<2, 2, 2, 16, 3, false, true>>("D16S BK16 o3 noPF SKIP", sh, f1, f2, off));
        CK(vs[0].launch(ref));
        for (auto &v : vs) {  // warm + correctness
            CK(hipMemset(out, 0, tot * 4));
            CK(v.launch(out));
            CK(hipDeviceSynchronize());
            unsigned long long *d, diff = 0;
            CK(hipMalloc(&d, sizeof(*d)));
            CK(hipMemset(d, 0, sizeof(*d)));
            hipLaunchKernelGGL(count_diff, dim3(2048), dim3(256), 0, 0, ref, out, tot, d);
            CK(hipMemcpy(&diff, d, sizeof(diff), hipMemcpyDeviceToHost));
            CK(hipFree(d));
            if (diff) printf("!! %s differs from v0 in %llu elements\n", v.name.c_str(), diff);
        }
        for (int r = 0; r < rounds; ++r)
            for (auto &v : vs) {
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < PER; ++i) CK(v.launch(out));
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.us.push_back(ms * 1e3f / PER);
            }
        const double flops = 2.0 * sh.B * (double)N * N * sh.D;
        for (auto &v : vs) {
            std::sort(v.us.begin(), v.us.end());
            const float med = v.us[v.us.size() / 2];
            printf("%-10s %s  median %8.2f us  min %8.2f us  %6.1f TF/s\n", sh.name, v.name.c_str(), med, v.us[0],
                   flops / (med * 1e-6) / 1e12);
        }
        CK(hipFree(f1));
        CK(hipFree(f2));
        CK(hipFree(ref));
        CK(hipFree(out));
    }
    return 0;
}
