// kbench_lookup.hip — A/B timing of lookup-kernel variants in ONE process, interleaved
// round-robin, random data, bitwise check of every variant against the production launch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o kbench_lookup tools/kbench_lookup.hip
//   ./kbench_lookup [rounds]
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../e-raft_amd/csrc/corr_lookup.hip"

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

// coords = pixel grid + uniform(-sigma, sigma) flow
__global__ void make_coords(float *c, int B, int H, int W, float sigma, unsigned seed) {
    const size_t N = (size_t)H * W;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)B * 2 * N; i += (size_t)gridDim.x * blockDim.x) {
        const size_t n = i % N, axis = (i / N) % 2;
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        const float u = ((x >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
        c[i] = (axis ? (float)(n / W) : (float)(n % W)) + sigma * u;
    }
}

// smooth flow: global non-integer shift + low-frequency field (what E-RAFT's GRU produces)
__global__ void make_coords_smooth(float *c, int B, int H, int W, float amp, unsigned seed) {
    const size_t N = (size_t)H * W;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)B * 2 * N; i += (size_t)gridDim.x * blockDim.x) {
        const size_t n = i % N, axis = (i / N) % 2;
        const float x = (float)(n % W), y = (float)(n / W);
        const float f = axis ? (-2.7f + amp * __cosf(0.11f * x - 0.07f * y + seed))
                             : (3.3f + amp * __sinf(0.09f * x + 0.13f * y + seed));
        c[i] = (axis ? y : x) + f;
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
    int B, H, W;
};

struct Variant {
    std::string name;
    std::function<hipError_t(float *)> launch;
    std::vector<float> us;
};

template <int QB, int ABL = 0, bool TIGHT = false>
static hipError_t launch_qb(const ConstLevelPtrs &pyr, const float *coords, int B, int H, int W, float *out) {
    const int nqb = (H * W + QB - 1) / QB;
    hipLaunchKernelGGL((lookup_kernel<9, QB, ABL, TIGHT>), dim3(nqb * B, 4), dim3(lookup_threads(9, QB)), 0, 0, pyr,
                       coords, B, H * W, H, W, 4, out);
    return hipGetLastError();
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 40;
    constexpr int PER = 12;  // one frame pair's worth of lookups per sample
    std::vector<Shape> shapes = {{"dsec", 1, 60, 80}, {"mvsec-pad", 16, 36, 44}, {"train", 8, 36, 48},
                                 {"1280x960", 1, 120, 160}, {"mvsec-crop", 16, 32, 32}, {"train-b4", 4, 36, 48},
                                 {"train-b12", 12, 36, 48}, {"1920x1280", 1, 160, 240}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Shape &sh : shapes) {
        if (argc > 2 && std::string(argv[2]) != sh.name) continue;  // one shape (PMC passes)
        const size_t N = (size_t)sh.H * sh.W, BN = (size_t)sh.B * N;
        size_t off[4], tot = 0;
        for (int l = 0; l < 4; ++l) {
            off[l] = tot;
            tot += BN * map_floats(sh.H >> l, sh.W >> l);  // the tiled pyramid (corr_common.h)
        }
        float *pyr, *coords, *ref, *out;
        const size_t n_out = (size_t)sh.B * 324 * N;
        CK(hipMalloc(&pyr, tot * 4));
        CK(hipMalloc(&coords, (size_t)sh.B * 2 * N * 4));
        CK(hipMalloc(&ref, n_out * 4));
        CK(hipMalloc(&out, n_out * 4));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, pyr, tot, 7u);
        hipLaunchKernelGGL(make_coords, dim3(1024), dim3(256), 0, 0, coords, sh.B, sh.H, sh.W, 6.0f, 9u);
        float *coords_s, *coords_g;
        CK(hipMalloc(&coords_s, (size_t)sh.B * 2 * N * 4));
        CK(hipMalloc(&coords_g, (size_t)sh.B * 2 * N * 4));
        hipLaunchKernelGGL(make_coords_smooth, dim3(1024), dim3(256), 0, 0, coords_s, sh.B, sh.H, sh.W, 4.0f, 3u);
        hipLaunchKernelGGL(make_coords, dim3(1024), dim3(256), 0, 0, coords_g, sh.B, sh.H, sh.W, 0.0f, 9u);
        ConstLevelPtrs lp{};
        for (int l = 0; l < 4; ++l) lp.p[l] = pyr + off[l];
        const int B = sh.B, H = sh.H, W = sh.W;
        std::vector<Variant> vs;
        vs.push_back({"prod launch_lookup", [=](float *o) { return launch_lookup(lp, coords, B, H * W, H, W, 4, 4, o, 0); }, {}});
        vs.push_back({"QB16", [=](float *o) { return launch_qb<16>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"QB32", [=](float *o) { return launch_qb<32>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"QB16 tight", [=](float *o) { return launch_qb<16, 0, true>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"QB32 tight", [=](float *o) { return launch_qb<32, 0, true>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"QB32 tight grid", [=](float *o) { return launch_qb<32, 0, true>(lp, coords_g, B, H, W, o); }, {}});
        vs.push_back({"prod smooth-flow", [=](float *o) { return launch_lookup(lp, coords_s, B, H * W, H, W, 4, 4, o, 0); }, {}});
        vs.push_back({"prod grid (integer)", [=](float *o) { return launch_lookup(lp, coords_g, B, H * W, H, W, 4, 4, o, 0); }, {}});
        vs.push_back({"QB16 smooth-flow", [=](float *o) { return launch_qb<16>(lp, coords_s, B, H, W, o); }, {}});
        vs.push_back({"abl QB32 noload", [=](float *o) { return launch_qb<32, 1>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"abl QB32 nostore", [=](float *o) { return launch_qb<32, 2>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"abl QB32 nocoords", [=](float *o) { return launch_qb<32, 4>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"abl QB32 noload nostore", [=](float *o) { return launch_qb<32, 3>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"abl QB32 none (taps only)", [=](float *o) { return launch_qb<32, 7>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"QB16 cached-stores", [=](float *o) { return launch_qb<16, 8>(lp, coords, B, H, W, o); }, {}});
        vs.push_back({"QB32 cached-stores", [=](float *o) { return launch_qb<32, 8>(lp, coords, B, H, W, o); }, {}});
        CK(vs[0].launch(ref));
        if (argc > 3) {  // one variant (PMC passes)
            std::vector<Variant> keep;
            for (auto &v : vs)
                if (v.name == argv[3]) keep.push_back(v);
            vs = keep;
        }
        float *ref_g;  // the integer-grid coords' reference (production launch)
        CK(hipMalloc(&ref_g, n_out * 4));
        CK(launch_lookup(lp, coords_g, B, H * W, H, W, 4, 4, ref_g, 0));
        for (auto &v : vs) {
            CK(hipMemset(out, 0, n_out * 4));
            CK(v.launch(out));
            CK(hipDeviceSynchronize());
            unsigned long long *d, diff = 0;
            CK(hipMalloc(&d, sizeof(*d)));
            CK(hipMemset(d, 0, sizeof(*d)));
            const bool grid = v.name.find("grid") != std::string::npos;
            hipLaunchKernelGGL(count_diff, dim3(2048), dim3(256), 0, 0, grid ? ref_g : ref, out, n_out, d);
            CK(hipMemcpy(&diff, d, sizeof(diff), hipMemcpyDeviceToHost));
            CK(hipFree(d));
            const bool same_inputs = v.name.rfind("abl", 0) != 0 && v.name.find("smooth") == std::string::npos;
            if (diff && same_inputs) printf("!! %s differs in %llu elements\n", v.name.c_str(), diff);
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
        const double bytes = (double)BN * (4 * 100 * 4 + 4 * 81 * 4 + 8);
        for (auto &v : vs) {
            std::sort(v.us.begin(), v.us.end());
            const float med = v.us[v.us.size() / 2];
            printf("%-10s %-22s median %8.2f us  min %8.2f us  %7.1f GB/s(alg)\n", sh.name, v.name.c_str(), med,
                   v.us[0], bytes / (med * 1e-6) / 1e9);
        }
        CK(hipFree(pyr));
        CK(hipFree(coords));
        CK(hipFree(ref));
        CK(hipFree(out));
        CK(hipFree(ref_g));
    }
    return 0;
}
