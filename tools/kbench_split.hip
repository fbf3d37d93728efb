// kbench_split.hip — the split (3 x f16 MFMA) build against the exact-fp32 MFMA build: accuracy
// (max |split - f32| / max |f32| over every pyramid level) and interleaved timing of geometry
// variants in one process (cdna_hip_programming.md §5.4 rule 24), random data.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o kbench_split tools/kbench_split.hip
//   ./kbench_split [rounds]
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../e-raft_amd/csrc/corr_build.hip"
#include "../e-raft_amd/csrc/corr_build_split.hip"

using namespace corr;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__global__ void fill(float *p, size_t n, unsigned seed, float scale) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (((x >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f) * scale;
    }
}

__global__ void maxdiff(const float *a, const float *b, size_t n, unsigned *dmax, unsigned *rmax) {
    float d = 0.f, r = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        d = fmaxf(d, fabsf(a[i] - b[i]));
        r = fmaxf(r, fabsf(a[i]));
    }
    atomicMax(dmax, __float_as_uint(d));
    atomicMax(rmax, __float_as_uint(r));
}

struct Shape {
    const char *name;
    int B, D, H, W;
};

struct Variant {
    std::string name;
    std::function<hipError_t(float *)> launch;
    std::vector<float> us;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 20;
    constexpr int PER = 4;
    std::vector<Shape> shapes = {{"dsec", 1, 256, 60, 80},
                                 {"mvsec-pad", 16, 256, 36, 44},
                                 {"train", 8, 256, 36, 48},
                                 {"odd", 2, 200, 17, 23},
                                 {"1280x960", 1, 256, 120, 160}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *only = argc > 2 ? argv[2] : nullptr;
    for (const Shape &sh : shapes) {
        if (only && strcmp(only, sh.name)) continue;
        const size_t N = (size_t)sh.H * sh.W, BN = (size_t)sh.B * N;
        static size_t off[4];
        size_t tot = 0;
        for (int l = 0; l < 4; ++l) {
            off[l] = tot;
            tot += (BN * (sh.H >> l) * (sh.W >> l) + 3) / 4 * 4;
        }
        const size_t fe = (size_t)sh.B * sh.D * N;
        float *f1, *f2, *ref, *out;
        void *ws;
        const size_t wsb = build_split_workspace(sh.B, sh.D, (int)N, sh.H, sh.W);
        CK(hipMalloc(&f1, fe * 4));
        CK(hipMalloc(&f2, fe * 4));
        CK(hipMalloc(&ref, tot * 4));
        CK(hipMalloc(&out, tot * 4));
        CK(hipMalloc(&ws, wsb));
        auto lp_of = [&](float *base) {
            LevelPtrs lp{};
            for (int l = 0; l < 4; ++l) lp.p[l] = base + off[l];
            return lp;
        };
        std::vector<Variant> vs;
        vs.push_back({"f32  BuildDefault", [&](float *o) {
                          return launch_build_cfg<BuildDefault>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), 0);
                      }});
        vs.push_back({"x3   pack+mfma default", [&](float *o) {
                          return launch_build_split_cfg<SplitDefault>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, 4,
                                                                      lp_of(o), ws, 0);
                      }});
        vs.push_back({"x3   pack only", [&](float *o) {
                          return launch_split_pack(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0);
                      }});
        vs.push_back({"x3   pack only LDS", [&](float *o) {
                          return launch_split_pack(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0, true);
                      }});
        vs.push_back({"x3   pack only px4", [&](float *o) {
                          return launch_split_pack_px<4>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0);
                      }});
        vs.push_back({"x3   pack only px8", [&](float *o) {
                          return launch_split_pack_px<8>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0);
                      }});
        vs.push_back({"x3   pack only px16", [&](float *o) {
                          return launch_split_pack_px<16>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0);
                      }});
        {  // the register pack and the LDS pack must write identical bytes
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f1, fe, 7u, 3.0f);
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f2, fe, 8u, 0.01f);
            std::vector<char> h0(wsb), h1(wsb);
            CK(hipMemset(ws, 0, wsb));
            CK(launch_split_pack(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0, true));
            CK(hipMemcpy(h0.data(), ws, wsb, hipMemcpyDeviceToHost));
            CK(hipMemset(ws, 0, wsb));
            CK(launch_split_pack(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0, false));
            CK(hipMemcpy(h1.data(), ws, wsb, hipMemcpyDeviceToHost));
            printf("%-10s pack reg vs LDS: %s\n", sh.name, std::memcmp(h0.data(), h1.data(), wsb) ? "DIFFER" : "bit-identical");
            for (int nw : {4, 8, 16}) {
                CK(hipMemset(ws, 0, wsb));
                CK(nw == 4    ? launch_split_pack_px<4>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0)
                   : nw == 8 ? launch_split_pack_px<8>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0)
                             : launch_split_pack_px<16>(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0));
                CK(hipMemcpy(h1.data(), ws, wsb, hipMemcpyDeviceToHost));
                printf("%-10s pack px%d vs LDS: %s\n", sh.name, nw,
                       std::memcmp(h0.data(), h1.data(), wsb) ? "DIFFER" : "bit-identical");
            }
        }
        const size_t first_mfma = vs.size();
#define MF(name, ...)                                                                                     \
        vs.push_back({name, [&](float *o) {                                                               \
                          return launch_split_mfma_cfg<__VA_ARGS__>((int)N, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), \
                                                                    ws, 0);                               \
                      }});
        MF("mfma 2x2 MQ2 o2", SplitCfg<2, 2, 2, 2>)
        MF("mfma 2x2 MQ2 o1", SplitCfg<2, 2, 2, 1>)
        MF("mfma 4x2 MQ2 o1", SplitCfg<4, 2, 2, 1>)
        MF("mfma 4x1 MQ2 o2", SplitCfg<4, 1, 2, 2>)
        MF("mfma 2x1 MQ2 o2", SplitCfg<2, 1, 2, 2>)
        MF("mfma 2x2 MQ1 o3", SplitCfg<2, 2, 1, 3>)
#define RG(name, st, ...)                                                                                 \
        vs.push_back({name, [&](float *o) {                                                               \
                          return launch_split_ring_cfg<__VA_ARGS__, st>((int)N, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), \
                                                                    ws, 0);                               \
                      }});
        RG("ring 4x2 MQ2 s4", 4, SplitCfg<4, 2, 2, 1>)
        RG("ring 4x2 MQ2 s3", 3, SplitCfg<4, 2, 2, 1>)
        RG("ring 2x2 MQ2 s4", 4, SplitCfg<2, 2, 2, 1>)
        RG("ring 4x1 MQ2 s4", 4, SplitCfg<4, 1, 2, 1>)
        vs.push_back({"mfma 2x2 MQ2 o2 NOSTORE", [&](float *o) {
                          return launch_split_mfma_cfg<SplitCfg<2, 2, 2, 2>>((int)N, sh.B, sh.D, sh.H, sh.W, 0,
                                                                             lp_of(o), ws, 0);
                      }});
        // accuracy on several operand scales (the split build rescales per pixel)
        for (float sc : {1.0f, 1e-3f, 300.0f}) {
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f1, fe, 1u, sc);
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f2, fe, 2u, sc);
            if (argc > 3) {  // keep the reference + variants whose name contains argv[3]
            std::vector<Variant> keep{vs[0]};
            for (size_t k = 1; k < vs.size(); ++k)
                if (vs[k].name.find(argv[3]) != std::string::npos) keep.push_back(vs[k]);
            vs = keep;
        }
        CK(vs[0].launch(ref));
            for (size_t k = 1; k < vs.size(); ++k) {
                if (vs[k].name.find("only") != std::string::npos || vs[k].name.find("NOSTORE") != std::string::npos)
                    continue;  // no output
                CK(hipMemset(out, 0, tot * 4));
                CK(launch_split_pack(f1, (int)N, f2, sh.B, sh.D, sh.H, sh.W, ws, 0));
                CK(vs[k].launch(out));
                unsigned *d;
                unsigned hv[2] = {0, 0};
                CK(hipMalloc(&d, 8));
                CK(hipMemset(d, 0, 8));
                hipLaunchKernelGGL(maxdiff, dim3(2048), dim3(256), 0, 0, ref, out, tot, d, d + 1);
                CK(hipMemcpy(hv, d, 8, hipMemcpyDeviceToHost));
                CK(hipFree(d));
                float dm, rm;
                std::memcpy(&dm, &hv[0], 4);
                std::memcpy(&rm, &hv[1], 4);
                printf("%-10s scale %-6g %-24s max|x3-f32|/max|f32| = %.3e\n", sh.name, sc, vs[k].name.c_str(),
                       dm / rm);
            }
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
            printf("%-10s %-24s median %8.2f us  min %8.2f us  %7.1f TF/s (fp32-equivalent)\n", sh.name,
                   v.name.c_str(), med, v.us[0], flops / (med * 1e-6) / 1e12);
        }
        CK(hipFree(f1));
        CK(hipFree(f2));
        CK(hipFree(ref));
        CK(hipFree(out));
        CK(hipFree(ws));
    }
    return 0;
}
