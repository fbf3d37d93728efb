// kbench_gemm.hip — the backward split GEMMs (corr_bwd_split.hip) at the train shape (B 8,
// D 256, 36x48): dF1 = F2 dC^T (row operands) and dF2 = F1 dC (dC columns), each with its
// split-K reduce, for several split counts, register-staged vs LDS-DMA operand ring (HIP events
// around back-to-back launches; results against the register-staged plan, which must match bitwise).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -o tools/_build/kbench_gemm tools/kbench_gemm.hip \
//         e-raft_amd/csrc/corr_bwd.hip e-raft_amd/csrc/corr_build.hip e-raft_amd/csrc/corr_lookup.hip
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../e-raft_amd/csrc/corr_bwd_split.hip"

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
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        p[i] = ((x >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
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

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    const int B = 8, D = 256, H = 36, W = 48, N = H * W, NQ = N;
    float *f1, *f2, *dc, *o1, *o2, *r1, *r2, *b1, *b2;
    CK(hipMalloc(&f1, (size_t)B * D * N * 4));
    CK(hipMalloc(&f2, (size_t)B * D * N * 4));
    CK(hipMalloc(&dc, (size_t)B * NQ * N * 4));
    CK(hipMalloc(&o1, (size_t)B * D * N * 4));
    CK(hipMalloc(&o2, (size_t)B * D * N * 4));
    CK(hipMalloc(&r1, (size_t)B * D * N * 4));
    CK(hipMalloc(&r2, (size_t)B * D * N * 4));
    CK(hipMalloc(&b1, (size_t)B * D * N * 4));
    CK(hipMalloc(&b2, (size_t)B * D * N * 4));
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f1, (size_t)B * D * N, 1u);
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f2, (size_t)B * D * N, 2u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, dc, (size_t)B * NQ * N, 3u);
    GemmTune big;
    big.splits = 16;  // the largest slab the variants need
    const size_t wsb = bwd_split_workspace_tuned(B, D, NQ, H, W, big);
    void *ws;
    CK(hipMalloc(&ws, wsb));
    const BwdWs w = carve(ws, B, D, NQ, N);
    CK(hipMemset(w.mx0, 0, w.mx_bytes));
    CK(absmax(dc, B, NQ, N, w.mxB, w.mxC, 0));
    CK(rowmax2(f2, N, w.mxA, f1, NQ, w.mxA2, B, D, 0));
    const float sD = 16.0f;
    // bf: the bf16x6 GEMMs (exact three-piece split, six products), checked against their own
    // register-staged plan
    auto g1 = [&](float *out, const GemmTune &t, bool bf = false) {
        return gemm_f32<false>(f2, (long)D * N, N, dc, (long)NQ * N, N, 1, w.mxA, w.mxB, B, D, NQ, N, sD, out, w.slab, 0, t,
                               bf);
    };
    auto g2 = [&](float *out, const GemmTune &t, bool bf = false) {
        return gemm_f32<true>(f1, (long)D * NQ, NQ, dc, (long)NQ * N, 1, N, w.mxA2, w.mxC, B, D, N, NQ, sD, out, w.slab, 0, t,
                              bf);
    };
    GemmTune ref;  // reference: register-staged, 128-row tiles, scalar reduce
    ref.dma = false, ref.wide = false, ref.reduce_vec4 = false;
    CK(g1(r1, ref));
    CK(g2(r2, ref));
    CK(g1(b1, ref, true));
    CK(g2(b2, ref, true));
    struct V {
        std::string name;
        std::function<hipError_t()> run;
        float *out, *ref;
        std::vector<float> us;
    };
    std::vector<V> vs;
    for (int cfg : {0, 1, 2}) {  // 128x256; 256x256; 256x256 with the split under the MFMAs
        const std::string tag = std::string("DMA mix splits plan, ") +
                                (cfg == 0 ? "128x256 tiles" : cfg == 1 ? "256x256 tiles (8 waves)" : "256x256 pipelined");
        GemmTune t;
        t.wide = cfg >= 1;
        t.pipe = cfg == 2;
        vs.push_back({"dF1 (rows) " + tag, [&, t] { return g1(o1, t); }, o1, r1, {}});
        vs.push_back({"dF2 (cols) " + tag, [&, t] { return g2(o2, t); }, o2, r2, {}});
    }
    for (int cfg : {1, 2}) {
        const std::string tag = std::string("bf16x6 ") + (cfg == 1 ? "256x256 tiles" : "256x256 pipelined");
        GemmTune t;
        t.pipe = cfg == 2;
        vs.push_back({"dF1 (rows) " + tag, [&, t] { return g1(o1, t, true); }, o1, b1, {}});
        vs.push_back({"dF2 (cols) " + tag, [&, t] { return g2(o2, t, true); }, o2, b2, {}});
    }
    for (int cfg : {0, 1}) {  // L2-cached epilogue stores (the default is non-temporal)
        GemmTune t;
        t.nt = false;
        const std::string tag = cfg ? "bf16x6 pipelined cached slabs" : "f16x3 pipelined cached slabs";
        vs.push_back({"dF1 (rows) " + tag, [&, t, cfg] { return g1(o1, t, cfg == 1); }, o1, cfg ? b1 : r1, {}});
        vs.push_back({"dF2 (cols) " + tag, [&, t, cfg] { return g2(o2, t, cfg == 1); }, o2, cfg ? b2 : r2, {}});
    }
    for (int sp : {4, 6, 8, 12}) {  // bf16x6 split-K counts (the plan's is 4 at this shape)
        GemmTune t;
        t.pipe = false;
        t.splits = sp;
        const std::string tag = "bf16x6 256x256 splits " + std::to_string(sp);
        vs.push_back({"dF1 (rows) " + tag, [&, t] { return g1(o1, t, true); }, o1, b1, {}});
        vs.push_back({"dF2 (cols) " + tag, [&, t] { return g2(o2, t, true); }, o2, b2, {}});
    }
    vs.push_back({"bf16x6 ref vs f16x3 ref dF1", [&] { return g1(o1, ref, true); }, o1, r1, {}});
    vs.push_back({"bf16x6 ref vs f16x3 ref dF2", [&] { return g2(o2, ref, true); }, o2, r2, {}});
    if (argc > 2) {  // only the variant named exactly argv[2] (PMC passes)
        std::vector<V> keep;
        for (auto &v : vs)
            if (v.name == argv[2]) keep.push_back(v);
        vs = keep;
    }
    for (auto &v : vs) {
        CK(v.run());
        unsigned *d;
        unsigned hv[2] = {0, 0};
        CK(hipMalloc(&d, 8));
        CK(hipMemset(d, 0, 8));
        hipLaunchKernelGGL(maxdiff, dim3(2048), dim3(256), 0, 0, v.ref, v.out, (size_t)B * D * N, d, d + 1);
        CK(hipMemcpy(hv, d, 8, hipMemcpyDeviceToHost));
        CK(hipFree(d));
        float dm, rm;
        std::memcpy(&dm, &hv[0], 4);
        std::memcpy(&rm, &hv[1], 4);
        printf("%-32s max|x - reg cvt plan| / max|ref| = %.3e\n", v.name.c_str(), dm / rm);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    constexpr int PER = 4;
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vs) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < PER; ++i) CK(v.run());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3f / PER);
        }
    const double fl = 2.0 * B * (double)D * N * NQ;
    for (auto &v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const float med = v.us[v.us.size() / 2];
        const bool bf = v.name.find("bf16x6") != std::string::npos;
        printf("%-32s median %8.2f us  min %8.2f us  %6.3f of 2.5 PF %s\n", v.name.c_str(), med, v.us[0],
               (bf ? 6.0 : 3.0) * fl / (med * 1e-6) / 2.5e15, bf ? "bf16 pipe (x6)" : "f16 pipe (x3)");
    }
    return 0;
}
