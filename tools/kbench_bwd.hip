// kbench_bwd.hip — where lookup_bwd_fold_kernel (corr_lookup.hip) spends its time at the train
// shape (B8, 36x48, r4, L4, 12 lookups): the full kernel against probes that drop the lookup
// loop, the fold (dC + maxima), or the LDS zero-init (timing only; wrong results).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -o tools/_build/kbench_bwd tools/kbench_bwd.hip
//   ./kbench_bwd [rounds]
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

__global__ void fill_coords(float *c, int B, int H, int W, unsigned seed) {
    const int N = H * W;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * 2 * N; i += gridDim.x * blockDim.x) {
        const int n = i % N, axis = (i / N) % 2;
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        const float noise = ((x >> 8) * (1.0f / 16777216.0f) - 0.5f) * 6.0f;
        c[i] = (axis == 0 ? (float)(n % W) : (float)(n / W)) + noise;
    }
}

__global__ void fill_grid(float *c, int B, int H, int W) {  // the integer pixel grid (cold start)
    const int N = H * W;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * 2 * N; i += gridDim.x * blockDim.x) {
        const int n = i % N, axis = (i / N) % 2;
        c[i] = axis == 0 ? (float)(n % W) : (float)(n / W);
    }
}

__global__ void fill(float *p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        p[i] = ((x >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
    }
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    constexpr int S = 9, K = S * S, PER = 4;
    const int B = 8, H = 36, W = 48, L = 4, N = H * W, T = 12;
    using ST = FusedStage<S>;
    std::vector<float *> cs(T), gs(T);
    for (int t = 0; t < T; ++t) {
        CK(hipMalloc(&cs[t], (size_t)B * 2 * N * 4));
        CK(hipMalloc(&gs[t], (size_t)B * L * K * N * 4));
        hipLaunchKernelGGL(fill_coords, dim3(256), dim3(256), 0, 0, cs[t], B, H, W, 17u + t);
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, gs[t], (size_t)B * L * K * N, 101u + t);
    }
    const int G = (N + ST::BQ - 1) / ST::BQ;
    float *dc, *cpart;
    unsigned *rmax;
    CK(hipMalloc(&dc, (size_t)B * N * N * 4));
    CK(hipMalloc(&cpart, (size_t)B * G * N * 4));
    CK(hipMalloc(&rmax, (size_t)B * N * 4));
    BwdLookups lk{};
    for (int t = 0; t < T; ++t) lk.coords[t] = cs[t], lk.grad[t] = gs[t];
    FusedOut o{};
    o.dc = dc, o.rmax = rmax, o.cmax = nullptr, o.cpart = cpart;
    o.B = B, o.NQ = N, o.H = H, o.W = W, o.L = L;
    o.nfold = G * B;  // no appended row-maxima blocks
    const size_t bytes = fused_lds_bytes<S>(H, W, L, &o);
    printf("LDS %zu B per workgroup, %d workgroups\n", bytes, G * B);
    struct V {
        std::string name;
        std::function<void()> run;
        std::vector<float> us;
    };
    float *cgrid;
    CK(hipMalloc(&cgrid, (size_t)B * 2 * N * 4));
    hipLaunchKernelGGL(fill_grid, dim3(256), dim3(256), 0, 0, cgrid, B, H, W);
    // lds > bytes: the same kernel with its LDS padded, i.e. fewer workgroups per CU (the
    // occupancy sensitivity of the lookup loop)
    FusedOut onm = o;  // the bf16x6 backward's fold: dC only, no maxima
    onm.rmax = nullptr, onm.cpart = nullptr;
    FusedOut os = o;  // the separable kernel's LDS image (no per-wave staging)
    const size_t bytes_sep = fused_lds_bytes<S, true>(H, W, L, &os);
    FusedOut osnm = os;
    osnm.rmax = nullptr, osnm.cpart = nullptr;
    printf("separable: LDS %zu B per workgroup\n", bytes_sep);
    auto launch = [&](auto kern, int t_count, bool grid0 = false, size_t lds = 0, const FusedOut *oo = nullptr) {
        BwdLookups l2 = lk;
        l2.T = t_count;
        if (grid0) l2.coords[0] = cgrid;
        const size_t b = lds ? lds : bytes;
        CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b));
        hipLaunchKernelGGL(kern, dim3((unsigned)(G * B)), dim3(64 * kFusedLv), b, 0, l2, oo ? *oo : o);
    };
    std::vector<V> vs;
    vs.push_back({"full T=12", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 12); }, {}});
    vs.push_back({"full T=12, no maxima (bf16x6)", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 12, false, 0, &onm); }, {}});
    vs.push_back({"SEP full T=12, no maxima (bf16x6)", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 12, false, bytes_sep, &osnm); }, {}});
    vs.push_back({"SEP LEAN full T=12, no maxima (bf16x6)", [&] { launch(lookup_bwd_fold_kernel<S, 0, true, true>, 12, false, bytes_sep, &osnm); }, {}});
    vs.push_back({"SEP LEAN T=12, cold", [&] { launch(lookup_bwd_fold_kernel<S, 0, true, true>, 12, false, bytes_sep, &osnm); }, {}});
    vs.push_back({"LEAN fold only (no zero)", [&] { launch(lookup_bwd_fold_kernel<S, 5, true, true>, 12, false, bytes_sep, &osnm); }, {}});
    vs.push_back({"SEP full T=12", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 12, false, bytes_sep, &os); }, {}});
    vs.push_back({"SEP full T=12, LDS padded to 3 WG/CU", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 12, false, 52 * 1024, &os); }, {}});
    // "cold": the upstream gradients evicted from the MALL before each launch (a 512 MB memset in
    // between, outside the timed region)
    vs.push_back({"SEP full T=12, cold", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 12, false, bytes_sep, &os); }, {}});
    vs.push_back({"SEP full T=12, trailing LDS wait", [&] { launch(lookup_bwd_fold_kernel<S, 16, true>, 12, false, bytes_sep, &os); }, {}});
    vs.push_back({"SEP full T=12, lookup 0 on the integer grid", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 12, true, bytes_sep, &os); }, {}});
    vs.push_back({"SEP full T=1", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 1, false, bytes_sep, &os); }, {}});
    vs.push_back({"SEP full T=1 on the integer grid", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 1, true, bytes_sep, &os); }, {}});
    vs.push_back({"full T=12, no maxima, cached dC", [&] { launch(lookup_bwd_fold_kernel<S, 8>, 12, false, 0, &onm); }, {}});
    vs.push_back({"no lookups, no maxima", [&] { launch(lookup_bwd_fold_kernel<S, 1>, 12, false, 0, &onm); }, {}});
    vs.push_back({"no lookups, no maxima, cached dC", [&] { launch(lookup_bwd_fold_kernel<S, 9>, 12, false, 0, &onm); }, {}});
    vs.push_back({"full T=1", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 1); }, {}});
    vs.push_back({"full T=12, 2 WG/CU (LDS padded to 64 KB)", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 12, false, 64 * 1024); }, {}});
    vs.push_back({"full T=1, 2 WG/CU", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 1, false, 64 * 1024); }, {}});
    vs.push_back({"full T=12, 1 WG/CU (LDS padded to 96 KB)", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 12, false, 96 * 1024); }, {}});
    vs.push_back({"full T=1, 1 WG/CU", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 1, false, 96 * 1024); }, {}});
    vs.push_back({"full T=12, lookup 0 on the integer grid", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 12, true); }, {}});
    vs.push_back({"full T=1 on the integer grid", [&] { launch(lookup_bwd_fold_kernel<S, 0>, 1, true); }, {}});
    vs.push_back({"no lookups (zero + fold)", [&] { launch(lookup_bwd_fold_kernel<S, 1>, 12); }, {}});
    vs.push_back({"no fold T=12", [&] { launch(lookup_bwd_fold_kernel<S, 2>, 12); }, {}});
    vs.push_back({"zero-init only", [&] { launch(lookup_bwd_fold_kernel<S, 3>, 12); }, {}});
    vs.push_back({"fold only (no zero)", [&] { launch(lookup_bwd_fold_kernel<S, 5>, 12); }, {}});
    vs.push_back({"empty (no zero, no fold)", [&] { launch(lookup_bwd_fold_kernel<S, 7>, 12); }, {}});
    if (argc > 2) {  // time only the variant named exactly argv[2] (for PMC passes)
        std::vector<V> keep;
        for (auto &v : vs)
            if (v.name == argv[2]) keep.push_back(v);
        vs = keep;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto &v : vs) v.run();
    CK(hipDeviceSynchronize());
    void *flush;
    const size_t flush_bytes = 512ull << 20;
    CK(hipMalloc(&flush, flush_bytes));
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vs) {
            if (v.name.find("cold") != std::string::npos) {
                float tot = 0.f;
                for (int i = 0; i < PER; ++i) {
                    CK(hipMemsetAsync(flush, i + r, flush_bytes, 0));
                    CK(hipEventRecord(e0, 0));
                    v.run();
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    tot += ms;
                }
                v.us.push_back(tot * 1e3f / PER);
                continue;
            }
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < PER; ++i) v.run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3f / PER);
        }
    {  // the generic fold phase and the LEAN one: dC bit-identical
        std::vector<unsigned> ref((size_t)B * N * N), got((size_t)B * N * N);
        launch(lookup_bwd_fold_kernel<S, 0, true, true>, 12, false, bytes_sep, &osnm);
        CK(hipMemcpy(ref.data(), dc, ref.size() * 4, hipMemcpyDeviceToHost));
        auto cmp = [&](const char *nm, std::function<void()> run) {
            CK(hipMemset(dc, 0xff, ref.size() * 4));
            run();
            CK(hipMemcpy(got.data(), dc, got.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < ref.size(); ++i) bad += ref[i] != got[i];
            printf("check %-28s vs LEAN: %s (%zu mismatches)\n", nm, bad ? "DIFFER" : "bit-identical", bad);
        };
        cmp("generic fold (SEP, no maxima)", [&] { launch(lookup_bwd_fold_kernel<S, 0, true>, 12, false, bytes_sep, &osnm); });
    }
    for (auto &v : vs) {
        std::sort(v.us.begin(), v.us.end());
        printf("%-42s median %8.2f us  min %8.2f us\n", v.name.c_str(), v.us[v.us.size() / 2], v.us[0]);
    }
    return 0;
}
