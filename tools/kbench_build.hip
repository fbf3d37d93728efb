// kbench_build.hip — the f16x3 build (corr_build_split.hip) against the exact-fp32 MFMA build
// (corr_build.hip), and variants of the MFMA kernel (tile order, fragment pipelining):
//   * accuracy: max |x - f32| / max |f32| over every pyramid level, three operand scales;
//   * pooling: levels 1-3 bit-identical to avg_pool2d of the kernel's own level 0 (host check);
//   * timing: interleaved rounds of every variant in one process, random data (HIP events
//     around PER back-to-back launches; cdna_hip_programming.md §5.4 rule 24).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -o tools/_build/kbench_build tools/kbench_build.hip
//   ./kbench_build [rounds] [shape]
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../e-raft_amd/csrc/corr_build.hip"
#include "../e-raft_amd/csrc/corr_build_split.hip"
#include "../e-raft_amd/csrc/corr_build_bf16.hip"

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
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
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
    bool has_output;
    std::vector<float> us;
};

static float pool_host(float a, float b, float c, float d) {
    volatile float t = a + b;
    t = t + c;
    t = t + d;
    return t * 0.25f;
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 20;
    const char *only = argc > 2 ? argv[2] : nullptr;
    const char *vfilter = argc > 3 ? argv[3] : nullptr;  // time only variants containing this
    constexpr int PER = 4;
    std::vector<Shape> shapes = {{"dsec", 1, 256, 60, 80},     {"mvsec-pad", 16, 256, 36, 44},
                                 {"mvsec-crop", 16, 256, 32, 32}, {"train", 8, 256, 36, 48},
                                 {"odd", 2, 200, 17, 23},      {"1280x960", 1, 256, 120, 160},
                                 {"1920x1280", 1, 256, 160, 240}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Shape &sh : shapes) {
        if (only && strcmp(only, "all") && strcmp(only, sh.name)) continue;
        const size_t N = (size_t)sh.H * sh.W, BN = (size_t)sh.B * N;
        size_t off[4], cnt[4], tot = 0;
        for (int l = 0; l < 4; ++l) {
            off[l] = tot;
            cnt[l] = BN * map_floats(sh.H >> l, sh.W >> l);  // the tiled pyramid (corr_common.h)
            tot += cnt[l];
        }
        const size_t fe = (size_t)sh.B * sh.D * N;
        float *f1, *f2, *ref, *out;
        void *ws, *wsbf;
        const size_t wsb = build_split_workspace(sh.B, sh.D, (int)N, sh.H, sh.W);
        const size_t wsbfb = build_bf16_workspace(sh.B, sh.D, (int)N, sh.H, sh.W);
        CK(hipMalloc(&wsbf, wsbfb));
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
        const int NQ = (int)N;
        std::vector<Variant> vs;
        vs.push_back({"f32 build (corr_build.hip)", [&](float *o) {
                          return launch_build_cfg<BuildDefault>(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), 0);
                      }, true});
        vs.push_back({"f32 noskip occ3", [&](float *o) {
                          return launch_build_cfg<BuildCfg<2, 2, 2, 8, 3, true, false>>(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), 0);
                      }, true});
        vs.push_back({"f32 skip occ4 (round-2 default)", [&](float *o) {
                          return launch_build_cfg<BuildCfg<2, 2, 2, 8, 4, true, true>>(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), 0);
                      }, true});
        vs.push_back({"f32 element level-1/2 stores", [&](float *o) {
                          return launch_build_cfg<BuildDefault>(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), 0, false);
                      }, true});
        vs.push_back({"f32 level 0 only", [&](float *o) {
                          return launch_build_cfg<BuildDefault>(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 1, lp_of(o), 0);
                      }, false});
        vs.push_back({"f32 default NOSTORE", [&](float *o) {
                          return launch_build_cfg<BuildCfg<2, 2, 2, 8, 4, true, false, true>>(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), 0);
                      }, false});
        vs.push_back({"bf16x6 pack+mfma", [&](float *o) {
                          return launch_build_bf16(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), wsbf, 0, 0);
                      }, true});
        vs.push_back({"bf16x6 pack only", [&](float *o) {
                          return launch_build_bf16(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), wsbf, 0, 1);
                      }, false});
        for (int rpw : {1, 2, 4})
            vs.push_back({"bf16x6 pack only rpw" + std::to_string(rpw), [&, rpw](float *) {
                              return bf16b::launch_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, wsbf, 0, 0, -1, true, rpw);
                          }, false});
        vs.push_back({"bf16x6 mfma only", [&](float *o) {
                          return launch_build_bf16(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), wsbf, 0, 2);
                      }, false});
        vs.push_back({"bf16x6 mfma tchain", [&](float *o) {
                          return bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), wsbf, 0, 1);
                      }, false});
        vs.push_back({"bf16x6 mfma tchain NOSTORE", [&](float *o) {
                          return bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 0, lp_of(o), wsbf, 0, 1);
                      }, false});
        for (int vv : {2, 3, 5}) {
            const char *nm[] = {"", "", "bf16x6 mfma hiddenQ", "bf16x6 mfma prio", "bf16x6 mfma hiddenQ+prio", "bf16x6 mfma no half path"};
            vs.push_back({nm[vv], [&, vv](float *o) {
                              return bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), wsbf, 0, vv);
                          }, false});
        }
        vs.push_back({"bf16x6 mfma order2 (XCD blocks)", [&](float *o) {
                          return bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), wsbf, 0, 0, 2);
                      }, false});
        for (int od : {0, 1})
            for (int gq : {4, 8, 16, 32}) {
                vs.push_back({"bf16x6 mfma order" + std::to_string(od) + " gq" + std::to_string(gq), [&, od, gq](float *o) {
                                  return bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), wsbf, 0, 0, od, 0, -1, gq);
                              }, false});
            }
        vs.push_back({"bf16x6 mfma NOSTORE", [&](float *o) {
                          return launch_build_bf16(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 0, lp_of(o), wsbf, 0, 2);
                      }, false});
        vs.push_back({"x3 pack+mfma", [&](float *o) {
                          return launch_build_split(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0);
                      }, true});
        vs.push_back({"x3 pack only", [&](float *) {
                          return launch_split_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, ws, 0);
                      }, false});
        vs.push_back({"x3 pack only px64", [&](float *) {
                          return launch_split_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, ws, 0, 64);
                      }, false});
        vs.push_back({"x3 mfma 1-tile order0", [&](float *o) {
                          return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0, true, 0, 0);
                      }, false});
        vs.push_back({"x3 mfma 1-tile NOSTORE", [&](float *o) {
                          return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 0, lp_of(o), ws, 0);
                      }, false});
        vs.push_back({"x3 mfma 1-tile order1", [&](float *o) {
                          return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0, true, 0, 1);
                      }, false});
        vs.push_back({"x3 mfma 1-tile no half path", [&](float *o) {
                          return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0, true, 2);
                      }, false});
        vs.push_back({"x3 mfma 1-tile nopipe (206 VGPR)", [&](float *o) {
                          return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0, true, 1);
                      }, false});
        for (float sc : {1.0f, 1e-3f, 300.0f}) {
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f1, fe, 1u, sc);
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, f2, fe, 2u, sc);
            CK(vs[0].launch(ref));
            for (size_t k = 1; k < vs.size(); ++k) {
                if (!vs[k].has_output) continue;
                CK(hipMemset(out, 0xff, tot * 4));
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
                printf("%-10s scale %-6g %-28s max|x-f32|/max|f32| = %.3e\n", sh.name, sc, vs[k].name.c_str(), dm / rm);
            }
        }
        // mismatching words over the real cells of every level (the tiled maps' padding cells are
        // anything: the builds may write them or not)
        auto count_bad = [&](const std::vector<unsigned> &ha, const std::vector<unsigned> &hb) {
            size_t bad = 0;
            for (int l = 0; l < 4; ++l) {
                const int Hl = sh.H >> l, Wl = sh.W >> l, TC = map_tcols(Wl);
                const size_t mf = map_floats(Hl, Wl);
                for (size_t i = off[l]; i < off[l] + cnt[l]; ++i) {
                    const size_t m = (i - off[l]) % mf, t = m / 16, e = m % 16;
                    const int y = (int)(t / TC) * 4 + (int)(e / 4), x = (int)(t % TC) * 4 + (int)(e % 4);
                    if (y < Hl && x < Wl) bad += ha[i] != hb[i];
                }
            }
            return bad;
        };
        {  // kernel variants against the one-tile-per-workgroup kernel (level-1/2 element stores): every level bitwise
            auto same = [&](const char *what, std::function<hipError_t(float *)> fa) {
                CK(launch_split_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, ws, 0));
                CK(hipMemset(out, 0xff, tot * 4));
                CK(hipMemset(ref, 0x7f, tot * 4));
                CK(fa(out));
                CK(launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(ref), ws, 0, false));
                std::vector<unsigned> ha(tot), hb(tot);
                CK(hipMemcpy(ha.data(), out, tot * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hb.data(), ref, tot * 4, hipMemcpyDeviceToHost));
                const size_t bad = count_bad(ha, hb);
                printf("%-10s %s vs 1-tile element stores, all levels: %s (%zu mismatches)\n", sh.name, what,
                       bad ? "DIFFER" : "bit-identical", bad);
            };
            same("16-B level 1/2 stores", [&](float *o) { return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0); });
            same("1-tile order0", [&](float *o) { return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0, true, 0, 0); });
            same("1-tile no half path", [&](float *o) { return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0, true, 2); });
            same("1-tile nopipe", [&](float *o) { return launch_split_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(o), ws, 0, true, 1); });
            if (sh.D == 256) {
                for (int vv : {2, 3, 5, 9, 10, 11}) {  // bf16x6 variants vs the default bf16x6 kernel (9: tile order 2; 10: order 0 gq 16; 11: order 1 gq 32)
                    CK(launch_build_bf16(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(ref), wsbf, 0, 0));
                    CK(hipMemset(out, 0xff, tot * 4));
                    CK(vv == 9    ? bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(out), wsbf, 0, 0, 2)
                       : vv == 10 ? bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(out), wsbf, 0, 0, 0, 0, -1, 16)
                       : vv == 11 ? bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(out), wsbf, 0, 0, 1, 0, -1, 32)
                                  : bf16b::launch_mfma(NQ, sh.B, sh.D, sh.H, sh.W, 4, lp_of(out), wsbf, 0, vv));
                    std::vector<unsigned> ha(tot), hb(tot);
                    CK(hipMemcpy(ha.data(), out, tot * 4, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(hb.data(), ref, tot * 4, hipMemcpyDeviceToHost));
                    const size_t bad = count_bad(ha, hb);
                    printf("%-10s bf16x6 variant %d vs default, all levels: %s (%zu mismatches)\n", sh.name, vv,
                           bad ? "DIFFER" : "bit-identical", bad);
                }
            }

        }
        {  // bf16x6 pack with 2 / 4 records per wave: byte-identical workspaces
            void *w2;
            CK(hipMalloc(&w2, wsbfb));
            for (int rpw : {2, 4}) {
                CK(hipMemset(wsbf, 0, wsbfb));
                CK(hipMemset(w2, 0, wsbfb));
                CK(bf16b::launch_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, wsbf, 0, 0, -1, true, 1));
                CK(bf16b::launch_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, w2, 0, 0, -1, true, rpw));
                std::vector<unsigned char> ha(wsbfb), hb(wsbfb);
                CK(hipMemcpy(ha.data(), wsbf, wsbfb, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hb.data(), w2, wsbfb, hipMemcpyDeviceToHost));
                printf("%-10s bf16x6 pack rpw%d vs default: %s\n", sh.name, rpw, ha == hb ? "byte-identical" : "DIFFER");
            }
            CK(hipFree(w2));
        }
        {  // pack variants: byte-identical workspaces
            void *ws2;
            CK(hipMalloc(&ws2, wsb));
            for (int px : {64}) {
                CK(hipMemset(ws, 0, wsb));
                CK(hipMemset(ws2, 0, wsb));
                CK(launch_split_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, ws, 0));
                CK(launch_split_pack(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, ws2, 0, px));
                std::vector<unsigned char> ha(wsb), hb(wsb);
                CK(hipMemcpy(ha.data(), ws, wsb, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hb.data(), ws2, wsb, hipMemcpyDeviceToHost));
                printf("%-10s pack px%d vs default: %s\n", sh.name, px, ha == hb ? "byte-identical" : "DIFFER");
            }
            CK(hipFree(ws2));
        }
        for (int which = 0; which < 2; ++which) {  // pooling: every level bit-identical to avg_pool2d of its own level 0
            if (which == 0) CK(launch_build_split(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(out), ws, 0));
            else CK(launch_build_bf16(f1, NQ, f2, sh.B, sh.D, sh.H, sh.W, 4, lp_of(out), wsbf, 0, 0));
            std::vector<float> h(tot);
            CK(hipMemcpy(h.data(), out, tot * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (int l = 1; l < 4; ++l) {
                const int Wp = sh.W >> (l - 1), Hl = sh.H >> l, Wl = sh.W >> l;
                const int TP = map_tcols(Wp), TL = map_tcols(Wl);
                const size_t MP = map_floats(sh.H >> (l - 1), Wp), ML = map_floats(Hl, Wl);
                const float *P = h.data() + off[l - 1], *C = h.data() + off[l];
                for (size_t q = 0; q < BN; ++q)
                    for (int y = 0; y < Hl; ++y)
                        for (int x = 0; x < Wl; ++x) {
                            const float *a = P + q * MP;
                            const float e = pool_host(a[map_cell(2 * y, 2 * x, TP)], a[map_cell(2 * y, 2 * x + 1, TP)],
                                                      a[map_cell(2 * y + 1, 2 * x, TP)],
                                                      a[map_cell(2 * y + 1, 2 * x + 1, TP)]);
                            const float g = C[q * ML + map_cell(y, x, TL)];
                            if (std::memcmp(&e, &g, 4)) ++bad;
                        }
            }
            printf("%-10s %s pooling levels 1-3 vs own level 0: %s (%zu mismatches)\n", sh.name, which ? "bf16x6" : "x3",
                   bad ? "DIFFER" : "bit-identical", bad);
        }
        if (vfilter) {
            std::vector<Variant> keep;
            for (auto &v : vs)
                if (v.name.find(vfilter) != std::string::npos) keep.push_back(v);
            vs = keep;
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
            printf("%-10s %-28s median %8.2f us  min %8.2f us  %7.1f TF/s fp32-equiv  %6.3f of 2.5 PF (x3)  %6.3f (x6)\n",
                   sh.name, v.name.c_str(), med, v.us[0], flops / (med * 1e-6) / 1e12,
                   3.0 * flops / (med * 1e-6) / 2.5e15, 6.0 * flops / (med * 1e-6) / 2.5e15);
        }
        fflush(stdout);
        CK(hipFree(f1));
        CK(hipFree(f2));
        CK(hipFree(ref));
        CK(hipFree(out));
        CK(hipFree(ws));
        CK(hipFree(wsbf));
    }
    return 0;
}
