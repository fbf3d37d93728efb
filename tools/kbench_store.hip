// kbench_store.hip — store-path microbenchmark for the build's pyramid write pattern (no
// MFMA): how fast can 768 resident workgroups write the level-0 volume [NQ][H][W] fp32 when
// each 16-B-per-lane store instruction covers Q queries x (1024/Q) contiguous bytes?
//   Q = 16: the build's pattern (16 queries x one 64-B row segment of a 16-column patch)
//   Q = 8, 4, 2, 1: fewer queries, longer contiguous runs per instruction (layout experiments)
// Every variant writes exactly the same bytes once (the whole volume).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o tools/_build/kbench_store tools/kbench_store.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Tile = 128 queries x (PR rows x PC columns) targets, PR * PC = 128; a wave owns 32 queries.
// Lane l of a wave: the store instruction k writes query (Q-group) + contiguous run.
// Generic form: per wave 32 queries x 128 targets = 16 KB = 16 store instructions of 1 KB.
// Instruction k, lane l: query qa = 32 w + (k * 64 + l) / (128 / 4) ... expressed as
// (query, target offset) with T contiguous targets per query per instruction (T = 256 / Q).
template <int PC>
__global__ __launch_bounds__(256) void store_kernel(float *out, int NQ, int H, int W, int ntile, int npc, int Q, int order) {
    constexpr int PR = 128 / PC;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nqg = (NQ + 127) / 128;
    for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
        int qg, py, pc;
        if (order == 0) {  // query group fastest (groups of 8), then patch
            const int np = ntile / nqg;
            const int g = t / (8 * np), r2 = t % (8 * np);
            const int gm = std::min(8, nqg - g * 8);
            const int patch = r2 / gm;
            qg = g * 8 + r2 % gm;
            py = patch / npc, pc = patch % npc;
        } else {  // patch column fastest
            qg = t / (ntile / nqg);
            const int patch = t % (ntile / nqg);
            py = patch / npc, pc = patch % npc;
        }
        const int y0 = py * PR, x0 = pc * PC;
        // 16 instructions per wave; each covers Q queries x (256 / Q) floats of contiguous
        // row segments (runs of up to PC floats, then the next row)
        const int T = 256 / Q;  // floats per query per instruction
        for (int k = 0; k < 16; ++k) {
            const int runs = 128 / T;                 // row segments per query in the patch
            const int qgrp = k / runs, tb = k % runs;  // instruction k: queries qgrp*Q.., segment tb
            const int q = qgrp * Q + lane / (T / 4);
            const int tgt = tb * T + (lane % (T / 4)) * 4;
            const int y = y0 + tgt / PC, x = x0 + tgt % PC;
            const int qq = qg * 128 + 32 * w + q;
            const f32x4 v = f32x4{(float)k, (float)lane, 1.f, 2.f};
            if (qq < NQ && y < H && x < W) *reinterpret_cast<f32x4 *>(out + ((size_t)qq * H + y) * W + x) = v;
        }
    }
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    struct Sh { const char *n; int H, W; } shapes[] = {{"dsec", 60, 80}, {"1280x960", 120, 160}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto sh : shapes) {
        const int NQ = sh.H * sh.W;
        const size_t bytes = (size_t)NQ * sh.H * sh.W * 4;
        float *out;
        CK(hipMalloc(&out, bytes));
        struct V { int pc, q, order, grid; };
        std::vector<V> vs = {{16, 16, 0, 768}, {16, 16, 1, 768}, {32, 8, 0, 768}, {32, 8, 1, 768}, {64, 4, 1, 768},
                             {128, 2, 1, 768}, {16, 16, 0, 4096}};
        for (auto v : vs) {
            const int PR = 128 / v.pc;
            const int npr = (sh.H + PR - 1) / PR, npc = (sh.W + v.pc - 1) / v.pc;
            const int ntile = npr * npc * ((NQ + 127) / 128);
            auto go = [&]() {
                switch (v.pc) {
                    case 16: hipLaunchKernelGGL(store_kernel<16>, dim3(v.grid), dim3(256), 0, 0, out, NQ, sh.H, sh.W, ntile, npc, v.q, v.order); break;
                    case 32: hipLaunchKernelGGL(store_kernel<32>, dim3(v.grid), dim3(256), 0, 0, out, NQ, sh.H, sh.W, ntile, npc, v.q, v.order); break;
                    case 64: hipLaunchKernelGGL(store_kernel<64>, dim3(v.grid), dim3(256), 0, 0, out, NQ, sh.H, sh.W, ntile, npc, v.q, v.order); break;
                    default: hipLaunchKernelGGL(store_kernel<128>, dim3(v.grid), dim3(256), 0, 0, out, NQ, sh.H, sh.W, ntile, npc, v.q, v.order); break;
                }
            };
            go();
            CK(hipDeviceSynchronize());
            std::vector<float> us;
            for (int r = 0; r < rounds; ++r) {
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < 4; ++i) go();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                us.push_back(ms * 250.f);
            }
            std::sort(us.begin(), us.end());
            printf("%-9s patch %3dx%-3d Q=%2d (%4d B runs) order %d grid %4d: median %8.1f us  %6.2f TB/s\n", sh.n, PR, v.pc, v.q,
                   1024 / v.q, v.order, v.grid, us[us.size() / 2], bytes / (us[us.size() / 2] * 1e-6) / 1e12);
        }
        CK(hipFree(out));
    }
    return 0;
}
