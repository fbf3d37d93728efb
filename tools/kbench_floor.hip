// kbench_floor.hip — the per-launch floor on this box: back-to-back launches of trivial
// kernels on one stream (eager and captured in a hipGraph), timed with HIP events.  Tells how
// much of a few-microsecond kernel (the DSEC lookup, the operand pack) is launch + completion
// overhead rather than its own work.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/_build/kbench_floor tools/kbench_floor.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__global__ void k_empty(float *) {}

__global__ void k_store(float *p) { p[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = 1.0f; }

// one dependent load -> store per thread (the lookup's minimal round trip)
__global__ void k_load_store(float *p) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    p[i + (1u << 22)] = p[i] + 1.0f;
}

// two dependent round trips (coords -> address -> window), like the lookup
__global__ void k_two_trips(float *p) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int j = (int)p[i] & 1023;
    p[i + (1u << 22)] = p[(1u << 21) + i + j] + 1.0f;
}

int main() {
    float *buf;
    CK(hipMalloc(&buf, 64ull << 20));
    CK(hipMemset(buf, 0, 64ull << 20));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    struct K {
        const char *name;
        void (*f)(float *);
    } ks[] = {{"empty", k_empty}, {"store", k_store}, {"load->store", k_load_store}, {"2 round trips", k_two_trips}};
    const int grids[] = {1, 256, 600, 2400};
    const int REP = 20;
    for (const K &k : ks)
        for (int g : grids)
            for (int graph = 0; graph < 2; ++graph) {
                hipGraphExec_t ge = nullptr;
                if (graph) {
                    hipGraph_t gr;
                    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                    for (int r = 0; r < REP; ++r) hipLaunchKernelGGL(k.f, dim3(g), dim3(320), 0, s, buf);
                    CK(hipStreamEndCapture(s, &gr));
                    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
                    CK(hipGraphDestroy(gr));
                }
                std::vector<float> us;
                for (int it = 0; it < 12; ++it) {
                    CK(hipEventRecord(a, s));
                    if (graph)
                        CK(hipGraphLaunch(ge, s));
                    else
                        for (int r = 0; r < REP; ++r) hipLaunchKernelGGL(k.f, dim3(g), dim3(320), 0, s, buf);
                    CK(hipEventRecord(z, s));
                    CK(hipEventSynchronize(z));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, z));
                    if (it >= 2) us.push_back(ms * 1e3f / REP);
                }
                std::sort(us.begin(), us.end());
                printf("%-14s grid %5d x 320  %-6s  per launch median %6.2f us  min %6.2f us\n", k.name, g,
                       graph ? "graph" : "eager", us[us.size() / 2], us[0]);
                if (ge) CK(hipGraphExecDestroy(ge));
            }
    CK(hipFree(buf));
    return 0;
}
