// kbench_fetchcal.hip — calibrates rocprofv3's FETCH_SIZE on gfx950 for the access widths this
// repo's kernels use (MI355X_MICROARCH.md: the x2 correction is established for 16-B/lane
// streaming reads only; other widths must be calibrated on a known byte count).  Three
// read-only kernels over a 1 GiB buffer (far beyond L2 and the 256 MiB MALL):
//   stream16  16 B per lane, coalesced, every byte once
//   stream4   4 B per lane, coalesced, every byte once
//   gather44  the lookup's window pattern: 11-float (44-B) row segments at random float offsets,
//             one 16-lane group per segment; the host counts the distinct 32/64/128-B lines
//             the segments touch.
//   gatherwin the tiled lookup's window pattern (corr_common.h map_cell, round 5): one 10 x 10
//             window per 32 x 40-cell map stored as 64-B tiles of 4 x 4 cells, gathered as one
//             16-B tile-row chunk per lane (window rows x tile columns), as lookup_kernel does;
//             the host counts the distinct 16-B chunks and 64/128-B lines.
// Run:  rocprofv3 --pmc FETCH_SIZE -d <dir> -o run --output-format csv -- tools/_build/kbench_fetchcal
// and divide each kernel's FETCH_SIZE (KiB) by the byte counts printed here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <unordered_set>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__global__ void stream16(const float4 *__restrict__ p, size_t n4, float *__restrict__ sink) {
    float a = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        a += v.x + v.y + v.z + v.w;
    }
    if (a == 1234.5f) sink[threadIdx.x] = a;  // never: keeps the loads, writes nothing
}

__global__ void stream4(const float *__restrict__ p, size_t n, float *__restrict__ sink) {
    float a = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a += p[i];
    if (a == 1234.5f) sink[threadIdx.x] = a;
}

// 4 segments per wave (16 lanes each, lanes 0..10 load); segment s starts at float offset st[s]
__global__ void gather44(const float *__restrict__ p, const unsigned *__restrict__ st, int nseg,
                         float *__restrict__ sink) {
    const int lane = threadIdx.x & 15;
    float a = 0.f;
    for (int s = (blockIdx.x * blockDim.x + threadIdx.x) >> 4; s < nseg; s += (gridDim.x * blockDim.x) >> 4)
        if (lane < 11) a += p[(size_t)st[s] + lane];
    if (a == 1234.5f) sink[threadIdx.x] = a;
}

// Tiled maps of 32 x 40 cells (8 tile rows x 10 tile columns of 64 B = 5120 B); window w at cell
// (wy[w], wx[w]) of map w, one wave per window, lane = (window row rr < 10, chunk column tc < 4).
constexpr int kMapH = 32, kMapW = 40, kTC = kMapW / 4, kMapFloats = kMapH * kMapW;
__global__ void gatherwin(const float4 *__restrict__ p, const unsigned short *__restrict__ wyx, int nwin,
                          float *__restrict__ sink) {
    const int lane = threadIdx.x & 63, rr = lane >> 2, tc = lane & 3;
    float a = 0.f;
    for (int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nwin; w += (gridDim.x * blockDim.x) >> 6) {
        const int y0 = wyx[2 * w], x0 = wyx[2 * w + 1], y = y0 + rr, t = (x0 >> 2) + tc;
        if (rr < 10 && 4 * t <= x0 + 9) {
            const size_t f = (size_t)w * kMapFloats + (((y >> 2) * kTC + t) * 4 + (y & 3)) * 4;
            const float4 v = p[f / 4];
            a += v.x + v.y + v.z + v.w;
        }
    }
    if (a == 1234.5f) sink[threadIdx.x] = a;
}

int main() {
    const size_t bytes = (size_t)1 << 30, n = bytes / 4;
    float *buf, *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(buf, 0, bytes));
    const int nseg = 4 << 20;  // 4M segments: 176 MiB of useful bytes
    std::vector<unsigned> st(nseg);
    unsigned x = 12345u;
    for (int i = 0; i < nseg; ++i) {
        x = x * 1664525u + 1013904223u;
        st[i] = (unsigned)(((unsigned long long)x * (n - 16)) >> 32);
    }
    size_t lines[3] = {0, 0, 0};
    const int gran[3] = {32, 64, 128};
    for (int g = 0; g < 3; ++g) {
        std::unordered_set<unsigned long long> seen;
        seen.reserve((size_t)nseg * 3);
        for (int i = 0; i < nseg; ++i) {
            const unsigned long long b0 = (unsigned long long)st[i] * 4, b1 = b0 + 43;
            for (unsigned long long l = b0 / gran[g]; l <= b1 / gran[g]; ++l) seen.insert(l);
        }
        lines[g] = seen.size() * gran[g];
    }
    const int nwin = (int)(bytes / (kMapFloats * 4));
    std::vector<unsigned short> wyx(2 * (size_t)nwin);
    size_t wchunks = 0, wl64 = 0, wl128 = 0;
    for (int w = 0; w < nwin; ++w) {
        x = x * 1664525u + 1013904223u;
        const int y0 = (x >> 8) % (kMapH - 9), x0 = (x >> 20) % (kMapW - 9);
        wyx[2 * w] = (unsigned short)y0, wyx[2 * w + 1] = (unsigned short)x0;
        std::unordered_set<unsigned> s64, s128;
        for (int y = y0; y < y0 + 10; ++y)
            for (int t = x0 >> 2; 4 * t <= x0 + 9; ++t) {
                const unsigned b = ((((y >> 2) * kTC + t) * 4 + (y & 3)) * 4) * 4;
                ++wchunks, s64.insert(b / 64), s128.insert(b / 128);
            }
        wl64 += s64.size() * 64, wl128 += s128.size() * 128;
    }
    unsigned short *dwyx;
    CK(hipMalloc(&dwyx, wyx.size() * 2));
    CK(hipMemcpy(dwyx, wyx.data(), wyx.size() * 2, hipMemcpyHostToDevice));
    unsigned *dst;
    CK(hipMalloc(&dst, (size_t)nseg * 4));
    CK(hipMemcpy(dst, st.data(), (size_t)nseg * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, (const float4 *)buf, n / 4, sink);
        hipLaunchKernelGGL(stream4, dim3(4096), dim3(256), 0, 0, buf, n, sink);
        hipLaunchKernelGGL(gather44, dim3(4096), dim3(256), 0, 0, buf, dst, nseg, sink);
        hipLaunchKernelGGL(gatherwin, dim3(4096), dim3(256), 0, 0, (const float4 *)buf, dwyx, nwin, sink);
    }
    CK(hipDeviceSynchronize());
    printf("stream16 bytes %zu\n", bytes);
    printf("stream4  bytes %zu\n", bytes);
    printf("gather44 useful %zu  lines32 %zu  lines64 %zu  lines128 %zu  (+ index array %zu)\n", (size_t)nseg * 44,
           lines[0], lines[1], lines[2], (size_t)nseg * 4);
    printf("gatherwin windows %d  useful %zu  chunks16 %zu  lines64 %zu  lines128 %zu  (+ index array %zu)\n", nwin,
           (size_t)nwin * 400, wchunks * 16, wl64, wl128, (size_t)nwin * 4);
    return 0;
}
