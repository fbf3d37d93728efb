// Helpers shared by the two all-pairs builds (corr_build.hip: exact fp32 MFMA;
// corr_build_split.hip: fp32 operands split into f16 pairs).  Internal, not part of the C-ABI.
#pragma once

#include <atomic>
#include <cmath>

#include "corr_common.h"

namespace corr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Blocks are dealt round-robin to the 8 XCDs; give each XCD a contiguous range of tiles
// (which share operands in its L2) — bijective for any nwg (speed only).
__device__ __forceinline__ int xcd_swizzle(int bid, int nwg) {
    const int xcd = bid & 7, loc = bid >> 3, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// avg_pool2d(2, 2) on CPU ATen: ((a + b) + c) + d, then * 1/4 (bit-identical).
__device__ __forceinline__ float pool4(float a, float b, float c, float d) {
    float t = a + b;
    t = t + c;
    t = t + d;
    return t * 0.25f;
}

// Raise a kernel's dynamic-LDS limit once per device: `done` holds one bit per device id, set
// after a successful hipFuncSetAttribute (thread-safe; two threads racing both set the same
// attribute, which is idempotent).  One `done` word per kernel instantiation.
inline hipError_t ensure_lds_limit(const void *fn, int bytes, std::atomic<unsigned long long> &done) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

// sqrt(D) is a power of two: x * (1/s) == x / s bit for bit.
inline bool is_pow2(float s) {
    int e;
    return std::frexp(s, &e) == 0.5f;
}

}  // namespace corr
