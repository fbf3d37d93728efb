// Helpers shared by the two all-pairs builds (corr_build.hip: exact fp32 MFMA;
// corr_build_split.hip: fp32 operands split into f16 pairs).  Internal, not part of the C-ABI.
#pragma once

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

// sqrt(D) is a power of two: x * (1/s) == x / s bit for bit.
inline bool is_pow2(float s) {
    int e;
    return std::frexp(s, &e) == 0.5f;
}

}  // namespace corr
