// Helpers shared by the two all-pairs builds (corr_build.hip: exact fp32 MFMA;
// corr_build_split.hip: fp32 operands split into f16 pairs).  Internal, not part of the C-ABI.
#pragma once

#include <atomic>
#include <cmath>

#include "corr_common.h"

namespace corr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;

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

// ---------------------------------------------------------------------------------------
// Shared by the two split builds (corr_build_split.hip, corr_build_bf16.hip): tile order and
// LDS-DMA pieces.
// ---------------------------------------------------------------------------------------
constexpr int kGroupQ = 8;  // query groups per L2 tile group

struct Tile {
    int b, qg, py, cb;
};

// Tile t of (batch item, query group, target patch).  order 0: per batch item, query groups in
// groups of kGroupQ; inside a group the query group runs fastest, then the patch (the ~64 tiles
// one XCD has in flight cover ~8 patches x 8 query groups).  order 1: a patch row's patches
// consecutive for one query group (the 64-B row segments of horizontally adjacent patches share
// 128-B lines and are written close in time on one XCD).
// gq: query groups per L2 tile group (kGroupQ unless a caller passes its own).
__device__ __forceinline__ Tile patch_tile(int t, int npatch, int NQG, int CB, int order, int gq = kGroupQ) {
    Tile o;
    const int per_b = npatch * NQG;
    o.b = t / per_b;
    const int r = t - o.b * per_b;
    const int g = r / (gq * npatch);
    const int gm = min(gq, NQG - g * gq);
    const int r2 = r - g * gq * npatch;
    if (order == 1) {
        o.py = r2 / (gm * CB);
        const int r3 = r2 - o.py * gm * CB;
        o.qg = g * gq + r3 / CB;
        o.cb = r3 - (r3 / CB) * CB;
        return o;
    }
    const int patch = r2 / gm;
    o.qg = g * gq + (r2 - patch * gm);
    o.py = patch / CB;
    o.cb = patch - o.py * CB;
    return o;
}

// s_waitcnt vmcnt(N) lgkmcnt(0) + s_barrier with N an immediate (the rings' hand-counted waits).
template <int N>
__device__ __forceinline__ void wait_vmcnt_barrier() {
    static_assert(N >= 0 && N < 64, "vmcnt immediate");
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// One LDS-DMA piece: 16 B per lane from g into LDS at lds + 16 * lane (global_load_lds_dwordx4;
// M0 = the wave-uniform LDS base).  Counted in vmcnt like any vector load.  Inline asm, so the
// compiler does not make every ds_read wait for all outstanding DMAs (it cannot tell ring slots
// apart); the callers count vmcnt themselves.
__device__ __forceinline__ void dma16(const void *g, uint32_t lds) {
    asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds) : "memory");
}

// One LDS-DMA dword per lane: g -> LDS at lds + 4 * lane.
__device__ __forceinline__ void dma4(const void *g, uint32_t lds) {
    asm volatile("global_load_lds_dword %0, off" ::"v"(g), "{m0}"(lds) : "memory");
}

// ---------------------------------------------------------------------------------------
// The exact three-piece bf16 split (corr_build_bf16.hip's operands, lookup_conv_bwd's).
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16s_pair __attribute__((ext_vector_type(2)));
typedef float bf16s_f32x2 __attribute__((ext_vector_type(2)));

// bf16 round-to-nearest-even of a pair, as fp32 values and as the packed pair.
__device__ __forceinline__ unsigned rn_pair(float a, float b, float &ha, float &hb) {
    const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(bf16s_f32x2{a, b}, bf16s_pair));
    ha = __builtin_bit_cast(float, u << 16);
    hb = __builtin_bit_cast(float, u & 0xffff0000u);
    return u;
}

// Split a pair of fp32 features into packed bf16 (hi, mid, lo) pairs, x = hi + mid + lo exactly.
// Guards: an infinite feature keeps hi = x and mid = lo = 0 (its hi*hi product is x * hi of the
// other operand; its products with the other operand's zero mid / lo pieces are NaN, which the
// consumers' split_sum discards when the hi*hi sum is infinite, corr_common.h); a finite feature
// whose hi rounds up past the bf16 range (|x| within 2^-9 of FLT_MAX) takes the truncated hi
// instead.  NaN propagates through hi.
__device__ __forceinline__ void split3(float a, float b, unsigned &hi, unsigned &mid, unsigned &lo) {
    float ha, hb;
    hi = rn_pair(a, b, ha, hb);
    if (__builtin_expect(__builtin_isinf(ha) | __builtin_isinf(hb), 0)) {
        const unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
        if (__builtin_isinf(ha) && !__builtin_isinf(a)) ha = __builtin_bit_cast(float, ua & 0xffff0000u);
        if (__builtin_isinf(hb) && !__builtin_isinf(b)) hb = __builtin_bit_cast(float, ub & 0xffff0000u);
        hi = (__builtin_bit_cast(unsigned, ha) >> 16) | (__builtin_bit_cast(unsigned, hb) & 0xffff0000u);
    }
    float ra = __builtin_isinf(a) ? 0.f : a - ha, rb = __builtin_isinf(b) ? 0.f : b - hb;
    float ma, mb;
    mid = rn_pair(ra, rb, ma, mb);
    float da, db;
    lo = rn_pair(ra - ma, rb - mb, da, db);  // exact: the residuals have <= 8 significant bits
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace corr
