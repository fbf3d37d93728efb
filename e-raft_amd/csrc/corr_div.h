// Correctly rounded division by a per-level constant for the lookup's tap arithmetic
// (bilinear_sampler's 2x / (W - 1), utils.py:11), without __fdiv_rn's scale / fixup sequence.
#pragma once

#include <hip/hip_runtime.h>

namespace corr {

// RN(1 / d) for an integer-valued d >= 1: v_rcp_f32 (1 ulp) and one Newton step.  Bit-identical
// to __fdiv_rn(1, d) for every d in [1, 2^20] (tools/kbench_div.hip); d = 0 gives NaN.
__device__ __forceinline__ float recip_rn(float d) {
    const float y0 = __builtin_amdgcn_rcpf(d);
    return __builtin_fmaf(__builtin_fmaf(-d, y0, 1.0f), y0, y0);
}

// RN(a / d) from y = RN(1 / d): q = RN(a y), the exact residual a - q d by fma, then Markstein's
// correction q + r y in one rounding (an infinite q is the quotient: its residual is NaN).
// Against __fdiv_rn(a, d), every float a, d = 1 .. 4096 (tools/kbench_div.hip): the same bits
// except where the quotient is subnormal or zero (the correction's rounding below 2^-126, the sign
// of a zero), all of which give the same a / d - 1, the only use here (bilinear_sampler's
// 2x/(W-1) - 1, utils.py:11) — checked on that value for the same inputs.  d = 0 (a one-cell
// level: y = NaN) gives NaN where __fdiv_rn gives +-inf or NaN; the tap arithmetic then
// multiplies by d = 0, so the tap is NaN either way.
__device__ __forceinline__ float div_rn(float a, float d, float y) {
    const float q = __fmul_rn(a, y);
    return __builtin_isinf(q) ? q : __builtin_fmaf(__builtin_fmaf(-q, d, a), y, q);
}

}  // namespace corr
