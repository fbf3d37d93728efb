// pack_256.hip — the round-1 operand pack (one 256-thread workgroup per 16-pixel block; thread =
// (pixel, k-octet)), replaced by split_pack_wide_kernel and kept here only for the bitwise A/B
// in tools/kbench_build.hip ("wide pack vs 256-thread pack, workspace: bit-identical").  Not
// part of the library.  Included after e-raft_amd/csrc/corr_build_split.hip.
#pragma once

namespace corr {

template <int CPT>
__global__ __launch_bounds__(256) void split_pack_kernel(PackArgs a) {
    __shared__ float red[4][16];
    const int z = blockIdx.z, b = blockIdx.y, blk = blockIdx.x;
    if (blk >= a.nblk[z]) return;  // the grid covers the larger image (uniform exit)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int ci = lane & 15, og = (w << 2) | (lane >> 4);
    int n, exi;
    bool valid;
    if (z == 0) {
        n = blk * 16 + ci;
        valid = n < a.np[0];
        exi = b * a.NQp + n;
    } else {
        const int y = blk / a.CB, x = (blk - y * a.CB) * 16 + ci;
        valid = y < a.H && x < a.W;
        n = y * a.W + x;
        exi = (b * a.Hp + y) * a.Wp + x;
    }
    const int NP = a.np[z], D = a.D;
    const float *src = a.f[z] + (size_t)b * D * NP + (valid ? n : 0);
    float v[CPT][8];
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int d = 8 * (og + 16 * c) + j;
            v[c][j] = (valid && d < D) ? src[(size_t)d * NP] : 0.f;
        }
    float m = 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[c][j]));
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    if (lane < 16) red[w][ci] = m;
    __syncthreads();
    const float mm = fmaxf(fmaxf(red[0][ci], red[1][ci]), fmaxf(red[2][ci], red[3][ci]));
    int s = 0;
    if (mm > 0.f && mm <= 3.402823466e38f) {
        int E;
        (void)frexpf(mm, &E);  // mm < 2^E
        s = 15 - E;            // mm * 2^s < 2^15: neither half overflows
    }
    if (tid < 16) a.ex[z][exi] = -s;
    const int OCT = 4 * a.S;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int o = og + 16 * c;
        if (o >= OCT) break;
        half8 hi8, lo8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float y = ldexpf(v[c][j], s);
            const _Float16 hi = (_Float16)y;
            hi8[j] = hi;
            lo8[j] = __builtin_isinf(y) ? (_Float16)0.f : (_Float16)(y - (float)hi);
        }
        u32x4 *rec = a.pk[z] + (((size_t)b * a.S + (o >> 2)) * a.nblk[z] + blk) * kRecU;
        rec[lane] = __builtin_bit_cast(u32x4, hi8);  // lane = 16 (o & 3) + ci
        rec[64 + lane] = __builtin_bit_cast(u32x4, lo8);
    }
}


hipError_t launch_split_pack_256(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, void *ws,
                                 hipStream_t s) {
    const SplitGeom g = split_geom(D, NQ, H, W);
    const SplitWs w = split_ws(ws, B, g);
    PackArgs a{};
    a.f[0] = f1, a.f[1] = f2;
    a.pk[0] = w.pq, a.pk[1] = w.pt;
    a.ex[0] = w.eq, a.ex[1] = w.et;
    a.np[0] = NQ, a.np[1] = H * W;
    a.nblk[0] = g.NQB, a.nblk[1] = g.Hp * g.CB;
    a.D = D, a.S = g.S, a.H = H, a.W = W, a.CB = g.CB, a.Hp = g.Hp, a.Wp = g.Wp, a.NQp = g.NQp;
    const dim3 grid((unsigned)std::max(a.nblk[0], a.nblk[1]), B, 2), blk(256);
    switch ((4 * g.S + 15) / 16) {
#define CORR_PACK_CASE(c) \
    case c: hipLaunchKernelGGL(split_pack_kernel<c>, grid, blk, 0, s, a); return hipGetLastError();
        CORR_PACK_CASE(1) CORR_PACK_CASE(2) CORR_PACK_CASE(3) CORR_PACK_CASE(4)
        CORR_PACK_CASE(5) CORR_PACK_CASE(6) CORR_PACK_CASE(7) CORR_PACK_CASE(8)
#undef CORR_PACK_CASE
        default: return hipErrorInvalidValue;
    }
}

}  // namespace corr
