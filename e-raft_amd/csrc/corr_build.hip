// corr_build.hip — all-pairs correlation + fused 4-level avg-pool pyramid on gfx950 MFMA.
//
// Replaces CorrBlock.corr (model/corr.py:52-60: matmul(F1^T, F2) / sqrt(D)) and the pyramid
// loop of CorrBlock.__init__ (model/corr.py:21-27: avg_pool2d(2, stride 2) x (L-1)).
//
// A workgroup of WQ x WT waves owns a tile of BQ = 32*QT*WQ query pixels x one 8 x (8*WT)
// patch of target pixels.  K = D is staged through LDS in BK-deep chunks (double-buffered;
// the global loads of chunk c+1 are in flight while chunk c feeds the MFMAs).  Each wave
// computes (32*QT) queries x an 8x8 target sub-patch with v_mfma_f32_32x32x2_f32 (exact
// fp32: a k-ordered fmaf chain): A = targets (MFMA rows), B = queries (MFMA columns), so every
// lane ends up owning ONE query and a 4x8 block of target pixels (lanes l, l+32 hold the two
// 4-wide halves of the 8x8).  The epilogue applies 1/sqrt(D), writes level 0 and pools levels
// 1..3 in registers (level 3 needs one cross-half shuffle) — every pyramid level leaves the
// chip exactly once; no level is re-read to build the next.
//
// The k-order of every accumulation (chunks in order, k = 2s + h inside a chunk) does not
// depend on the tile geometry, so all BuildCfg instantiations give bit-identical results.
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "corr_build_common.h"

namespace corr {


// Tile geometry.  WQ x WT waves; each wave QT query tiles of 32 x one 8x8 target sub-patch.
// PF: read all of a chunk's MFMA operands from LDS before issuing its MFMAs.
// SKIP: skip the MFMAs of a 4-row target tile that lies entirely below the map.
// NOSTORE: measurement instantiation only (tools/kbench_build.hip): no pyramid stores.
template <int WQ_, int WT_, int QT_, int BK_, int OCC_, bool PF_ = false, bool SKIP_ = true, bool NOSTORE_ = false>
struct BuildCfg {
    static constexpr int WQ = WQ_, WT = WT_, QT = QT_, BK = BK_, OCC = OCC_;
    static constexpr bool PF = PF_, SKIP = SKIP_, NOSTORE = NOSTORE_;
    static constexpr int NT = 64 * WQ * WT;  // threads
    static constexpr int BQ = 32 * QT * WQ;  // queries per tile
    static constexpr int PW = 8 * WT;        // target patch columns (8 rows)
    static constexpr int BT = 64 * WT;       // targets per tile
    static constexpr int QPT = BK * BQ / 4 / NT;  // float4 staged per thread per chunk (queries)
    static constexpr int TPT = BK * BT / 4 / NT;  // ... (targets)
    static constexpr size_t LDS = 2ull * BK * (BQ + BT) * sizeof(float);
    static_assert(BK * BQ / 4 % NT == 0 && BK * BT / 4 % NT == 0, "staging must tile the chunk");
    static_assert(NT % (BQ / 4) == 0 && NT % (BT / 4) == 0, "fixed staging column per thread");
};

// Default geometry (selected by tools/kbench_build.hip measurements).  No SKIP:
// the second (half-tile) kernel body costs more than the MFMAs it skips (DSEC 126 -> 123 us,
// train 139 -> 137 us; profiles/r03f_kbench_build_fp32.txt).
using BuildDefault = BuildCfg<2, 2, 2, 8, 4, true, false>;

struct BuildParams {
    const float *f1;
    const float *f2;
    float *lvl[kFusedLevels];
    int B, D, H, W, N;  // N = H*W target pixels per batch item
    int NQ;             // query pixels per batch item (N, or a row slab of it)
    int nlev;           // levels written by the epilogue (1..4)
    int nq, npx, npy;   // query blocks, patch columns, patch rows
    float inv_s, s;
    int exact_mul;      // sqrt(D) is a power of two: x * (1/s) == x / s bit-for-bit
};



// Epilogue: scale, level 0, in-register pyramid, into the tiled pyramid (corr_common.h).
// acc[qt][tt][r]: query qw + qt*32 + l32, target (y, x) of the wave's 8x8 sub-patch at
// (py*8, xw) with y = tt*4 + (r >> 2), x = 4h + (r & 3)   (32x32 C/D map).
// Level 0 leaves as 16-B tile rows (columns X0 .. X0 + 3); for level 1 the two lane halves (h = 0,
// 1: the same query, target columns 0-3 / 4-7) swap half of their rows, so a lane writes 2 level-1
// tile rows of 4 columns; level 2 as one 8-B pair, level 3 one cell.  A store runs whenever its
// tile row lies in the padded map (cells past W_l / H_l are padding: the zero-padded target
// operands make them finite, nothing reads them).
template <int QT>
__device__ __forceinline__ void store_pyramid(const BuildParams &p, f32x16 (&acc)[QT][2], const int b,
                                              const int qw, const int xw, const int py, const int h,
                                              const int l32) {
    const int NQ = p.NQ, W = p.W, H = p.H;
    const int H1 = H >> 1, W1 = W >> 1, H2 = H >> 2, W2 = W >> 2, H3 = H >> 3, W3 = W >> 3;
    const int TW0 = map_tcols(W), TW1 = map_tcols(W1), TW2 = map_tcols(W2), TW3 = map_tcols(W3);
    const int R0 = 4 * map_tiles(H), R1 = 4 * map_tiles(H1), R2 = 4 * map_tiles(H2), R3 = 4 * map_tiles(H3);
    const size_t M0 = map_floats(H, W), M1 = map_floats(H1, W1), M2 = map_floats(H2, W2), M3 = map_floats(H3, W3);
    const int X0 = xw + 4 * h, Y0 = py * 8;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int q = qw + qt * 32 + l32;
        const bool qok = q < NQ;
        const size_t qrow = (size_t)b * NQ + q;
        float v[8][4];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float x = acc[qt][tt][r];
                v[tt * 4 + (r >> 2)][r & 3] = p.exact_mul ? x * p.inv_s : x / p.s;
            }
        // level 0
        if (qok && X0 < W) {
            float *o = p.lvl[0] + qrow * M0;
#pragma unroll
            for (int y = 0; y < 8; ++y)
                if (Y0 + y < R0)
                    *reinterpret_cast<float4 *>(o + map_row4(Y0 + y, X0 >> 2, TW0)) = make_float4(v[y][0], v[y][1], v[y][2], v[y][3]);
        }
        if (p.nlev < 2) continue;
        // level 1: 4 rows x 2 cols per lane
        float l1[4][2];
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int x = 0; x < 2; ++x)
                l1[y][x] = pool4(v[2 * y][2 * x], v[2 * y][2 * x + 1], v[2 * y + 1][2 * x],
                                 v[2 * y + 1][2 * x + 1]);
        {
            // h = 0 keeps rows 0-1 and receives columns 2-3 of them; h = 1 keeps rows 2-3 and
            // receives columns 0-1 of them
            float r[2][4];
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    const float give = h ? l1[y][x] : l1[y + 2][x];
                    const float got = __shfl_xor(give, 32);
                    const float mine = h ? l1[y + 2][x] : l1[y][x];
                    r[y][2 * h + x] = mine;
                    r[y][2 * (1 - h) + x] = got;
                }
            const int X1 = xw >> 1;  // a multiple of 4
            if (qok && X1 < W1) {
                float *o = p.lvl[1] + qrow * M1;
#pragma unroll
                for (int y = 0; y < 2; ++y) {
                    const int Y = py * 4 + 2 * h + y;
                    if (Y < R1)
                        *reinterpret_cast<float4 *>(o + map_row4(Y, X1 >> 2, TW1)) = make_float4(r[y][0], r[y][1], r[y][2], r[y][3]);
                }
            }
        }
        if (p.nlev < 3) continue;
        // level 2: 2 rows x 1 col per lane
        float l2[2];
#pragma unroll
        for (int y = 0; y < 2; ++y) l2[y] = pool4(l1[2 * y][0], l1[2 * y][1], l1[2 * y + 1][0], l1[2 * y + 1][1]);
        // the partner half's level-2 pair (x = 1 - h): for the 8-B level-2 stores and level 3
        const float o0 = __shfl_xor(l2[0], 32);
        const float o1 = __shfl_xor(l2[1], 32);
        {  // h = 0 writes row 0 (x = 0, 1), h = 1 row 1; xw / 4 is even, so the pair is 8-B aligned
            const int Y = py * 2 + h, X2 = xw >> 2;
            if (qok && X2 < kTileW * TW2 && Y < R2)
                *reinterpret_cast<float2 *>(p.lvl[2] + qrow * M2 + map_cell(Y, X2, TW2)) =
                    h ? make_float2(o1, l2[1]) : make_float2(l2[0], o0);
        }
        if (p.nlev < 4) continue;
        // level 3: the 2x2 level-2 block is split across lane halves h = 0 (x = 0), 1 (x = 1)
        if (h == 0 && qok) {
            const float l3 = pool4(l2[0], o0, l2[1], o1);
            const int Y = py, X = X0 >> 3;
            if (Y < R3 && X < kTileW * TW3) p.lvl[3][qrow * M3 + map_cell(Y, X, TW3)] = l3;
        }
    }
}

// One output tile.  smem: [stage][BK][BQ + BT].
// VM: 0 = element loads / stores, 1 = 16-B staging loads and level-0 stores, 2 = also 16-B
// level-1 and 8-B level-2 stores (store_pyramid's VEC1).
template <class Cfg, int VM, bool TT1>
__device__ __forceinline__ void build_tile(const BuildParams &p, float *smem, const int tile) {
    constexpr int NT = Cfg::NT, BQ = Cfg::BQ, BT = Cfg::BT, BK = Cfg::BK, QT = Cfg::QT;
    constexpr int PW = Cfg::PW, QPT = Cfg::QPT, TPT = Cfg::TPT;

    const int px = tile % p.npx;
    const int py = (tile / p.npx) % p.npy;
    const int qb = (tile / (p.npx * p.npy)) % p.nq;
    const int b = tile / (p.npx * p.npy * p.nq);
    const int q0 = qb * BQ;
    const int N = p.N, NQ = p.NQ, W = p.W, H = p.H, D = p.D;

    const int tid = threadIdx.x;
    const int lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wv = tid >> 6, wq = wv / Cfg::WT, wt = wv % Cfg::WT;

    // ---- staging: thread -> fixed column (4 consecutive idx), rows k advance by a stride ----
    constexpr int QCOLS = BQ / 4, TCOLS = BT / 4;
    constexpr int QKSTEP = NT / QCOLS, TKSTEP = NT / TCOLS;
    const int qk = tid / QCOLS, qc4 = (tid % QCOLS) * 4;
    const int tk = tid / TCOLS, tc4 = (tid % TCOLS) * 4;
    const int qidx = q0 + qc4;
    // target patch layout inside a tile: idx = wt*64 + tt*32 + y4*8 + x8
    const int sy = ((tc4 >> 5) & 1) * 4 + ((tc4 >> 3) & 3);
    const int sx = (tc4 >> 6) * 8 + (tc4 & 7);
    const int tY = py * 8 + sy, tX = px * PW + sx;
    const size_t tOff = (size_t)tY * W + tX;
    const bool tvalid = tY < H && tX < W;
    const float *f1b = p.f1 + (size_t)b * D * NQ;
    const float *f2b = p.f2 + (size_t)b * D * N;

    float4 rq[QPT], rt[TPT];
    auto load_chunk = [&](int k0) {
#pragma unroll
        for (int i = 0; i < QPT; ++i) {
            const int k = k0 + qk + QKSTEP * i;
            if (VM >= 1) {
                rq[i] = (k < D && qidx < NQ) ? *reinterpret_cast<const float4 *>(f1b + (size_t)k * NQ + qidx)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = (k < D && qidx + e < NQ) ? f1b[(size_t)k * NQ + qidx + e] : 0.f;
                rq[i] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
#pragma unroll
        for (int i = 0; i < TPT; ++i) {
            const int k = k0 + tk + TKSTEP * i;
            if (VM >= 1) {
                rt[i] = (k < D && tvalid) ? *reinterpret_cast<const float4 *>(f2b + (size_t)k * N + tOff)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = (k < D && tY < H && tX + e < W) ? f2b[(size_t)k * N + tOff + e] : 0.f;
                rt[i] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    };
    auto store_chunk = [&](int st) {
        float *Qs = smem + (size_t)st * BK * (BQ + BT);
        float *Ts = Qs + BK * BQ;
#pragma unroll
        for (int i = 0; i < QPT; ++i)
            *reinterpret_cast<float4 *>(&Qs[(qk + QKSTEP * i) * BQ + qc4]) = rq[i];
#pragma unroll
        for (int i = 0; i < TPT; ++i)
            *reinterpret_cast<float4 *>(&Ts[(tk + TKSTEP * i) * BT + tc4]) = rt[i];
    };

    f32x16 acc[QT][2];
#pragma unroll
    for (int i = 0; i < QT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nchunks = (D + BK - 1) / BK;
    load_chunk(0);
    store_chunk(0);
    __syncthreads();

    for (int c = 0; c < nchunks; ++c) {
        const int st = c & 1;
        if (c + 1 < nchunks) load_chunk((c + 1) * BK);
        const float *Qs = smem + (size_t)st * BK * (BQ + BT);
        const float *Ts = Qs + BK * BQ;
        // TT1 = false: the lower 4-row target tile lies entirely below the map (H % 8 in
        // 1..4) — its MFMAs would only produce discarded padding, so they are not issued.
        if constexpr (Cfg::PF) {
            float bq[BK / 2][QT], a0[BK / 2], a1[BK / 2];
#pragma unroll
            for (int s = 0; s < BK / 2; ++s) {
                const int k = 2 * s + h;
#pragma unroll
                for (int i = 0; i < QT; ++i) bq[s][i] = Qs[k * BQ + wq * (32 * QT) + i * 32 + l32];
                a0[s] = Ts[k * BT + wt * 64 + l32];
                if (TT1) a1[s] = Ts[k * BT + wt * 64 + 32 + l32];
            }
#pragma unroll
            for (int s = 0; s < BK / 2; ++s)
#pragma unroll
                for (int i = 0; i < QT; ++i) {
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], bq[s][i], acc[i][0], 0, 0, 0);
                    if (TT1)
                        acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], bq[s][i], acc[i][1], 0, 0, 0);
                }
        } else {
#pragma unroll
            for (int s = 0; s < BK / 2; ++s) {
                const int k = 2 * s + h;
                float bq[QT];
#pragma unroll
                for (int i = 0; i < QT; ++i) bq[i] = Qs[k * BQ + wq * (32 * QT) + i * 32 + l32];
                const float a0 = Ts[k * BT + wt * 64 + l32];
                const float a1 = TT1 ? Ts[k * BT + wt * 64 + 32 + l32] : 0.0f;
#pragma unroll
                for (int i = 0; i < QT; ++i) {
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bq[i], acc[i][0], 0, 0, 0);
                    if (TT1) acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bq[i], acc[i][1], 0, 0, 0);
                }
            }
        }
        if (c + 1 < nchunks) store_chunk(st ^ 1);
        __syncthreads();
    }

    if constexpr (Cfg::NOSTORE) {  // keep the MFMAs live without writing the pyramid
        float x = 0.f;
#pragma unroll
        for (int i = 0; i < QT; ++i) x += acc[i][0][0] + acc[i][1][15];
        if (x == 1234.5f) p.lvl[0][tid] = x;
    } else {
        store_pyramid<QT>(p, acc, b, q0 + wq * 32 * QT, px * PW + wt * 8, py, h, l32);
    }
}

template <class Cfg, int VM>
__global__ __launch_bounds__(Cfg::NT, Cfg::OCC) void corr_build_kernel(BuildParams p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tile = xcd_swizzle(blockIdx.x, gridDim.x);
    const int py = (tile / p.npx) % p.npy;
    // one tile-uniform branch between two complete bodies (register pressure = the max of the
    // two, not their union)
    if (!Cfg::SKIP || py * 8 + 4 < p.H)
        build_tile<Cfg, VM, true>(p, smem, tile);
    else
        build_tile<Cfg, VM, false>(p, smem, tile);
}

namespace {

// Levels beyond the fused four: plain 2x2 average pool of level l-1 into level l, both tiled
// (one thread per cell of level l, padding cells included: they pool padding).
__global__ __launch_bounds__(256) void pool2x2_kernel(const float *__restrict__ in,
                                                      float *__restrict__ out, long BN, int H,
                                                      int W) {
    const int Ho = H >> 1, Wo = W >> 1;
    const int TWi = map_tcols(W), TWo = map_tcols(Wo);
    const size_t Mi = map_floats(H, W), Mo = map_floats(Ho, Wo);
    const size_t total = (size_t)BN * Mo;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const size_t q = i / Mo;
        const int rem = (int)(i - q * Mo);
        const int t = rem / (4 * kTileW), c = rem % (4 * kTileW);
        const int ty = t / TWo, tx = t - ty * TWo;
        const int y = 4 * ty + c / kTileW, x = kTileW * tx + c % kTileW;
        if (y >= Ho || x >= Wo) continue;  // padding of level l: never read
        const float *I = in + q * Mi;
        out[i] = pool4(I[map_cell(2 * y, 2 * x, TWi)], I[map_cell(2 * y, 2 * x + 1, TWi)],
                       I[map_cell(2 * y + 1, 2 * x, TWi)], I[map_cell(2 * y + 1, 2 * x + 1, TWi)]);
    }
}


}  // namespace

hipError_t launch_pool_levels(const LevelPtrs &pyr, int l_from, int levels, long BN, int H, int W,
                              hipStream_t s) {
    for (int l = l_from; l < levels; ++l) {
        const int Hi = H >> (l - 1), Wi = W >> (l - 1);
        const size_t total = (size_t)BN * map_floats(Hi >> 1, Wi >> 1);
        const int grid = (int)std::min<size_t>((total + 255) / 256, 4096);
        hipLaunchKernelGGL(pool2x2_kernel, dim3(grid), dim3(256), 0, s, pyr.p[l - 1], pyr.p[l], BN,
                           Hi, Wi);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Launch one build with tile geometry Cfg (exposed for tools/kbench_build.hip).
// vec1_ok: 16-B level-1 stores when the shape allows (tools/kbench_build.hip turns them off for
// its A/B).
template <class Cfg>
hipError_t launch_build_cfg(const float *f1, int NQ, const float *f2, int B, int D, int H, int W,
                            int levels, const LevelPtrs &pyr, hipStream_t s, bool vec1_ok = true) {
    BuildParams p{};
    p.f1 = f1;
    p.f2 = f2;
    p.B = B;
    p.D = D;
    p.H = H;
    p.W = W;
    p.N = H * W;
    p.NQ = NQ;
    p.nlev = levels < kFusedLevels ? levels : kFusedLevels;
    for (int l = 0; l < kFusedLevels; ++l) p.lvl[l] = l < p.nlev ? pyr.p[l] : nullptr;
    p.nq = (NQ + Cfg::BQ - 1) / Cfg::BQ;
    p.npx = (W + Cfg::PW - 1) / Cfg::PW;
    p.npy = (H + 7) / 8;
    p.s = std::sqrt((float)D);
    p.exact_mul = is_pow2(p.s);
    p.inv_s = 1.0f / p.s;

    // float4 staging / level-0 stores need 16-B aligned rows and patch columns.
    const bool vec = (W % 4 == 0) && (NQ % 4 == 0) && ((uintptr_t)pyr.p[0] % 16 == 0) &&
                     ((uintptr_t)f1 % 16 == 0) && ((uintptr_t)f2 % 16 == 0);
    const long tiles = (long)p.nq * p.npx * p.npy * B;
    if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
    (void)vec1_ok;  // the tiled pyramid's stores are always 16-B tile rows: VM 2 == VM 1
    const bool vec1 = false;
    static std::atomic<unsigned long long> lds_done[3];
    auto go = [&](auto vm_tag) {
        constexpr int VM = decltype(vm_tag)::value;
        hipError_t e = ensure_lds_limit((const void *)corr_build_kernel<Cfg, VM>, (int)Cfg::LDS, lds_done[VM]);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((corr_build_kernel<Cfg, VM>), dim3((unsigned)tiles), dim3(Cfg::NT), Cfg::LDS, s, p);
        return hipSuccess;
    };
    hipError_t e0 = vec1 ? go(std::integral_constant<int, 2>{})
                  : vec  ? go(std::integral_constant<int, 1>{})
                         : go(std::integral_constant<int, 0>{});
    if (e0 != hipSuccess) return e0;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (levels > kFusedLevels) return launch_pool_levels(pyr, kFusedLevels, levels, (long)B * NQ, H, W, s);
    return hipSuccess;
}

hipError_t launch_build(const float *f1, int NQ, const float *f2, int B, int D, int H, int W,
                        int levels, const LevelPtrs &pyr, hipStream_t s) {
    return launch_build_cfg<BuildDefault>(f1, NQ, f2, B, D, H, W, levels, pyr, s);
}

}  // namespace corr
