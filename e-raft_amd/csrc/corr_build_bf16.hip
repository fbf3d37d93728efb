// corr_build_bf16.hip — the all-pairs build and its pyramid on gfx950's bf16 MFMA, at no less
// than fp32 accuracy.  Replaces CorrBlock.corr (model/corr.py:52-60: matmul(F1^T, F2) / sqrt(D))
// and the pyramid loop of CorrBlock.__init__ (model/corr.py:21-27).
//
// Operands.  bf16 has fp32's exponent range and 8 significant bits, so every fp32 feature is
// EXACTLY the sum of three bf16 pieces,
//     x = hi + mid + lo,   hi = bf16_rn(x),  mid = bf16_rn(x - hi),  lo = x - hi - mid,
// (x - hi and x - hi - mid are exact in fp32; lo has at most 8 significant bits, so it is a bf16
// value as it stands) with |mid| <= 2^-8 |x| and |lo| <= 2^-16 |x|.  No per-pixel scale and no
// flush: the only exception is the bf16 subnormal floor for lo (|x| below ~2^-110).  A dot
// product takes, per 32-deep K step, the six bf16 MFMAs of largest weight chained from zero,
//     t = lo_t hi_q + hi_t lo_q + mid_t mid_q + mid_t hi_q + hi_t mid_q + hi_t hi_q
// (smallest first; bf16 x bf16 products are exact in fp32), and adds t to its fp32
// accumulator: the accumulator rounds ONCE per K step (D / 32 times per dot product, where an
// fp32 fmaf chain rounds D times), t's own roundings happen at one K step's magnitude.  What is
// dropped (mid lo + lo mid + lo lo) is <= 2^-23 |x_t x_q| per term.  The fp64-oracle test holds this build's per-row error to at most the
// exact-fp32 MFMA build's (tests/test_gpu_parity.py::test_build_bf16x6_not_narrower_than_fp32).
//
// MFMA orientation (as corr_build_split.hip): v_mfma_f32_16x16x32_bf16 with A = TARGETS (rows)
// and B = QUERIES (columns); lane l = 16 grp + ci owns query ci of a 16-query block and targets
// 4 grp .. 4 grp + 3 of a 16-target block (one map row x 16 columns), so a lane holds runs of
// 4 consecutive pixels of one query's map: level 0 leaves as 16-B row stores, the 2x2 / 4x4
// windows of levels 1-2 sit inside one lane, level 3 pairs lanes 16 apart.
//
// Workgroup = 4 waves x 32 queries against one 8 x 16 target patch (2 x 4 tiles).  The patch's records
// (24 KiB per 32-deep K step) stream into a 3-slot LDS ring by LDS-DMA two steps ahead; each
// wave loads its own queries' records into registers, also two steps ahead.  One barrier per K
// step.  Two workgroups per CU (72 KiB LDS each).
//
// Packed operand images (bf16_pack_kernel), one 3 KiB record per (K step s, 16-pixel block):
//   bytes [0, 1024)      hi:  lane l = 16 grp + ci at 16 l: 8 bf16 of k = 32 s + 8 grp + j, pixel ci
//   bytes [1024, 2048)   mid: the same positions
//   bytes [2048, 3072)   lo:  the same positions
// i.e. exactly the MFMA fragment images of that block: the LDS fill and every fragment read are
// contiguous 1 KiB (conflict-free ds_read_b128, coalesced loads).
//   pq [B][S][NQB][3 KiB]          queries: block = 16 consecutive query pixels, NQp = NQB*16
//   pt [B][S][Hp/4][4 CB][3 KiB]   targets: block = the 4x4 tile (rows 4 ty .., columns 4 tx ..),
//                                  pixel ci at (ci / 4, ci % 4) — the pyramid's tile
//                                  (corr_common.h), so each 16x16 output block of an MFMA is one
//                                  tile: lane (grp, ci) holds its row grp for query ci, and the
//                                  four lanes of a query store a whole 64-B tile per instruction
// Padding pixels and k >= D are zero.
#include <algorithm>
#include <atomic>
#include <cmath>

#include "corr_build_common.h"

namespace corr {

typedef __bf16 bfx8_t __attribute__((ext_vector_type(8)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

namespace bf16b {

constexpr int kStepK = 32;                              // k per MFMA step
constexpr int kPieces = 3;                              // hi, mid, lo
constexpr int kRecU = kPieces * 64;                     // u32x4 per record (3 KiB)
constexpr int kPatchRows = 8;                           // target patch: 8 rows x 16 columns
constexpr int kWaves = 4, kQPerWave = 32;               // 2 query blocks per wave
constexpr int kQPerWG = kWaves * kQPerWave;             // 128
constexpr int kRing = 3;                                // LDS ring slots (prefetch distance 2)
constexpr int kSlotBytes = kPatchRows * kPieces * 1024; // 24 KiB per K step
constexpr int kLds = kRing * kSlotBytes;                // 72 KiB
constexpr int kDmaPerWave = kPatchRows * kPieces / kWaves;  // 6 LDS-DMA pieces per wave and step
constexpr int kQLoads = 2 * kPieces;                    // query loads per wave and step
constexpr int kPixBytes = kStepK * kPieces * 2;         // workspace bytes per pixel and K step

struct Geom {
    int S, NQp, NQB, NQG, Hp, CB, Wp;
};

inline Geom geom(int D, int NQ, int H, int W) {
    Geom g;
    g.S = (D + kStepK - 1) / kStepK;
    g.NQp = (NQ + kQPerWG - 1) / kQPerWG * kQPerWG;
    g.NQB = g.NQp / 16;
    g.NQG = g.NQp / kQPerWG;
    g.Hp = (H + kPatchRows - 1) / kPatchRows * kPatchRows;
    g.CB = (W + 15) / 16;
    g.Wp = g.CB * 16;
    return g;
}

// ---------------------------------------------------------------------------------------
// Operand pack: one wave per record (K step, 16-pixel block) of one batch item and tensor;
// lane = 16 grp + ci holds the 8 k of its fragment position, splits them and writes 16 B of
// each piece (each store instruction writes one contiguous 1 KiB piece).
// ---------------------------------------------------------------------------------------
// Target region (corr_build_region): the target image's patch-padded rows [y0, y0 + nyp) are
// packed from a slab holding rows [y0, y1) of fmap2 ([B][D][y1 - y0][W]); the full build is the
// region [0, H).  z = 0 packs the queries (skipped when z0 = 1), z = 1 the targets.
struct PackArgs {
    const float *f[2];
    u32x4_t *pk[2];
    int np[2];    // source pixels per batch item: NQ, (y1 - y0) * W
    int nblk[2];  // blocks per batch item to pack: NQB, nyp * CB
    int img[2];   // blocks per batch item in the packed image: NQB, Hp * CB
    int D, S, W, CB, y0, y1, z0;
};

// R: records per wave, all R records' loads issued before any split or store (more bytes in
// flight per wave); the workgroup's 4 waves take 4 consecutive records at each r, so a k row is
// still read as one 256-B run per workgroup.
template <int R = 1>
__global__ __launch_bounds__(256) void bf16_pack_kernel(PackArgs a) {
    const int z = blockIdx.z + a.z0, b = blockIdx.y;
    const int nblk = a.nblk[z];
    const int lane = threadIdx.x & 63, ci = lane & 15, grp = lane >> 4;
    const int NP = a.np[z];
    float v[R][8];
    bool live[R];
    size_t dst[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int rec = (blockIdx.x * R + r) * 4 + (threadIdx.x >> 6);  // record = s * nblk + blk
        live[r] = rec < a.S * nblk;
        const int s = live[r] ? rec / nblk : 0, blk = live[r] ? rec - s * nblk : 0;
        int n, iblk;  // source pixel in the slab, block in the packed image
        bool valid;
        if (z == 0) {
            n = blk * 16 + ci;
            valid = n < a.np[0];
            iblk = blk;
        } else {
            // target block = a 4x4 tile of the map (tile row ty, column tx; 4 CB tiles per row), pixel
            // ci at (ci / 4, ci % 4): the MFMA's output rows then hold whole tile rows of the pyramid
            const int TCp = 4 * a.CB, ty = blk / TCp, tx = blk - ty * TCp;
            const int ly = 4 * ty + (ci >> 2), x = 4 * tx + (ci & 3);
            valid = a.y0 + ly < a.y1 && x < a.W;
            n = ly * a.W + x;
            iblk = (a.y0 >> 2) * TCp + blk;
        }
        valid = valid && live[r];
        const int k0 = s * kStepK + 8 * grp;
        const float *src = a.f[z] + (size_t)b * a.D * NP + (valid ? n : 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[r][j] = (valid && k0 + j < a.D) ? src[(size_t)(k0 + j) * NP] : 0.f;
        dst[r] = (((size_t)b * a.S + s) * a.img[z] + iblk) * kRecU + lane;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!live[r]) continue;
        unsigned hh[4], mm[4], ll[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) split3(v[r][2 * j], v[r][2 * j + 1], hh[j], mm[j], ll[j]);
        const u32x4_t h{hh[0], hh[1], hh[2], hh[3]}, m{mm[0], mm[1], mm[2], mm[3]}, l{ll[0], ll[1], ll[2], ll[3]};
        u32x4_t *out = a.pk[z] + dst[r];
        out[0] = h;
        out[64] = m;
        out[128] = l;
    }
}

// ---------------------------------------------------------------------------------------
// The MFMA build.
// ---------------------------------------------------------------------------------------
struct Args {
    const u32x4_t *pq, *pt;
    float *lvl[kFusedLevels];
    int B, H, W, N, NQ, S, nlev;
    int NQp, NQB, NQG, Hp, CB, npatch;  // npatch: patches of the target region
    int py0;                            // first patch row of the target region
    int exact;         // 1/sqrt(D) is a power of two (x * 1/s == x / s); else x * RN(1/s), within ~1 ulp
    float inv_s, s;
    int order;  // tile order: 0, 1 = patch_tile's; 2 = XCD blocks (xcd_block_tile)
    int gq;     // orders 0 / 1: query groups per L2 tile group (patch_tile)
    int nqh, npq;  // order 2: query-group and patch splits of a batch item into XCD blocks
};

// Tile order 2: tile index t (XCD x owns the contiguous range [x T / 8, (x + 1) T / 8) after
// xcd_swizzle) enumerates, per batch item, qh x pq blocks (query-group range x patch range),
// and inside a block the query group slowest and the patch fastest.  With qh x pq = 8 / B
// blocks per batch item (B < 8), every XCD's L2 holds one block's target patches for its whole
// life and streams each of its query groups once: each packed operand byte crosses the MALL ->
// L2 boundary about once per XCD that needs it (DSEC: 2 x 4 blocks).  Measured no faster than
// order 1 (DSEC 65.8 vs 64.9 us, train 70.2 vs 66.5, MVSEC 137.0 vs 138.7:
// profiles/r04e_kbench_build_bf16x6_order.txt): the library uses order 1; kbench A/B only.
__device__ __forceinline__ Tile xcd_block_tile(const Args &p, int t) {
    Tile o;
    const int per_b = p.npatch * p.NQG;
    o.b = t / per_b;
    int r = t - o.b * per_b;
    // block (i, j): query groups [i NQG / qh, (i + 1) NQG / qh), patches [j np / pq, (j + 1) np / pq)
    // — blocks laid out in order, each of size nq_i * np_j
    int q0 = 0, q1 = 0, p0 = 0, p1 = 0;
    for (int i = 0; i < p.nqh; ++i) {
        const int qa = i * p.NQG / p.nqh, qb = (i + 1) * p.NQG / p.nqh;
        const int rows = (qb - qa) * p.npatch;
        if (r < rows) {
            for (int j = 0; j < p.npq; ++j) {
                const int pa = j * p.npatch / p.npq, pb = (j + 1) * p.npatch / p.npq;
                const int sz = (qb - qa) * (pb - pa);
                if (r < sz) {
                    q0 = qa, q1 = qb, p0 = pa, p1 = pb;
                    break;
                }
                r -= sz;
            }
            break;
        }
        r -= rows;
    }
    (void)q1;
    const int np = p1 - p0;
    o.qg = q0 + r / np;
    const int patch = p0 + r % np;
    o.py = patch / p.CB;
    o.cb = patch - o.py * p.CB;
    return o;
}

// SS > 0: S = SS K steps, fully unrolled (straight-line code: the compiler's own waits on the
// query registers are exact and never drain the prefetch).  SS = 0: any S, runtime loop.
// NR: map rows of the patch whose MFMAs run (8; 4 for a patch with at most 4 rows inside the
// map — its rows 4-7 are padding whose accumulators stay zero and whose stores are dropped).
// ACC2 (default): the five small piece products of every K step accumulate in a second fp32
// accumulator and hi*hi alone in the first; they meet once, in the epilogue.  The first
// accumulator rounds D / 32 times per dot product, the second's roundings are 2^-8 smaller.  Its
// 64 extra registers leave room for three query register slots (prefetch distance 2; the
// compiler's own wait on them then also covers the next step's query loads, which have landed
// by then).  ACC2 = false: the six products of a K step chained from zero into a transient and
// added to one accumulator by VALU (four query slots) — the same rounding count, measured slower.
// VF (measurement variants, tools/kbench_build.hip; 0 in the library): bit 0 = query loads by
// inline asm (the compiler then adds no wait of its own on them), bit 1 = s_setprio 1 over the
// K loop (the epilogue of a neighbouring workgroup yields issue slots to MFMA-phase waves), bit 2 =
// no half-patch body (padding rows computed and discarded: one kernel body).
// (8 waves per workgroup — 256 queries against the patch, so its LDS-DMA records feed twice the
// MFMAs and the L2 operand traffic per flop drops by a quarter, one workgroup per CU — was
// measured and dropped: bit-identical, 5-15 % slower at every size,
// profiles/r06k_kbench_build_8waves_dropped.txt.)
// FAST: levels == 4 (no level-count branches in the epilogue).
template <int SS, int NR, bool ACC2, int VF = 0, bool FAST = false>
__device__ __forceinline__ void build_tile(const Args &p, const Tile tl) {
    constexpr int QS = ACC2 ? 3 : 4, QD = QS - 1;
    constexpr int WV = kWaves, QPWG = kQPerWG, DPW = kDmaPerWave;
    extern __shared__ __attribute__((aligned(16))) char smem_bf16[];
    char *smem = smem_bf16;

    const int b = tl.b, y0 = tl.py * kPatchRows, x0 = tl.cb * 16;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ci = lane & 15, grp = lane >> 4;
    const int qb0 = tl.qg * (QPWG / 16) + 2 * w;  // this wave's first 16-query block
    const int S = SS > 0 ? SS : p.S;
    const bool qact = qb0 * 16 < p.NQ;  // wave-uniform

    // LDS-DMA pieces of this wave: pc = w + 4 m (m < 6) -> patch record rp = pc / 3 (tile row rp / 4,
    // tile column rp % 4 of the patch), piece pc % 3, landing at slot offset pc KiB (record rp's
    // pieces at 3 rp .. 3 rp + 2).
    const int TCp = 4 * p.CB;                          // tiles per row of the target image
    const size_t tstep = (size_t)p.Hp * p.CB * kRecU;  // u32x4 per K step of the target image
    const u32x4_t *tbase = p.pt + (((size_t)b * S * (p.Hp >> 2) + (y0 >> 2)) * TCp + 4 * tl.cb) * kRecU + lane;
    unsigned toff[DPW];
#pragma unroll
    for (int m = 0; m < DPW; ++m) {
        const int pc = w + WV * m, rp = pc / kPieces;
        toff[m] = (unsigned)(((rp >> 2) * TCp + (rp & 3)) * kRecU + (pc % kPieces) * 64);
    }
    const size_t qstep = (size_t)p.NQB * kRecU;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_void_t *)smem;
    const u32x4_t *qsrc = p.pq + ((size_t)b * S * p.NQB + qb0) * kRecU + lane;

    // Issue schedule (SS > 0): step k issues the wave's 6 query loads of step k + 3 (register
    // slot (k + 3) % 4), then its 6 LDS-DMA pieces of step k + 2 (ring slot (k + 2) % 3); the
    // prologue plays Q0 Q1 T0 Q2 T1.  At step k's barrier the operations younger than T(k) are
    // exactly step k - 1's group (Q(k + 2), T(k + 1): vmcnt(12) while both exist), and Q(k) is
    // older than T(k); the query registers then pass through an empty asm, before which the
    // compiler's own wait (it counts only the query loads: Q(k + 1), Q(k + 2) younger) is
    // already satisfied: no drain.
    u32x4_t qv[QS][2][kPieces];
    auto issue_q = [&](int s, int slot) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int c = 0; c < kPieces; ++c) {
                if constexpr (VF & 1)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qv[slot][i][c]) : "v"(qsrc + s * qstep + i * kRecU + c * 64) : "memory");
                else
                    qv[slot][i][c] = qsrc[s * qstep + i * kRecU + c * 64];
            }
    };
    auto issue_t = [&](int s, int slot) __attribute__((always_inline)) {
        const uint32_t base = lds_base + slot * kSlotBytes;
        const u32x4_t *src = tbase + s * tstep;
#pragma unroll
        for (int m = 0; m < DPW; ++m) dma16(src + toff[m], base + (w + WV * m) * 1024);
    };

    f32x4_t acc[2][kPatchRows], acs[2][kPatchRows];  // hi*hi; the small products (ACC2)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < kPatchRows; ++r) acc[i][r] = acs[i][r] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // One K step: per map row, its three target fragments (read one row ahead) and 12 MFMAs.
    auto compute = [&](int tslot, int qslot) __attribute__((always_inline)) {
        const u32x4_t *A = reinterpret_cast<const u32x4_t *>(smem + tslot * kSlotBytes);
        bfx8_t qh[2], qm[2], ql[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            qh[i] = __builtin_bit_cast(bfx8_t, qv[qslot][i][0]);
            qm[i] = __builtin_bit_cast(bfx8_t, qv[qslot][i][1]);
            ql[i] = __builtin_bit_cast(bfx8_t, qv[qslot][i][2]);
        }
        bfx8_t th[2], tm[2], tl8[2];
        th[0] = __builtin_bit_cast(bfx8_t, A[lane]);
        tm[0] = __builtin_bit_cast(bfx8_t, A[64 + lane]);
        tl8[0] = __builtin_bit_cast(bfx8_t, A[128 + lane]);
        if constexpr (ACC2) {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int c = r & 1;
                if (r + 1 < NR) {
                    th[c ^ 1] = __builtin_bit_cast(bfx8_t, A[(3 * r + 3) * 64 + lane]);
                    tm[c ^ 1] = __builtin_bit_cast(bfx8_t, A[(3 * r + 4) * 64 + lane]);
                    tl8[c ^ 1] = __builtin_bit_cast(bfx8_t, A[(3 * r + 5) * 64 + lane]);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i) acs[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tl8[c], qh[i], acs[i][r], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) acs[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th[c], ql[i], acs[i][r], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) acs[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tm[c], qm[i], acs[i][r], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) acs[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tm[c], qh[i], acs[i][r], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) acs[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th[c], qm[i], acs[i][r], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th[c], qh[i], acc[i][r], 0, 0, 0);
            }
            // schedule: row 0's reads, then per row the next row's 3 reads ahead of its 12 MFMAs
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (r + 1 < NR) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
            }
        } else {
            f32x4_t t[2][2];  // per row: the six products of one K step, summed from zero (row parity)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int c = r & 1;
                if (r + 1 < NR) {
                    th[c ^ 1] = __builtin_bit_cast(bfx8_t, A[(3 * r + 3) * 64 + lane]);
                    tm[c ^ 1] = __builtin_bit_cast(bfx8_t, A[(3 * r + 4) * 64 + lane]);
                    tl8[c ^ 1] = __builtin_bit_cast(bfx8_t, A[(3 * r + 5) * 64 + lane]);
                }
                const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 2; ++i) t[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tl8[c], qh[i], z, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) t[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th[c], ql[i], t[c][i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) t[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tm[c], qm[i], t[c][i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) t[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tm[c], qh[i], t[c][i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) t[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th[c], qm[i], t[c][i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 2; ++i) t[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th[c], qh[i], t[c][i], 0, 0, 0);
                // the previous row's step sum joins its accumulator (one rounding per K step) while
                // this row's MFMAs run
                if (r > 0) {
#pragma unroll
                    for (int i = 0; i < 2; ++i) acc[i][r - 1] += t[c ^ 1][i];
                }
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) acc[i][NR - 1] += t[(NR - 1) & 1][i];
            // schedule: row 0's reads, then per row the next row's 3 reads ahead of its 12 MFMAs and
            // the previous row's 8 accumulator adds behind them
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (r + 1 < NR) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
                if (r > 0) __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        }
    };

    if constexpr (SS > 0) {
        if constexpr ((VF & 2) != 0) __builtin_amdgcn_s_setprio(1);
        issue_q(0, 0);
        if (SS > 1) issue_q(1, 1);
        issue_t(0, 0);
        if (QD > 2 && SS > 2) issue_q(2, 2);
        if (SS > 1) issue_t(1, 1);
#pragma unroll
        for (int s = 0; s < SS; ++s) {
            // operations younger than T(s): at step 0 the prologue's [Q2,] T1; else step s - 1's
            // group Q(s - 1 + QD), T(s + 1) — where they exist
            const int younger = s == 0 ? (QD > 2 && SS > 2 ? kQLoads : 0) + (SS > 1 ? DPW : 0)
                                       : (s - 1 + QD < SS ? kQLoads : 0) + (s + 1 < SS ? DPW : 0);
            if (younger == kQLoads + DPW) wait_vmcnt_barrier<kQLoads + DPW>();
            else if (younger == DPW) wait_vmcnt_barrier<DPW>();
            else if (younger == kQLoads) wait_vmcnt_barrier<kQLoads>();
            else wait_vmcnt_barrier<0>();
            const int qs = s % QS;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                asm volatile("" : "+v"(qv[qs][i][0]), "+v"(qv[qs][i][1]), "+v"(qv[qs][i][2]));
            if (s + QD < SS) issue_q(s + QD, (s + QD) % QS);
            if (s + 2 < SS) issue_t(s + 2, (s + 2) % kRing);
            if (qact) compute(s % kRing, qs);  // a wave whose queries all lie past NQ skips its MFMAs
        }
        if constexpr ((VF & 2) != 0) __builtin_amdgcn_s_setprio(0);
    } else {
        // any S: no prefetch (one group in flight, drained every step)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int s = 0; s < S; ++s) {
            issue_q(s, 0);
            issue_t(s, 0);
            wait_vmcnt_barrier<0>();
            if (qact) compute(0, 0);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // slot 0 is refilled next
        }
    }

    // ---- epilogue: 1/sqrt(D), level 0 from registers, levels 1-3 in registers ----
    // MFMA block rp (patch tile (rp / 4, rp % 4)) leaves lane (grp, ci) with row grp of that tile
    // for query ci.  Writing lane grp = 2 h + k:
    //   level 0: one 16-B tile row per block; the four lanes of a query fill one 64-B tile per
    //            store instruction (the pyramid's tile, corr_common.h);
    //   level 1: row Y = 2 tr + h of the patch's level 1 comes from tile rows 2h, 2h + 1 — lanes
    //            (h, 0) and (h, 1), 16 apart: each takes level-1 tile k (columns 4k .. 4k + 3) and
    //            trades the other tile pair's row with its partner; one 16-B store per tr;
    //   level 2: row Y2 = h from level-1 rows 2h, 2h + 1 — lanes (0, k), (1, k), 32 apart; the
    //            lanes (h, 0), (h, 1) then meet for the 16-B row, one store per lane over the two
    //            query blocks; level 3 as level 2 with the pair 32 apart, one cell per lane.
    // Every pool is ((a + b) + c) + d in avg_pool2d's order (bit-identical).  A store runs whenever
    // its tile row lies in the padded map (cells past W_l / H_l are padding: the zero-padded target
    // records make them finite, nothing reads them).
    const int H = p.H, W = p.W, NQ = p.NQ, nlev = FAST ? 4 : p.nlev;
    const int H1 = H >> 1, W1 = W >> 1, H2 = H >> 2, W2 = W >> 2, H3 = H >> 3, W3 = W >> 3;
    const int TC0 = map_tcols(W), TC1 = map_tcols(W1), TC2 = map_tcols(W2), TC3 = map_tcols(W3);
    const int R0 = 4 * map_tiles(H), R1 = 4 * map_tiles(H1), R2 = 4 * map_tiles(H2), R3 = 4 * map_tiles(H3);
    const size_t M0 = map_floats(H, W), M1 = map_floats(H1, W1), M2 = map_floats(H2, W2), M3 = map_floats(H3, W3);
    const int h = grp >> 1, k = grp & 1;
    float l2s[2][2];  // level 2 of both query blocks: (Y2 = h, X2 = 2k + j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = (qb0 + i) * 16 + ci;
        const bool qok = q < NQ;
        const size_t qrow = (size_t)b * NQ + q;
        float v[kPatchRows][4];  // v[rp][c]: patch cell (4 (rp >> 2) + grp, 4 (rp & 3) + c)
#pragma unroll
        for (int r = 0; r < kPatchRows; ++r)
#pragma unroll
            for (int g = 0; g < 4; ++g) v[r][g] = (ACC2 ? split_sum(acc[i][r][g], acs[i][r][g]) : acc[i][r][g]) * p.inv_s;
        if (qok && nlev > 0) {
            float *m0 = p.lvl[0] + qrow * M0;
#pragma unroll
            for (int rp = 0; rp < kPatchRows; ++rp) {
                const int Y = y0 + 4 * (rp >> 2) + grp, T = (x0 >> 2) + (rp & 3);
                if (Y < R0 && 4 * T < W)
                    *reinterpret_cast<float4 *>(m0 + map_row4(Y, T, TC0)) = make_float4(v[rp][0], v[rp][1], v[rp][2], v[rp][3]);
            }
        }
        float l1[2][4];  // l1[tr][m]: level-1 cell (2 tr + h, 4k + m) of the patch
#pragma unroll
        for (int tr = 0; tr < 2; ++tr) {
            float top[2][4], bot[2][4];  // rows 2h, 2h + 1 of tiles 4 tr + 2k + j
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float mine = k ? v[4 * tr + 2 + j][c] : v[4 * tr + j][c];
                    const float give = k ? v[4 * tr + j][c] : v[4 * tr + 2 + j][c];
                    const float got = __shfl_xor(give, 16);
                    top[j][c] = k ? got : mine;
                    bot[j][c] = k ? mine : got;
                }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int j = m >> 1, c = 2 * (m & 1);
                l1[tr][m] = pool4(top[j][c], top[j][c + 1], bot[j][c], bot[j][c + 1]);
            }
            const int Y1 = (y0 >> 1) + 2 * tr + h, T1 = (x0 >> 3) + k;
            if (qok && nlev > 1 && Y1 < R1 && 4 * T1 < W1)
                *reinterpret_cast<float4 *>(p.lvl[1] + qrow * M1 + map_row4(Y1, T1, TC1)) =
                    make_float4(l1[tr][0], l1[tr][1], l1[tr][2], l1[tr][3]);
        }
        // level 2 (Y2 = h, X2 = 2k + j): level-1 rows 2h (lane (0, k), tr = h) and 2h + 1 (lane (1, k))
        float top[4], bot[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float give = h ? l1[0][m] : l1[1][m];
            const float got = __shfl_xor(give, 32);
            top[m] = h ? got : l1[0][m];
            bot[m] = h ? l1[1][m] : got;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) l2s[i][j] = pool4(top[2 * j], top[2 * j + 1], bot[2 * j], bot[2 * j + 1]);
    }
    {
        // Level 2 rows of BOTH blocks, one 16-B store per lane: lane (h, k) stores row h of block k;
        // lanes (h, 0), (h, 1) hold columns 0-1 / 2-3 and trade the other block's pair.
        const float g0 = __shfl_xor(k ? l2s[0][0] : l2s[1][0], 16), g1 = __shfl_xor(k ? l2s[0][1] : l2s[1][1], 16);
        const float o0 = k ? l2s[1][0] : l2s[0][0], o1 = k ? l2s[1][1] : l2s[0][1];
        const float4 o = k ? make_float4(g0, g1, o0, o1) : make_float4(o0, o1, g0, g1);
        const int q = (qb0 + k) * 16 + ci, Y2 = (y0 >> 2) + h;
        if (q < NQ && nlev > 2 && Y2 < R2 && (x0 >> 2) < W2)
            *reinterpret_cast<float4 *>(p.lvl[2] + ((size_t)b * NQ + q) * M2 + map_row4(Y2, x0 >> 4, TC2)) = o;
    }
    {
        // Level 3, cell X3 = k of block h: level-2 rows 0 (lanes (0, k)) and 1 (lanes (1, k)).
        const float g0 = __shfl_xor(h ? l2s[0][0] : l2s[1][0], 32), g1 = __shfl_xor(h ? l2s[0][1] : l2s[1][1], 32);
        const float l3 = h ? pool4(g0, g1, l2s[1][0], l2s[1][1]) : pool4(l2s[0][0], l2s[0][1], g0, g1);
        const int q = (qb0 + h) * 16 + ci;
        const int Y3 = y0 >> 3, X3 = (x0 >> 3) + k;
        if (q < NQ && nlev > 3 && Y3 < R3 && X3 < kTileW * TC3) p.lvl[3][((size_t)b * NQ + q) * M3 + map_cell(Y3, X3, TC3)] = l3;
    }
}

template <int SS, bool ACC2 = true, int VF = 0, bool FAST = false>
__global__ __launch_bounds__(256, 2) void corr_build_bf16_kernel(Args p) {
    const int t = xcd_swizzle(blockIdx.x, gridDim.x);
    Tile tl = p.order == 2 ? xcd_block_tile(p, t) : patch_tile(t, p.npatch, p.NQG, p.CB, p.order, p.gq);
    tl.py += p.py0;
    // two whole code paths (no value flows out of either): a half patch runs half the MFMAs
    if (!(VF & 4) && SS > 0 && tl.py * kPatchRows + kPatchRows / 2 >= p.H)
        build_tile<SS, kPatchRows / 2, ACC2, VF, FAST>(p, tl);
    else
        build_tile<SS, kPatchRows, ACC2, VF, FAST>(p, tl);
}

struct Ws {
    u32x4_t *pq, *pt;
};

inline Ws workspace_of(void *ws, int B, const Geom &g) {
    char *w = (char *)ws;
    Ws r;
    r.pq = (u32x4_t *)w;
    w += align256((size_t)B * g.S * g.NQp * kPixBytes);
    r.pt = (u32x4_t *)w;
    return r;
}

template <int SS, bool ACC2 = true, int VF = 0>
hipError_t launch_kernel(dim3 grid, const Args &p, hipStream_t s) {
    const bool fast = p.nlev == 4;
    static std::atomic<unsigned long long> lds_done[2];
    const void *fn = fast ? (const void *)corr_build_bf16_kernel<SS, ACC2, VF, true>
                          : (const void *)corr_build_bf16_kernel<SS, ACC2, VF, false>;
    const hipError_t e = ensure_lds_limit(fn, kLds, lds_done[fast]);
    if (e != hipSuccess) return e;
    const dim3 blk(256);
    if (fast)
        hipLaunchKernelGGL((corr_build_bf16_kernel<SS, ACC2, VF, true>), grid, blk, kLds, s, p);
    else
        hipLaunchKernelGGL((corr_build_bf16_kernel<SS, ACC2, VF, false>), grid, blk, kLds, s, p);
    return hipGetLastError();
}


// Workspace: the packed query and target images (3 KiB per K step and 16-pixel block).
size_t workspace_bytes(int B, int D, int NQ, int H, int W) {
    const Geom g = geom(D, NQ, H, W);
    return align256((size_t)B * g.S * g.NQp * kPixBytes) + align256((size_t)B * g.S * g.Hp * g.Wp * kPixBytes);
}

// Packs the queries (pack_q) and the target rows [y0, y1) (f2 = that slab, [B][D][y1 - y0][W];
// y0 a multiple of 8, y1 a multiple of 8 or H): the patch rows [y0 / 8, ceil(y1 / 8)).
// rpw: records per wave (bf16_pack_kernel's R); 0 = by size: 4 once there are >= 8192 records
// (train B8 15.4 -> 14.0 us, MVSEC B16 29.9 -> 27.7 us), else 1 (DSEC's 4,800 records: 6.3 us
// with one, 8.5 with four — a single round of workgroups, profiles/r06g_kbench_pack_rpw.txt).
hipError_t launch_pack(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, void *ws,
                       hipStream_t s, int y0 = 0, int y1 = -1, bool pack_q = true, int rpw = 0) {
    if (y1 < 0) y1 = H;
    const Geom g = geom(D, NQ, H, W);
    const Ws w = workspace_of(ws, B, g);
    PackArgs a{};
    a.f[0] = f1, a.f[1] = f2;
    a.pk[0] = w.pq, a.pk[1] = w.pt;
    a.np[0] = NQ, a.np[1] = (y1 - y0) * W;
    const int nyp = (y1 + kPatchRows - 1) / kPatchRows * kPatchRows - y0;
    a.nblk[0] = g.NQB, a.nblk[1] = nyp * g.CB;
    a.img[0] = g.NQB, a.img[1] = g.Hp * g.CB;
    a.D = D, a.S = g.S, a.W = W, a.CB = g.CB, a.y0 = y0, a.y1 = y1;
    a.z0 = pack_q ? 0 : 1;
    const int recs = g.S * std::max(pack_q ? a.nblk[0] : 0, a.nblk[1]);
    if (rpw == 0) rpw = (long)recs * B * (pack_q ? 2 : 1) >= 8192 ? 4 : 1;
    const dim3 blk(256);
    if (rpw == 4)
        hipLaunchKernelGGL(bf16_pack_kernel<4>, dim3((unsigned)((recs + 15) / 16), B, pack_q ? 2 : 1), blk, 0, s, a);
    else if (rpw == 2)
        hipLaunchKernelGGL(bf16_pack_kernel<2>, dim3((unsigned)((recs + 7) / 8), B, pack_q ? 2 : 1), blk, 0, s, a);
    else
        hipLaunchKernelGGL(bf16_pack_kernel<1>, dim3((unsigned)((recs + 3) / 4), B, pack_q ? 2 : 1), blk, 0, s, a);
    return hipGetLastError();
}

// The MFMA part (operands already packed in ws).  levels == 0: the MFMAs and epilogue
// arithmetic without stores (measurement).  variant (tools/kbench_build.hip A/B, D = 256 only):
// 1 = the single-accumulator form (ACC2 = false), 2..4 = VF 1..3, 5 = VF 4.
// y0, y1: the target region (as launch_pack), whose pyramid rows [y0 >> l, ceil(y1 / 2^l)) of
// every level it writes.
hipError_t launch_mfma(int NQ, int B, int D, int H, int W, int levels, const LevelPtrs &pyr, void *ws,
                       hipStream_t s, int variant = 0, int order = 1, int y0 = 0, int y1 = -1, int gq = 0) {
    if (y1 < 0) y1 = H;
    const Geom g = geom(D, NQ, H, W);
    const Ws w = workspace_of(ws, B, g);
    Args p{};
    p.pq = w.pq, p.pt = w.pt;
    p.B = B, p.H = H, p.W = W, p.N = H * W, p.NQ = NQ, p.S = g.S;
    p.nlev = std::min(levels, kFusedLevels);
    for (int l = 0; l < kFusedLevels; ++l) p.lvl[l] = l < p.nlev ? pyr.p[l] : nullptr;
    p.NQp = g.NQp, p.NQB = g.NQB, p.NQG = g.NQG, p.Hp = g.Hp, p.CB = g.CB;
    p.py0 = y0 / kPatchRows;
    p.npatch = ((y1 + kPatchRows - 1) / kPatchRows - p.py0) * g.CB;
    p.s = std::sqrt((float)D);
    p.inv_s = 1.0f / p.s;
    p.exact = is_pow2(p.s);
    // XCD blocks: split each batch item into 8 / B blocks (2 x 4 for one item), so the 8 XCDs
    // get disjoint operand sets; B >= 8: one or more whole batch items per XCD
    p.order = order;
    // query groups per L2 band: 4 for one batch item (DSEC 78.7 -> 75.2 us, 1280x960 1,042 -> 1,019,
    // 1920x1280 4,321 -> 4,276), the default 8 for batches (MVSEC B16 prefers it: 141 vs 146 us;
    // train B8 even) — profiles/r06d_kbench_build_tile_groups_dropped.txt, r06k_*
    p.gq = gq > 0 ? gq : (B == 1 ? 4 : kGroupQ);
    const int per = B >= 8 ? 1 : 8 / B;
    p.nqh = per >= 2 && g.NQG >= 2 ? 2 : 1;
    p.npq = std::max(1, std::min(per / p.nqh, p.npatch));
    const long tiles = (long)B * p.npatch * p.NQG;
    if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
    const dim3 grid((unsigned)tiles);
    hipError_t e;
    if (variant != 0) {
        if (g.S != 8) return hipErrorInvalidValue;
        switch (variant) {
            case 1: e = launch_kernel<8, false>(grid, p, s); break;
            case 2: e = launch_kernel<8, true, 1>(grid, p, s); break;
            case 3: e = launch_kernel<8, true, 2>(grid, p, s); break;
            case 4: e = launch_kernel<8, true, 3>(grid, p, s); break;
            case 5: e = launch_kernel<8, true, 4>(grid, p, s); break;
            default: return hipErrorInvalidValue;
        }
    } else switch (g.S <= 8 ? g.S : 0) {
#define CORR_BF16_CASE(c) \
    case c: e = launch_kernel<c>(grid, p, s); break;
        CORR_BF16_CASE(0) CORR_BF16_CASE(1) CORR_BF16_CASE(2) CORR_BF16_CASE(3) CORR_BF16_CASE(4)
        CORR_BF16_CASE(5) CORR_BF16_CASE(6) CORR_BF16_CASE(7) CORR_BF16_CASE(8)
#undef CORR_BF16_CASE
        default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    if (levels > kFusedLevels) return launch_pool_levels(pyr, kFusedLevels, levels, (long)B * NQ, H, W, s);
    return hipSuccess;
}

}  // namespace bf16b

size_t build_bf16_workspace(int B, int D, int NQ, int H, int W) {
    return bf16b::workspace_bytes(B, D, NQ, H, W);
}

// part: 0 = pack + MFMA; 1 = the pack alone; 2 = the MFMA kernel alone (measurement: the
// workspace must already hold this pair's pack).
hipError_t launch_build_bf16(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, int levels,
                             const LevelPtrs &pyr, void *ws, hipStream_t s, int part) {
    if (part != 2) {
        const hipError_t e = bf16b::launch_pack(f1, NQ, f2, B, D, H, W, ws, s);
        if (e != hipSuccess || part == 1) return e;
    }
    return bf16b::launch_mfma(NQ, B, D, H, W, levels, pyr, ws, s);
}

// One target region [y0, y1) of the build (corr_build_region): f2_rows holds those fmap2 rows.
hipError_t launch_build_bf16_region(const float *f1, int NQ, const float *f2_rows, int y0, int y1, int B, int D,
                                    int H, int W, int levels, const LevelPtrs &pyr, void *ws, bool pack_q,
                                    hipStream_t s) {
    const hipError_t e = bf16b::launch_pack(f1, NQ, f2_rows, B, D, H, W, ws, s, y0, y1, pack_q);
    if (e != hipSuccess) return e;
    return bf16b::launch_mfma(NQ, B, D, H, W, levels, pyr, ws, s, 0, 1, y0, y1);
}

}  // namespace corr
