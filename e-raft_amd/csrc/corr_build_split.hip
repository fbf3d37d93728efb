// corr_build_split.hip — the all-pairs build and its pyramid on gfx950's f16 MFMA at fp32
// accuracy.  Replaces CorrBlock.corr (model/corr.py:52-60: matmul(F1^T, F2) / sqrt(D)) and the
// pyramid loop of CorrBlock.__init__ (model/corr.py:21-27).
//
// Operands.  Every fp32 feature x of pixel n is rewritten as
//     x = 2^e_n * (hi + lo) + O(2^-22 |x|),   hi = f16(x * 2^-e_n),  lo = f16(x * 2^-e_n - hi)
// with a per-pixel power-of-two e_n that puts the pixel's largest |x| in [2^14, 2^15): neither
// half overflows, and the f16 subnormal floor lies 2^-38 below the pixel's largest value.  A dot
// product is then three f16 MFMAs into ONE fp32 accumulator,
//     acc += lo_t * hi_q;   acc += hi_t * lo_q;   acc += hi_t * hi_q,
// whose f16 x f16 products are exact in fp32; what is dropped (lo*lo, the lo rounding) is
// <= 2^-22 relative per term.  The epilogue restores 2^(e_q + e_t) (exact ldexp) and applies
// 1/sqrt(D) as the fp32 build does.
//
// MFMA orientation.  v_mfma_f32_16x16x32_f16 with A = TARGETS (rows) and B = QUERIES (columns):
// lane l = 16 grp + ci owns query ci of a 16-query block and, in its 4 accumulator registers,
// targets 4 grp .. 4 grp + 3 of a 16-target block.  A target block is one 4x4 tile of the
// pyramid (corr_common.h), so lane (grp, ci) holds tile row grp for query ci and the four lanes
// of a query store the whole 64-B tile in one store instruction; a wave's 8 blocks are an 8 x 16
// target patch (2 x 4 tiles), whose levels 1-3 pool across lanes 16 / 32 apart in the
// reference's ((a+b)+c)+d order (shuffles, no LDS staging).
//
// Workgroup = 4 waves x 32 queries against ONE 8 x 16 target patch.  The patch's operand
// records (16 KiB per 32-deep K step) stream into a 3-slot LDS ring by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction) two steps ahead, shared by the four
// waves; each wave loads its own queries' records straight into registers, also two steps
// ahead.  One barrier per K step.  Two workgroups per CU (49.7 KiB LDS each, <= 256 VGPRs).
//
// Packed operand images (split_pack_wide_kernel), one 2 KiB record per (K step s, 16-pixel block):
//   bytes [0, 1024)    hi: lane l = 16 grp + ci at 16 l: 8 f16 of k = 32 s + 8 grp + j, pixel ci
//   bytes [1024, 2048) lo: the same positions
// i.e. exactly the MFMA fragment image of that block, so the LDS fill and every fragment read
// are contiguous 1 KiB (conflict-free ds_read_b128, coalesced loads).
//   pq [B][S][NQB][2 KiB]     queries: block = 16 consecutive query pixels, NQp = NQB*16
//   pt [B][S][Hp/4][4 CB][2 KiB]  targets: block = the 4x4 tile (rows 4 ty .., columns 4 tx ..),
//                                 pixel ci at (ci / 4, ci % 4) — the pyramid's tile (corr_common.h)
//   eq [B][NQp], et [B][Hp][Wp] int32 exponents.  Padding pixels are zero (exponent 0).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <utility>

#include "corr_build_common.h"

namespace corr {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kStepK = 32;                          // k per MFMA step
constexpr int kRecU = 128;                          // u32x4 per record (2 KiB)
constexpr int kPatchRows = 8;                       // target patch: 8 rows x 16 columns
constexpr int kWaves = 4, kQPerWave = 32;           // 2 query blocks per wave
constexpr int kQPerWG = kWaves * kQPerWave;         // 128
constexpr int kRing = 3;                            // LDS ring slots (prefetch distance 2)
constexpr int kSlotBytes = kPatchRows * 2 * 1024;   // 16 KiB per K step
constexpr int kBuildLds = kRing * kSlotBytes + kPatchRows * 16 * 4;
constexpr int kMaxPackCpt = 8;                      // D <= 1024

struct SplitGeom {
    int S, NQp, NQB, NQG, Hp, CB, Wp;
};

inline SplitGeom split_geom(int D, int NQ, int H, int W) {
    SplitGeom g;
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
// Operand pack.  One workgroup per (16-pixel block, batch item, tensor); thread = (pixel ci,
// k-octet).  A wave's store instructions each write one record half: 1 KiB contiguous.
// ---------------------------------------------------------------------------------------
struct PackArgs {
    const float *f[2];
    u32x4 *pk[2];
    int *ex[2];
    int np[2];    // source pixels per batch item: NQ, H*W
    int nblk[2];  // blocks per batch item in the image: NQB, Hp*CB
    int D, S, H, W, CB, Hp, Wp, NQp;
};

// Operand pack, wide form: one workgroup per PX pixels (PX / 16 image blocks) of one batch
// item and tensor; wave w owns K steps [SPW w, SPW (w + 1)), lane = (pixel, octet half): with
// PX = 64 a lane holds its pixel's 4 k octets of a step, with PX = 32 two of them.  Every load
// instruction reads whole feature rows of the PX pixels (PX * 4-B runs where the blocks are
// contiguous), the pixel maxima meet in LDS, and each lane writes its own 16-B pieces of the
// records.
template <int SPW, int PX>
__global__ __launch_bounds__(512) void split_pack_wide_kernel(PackArgs a) {
    constexpr int OPL = 4 * PX / 64;  // k octets per lane and step
    __shared__ float red[8][64];
    const int z = blockIdx.z, b = blockIdx.y;
    const int nblk = a.nblk[z];
    if ((int)blockIdx.x * (PX / 16) >= nblk) return;  // the grid covers the larger image (uniform exit)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
    const int pix = lane % PX, o0 = (lane / PX) * OPL;
    const int blk = blockIdx.x * (PX / 16) + (pix >> 4), ci = pix & 15;
    int n, exi;
    bool valid;
    if (z == 0) {
        n = blk * 16 + ci;
        valid = blk < nblk && n < a.np[0];
        exi = b * a.NQp + n;
    } else {
        // target block = the 4x4 tile (tile row ty, column tx; 4 CB tiles per row), pixel ci at
        // (ci / 4, ci % 4): each 16x16 MFMA output block is one pyramid tile (as in the bf16x6 pack)
        const int TCp = 4 * a.CB, ty = blk / TCp, tx = blk - ty * TCp;
        const int y = 4 * ty + (ci >> 2), x = 4 * tx + (ci & 3);
        valid = blk < nblk && y < a.H && x < a.W;
        n = y * a.W + x;
        exi = (b * a.Hp + y) * a.Wp + x;
    }
    const int NP = a.np[z], D = a.D;
    const float *src = a.f[z] + (size_t)b * D * NP + (valid ? n : 0);
    float v[SPW][8 * OPL];
#pragma unroll
    for (int c = 0; c < SPW; ++c)
#pragma unroll
        for (int j = 0; j < 8 * OPL; ++j) {
            const int d = (SPW * w + c) * kStepK + 8 * o0 + j;
            v[c][j] = (valid && d < D) ? src[(size_t)d * NP] : 0.f;
        }
    float m = 0.f;
#pragma unroll
    for (int c = 0; c < SPW; ++c)
#pragma unroll
        for (int j = 0; j < 8 * OPL; ++j) m = fmaxf(m, fabsf(v[c][j]));
    red[w][lane] = m;
    __syncthreads();
    float mm = 0.f;
    for (int i = 0; i < nw; ++i)
#pragma unroll
        for (int h = 0; h < 64 / PX; ++h) mm = fmaxf(mm, red[i][pix + PX * h]);
    int s = 0;
    if (mm > 0.f && mm <= 3.402823466e38f) {
        int E;
        (void)frexpf(mm, &E);  // mm < 2^E
        s = 15 - E;            // mm * 2^s < 2^15: neither half overflows
    }
    if (w == 0 && lane < PX && blk < nblk) a.ex[z][exi] = -s;
#pragma unroll
    for (int c = 0; c < SPW; ++c) {
        const int ks = SPW * w + c;  // K step
        if (ks >= a.S || blk >= nblk) break;
        u32x4 *rec = a.pk[z] + (((size_t)b * a.S + ks) * nblk + blk) * kRecU;
#pragma unroll
        for (int oo = 0; oo < OPL; ++oo) {  // k octet of the step = fragment lane group
            const int o = o0 + oo;
            half8 hi8, lo8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float y = ldexpf(v[c][8 * oo + j], s);
                const _Float16 hi = (_Float16)y;
                hi8[j] = hi;
                lo8[j] = __builtin_isinf(y) ? (_Float16)0.f : (_Float16)(y - (float)hi);
            }
            rec[16 * o + ci] = __builtin_bit_cast(u32x4, hi8);
            rec[64 + 16 * o + ci] = __builtin_bit_cast(u32x4, lo8);
        }
    }
}

// ---------------------------------------------------------------------------------------
// The MFMA build.
// ---------------------------------------------------------------------------------------
struct BuildArgs {
    const u32x4 *pq, *pt;
    const int *eq, *et;
    float *lvl[kFusedLevels];
    int B, H, W, N, NQ, S, nlev;
    int NQp, NQB, NQG, Hp, CB, Wp, npatch;
    int eshift;      // log2(1/sqrt(D)) when that is exact (folded into the exponent), else 0
    int exact;       // 1/sqrt(D) is a power of two
    float inv_s;     // 1/sqrt(D) otherwise (multiplied: within tolerance, not bitwise)
    int order;       // tile order: 0 = query group fastest (groups of kGroupQ), 1 = patch column fastest
};

__device__ __forceinline__ Tile tile_of(const BuildArgs &p, int t) {
    return patch_tile(t, p.npatch, p.NQG, p.CB, p.order);
}

// SS > 0: S = SS K steps, fully unrolled (straight-line code: the compiler's own waits on the
// query registers are then exact and never drain the prefetch).  SS = 0: any S, runtime loop.
// QS: query register slots (the query prefetch distance is QS - 1 K steps).  PIPE: the target
// fragments of map row r + 1 are read from LDS while row r's six MFMAs issue (the LDS latency
// is hidden instead of exposed once per row); the per-accumulator product order is unchanged.
// NR: map rows of the patch whose MFMAs run (8; 4 for a patch with at most 4 rows inside the
// map: the last patch row when H % 8 is 1-4, i.e. DSEC, train, MVSEC — its rows 4-7 are padding
// whose accumulators stay zero and whose stores are dropped).
template <int SS, int QS, bool PIPE, int NR>
__device__ __forceinline__ void build_tile(const BuildArgs &p, const Tile tl) {
    static_assert(QS == 3 || QS == 4, "query slots (prefetch distance 2 or 3)");
    extern __shared__ __attribute__((aligned(16))) char smem_build[];
    char *smem = smem_build;
    int *lds_et = reinterpret_cast<int *>(smem + kRing * kSlotBytes);

    const int b = tl.b, y0 = tl.py * kPatchRows, x0 = tl.cb * 16;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ci = lane & 15, grp = lane >> 4;
    const int qb0 = tl.qg * (kQPerWG / 16) + 2 * w;  // this wave's first 16-query block
    const int S = SS > 0 ? SS : p.S;
    const bool qact = qb0 * 16 < p.NQ;  // wave-uniform

    // The patch's target exponents -> LDS by LDS-DMA (waves 0 and 1, one dword per lane) and
    // the query exponents -> registers, issued ahead of the operand stream and never waited for
    // on their own: they are older than every counted DMA, so step 0's wait covers them (the
    // epilogue reads them after several barriers).  No memory round trip before the first load.
    if (SS > 0 && w < 2) {
        const int idx = w * 64 + lane;
        dma4(p.et + ((size_t)b * p.Hp + y0 + (idx >> 4)) * p.Wp + x0 + (idx & 15),
             (uint32_t)(uintptr_t)(lds_void_t *)lds_et + w * 256);
    } else if (SS == 0 && tid < kPatchRows * 16) {
        lds_et[tid] = p.et[((size_t)b * p.Hp + y0 + (tid >> 4)) * p.Wp + x0 + (tid & 15)];
    }
    int eqv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) eqv[i] = p.eq[(size_t)b * p.NQp + (qb0 + i) * 16 + ci] + p.eshift;

    // LDS-DMA pieces of this wave: pc = w + 4 m -> patch block rp = pc >> 1 (tile row rp / 4, tile
    // column rp % 4 of the patch), half pc & 1
    const int TCp = 4 * p.CB;                           // tiles per row of the target image
    const size_t tstep = (size_t)p.Hp * p.CB * kRecU;  // u32x4 per K step of the target image
    const u32x4 *tsrc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int pc = w + 4 * m, rp = pc >> 1;
        tsrc[m] = p.pt + (((size_t)b * S * (p.Hp >> 2) + (y0 >> 2) + (rp >> 2)) * TCp + 4 * tl.cb + (rp & 3)) * kRecU +
                  (pc & 1) * 64 + lane;
    }
    const size_t qstep = (size_t)p.NQB * kRecU;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_void_t *)smem;
    const u32x4 *qsrc = p.pq + ((size_t)b * S * p.NQB + qb0) * kRecU + lane;

    // Issue schedule (SS > 0, fully unrolled): step k issues the wave's 4 query loads of step
    // k + QS - 1 (into register slot (k + QS - 1) % QS), then its 4 LDS-DMA pieces of step k + 2
    // (ring slot (k + 2) % 3); the prologue plays the steps before 0.  The DMA is inline asm, so
    // the compiler does not make every ds_read wait for ALL outstanding DMAs (it cannot tell the
    // ring slots apart).  At step k's barrier the operations younger than its DMA are exactly
    // the later groups (vmcnt(8) or (4)), and every query load of step k is older; the query
    // registers are then passed through an empty asm, before which the compiler's own wait
    // (counting only the query loads it knows of) is already satisfied: no drain.
    u32x4 qv[QS][2][2];  // [register slot][query block][hi, lo]
    auto issue_q = [&](int s, int slot) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const u32x4 *q = qsrc + s * qstep + i * kRecU;
            qv[slot][i][0] = q[0];
            qv[slot][i][1] = q[64];
        }
    };
    auto issue_t = [&](int s, int slot) __attribute__((always_inline)) {
        const uint32_t base = lds_base + slot * kSlotBytes;
#pragma unroll
        for (int m = 0; m < 4; ++m) dma16(tsrc[m] + s * tstep, base + (w + 4 * m) * 1024);
    };

    f32x4 acc[2][kPatchRows];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < kPatchRows; ++r) acc[i][r] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int tslot, int qslot) __attribute__((always_inline)) {
        const u32x4 *A = reinterpret_cast<const u32x4 *>(smem + tslot * kSlotBytes);
        half8 qh[2], ql[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            qh[i] = __builtin_bit_cast(half8, qv[qslot][i][0]);
            ql[i] = __builtin_bit_cast(half8, qv[qslot][i][1]);
        }
        if constexpr (PIPE) {
            half8 fh[2], fl[2];
            fh[0] = __builtin_bit_cast(half8, A[lane]);
            fl[0] = __builtin_bit_cast(half8, A[64 + lane]);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int c = r & 1;
                if (r + 1 < NR) {
                    fh[c ^ 1] = __builtin_bit_cast(half8, A[(2 * r + 2) * 64 + lane]);
                    fl[c ^ 1] = __builtin_bit_cast(half8, A[(2 * r + 3) * 64 + lane]);
                }
                acc[0][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fl[c], qh[0], acc[0][r], 0, 0, 0);
                acc[1][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fl[c], qh[1], acc[1][r], 0, 0, 0);
                acc[0][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[c], ql[0], acc[0][r], 0, 0, 0);
                acc[1][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[c], ql[1], acc[1][r], 0, 0, 0);
                acc[0][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[c], qh[0], acc[0][r], 0, 0, 0);
                acc[1][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[c], qh[1], acc[1][r], 0, 0, 0);
            }
            // schedule: row 0's reads, then per row the next row's 2 reads ahead of its 6 MFMAs
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (r + 1 < NR) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
            }
        } else {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const half8 ah = __builtin_bit_cast(half8, A[(2 * r) * 64 + lane]);
                const half8 al = __builtin_bit_cast(half8, A[(2 * r + 1) * 64 + lane]);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    acc[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, qh[i], acc[i][r], 0, 0, 0);
                    acc[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, ql[i], acc[i][r], 0, 0, 0);
                    acc[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, qh[i], acc[i][r], 0, 0, 0);
                }
            }
        }
    };

    if constexpr (SS > 0) {
        constexpr int QD = QS - 1;  // query prefetch distance (>= 2: Q(s) is issued before T(s))
        // prologue: Q0 Q1 T0 [Q2] T1 (Q0 T0 Q1 T1 Q2 with the query loads hidden from the
        // compiler's vmcnt accounting measured no faster: profiles/r03c_kbench_build_early_dropped.txt)
        issue_q(0, 0);
        if (SS > 1) issue_q(1, 1);
        issue_t(0, 0);
        if (QD > 2 && SS > 2) issue_q(2, 2);
        if (SS > 1) issue_t(1, 1);
#pragma unroll
        for (int s = 0; s < SS; ++s) {
            // operations younger than step s's DMA T(s): at step 0 the prologue's later loads,
            // else step s - 1's group (Q(s - 1 + QD), T(s + 1), where they exist)
            const int younger = s == 0 ? (QD > 2 && SS > 2 ? 4 : 0) + (SS > 1 ? 4 : 0)
                                       : (s - 1 + QD < SS ? 4 : 0) + (s + 1 < SS ? 4 : 0);
            if (younger == 8) wait_vmcnt_barrier<8>();
            else if (younger == 4) wait_vmcnt_barrier<4>();
            else wait_vmcnt_barrier<0>();
            const int qs = s % QS;
            asm volatile("" : "+v"(qv[qs][0][0]), "+v"(qv[qs][0][1]), "+v"(qv[qs][1][0]), "+v"(qv[qs][1][1]));
            if (s + QD < SS) issue_q(s + QD, (s + QD) % QS);
            if (s + 2 < SS) issue_t(s + 2, (s + 2) % kRing);
            if (qact) compute(s % kRing, qs);  // a wave whose queries all lie past NQ skips its MFMAs
        }
    } else {
        // any S: no prefetch (one group in flight, drained every step)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int s = 0; s < S; ++s) {
            issue_q(s, 0);
            issue_t(s, 0);
            wait_vmcnt_barrier<0>();
            compute(0, 0);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // slot 0 is refilled next
        }
    }

    // ---- epilogue: exponents, 1/sqrt(D), level 0 from registers, levels 1-3 in registers ----
    // MFMA block r (patch tile (r / 4, r % 4)) leaves lane (grp, ci) with row grp of that tile for
    // query ci: level 0 as whole 64-B tiles per store instruction, levels 1-3 pooled across lanes
    // 16 / 32 apart — corr_build_bf16.hip's epilogue, which describes the lane roles.
    const int h = grp >> 1, k = grp & 1;
    int et[kPatchRows][4];  // exponents of patch cell (4 (r >> 2) + grp, 4 (r & 3) + g)
#pragma unroll
    for (int r = 0; r < kPatchRows; ++r) {
        const int4 e4 = reinterpret_cast<const int4 *>(lds_et)[(4 * (r >> 2) + grp) * 4 + (r & 3)];
        et[r][0] = e4.x, et[r][1] = e4.y, et[r][2] = e4.z, et[r][3] = e4.w;
    }
    const int H = p.H, W = p.W, NQ = p.NQ, nlev = p.nlev;
    const int H1 = H >> 1, W1 = W >> 1, H2 = H >> 2, W2 = W >> 2, H3 = H >> 3, W3 = W >> 3;
    const int TC0 = map_tcols(W), TC1 = map_tcols(W1), TC2 = map_tcols(W2), TC3 = map_tcols(W3);
    const int R0 = 4 * map_tiles(H), R1 = 4 * map_tiles(H1), R2 = 4 * map_tiles(H2), R3 = 4 * map_tiles(H3);
    const size_t M0 = map_floats(H, W), M1 = map_floats(H1, W1), M2 = map_floats(H2, W2), M3 = map_floats(H3, W3);
    float l2s[2][2];  // level 2 of both query blocks: (Y2 = h, X2 = 2k + j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = (qb0 + i) * 16 + ci;
        const bool qok = q < NQ;
        const size_t qrow = (size_t)b * NQ + q;
        float v[kPatchRows][4];  // v[r][c]: patch cell (4 (r >> 2) + grp, 4 (r & 3) + c)
#pragma unroll
        for (int r = 0; r < kPatchRows; ++r)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float x = ldexpf(acc[i][r][g], eqv[i] + et[r][g]);
                if (!p.exact) x = x * p.inv_s;
                v[r][g] = x;
            }
        if (qok && nlev > 0) {
            float *m0 = p.lvl[0] + qrow * M0;
#pragma unroll
            for (int r = 0; r < kPatchRows; ++r) {
                const int Y = y0 + 4 * (r >> 2) + grp, T = (x0 >> 2) + (r & 3);
                if (Y < R0 && 4 * T < W)
                    *reinterpret_cast<float4 *>(m0 + map_row4(Y, T, TC0)) = make_float4(v[r][0], v[r][1], v[r][2], v[r][3]);
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

// HALF = false: measurement instantiation (one body; half patches compute their padding rows).
template <int SS, int QS = 4, bool PIPE = false, bool HALF = true>
__global__ __launch_bounds__(256, 2) void corr_build_split_kernel(BuildArgs p) {
    const Tile tl = tile_of(p, xcd_swizzle(blockIdx.x, gridDim.x));
    // two whole code paths (no value flows out of either): a half patch runs half the MFMAs
    if (HALF && SS > 0 && tl.py * kPatchRows + kPatchRows / 2 >= p.H) build_tile<SS, QS, PIPE, kPatchRows / 2>(p, tl);
    else build_tile<SS, QS, PIPE, kPatchRows>(p, tl);
}

// ---------------------------------------------------------------------------------------
// Host side.
// ---------------------------------------------------------------------------------------
namespace {
struct SplitWs {
    u32x4 *pq, *pt;
    int *eq, *et;
};

SplitWs split_ws(void *ws, int B, const SplitGeom &g) {
    char *w = (char *)ws;
    SplitWs r;
    r.pq = (u32x4 *)w;
    w += align256((size_t)B * g.S * g.NQp * 128);
    r.pt = (u32x4 *)w;
    w += align256((size_t)B * g.S * g.Hp * g.Wp * 128);
    r.eq = (int *)w;
    w += align256((size_t)B * g.NQp * 4);
    r.et = (int *)w;
    return r;
}

}  // namespace

size_t build_split_workspace(int B, int D, int NQ, int H, int W) {
    const SplitGeom g = split_geom(D, NQ, H, W);
    return align256((size_t)B * g.S * g.NQp * 128) + align256((size_t)B * g.S * g.Hp * g.Wp * 128) +
           align256((size_t)B * g.NQp * 4) + align256((size_t)B * g.Hp * g.Wp * 4);
}

bool build_split_supported(int D) { return D >= 1 && (D + kStepK - 1) / kStepK * 4 <= 16 * kMaxPackCpt; }

// px: pixels per workgroup, 0 = by grid size (32 px unless that grid reaches 1,024 workgroups:
// DSEC 7.4 us at 32 px vs 8.4 at 64; 1280x960 17.8 vs 15.7).
hipError_t launch_split_pack(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, void *ws,
                             hipStream_t s, int px = 0) {
    const SplitGeom g = split_geom(D, NQ, H, W);
    const SplitWs w = split_ws(ws, B, g);
    PackArgs a{};
    a.f[0] = f1, a.f[1] = f2;
    a.pk[0] = w.pq, a.pk[1] = w.pt;
    a.ex[0] = w.eq, a.ex[1] = w.et;
    a.np[0] = NQ, a.np[1] = H * W;
    a.nblk[0] = g.NQB, a.nblk[1] = g.Hp * g.CB;
    a.D = D, a.S = g.S, a.H = H, a.W = W, a.CB = g.CB, a.Hp = g.Hp, a.Wp = g.Wp, a.NQp = g.NQp;
    const int waves = std::min(g.S, 8), spw = (g.S + waves - 1) / waves;
    const int nb = std::max(a.nblk[0], a.nblk[1]);
    const dim3 blk(64 * waves);
    const dim3 g64((unsigned)((nb + 3) / 4), B, 2), g32((unsigned)((nb + 1) / 2), B, 2);
    const bool px32 = px == 32 || (px == 0 && (long)g32.x * B * 2 < 1024);
    switch (spw) {
        case 1:
            if (px32) hipLaunchKernelGGL((split_pack_wide_kernel<1, 32>), g32, blk, 0, s, a);
            else hipLaunchKernelGGL((split_pack_wide_kernel<1, 64>), g64, blk, 0, s, a);
            return hipGetLastError();
        case 2: hipLaunchKernelGGL((split_pack_wide_kernel<2, 64>), g64, blk, 0, s, a); return hipGetLastError();
        case 3:
        case 4: hipLaunchKernelGGL((split_pack_wide_kernel<4, 64>), g64, blk, 0, s, a); return hipGetLastError();
        default: return hipErrorInvalidValue;
    }
}

// One instantiation of the one-tile-per-workgroup kernel, its dynamic-LDS limit raised once.
template <int SS, int QS, bool PIPE, bool HALF = true>
hipError_t launch_build_kernel(dim3 grid, const BuildArgs &p, hipStream_t s) {
    static std::atomic<unsigned long long> lds_done{0};
    const hipError_t e = ensure_lds_limit((const void *)corr_build_split_kernel<SS, QS, PIPE, HALF>, kBuildLds, lds_done);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((corr_build_split_kernel<SS, QS, PIPE, HALF>), grid, dim3(256), kBuildLds, s, p);
    return hipGetLastError();
}

// The MFMA part (operands already packed in ws).  levels == 0: the MFMAs and epilogue
// arithmetic without stores (measurement).  cons: unused (the tiled pyramid's stores are always
// 16-B tile rows; kept for tools/kbench_build.hip's call signature).
// order: the build's tile order (BuildArgs::order): 1 = a patch row's patches consecutive for
// one query group (the default: 1280x960 1006 -> 948 us, DSEC / train / MVSEC 1-4 % faster,
// profiles/r03b_kbench_build_order.txt); tools/kbench_build.hip passes 0 for the A/B.
hipError_t launch_split_mfma(int NQ, int B, int D, int H, int W, int levels, const LevelPtrs &pyr, void *ws,
                             hipStream_t s, bool cons = true, int variant = 0, int order = 1) {
    const SplitGeom g = split_geom(D, NQ, H, W);
    const SplitWs w = split_ws(ws, B, g);
    BuildArgs p{};
    p.pq = w.pq, p.pt = w.pt, p.eq = w.eq, p.et = w.et;
    p.B = B, p.H = H, p.W = W, p.N = H * W, p.NQ = NQ, p.S = g.S;
    p.nlev = std::min(levels, kFusedLevels);
    for (int l = 0; l < kFusedLevels; ++l) p.lvl[l] = l < p.nlev ? pyr.p[l] : nullptr;
    p.NQp = g.NQp, p.NQB = g.NQB, p.NQG = g.NQG, p.Hp = g.Hp, p.CB = g.CB, p.Wp = g.Wp;
    p.npatch = (g.Hp / kPatchRows) * g.CB;
    const float sD = std::sqrt((float)D);
    p.inv_s = 1.0f / sD;
    p.exact = is_pow2(sD);
    p.eshift = 0;
    if (p.exact) {
        int e;
        std::frexp(p.inv_s, &e);
        p.eshift = e - 1;  // 1/s = 2^(e-1)
    }
    (void)cons;
    p.order = order;
    const long tiles = (long)B * p.npatch * g.NQG;
    if (tiles > 0x7fffffffL) return hipErrorInvalidValue;
    const dim3 grid((unsigned)tiles);
    const int ss = g.S <= 8 ? g.S : 0;
    hipError_t e;
    if (variant != 0 && ss == 8) {
        switch (variant) {
            case 1: e = launch_build_kernel<8, 4, false>(grid, p, s); break;
            case 2: e = launch_build_kernel<8, 4, true, false>(grid, p, s); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (ss) {
#define CORR_BUILD_CASE(c) \
    case c: e = launch_build_kernel<c, 4, true>(grid, p, s); break;
            CORR_BUILD_CASE(0) CORR_BUILD_CASE(1) CORR_BUILD_CASE(2) CORR_BUILD_CASE(3) CORR_BUILD_CASE(4)
            CORR_BUILD_CASE(5) CORR_BUILD_CASE(6) CORR_BUILD_CASE(7) CORR_BUILD_CASE(8)
#undef CORR_BUILD_CASE
            default: return hipErrorInvalidValue;
        }
    }
    if (e != hipSuccess) return e;
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (levels > kFusedLevels) return launch_pool_levels(pyr, kFusedLevels, levels, (long)B * NQ, H, W, s);
    return hipSuccess;
}

// part: 0 = pack + MFMA; 1 = the pack alone; 2 = the MFMA kernel alone (measurement: the
// workspace must already hold this pair's pack).
hipError_t launch_build_split(const float *f1, int NQ, const float *f2, int B, int D, int H, int W, int levels,
                              const LevelPtrs &pyr, void *ws, hipStream_t s, int part) {
    if (part != 2) {
        const hipError_t e = launch_split_pack(f1, NQ, f2, B, D, H, W, ws, s);
        if (e != hipSuccess || part == 1) return e;
    }
    return launch_split_mfma(NQ, B, D, H, W, levels, pyr, ws, s);
}

}  // namespace corr
