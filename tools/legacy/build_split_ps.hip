// build_split_ps.hip — measured and dropped (round 2): the persistent role-split build kernel.
// Included by tools/kbench_build.hip after e-raft_amd/csrc/corr_build_split.hip; not part of
// the library.  Bit-identical to corr_build_split_kernel, but slower on every shape measured
// (profiles/r02p_kbench_build_ps_nt_stagger_ab.txt: DSEC 52-56 vs 49-52 us, 1280x960 1389 vs 1007 us): with
// one workgroup per CU each SIMD runs ONE MFMA wave, so the MFMA phase loses the latency
// hiding of three co-resident workgroups (no-store 39 vs 34 us at DSEC), and the stores still
// cost what they cost in the one-tile kernel (about 40 cycles of CU time per store
// instruction), now on the critical path of the store waves' barriers.
#pragma once
#include <utility>

namespace corr {

// ---------------------------------------------------------------------------------------
// Persistent role-split build (S = 4 or 8 K steps: D in (96, 128] or (224, 256]).
//
// Why: in the kernel above every workgroup reaches its epilogue at about the same time, so the
// chip alternates between an MFMA phase with idle HBM and a store burst with idle matrix pipes
// (at 1280x960: 468 us without stores, 907 us with them).  Here one 768-thread workgroup per CU
// loops over its tiles with three roles, one wave of each per SIMD:
//   waves 0-3  MFMA: the same 32-query x 8x16-target blocks and MFMA order as above (so the
//              accumulators are bit-identical); query records loaded into registers 3 steps
//              ahead; at a tile's last K step the raw accumulators go to an LDS staging tile;
//   waves 4-7  DMA: the target records into the 3-slot ring by LDS-DMA, 2 steps ahead, plus
//              the tile's exponents (et, eq) into a 2-deep LDS buffer;
//   waves 8-11 store: during tile k's K loop they take tile k-1's accumulators from the
//              staging tile and run the epilogue (exponents, 1/sqrt(D), pooling, stores) in
//              slices between the barriers.
// vmcnt is per wave, so the MFMA waves' waits count only their query loads and the DMA waves'
// only their DMAs: the stores never hold up a K step, they drain under the next tile's MFMAs.
// Every wave passes the same barriers (one per K step of every tile, plus one to hand over the
// last tile), and there is no cross-workgroup synchronisation: any number of workgroups may
// be resident.  Loads past the last tile re-read its last records (uniform wait counts).
// ---------------------------------------------------------------------------------------
constexpr int kPsThreads = 768;
constexpr int kStQStride = kPatchRows * 16 + 4;  // floats per query in the staging tile (bank stagger)
constexpr int kStBytes = kQPerWG * kStQStride * 4;
constexpr int kEBytes = 2 * kQPerWG * 4;         // et (128 ints) then eq (128 ints)
constexpr int kPsRing = 5;                       // ring slots: DMA 4 K steps ahead
constexpr int ps_lds(int ring) { return ring * kSlotBytes + kStBytes + 2 * kEBytes; }
constexpr int kPsLds = ps_lds(kPsRing);

// s_waitcnt vmcnt(N) + s_barrier, N an immediate.
template <int N>
__device__ __forceinline__ void wait_vm_bar() {
    static_assert(N >= 0 && N <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}


__device__ __forceinline__ void bar_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The epilogue of one 16-query block (lane = query ci, columns X0..X0+3 of the patch's 8 rows):
// level 0 rows [r0, r0 + 4) when (parts & 1) (r0 = 0) / (parts & 2) (r0 = 4), levels 1-3 when
// (parts & 4).  The values, ops and order are those of corr_build_split_kernel's epilogue.
__device__ __forceinline__ void emit_block(const BuildArgs &p, size_t qrow, bool qok, int y0, int X0, int grp,
                                           const float (&v)[kPatchRows][4], int parts) {
    const int H = p.H, W = p.W, N = p.N, nlev = p.nlev;
    if (qok && nlev > 0) {
        float *row0 = p.lvl[0] + qrow * N;
#pragma unroll
        for (int r = 0; r < kPatchRows; ++r)
            if ((parts >> (r >> 2)) & 1)
                if (y0 + r < H) store4(row0 + (size_t)(y0 + r) * W, X0, W, v[r], p.mode0);
    }
    if (!(parts & 4)) return;
    const int H1 = H >> 1, W1 = W >> 1, H2 = H >> 2, W2 = W >> 2, H3 = H >> 3, W3 = W >> 3;
    float l1[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        l1[r][0] = pool4(v[2 * r][0], v[2 * r][1], v[2 * r + 1][0], v[2 * r + 1][1]);
        l1[r][1] = pool4(v[2 * r][2], v[2 * r][3], v[2 * r + 1][2], v[2 * r + 1][3]);
    }
    if (qok && nlev > 1) {
        float *row1 = p.lvl[1] + qrow * (H1 * W1);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if ((y0 >> 1) + r < H1) store2(row1 + (size_t)((y0 >> 1) + r) * W1, X0 >> 1, W1, l1[r][0], l1[r][1], p.mode1);
    }
    float l2[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) l2[r] = pool4(l1[2 * r][0], l1[2 * r][1], l1[2 * r + 1][0], l1[2 * r + 1][1]);
    if (qok && nlev > 2) {
        float *row2 = p.lvl[2] + qrow * (H2 * W2);
#pragma unroll
        for (int r = 0; r < 2; ++r)
            if ((y0 >> 2) + r < H2 && (X0 >> 2) < W2) row2[((y0 >> 2) + r) * W2 + (X0 >> 2)] = l2[r];
    }
    const float b0 = __shfl_xor(l2[0], 16), b1 = __shfl_xor(l2[1], 16);
    if (qok && nlev > 3 && (grp & 1) == 0) {
        const float l3 = pool4(l2[0], b0, l2[1], b1);
        const int Y3 = y0 >> 3, X3 = X0 >> 3;
        if (Y3 < H3 && X3 < W3) p.lvl[3][qrow * (H3 * W3) + Y3 * W3 + X3] = l3;
    }
}

// R = LDS ring slots (the DMA runs DD = R - 1 K steps ahead); PRIO = s_setprio of the MFMA waves.
template <int SS, int R = kPsRing, int PRIO = 0>
__global__ __launch_bounds__(kPsThreads, 1) void corr_build_split_ps_kernel(BuildArgs p) {
    static_assert(SS % 4 == 0, "query register slots are static per tile");
    constexpr int DD = R - 1;
    static_assert(DD >= 2 && DD <= SS, "DMA distance");
    extern __shared__ __attribute__((aligned(16))) char smem_build[];
    char *smem = smem_build;
    float *st = reinterpret_cast<float *>(smem + R * kSlotBytes);
    const int *ebuf = reinterpret_cast<const int *>(smem + R * kSlotBytes + kStBytes);
    const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_void_t *)smem;
    const uint32_t lds_e = lds_base + R * kSlotBytes + kStBytes;

    const int ntot = p.B * p.npatch * p.NQG, nwg = gridDim.x, wg = blockIdx.x;
    const int my_tiles = wg < ntot ? (ntot - 1 - wg) / nwg + 1 : 0;
    if (my_tiles == 0) return;  // uniform over the workgroup
    auto tile_k = [&](int k) __attribute__((always_inline)) { return tile_of(p, xcd_swizzle(k * nwg + wg, ntot)); };

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int role = w >> 2, rw = w & 3;
    const int ci = lane & 15, grp = lane >> 4;

    if (role == 0) {
        // ---------------- MFMA waves ----------------
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
        auto qbase = [&](const Tile &t) __attribute__((always_inline)) {
            return p.pq + ((size_t)t.b * SS * p.NQB + t.qg * (kQPerWG / 16) + 2 * rw) * kRecU + lane;
        };
        const size_t qstep = (size_t)p.NQB * kRecU;
        u32x4 qv[4][2][2];
        auto issue_q = [&](const u32x4 *src, int s, int slot) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const u32x4 *q = src + s * qstep + i * kRecU;
                qv[slot][i][0] = q[0];
                qv[slot][i][1] = q[64];
            }
        };
        f32x4 acc[2][kPatchRows];
        auto compute = [&](int tslot, int qs, bool first) __attribute__((always_inline)) {
            const u32x4 *A = reinterpret_cast<const u32x4 *>(smem + tslot * kSlotBytes);
            half8 qh[2], ql[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                qh[i] = __builtin_bit_cast(half8, qv[qs][i][0]);
                ql[i] = __builtin_bit_cast(half8, qv[qs][i][1]);
            }
#pragma unroll
            for (int r = 0; r < kPatchRows; ++r) {
                const half8 ah = __builtin_bit_cast(half8, A[(2 * r) * 64 + lane]);
                const half8 al = __builtin_bit_cast(half8, A[(2 * r + 1) * 64 + lane]);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 c = first ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][r];
                    acc[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, qh[i], c, 0, 0, 0);
                    acc[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, ql[i], acc[i][r], 0, 0, 0);
                    acc[i][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, qh[i], acc[i][r], 0, 0, 0);
                }
            }
        };
        const u32x4 *qcur = qbase(tile_k(0));
        // in step order (the empty asm keeps the compiler from reordering them): the loop's
        // waits then see the same load order on entry as around its back edge
        issue_q(qcur, 0, 0);
        asm volatile("" ::: "memory");
        issue_q(qcur, 1, 1);
        asm volatile("" ::: "memory");
        issue_q(qcur, 2, 2);
        asm volatile("" ::: "memory");
        float *stw = st + (32 * rw + ci) * kStQStride + 4 * grp;
        for (int k = 0; k < my_tiles; ++k) {
            const u32x4 *qnext = k + 1 < my_tiles ? qbase(tile_k(k + 1)) : qcur;
            const int rbase = (k * SS) % R;
#pragma unroll
            for (int s = 0; s < SS; ++s) {
                bar_lgkm();
                if (s + 3 < SS) issue_q(qcur, s + 3, (s + 3) & 3);
                else issue_q(qnext, s + 3 - SS, (s + 3) & 3);
                int slot = rbase + s % R;
                slot = slot >= R ? slot - R : slot;
                compute(slot, s & 3, s == 0);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < kPatchRows; ++r)
                    *reinterpret_cast<f32x4 *>(stw + 16 * i * kStQStride + r * 16) = acc[i][r];
            qcur = qnext;
        }
        bar_lgkm();  // hands the last tile to the store waves
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (role == 1) {
        // ---------------- DMA waves ----------------
        const size_t tstep = (size_t)p.Hp * p.CB * kRecU;
        auto tbase = [&](const Tile &t) __attribute__((always_inline)) {
            // piece pc = rw + 4 m: patch row pc >> 1, half pc & 1 (m adds 2 rows)
            return p.pt + (((size_t)t.b * SS * p.Hp + t.py * kPatchRows + (rw >> 1)) * p.CB + t.cb) * kRecU +
                   (rw & 1) * 64 + lane;
        };
        const size_t mstep = (size_t)2 * p.CB * kRecU;  // +2 patch rows per m
        auto issue_t = [&](const u32x4 *src, int s, int slot) __attribute__((always_inline)) {
            const uint32_t base = lds_base + slot * kSlotBytes;
#pragma unroll
            for (int m = 0; m < 4; ++m) dma16(src + s * tstep + m * mstep, base + (rw + 4 * m) * 1024);
        };
        auto issue_e = [&](const Tile &t, int k) __attribute__((always_inline)) {
            const int idx = rw * 64 + lane;  // 0..255: et row-major 8 x 16, then eq
            const int *src;
            if (idx < kQPerWG)
                src = p.et + ((size_t)t.b * p.Hp + t.py * kPatchRows + (idx >> 4)) * p.Wp + t.cb * 16 + (idx & 15);
            else
                src = p.eq + (size_t)t.b * p.NQp + t.qg * kQPerWG + (idx - kQPerWG);
            dma4(src, lds_e + (k & 1) * kEBytes + rw * 256);
        };
        Tile tc = tile_k(0);
        const u32x4 *tcur = tbase(tc);
#pragma unroll
        for (int j = 0; j < DD; ++j) issue_t(tcur, j, j);  // DD <= SS: all in the first tile
        for (int k = 0; k < my_tiles; ++k) {
            const Tile tn = k + 1 < my_tiles ? tile_k(k + 1) : tc;
            const u32x4 *tnext = tbase(tn);
            const int rbase = (k * SS) % R;
            [&]<int... S>(std::integer_sequence<int, S...>) __attribute__((always_inline)) {
                (
                    [&] {
                        // this step's ring slot has landed: younger than its DMA are the DD - 1
                        // later steps' 4 pieces each, plus the exponent DMA a tile's first step
                        // issues (before its ring pieces) when that step is among them
                        wait_vm_bar<4 * (DD - 1) + ((S >= 1 && S <= DD - 1) ? 1 : 0)>();
                        if constexpr (S == 0) issue_e(tc, k);
                        int slot = rbase + (S + DD) % R;
                        slot = slot >= R ? slot - R : slot;
                        if constexpr (S + DD < SS) issue_t(tcur, S + DD, slot);
                        else issue_t(tnext, S + DD - SS, slot);
                    }(),
                    ...);
            }(std::make_integer_sequence<int, SS>{});
            tc = tn;
            tcur = tnext;
        }
        asm volatile("s_barrier" ::: "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA in flight at exit
    } else {
        // ---------------- store waves ----------------
        const float *str = st + (32 * rw + ci) * kStQStride + 4 * grp;
        const int *er = ebuf;
        float v[2][kPatchRows][4];
        Tile tp{};
        for (int k = 0; k <= my_tiles; ++k) {
            bar_lgkm();
            const bool have = k >= 1;
            if (have) {
                const int *e = er + ((k - 1) & 1) * (kEBytes / 4);
                f32x4 a[2][kPatchRows];
                int4 e4[kPatchRows];
                int eqv[2];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int r = 0; r < kPatchRows; ++r)
                        a[i][r] = *reinterpret_cast<const f32x4 *>(str + 16 * i * kStQStride + r * 16);
#pragma unroll
                for (int r = 0; r < kPatchRows; ++r) e4[r] = reinterpret_cast<const int4 *>(e)[r * 4 + grp];
#pragma unroll
                for (int i = 0; i < 2; ++i) eqv[i] = e[kQPerWG + 32 * rw + 16 * i + ci] + p.eshift;
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int r = 0; r < kPatchRows; ++r) {
                        const int et[4] = {e4[r].x, e4[r].y, e4[r].z, e4[r].w};
#pragma unroll
                        for (int g = 0; g < 4; ++g) {
                            float x = ldexpf(a[i][r][g], eqv[i] + et[g]);
                            if (!p.exact) x = x * p.inv_s;
                            v[i][r][g] = x;
                        }
                    }
            }
            const int y0 = tp.py * kPatchRows, X0 = tp.cb * 16 + 4 * grp;
            // slice J = 0..5: block J / 3, part J % 3 (level-0 rows 0-3, rows 4-7, levels 1-3)
            auto slices = [&]<int LO, int HI>() __attribute__((always_inline)) {
                [&]<int... J>(std::integer_sequence<int, J...>) __attribute__((always_inline)) {
                    (
                        [&] {
                            constexpr int j = LO + J, i = j / 3;
                            const int q = (tp.qg * (kQPerWG / 16) + 2 * rw + i) * 16 + ci;
                            emit_block(p, (size_t)tp.b * p.NQ + q, q < p.NQ, y0, X0, grp, v[i], 1 << (j % 3));
                        }(),
                        ...);
                }(std::make_integer_sequence<int, HI - LO>{});
            };
            if (k == my_tiles) {  // the last tile: no K steps left to spread it over
                slices.template operator()<0, 6>();
                break;
            }
            // K step s runs slices [6s / SS, 6(s + 1) / SS)
            [&]<int... S>(std::integer_sequence<int, S...>) __attribute__((always_inline)) {
                (
                    [&] {
                        if constexpr (S > 0) bar_lgkm();
                        if (have) slices.template operator()<6 * S / SS, 6 * (S + 1) / SS>();
                    }(),
                    ...);
            }(std::make_integer_sequence<int, SS>{});
            tp = tile_k(k);
        }
    }
}


template <int PR = kPsRing, int PP = 0>
hipError_t launch_split_mfma_ps(int NQ, int B, int D, int H, int W, int levels, const LevelPtrs &pyr, void *ws,
                                hipStream_t s) {
    const SplitGeom g = split_geom(D, NQ, H, W);
    if (g.S != 4 && g.S != 8) return hipErrorInvalidValue;
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
    if (p.exact) {
        int e;
        std::frexp(p.inv_s, &e);
        p.eshift = e - 1;
    }
    p.mode0 = p.nlev > 0 ? store_mode(W, pyr.p[0]) : 0;
    p.mode1 = p.nlev > 1 ? store_mode(W >> 1, pyr.p[1]) : 0;
    const long tiles = (long)B * p.npatch * g.NQG;
    hipError_t e;
    {
        static std::atomic<unsigned long long> ps_done[2];
        static std::atomic<int> ncu_cache[64];
        int dev = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        int ncu = ncu_cache[dev & 63].load(std::memory_order_relaxed);
        if (ncu <= 0) {
            if ((e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
            ncu_cache[dev & 63].store(ncu, std::memory_order_relaxed);
        }
        const dim3 pgrid((unsigned)std::min<long>(tiles, ncu)), pblk(kPsThreads);
        if (g.S == 8) {
            if ((e = ensure_lds_limit((const void *)corr_build_split_ps_kernel<8, PR, PP>, ps_lds(PR), ps_done[1])) !=
                hipSuccess)
                return e;
            hipLaunchKernelGGL((corr_build_split_ps_kernel<8, PR, PP>), pgrid, pblk, ps_lds(PR), s, p);
        } else {
            if ((e = ensure_lds_limit((const void *)corr_build_split_ps_kernel<4, PR, PP>, ps_lds(PR), ps_done[0])) !=
                hipSuccess)
                return e;
            hipLaunchKernelGGL((corr_build_split_ps_kernel<4, PR, PP>), pgrid, pblk, ps_lds(PR), s, p);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (levels > kFusedLevels) return launch_pool_levels(pyr, kFusedLevels, levels, (long)B * NQ, H, W, s);
        return hipSuccess;
    }
    return hipSuccess;
}

}  // namespace corr
