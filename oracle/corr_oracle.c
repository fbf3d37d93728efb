/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp32 unless noted) of the reference E-RAFT CorrBlock hot path,
 * used as the checker for the HIP kernels in e-raft_amd/csrc.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library; the
 * product path (eraft_amd) never links, loads or calls it.
 *
 * Parity is PINNED: tests/test_oracle.py checks every function below against golden
 * vectors produced by the reference itself (tests/golden/make_golden.py imports
 * /root/reference/model/corr.py in the survey container).  Pool and lookup are bit-exact
 * against the reference; the all-pairs product is within 1e-6 norm-relative (the
 * reference's BLAS accumulation order is not reproducible).
 *
 * Reference (AhmedHumais/E-RAFT @ 2025-02-28):
 *   model/corr.py:52-60   CorrBlock.corr            -> oracle_corr_rows
 *   model/corr.py:25-27   avg_pool2d(2, stride 2)   -> oracle_avg_pool2x2
 *   model/corr.py:29-50   CorrBlock.__call__        -> oracle_lookup
 *   model/utils.py:7-21   bilinear_sampler          -> (inside oracle_lookup)
 *   autograd of the above (eraft.py:128 detaches coords)
 *                                                   -> oracle_lookup_bwd, oracle_pool_bwd,
 *                                                      oracle_corr_bwd
 *   utils/image_utils.py:10-83  forward_interpolate_pytorch / grid_sample_values
 *                         (warm-start forward splat) -> oracle_forward_splat
 *   utils/dsec_utils.py:26-64   VoxelGrid.convert    -> oracle_voxel_grid
 *   utils/transformers.py:36-126 EventSequenceToVoxelGrid_Pytorch
 *                                                   -> oracle_voxel_grid_tbilinear
 *
 * Build with -ffp-contract=off: every fp32 operation below is meant to round exactly once,
 * and fmaf() is used only where the reference's ATen kernel fuses.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* avg_pool2d floor mode: level l has dims floor(d / 2^l) (corr.py:26). */
static int level_dim(int d, int l) { return d >> l; }

/*
 * model/corr.py:52-60.  C[b, n, m] = (sum_d f1[b,d,n] * f2[b,d,m]) / sqrt(float(D)).
 * f1, f2: [B, D, N] contiguous.  Computes query rows n in [q0, q1) of every batch item and
 * writes out[b][n - q0][m] ([B][q1-q0][N]).  The dot product is accumulated in double and
 * rounded once to fp32 (the most accurate fp32 matmul result), then divided by the fp32
 * sqrt(D) exactly as corr.py:60 does.
 */
void oracle_corr_rows(const float *f1, const float *f2, int B, int D, int N, int q0, int q1,
                      float *out) {
    const float s = sqrtf((float)D);
    double *acc = (double *)malloc(sizeof(double) * (size_t)N);
    for (int b = 0; b < B; ++b) {
        const float *F1 = f1 + (size_t)b * D * N;
        const float *F2 = f2 + (size_t)b * D * N;
        for (int n = q0; n < q1; ++n) {
            for (int m = 0; m < N; ++m) acc[m] = 0.0;
            for (int d = 0; d < D; ++d) {
                const double a = (double)F1[(size_t)d * N + n];
                const float *row = F2 + (size_t)d * N;
                for (int m = 0; m < N; ++m) acc[m] += a * (double)row[m];
            }
            float *o = out + ((size_t)b * (q1 - q0) + (n - q0)) * N;
            for (int m = 0; m < N; ++m) o[m] = (float)acc[m] / s;
        }
    }
    free(acc);
}

/*
 * model/corr.py:26  F.avg_pool2d(corr, 2, stride=2): in [BN][H][W] -> out [BN][H/2][W/2]
 * (floor).  Sum order ((a + b) + c) + d then * 0.25 — bit-identical to ATen's CPU kernel
 * (pinned by tests/test_oracle.py::test_pool_bitexact).
 */
void oracle_avg_pool2x2(const float *in, long BN, int H, int W, float *out) {
    const int Ho = H / 2, Wo = W / 2;
    for (long q = 0; q < BN; ++q) {
        const float *I = in + (size_t)q * H * W;
        float *O = out + (size_t)q * Ho * Wo;
        for (int y = 0; y < Ho; ++y)
            for (int x = 0; x < Wo; ++x) {
                const float a = I[(2 * y) * W + 2 * x], b = I[(2 * y) * W + 2 * x + 1];
                const float c = I[(2 * y + 1) * W + 2 * x], d = I[(2 * y + 1) * W + 2 * x + 1];
                float t = a + b;
                t = t + c;
                t = t + d;
                O[y * Wo + x] = t * 0.25f;
            }
    }
}

/*
 * model/corr.py:41-43 + model/utils.py:11-15: tap coordinate along one axis of level l.
 * X = c / 2^l + (t - r); x' = 2X / (size - 1) - 1; grid_sample(align_corners=True)
 * unnormalises ix = ((x' + 1) / 2) * (size - 1).  Each step is one fp32 rounding, in this
 * order.  Returns ix and fills the corner origin (floor) and the two 1-D weights
 * w_hi = ix - x0 (toward x0 + 1) and w_lo = (x0 + 1) - ix (toward x0).
 */
static void tap_axis(float c, int l, int t, int r, int size, float *x0f, float *w_lo,
                     float *w_hi) {
    const float cl = c / (float)(1 << l);
    const float X = cl + (float)(t - r);
    const float den = (float)(size - 1);
    const float xn = ((2.0f * X) / den) - 1.0f;
    const float ix = ((xn + 1.0f) / 2.0f) * den;
    const float f = floorf(ix);
    *x0f = f;
    *w_hi = ix - f;
    *w_lo = (f + 1.0f) - ix;
}

static float corner(const float *P, int Hl, int Wl, float xf, float yf) {
    /* zero padding (grid_sample default); NaN / inf coordinates fail both tests */
    if (xf >= 0.0f && xf < (float)Wl && yf >= 0.0f && yf < (float)Hl)
        return P[(int)yf * Wl + (int)xf];
    return 0.0f;
}

/*
 * model/corr.py:29-50.  pyr[l]: [B*H*W][H>>l][W>>l]; coords: [B][2][H][W] (ch0 = x,
 * ch1 = y, utils.py:24-27); out: [B][L*(2r+1)^2][H][W], channel l*K + i*(2r+1) + j samples
 * at (x/2^l + i - r, y/2^l + j - r) — the slow window index moves x (corr.py:37-43).
 * Bilinear weights nw = ey*ex, ne = ey*wx, sw = ny*ex, se = ny*wx, accumulated
 * acc = v_nw*w_nw, then fmaf for ne, sw, se — bit-exact vs ATen grid_sampler_2d (CPU).
 */
void oracle_lookup_rows(const float *const *pyr, const float *coords, int B, int NQ, int H,
                        int W, int L, int r, float *out) {
    /* NQ query pixels per batch item (H*W, or a row slab); (H, W) = the target map */
    const int N = NQ, S = 2 * r + 1, K = S * S;
    for (int b = 0; b < B; ++b)
        for (int n = 0; n < N; ++n) {
            const float x = coords[((size_t)b * 2 + 0) * N + n];
            const float y = coords[((size_t)b * 2 + 1) * N + n];
            for (int l = 0; l < L; ++l) {
                const int Hl = level_dim(H, l), Wl = level_dim(W, l);
                const float *P = pyr[l] + ((size_t)b * N + n) * Hl * Wl;
                for (int i = 0; i < S; ++i) {
                    float x0, ex, wx;
                    tap_axis(x, l, i, r, Wl, &x0, &ex, &wx);
                    for (int j = 0; j < S; ++j) {
                        float y0, ey, ny;
                        tap_axis(y, l, j, r, Hl, &y0, &ey, &ny);
                        const float vnw = corner(P, Hl, Wl, x0, y0);
                        const float vne = corner(P, Hl, Wl, x0 + 1.0f, y0);
                        const float vsw = corner(P, Hl, Wl, x0, y0 + 1.0f);
                        const float vse = corner(P, Hl, Wl, x0 + 1.0f, y0 + 1.0f);
                        float acc = vnw * (ey * ex);
                        acc = fmaf(vne, ey * wx, acc);
                        acc = fmaf(vsw, ny * ex, acc);
                        acc = fmaf(vse, ny * wx, acc);
                        out[((size_t)b * L * K + (size_t)l * K + i * S + j) * N + n] = acc;
                    }
                }
            }
        }
}

static void corner_add(float *G, int Hl, int Wl, float xf, float yf, float v) {
    if (xf >= 0.0f && xf < (float)Wl && yf >= 0.0f && yf < (float)Hl)
        G[(int)yf * Wl + (int)xf] += v;
}

/*
 * Autograd of corr.py:45 (grid_sampler_2d backward, input gradient only: coords are
 * detached at eraft.py:128).  grad_out: [B][L*K][H][W]; grad_pyr[l]: [B*H*W][H>>l][W>>l],
 * ACCUMULATED into (the caller zeroes it once per build).  Contributions of a query stay in
 * its own map.  Order: taps (i, j) row-major, corners nw, ne, sw, se.
 */
void oracle_lookup_bwd_rows(const float *coords, const float *grad_out, int B, int NQ, int H,
                            int W, int L, int r, float *const *grad_pyr) {
    const int N = NQ, S = 2 * r + 1, K = S * S;
    for (int b = 0; b < B; ++b)
        for (int n = 0; n < N; ++n) {
            const float x = coords[((size_t)b * 2 + 0) * N + n];
            const float y = coords[((size_t)b * 2 + 1) * N + n];
            for (int l = 0; l < L; ++l) {
                const int Hl = level_dim(H, l), Wl = level_dim(W, l);
                float *G = grad_pyr[l] + ((size_t)b * N + n) * Hl * Wl;
                for (int i = 0; i < S; ++i) {
                    float x0, ex, wx;
                    tap_axis(x, l, i, r, Wl, &x0, &ex, &wx);
                    for (int j = 0; j < S; ++j) {
                        float y0, ey, ny;
                        tap_axis(y, l, j, r, Hl, &y0, &ey, &ny);
                        const float g =
                            grad_out[((size_t)b * L * K + (size_t)l * K + i * S + j) * N + n];
                        corner_add(G, Hl, Wl, x0, y0, g * (ey * ex));
                        corner_add(G, Hl, Wl, x0 + 1.0f, y0, g * (ey * wx));
                        corner_add(G, Hl, Wl, x0, y0 + 1.0f, g * (ny * ex));
                        corner_add(G, Hl, Wl, x0 + 1.0f, y0 + 1.0f, g * (ny * wx));
                    }
                }
            }
        }
}

/*
 * Autograd of corr.py:25-27 (avg_pool2d backward), folded coarse -> fine:
 * grad_pyr[l-1][2y+a][2x+b] += grad_pyr[l][y][x] * 0.25 for y < H_l, x < W_l; rows/cols
 * dropped by the floor receive nothing.  After the call grad_pyr[0] holds dL/dC (level 0).
 */
void oracle_pool_bwd(float *const *grad_pyr, long BN, int H, int W, int L) {
    for (int l = L - 1; l >= 1; --l) {
        const int Hc = level_dim(H, l), Wc = level_dim(W, l);
        const int Hf = level_dim(H, l - 1), Wf = level_dim(W, l - 1);
        for (long q = 0; q < BN; ++q) {
            const float *Gc = grad_pyr[l] + (size_t)q * Hc * Wc;
            float *Gf = grad_pyr[l - 1] + (size_t)q * Hf * Wf;
            for (int y = 0; y < Hc; ++y)
                for (int x = 0; x < Wc; ++x) {
                    const float v = Gc[y * Wc + x] * 0.25f;
                    Gf[(2 * y) * Wf + 2 * x] += v;
                    Gf[(2 * y) * Wf + 2 * x + 1] += v;
                    Gf[(2 * y + 1) * Wf + 2 * x] += v;
                    Gf[(2 * y + 1) * Wf + 2 * x + 1] += v;
                }
        }
    }
}

/*
 * Autograd of corr.py:58-60: with dC = grad_c / sqrt(D) ([B][N][N], query-major),
 * df1[b,d,n] = sum_m dC[n,m] f2[b,d,m] and df2[b,d,m] = sum_n f1[b,d,n] dC[n,m].
 * Accumulated in double, rounded once.
 */
void oracle_corr_bwd(const float *grad_c, const float *f1, const float *f2, int B, int D, int N,
                     float *df1, float *df2) {
    const float s = sqrtf((float)D);
    double *a1 = (double *)malloc(sizeof(double) * (size_t)D * N);
    double *a2 = (double *)malloc(sizeof(double) * (size_t)D * N);
    float *dc = (float *)malloc(sizeof(float) * (size_t)N);
    for (int b = 0; b < B; ++b) {
        const float *F1 = f1 + (size_t)b * D * N, *F2 = f2 + (size_t)b * D * N;
        memset(a1, 0, sizeof(double) * (size_t)D * N);
        memset(a2, 0, sizeof(double) * (size_t)D * N);
        for (int n = 0; n < N; ++n) {
            const float *G = grad_c + ((size_t)b * N + n) * N;
            for (int m = 0; m < N; ++m) dc[m] = G[m] / s;
            for (int d = 0; d < D; ++d) {
                const float *f2r = F2 + (size_t)d * N;
                double acc = 0.0;
                for (int m = 0; m < N; ++m) acc += (double)dc[m] * (double)f2r[m];
                a1[(size_t)d * N + n] += acc;
                const double f1v = (double)F1[(size_t)d * N + n];
                double *a2r = a2 + (size_t)d * N;
                for (int m = 0; m < N; ++m) a2r[m] += f1v * (double)dc[m];
            }
        }
        for (size_t i = 0; i < (size_t)D * N; ++i) {
            df1[(size_t)b * D * N + i] = (float)a1[i];
            df2[(size_t)b * D * N + i] = (float)a2[i];
        }
    }
    free(a1);
    free(a2);
    free(dc);
}

/* Reference-shaped forms (every pixel of fmap1 is a query). */
void oracle_lookup(const float *const *pyr, const float *coords, int B, int H, int W, int L,
                   int r, float *out) {
    oracle_lookup_rows(pyr, coords, B, H * W, H, W, L, r, out);
}

void oracle_lookup_bwd(const float *coords, const float *grad_out, int B, int H, int W, int L,
                       int r, float *const *grad_pyr) {
    oracle_lookup_bwd_rows(coords, grad_out, B, H * W, H, W, L, r, grad_pyr);
}

/*
 * Warm-start forward splat, utils/image_utils.py:52-83 (forward_interpolate_pytorch) and
 * :10-50 (grid_sample_values), per batch item and channel:
 *   x = x0 + dx, y = y0 + dy (fp32); for x_v in (floor x, ceil x), then y_v in (floor y,
 *   ceil y) (:27-28): w = (1 - |x - x_v|) * (1 - |y - y_v|) (:33); in-bounds points
 *   (0 <= x_v < W, 0 <= y_v < H, :30) accumulate z*w and w at index x_v + W*y_v with
 *   put_(accumulate=True) (:37-38) — on CPU a sequential pass in source order, one pass per
 *   corner; an integer x or y has floor == ceil, so that corner is counted twice (kept).
 *   out = values / (weights + 1e-15) (:46).  flow, out: [B][2][H][W].
 */
void oracle_forward_splat(const float *flow, int B, int H, int W, float *out) {
    const long N = (long)H * W;
    float *val = (float *)malloc(sizeof(float) * N);
    float *acc = (float *)malloc(sizeof(float) * N);
    for (int b = 0; b < B; ++b) {
        const float *dx = flow + ((long)b * 2 + 0) * N, *dy = flow + ((long)b * 2 + 1) * N;
        for (int c = 0; c < 2; ++c) {
            const float *z = c == 0 ? dx : dy;
            memset(val, 0, sizeof(float) * N);
            memset(acc, 0, sizeof(float) * N);
            for (int px = 0; px < 2; ++px)
                for (int py = 0; py < 2; ++py)
                    for (long p = 0; p < N; ++p) {
                        const float x = (float)(p % W) + dx[p], y = (float)(p / W) + dy[p];
                        const float xv = px ? ceilf(x) : floorf(x), yv = py ? ceilf(y) : floorf(y);
                        if (!(xv < (float)W && xv >= 0.0f && yv < (float)H && yv >= 0.0f)) continue;
                        const float w = (1.0f - fabsf(x - xv)) * (1.0f - fabsf(y - yv));
                        const long idx = (long)(xv + (float)W * yv);
                        val[idx] = val[idx] + z[p] * w;
                        acc[idx] = acc[idx] + w;
                    }
            float *o = out + ((long)b * 2 + c) * N;
            for (long t = 0; t < N; ++t) o[t] = val[t] / (acc[t] + 1e-15f);
        }
    }
    free(val);
    free(acc);
}

/*
 * DSEC event -> voxel grid, utils/dsec_utils.py:26-64 (VoxelGrid.convert), events as
 * loader/loader_dsec.py:245-257 prepares them (float32 x, y, t in [0, 1], p in {0, 1}):
 *   t_n = ((C-1) * (t - t[0])) / (t[M-1] - t[0]) (:33); x0, y0, t0 = trunc(x, y, t_n) (:35-37);
 *   value = 2p - 1 (:39); corners x_l in (x0, x0+1) outer, y_l in (y0, y0+1) inner, t_l = t0
 *   (:41-44, the t loop is commented out in the reference); in-bounds corners (:45) add
 *   ((value * (1-|x_l-x|)) * (1-|y_l-y|)) * (1-|t_l-t_n|) (:46) at H*W*t_l + W*y_l + x_l with
 *   put_(accumulate=True) (:52) — sequential per corner pass, in event order.
 *   normalize (:54-62): over the nonzero cells, v = (v - mean) / std (unbiased std; when
 *   std is not > 0: v - mean).  mean and std are accumulated in fp64 here and rounded to
 *   fp32 (the reference's fp32 reduction order is ATen's: tolerance-level for this step).
 */
void oracle_voxel_grid(const float *x, const float *y, const float *t, const float *p, long M, int C, int H,
                       int W, int normalize, float *out) {
    const long CHW = (long)C * H * W;
    memset(out, 0, sizeof(float) * CHW);
    if (M < 1) return;
    const float t0 = t[0], dt = t[M - 1] - t[0];
    for (int xi = 0; xi < 2; ++xi)
        for (int yi = 0; yi < 2; ++yi)
            for (long e = 0; e < M; ++e) {
                const float tn = ((float)(C - 1) * (t[e] - t0)) / dt;
                const int xl = (int)x[e] + xi, yl = (int)y[e] + yi, tl = (int)tn;
                if (!(xl < W && xl >= 0 && yl < H && yl >= 0 && tl >= 0 && tl < C)) continue;
                const float value = 2.0f * p[e] - 1.0f;
                const float w = value * (1.0f - fabsf((float)xl - x[e])) * (1.0f - fabsf((float)yl - y[e])) *
                                (1.0f - fabsf((float)tl - tn));
                const long idx = (long)H * W * tl + (long)W * yl + xl;
                out[idx] = out[idx] + w;
            }
    if (!normalize) return;
    long n = 0;
    double s = 0.0;
    for (long i = 0; i < CHW; ++i)
        if (out[i] != 0.0f) {
            s += out[i];
            ++n;
        }
    if (n == 0) return;
    const double mean = s / (double)n;
    double q = 0.0;
    for (long i = 0; i < CHW; ++i)
        if (out[i] != 0.0f) q += ((double)out[i] - mean) * ((double)out[i] - mean);
    const float mf = (float)mean;
    const float sf = n > 1 ? (float)sqrt(q / (double)(n - 1)) : NAN;
    for (long i = 0; i < CHW; ++i)
        if (out[i] != 0.0f) out[i] = sf > 0.0f ? (out[i] - mf) / sf : out[i] - mf;
}

/*
 * MVSEC event -> voxel grid, utils/transformers.py:36-126 (EventSequenceToVoxelGrid_Pytorch,
 * the representation of loader/loader_mvsec_flow.py:35), events [M][4] float64 rows
 * (t, x, y, p) as .astype('float') makes them (:46):
 *   t_n = ((C-1) * (t - t[0])) / dT, dT = t[M-1] - t[0] or 1 when 0 (:66-77, fp64);
 *   tis = floor(t_n), dts = fp32(t_n - tis) (:85-87); pol = fp32(p), 0 -> -1 (:81-82);
 *   left  = pol * (1 - dts) at bin tis      for 0 <= tis < C      (:88, :91-103);
 *   right = pol * dts       at bin tis + 1  for 0 <= tis, tis+1 < C (:89, :106-112);
 *   flat index trunc(x) + trunc(y) * W + bin * W * H; index_add_ on CPU adds sequentially in
 *   index order: all left entries in event order, then all right entries.  An index outside
 *   the grid (the reference raises) is skipped.  normalize: as oracle_voxel_grid.
 */
void oracle_voxel_grid_tbilinear(const double *ev, long M, int C, int H, int W, int normalize, float *out) {
    const long CHW = (long)C * H * W, HW = (long)H * W;
    memset(out, 0, sizeof(float) * CHW);
    if (M >= 1) {
        const double t0 = ev[0];
        double dT = ev[(M - 1) * 4] - t0;
        if (dT == 0.0) dT = 1.0;
        for (int side = 0; side < 2; ++side)
            for (long e = 0; e < M; ++e) {
                const double *q = ev + e * 4;
                const double ts = ((double)(C - 1) * (q[0] - t0)) / dT;
                const double tis = floor(ts);
                const float dts = (float)(ts - tis);
                float pol = (float)q[3];
                if (pol == 0.0f) pol = -1.0f;
                const double bin = tis + side;
                if (!(tis >= 0.0 && bin < (double)C)) continue;
                if (!(fabs(q[1]) < 2147483648.0 && fabs(q[2]) < 2147483648.0)) continue;
                const long idx = (long)q[1] + (long)q[2] * W + (long)bin * HW;
                if (idx < 0 || idx >= CHW) continue;
                const float v = side ? pol * dts : pol * (1.0f - dts);
                out[idx] = out[idx] + v;
            }
    }
    if (!normalize) return;
    long n = 0;
    double s = 0.0;
    for (long i = 0; i < CHW; ++i)
        if (out[i] != 0.0f) {
            s += out[i];
            ++n;
        }
    if (n == 0) return;
    const double mean = s / (double)n;
    double qq = 0.0;
    for (long i = 0; i < CHW; ++i)
        if (out[i] != 0.0f) qq += ((double)out[i] - mean) * ((double)out[i] - mean);
    const float mf = (float)mean;
    const float sf = n > 1 ? (float)sqrt(qq / (double)(n - 1)) : NAN;
    for (long i = 0; i < CHW; ++i)
        if (out[i] != 0.0f) out[i] = sf > 0.0f ? (out[i] - mf) / sf : out[i] - mf;
}
