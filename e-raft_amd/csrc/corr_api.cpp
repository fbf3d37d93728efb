// corr_api.cpp — the extern "C" boundary of libcorr_mi355x.so (declared in
// include/corr_mi355x.h).  Validates arguments, records thread-local errors and forwards to
// the gfx950 launchers.  No allocation and no synchronisation.  Global state: the thread-local
// error message, and per-kernel per-device "dynamic-LDS limit raised" bits (atomic, idempotent;
// ensure_lds_limit in corr_build_common.h) — re-entrant across threads, streams and devices.
//
// The reference-shaped entry points (corr_build, corr_lookup, ...) are the row-slab
// variants (corr_*_rows) with the slab = every query pixel (NQ = H*W).
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "corr_common.h"

namespace corr {

static thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int hip_status(hipError_t e, const char *what) {
    if (e == hipSuccess) return CORR_OK;
    return fail(CORR_EHIP, "%s: %s", what, hipGetErrorString(e));
}

static int check_dims(const char *fn, int B, int NQ, int H, int W, int levels) {
    if (B < 1 || H < 1 || W < 1)
        return fail(CORR_EINVAL, "%s: B, H, W must be >= 1 (got %d, %d, %d)", fn, B, H, W);
    if (NQ < 1 || NQ > H * (long long)W)
        return fail(CORR_EINVAL, "%s: NQ must be in [1, H*W] (got %d)", fn, NQ);
    if (levels < 1 || levels > CORR_MAX_LEVELS)
        return fail(CORR_EINVAL, "%s: levels must be in [1, %d] (got %d)", fn, CORR_MAX_LEVELS, levels);
    // avg_pool2d(2, 2) on a 1-pixel dimension raises in the reference (corr.py:26)
    if ((H >> (levels - 1)) < 1 || (W >> (levels - 1)) < 1)
        return fail(CORR_EINVAL, "%s: %dx%d is too small for %d pyramid levels", fn, H, W, levels);
    // the lookup's neighbourhood anchors assume |coordinate floors| of in-map taps < 2^20
    if (H > (1 << 20) || W > (1 << 20))
        return fail(CORR_EINVAL, "%s: H and W must be <= 2^20", fn);
    const long long N = (long long)H * W;
    if (N > (1LL << 30) || (long long)B * NQ > (1LL << 31) - 1)
        return fail(CORR_EINVAL, "%s: B*H*W too large", fn);
    return CORR_OK;
}

static int check_ptr(const char *fn, const void *p, const char *name) {
    if (!p) return fail(CORR_EINVAL, "%s: %s is NULL", fn, name);
    if ((uintptr_t)p % 4) return fail(CORR_EINVAL, "%s: %s is not 4-byte aligned", fn, name);
    return CORR_OK;
}

template <class P>
static int check_levels(const char *fn, P *const *src, int levels, const char *name, P **dst) {
    if (!src) return fail(CORR_EINVAL, "%s: %s is NULL", fn, name);
    for (int l = 0; l < levels; ++l) {
        int rc = check_ptr(fn, src[l], name);
        if (rc) return rc;
        dst[l] = src[l];
    }
    return CORR_OK;
}

// Value pyramids (tiled, corr_common.h): 16-B tile rows, so 16-B aligned level bases.
template <class P>
static int check_pyramid(const char *fn, P *const *src, int levels, const char *name, P **dst) {
    int rc = check_levels(fn, src, levels, name, dst);
    if (rc) return rc;
    for (int l = 0; l < levels; ++l)
        if ((uintptr_t)src[l] % 16) return fail(CORR_EINVAL, "%s: %s[%d] is not 16-byte aligned", fn, name, l);
    return CORR_OK;
}

static int check_radius(const char *fn, int radius) {
    if (radius < 0 || radius > CORR_MAX_RADIUS)
        return fail(CORR_EINVAL, "%s: radius must be in [0, %d] (got %d)", fn, CORR_MAX_RADIUS, radius);
    return CORR_OK;
}

}  // namespace corr

using namespace corr;

extern "C" {

int corr_version(void) { return 202; }

const char *corr_last_error(void) { return g_err; }

size_t corr_map_floats(int Hl, int Wl) {
    if (Hl < 1 || Wl < 1) return 0;
    return map_floats(Hl, Wl);
}

int corr_pyramid_export(const float *const *pyr, int BN, int H, int W, int levels, float *const *out, void *stream) {
    static const char *fn = "corr_pyramid_export";
    g_err[0] = 0;
    int rc = check_dims(fn, 1, 1, H, W, levels);
    if (rc) return rc;
    if (BN < 1) return fail(CORR_EINVAL, "%s: BN must be >= 1", fn);
    ConstLevelPtrs src{};
    LevelPtrs dst{};
    if ((rc = check_pyramid(fn, pyr, levels, "pyr", src.p)) || (rc = check_levels(fn, out, levels, "out", dst.p)))
        return rc;
    return hip_status(launch_pyramid_export(src, BN, H, W, levels, dst, (hipStream_t)stream), fn);
}

int corr_pyramid_import(const float *const *src, int BN, int H, int W, int levels, float *const *pyr, void *stream) {
    static const char *fn = "corr_pyramid_import";
    g_err[0] = 0;
    int rc = check_dims(fn, 1, 1, H, W, levels);
    if (rc) return rc;
    if (BN < 1) return fail(CORR_EINVAL, "%s: BN must be >= 1", fn);
    ConstLevelPtrs s{};
    LevelPtrs dst{};
    if ((rc = check_levels(fn, src, levels, "src", s.p)) || (rc = check_pyramid(fn, pyr, levels, "pyr", dst.p)))
        return rc;
    return hip_status(launch_pyramid_import(s, BN, H, W, levels, dst, (hipStream_t)stream), fn);
}

int corr_build_rows(const float *fmap1_rows, int NQ, const float *fmap2, int B, int D, int H,
                    int W, int levels, float *const *pyr, void *stream) {
    static const char *fn = "corr_build";
    g_err[0] = 0;
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc) return rc;
    if (D < 1) return fail(CORR_EINVAL, "%s: D must be >= 1 (got %d)", fn, D);
    if ((rc = check_ptr(fn, fmap1_rows, "fmap1")) || (rc = check_ptr(fn, fmap2, "fmap2"))) return rc;
    LevelPtrs lp{};
    if ((rc = check_pyramid(fn, pyr, levels, "pyr", lp.p))) return rc;
    return hip_status(launch_build(fmap1_rows, NQ, fmap2, B, D, H, W, levels, lp, (hipStream_t)stream), fn);
}

size_t corr_build_workspace(int algo, int B, int D, int NQ, int H, int W) {
    if (B < 1 || D < 1 || NQ < 1 || H < 1 || W < 1) return 0;
    if (algo == CORR_BUILD_F16X3)
        return build_split_supported(D) ? build_split_workspace(B, D, NQ, H, W) : (size_t)-1;
    if (algo == CORR_BUILD_BF16X6) return build_bf16_workspace(B, D, NQ, H, W);
    if (algo == CORR_BUILD_FP32) return 0;
    return (size_t)-1;
}

int corr_build_ex(int algo, const float *fmap1_rows, int NQ, const float *fmap2, int B, int D,
                  int H, int W, int levels, float *const *pyr, void *workspace,
                  size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_build_ex";
    if (algo == CORR_BUILD_FP32) return corr_build_rows(fmap1_rows, NQ, fmap2, B, D, H, W, levels, pyr, stream);
    g_err[0] = 0;
    const int phase = algo & (CORR_BUILD_ONLY_PACK | CORR_BUILD_ONLY_MFMA);
    algo &= ~(CORR_BUILD_ONLY_PACK | CORR_BUILD_ONLY_MFMA);
    if ((algo != CORR_BUILD_F16X3 && algo != CORR_BUILD_BF16X6) ||
        phase == (CORR_BUILD_ONLY_PACK | CORR_BUILD_ONLY_MFMA))
        return fail(CORR_EINVAL, "%s: unknown algorithm %d", fn, algo | phase);
    const bool bf = algo == CORR_BUILD_BF16X6;
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc) return rc;
    if (D < 1) return fail(CORR_EINVAL, "%s: D must be >= 1 (got %d)", fn, D);
    if (!bf && !build_split_supported(D))
        return fail(CORR_EUNSUPPORTED, "%s: D = %d is too large for CORR_BUILD_F16X3", fn, D);
    if ((rc = check_ptr(fn, fmap1_rows, "fmap1")) || (rc = check_ptr(fn, fmap2, "fmap2"))) return rc;
    if ((uintptr_t)workspace % 256) return fail(CORR_EINVAL, "%s: workspace is not 256-byte aligned", fn);
    const size_t need = bf ? build_bf16_workspace(B, D, NQ, H, W) : build_split_workspace(B, D, NQ, H, W);
    if (workspace_bytes < need || !workspace)
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    LevelPtrs lp{};
    if ((rc = check_pyramid(fn, pyr, levels, "pyr", lp.p))) return rc;
    const int part = phase == CORR_BUILD_ONLY_PACK ? 1 : phase == CORR_BUILD_ONLY_MFMA ? 2 : 0;
    if (bf)
        return hip_status(
            launch_build_bf16(fmap1_rows, NQ, fmap2, B, D, H, W, levels, lp, workspace, (hipStream_t)stream, part), fn);
    return hip_status(launch_build_split(fmap1_rows, NQ, fmap2, B, D, H, W, levels, lp, workspace, (hipStream_t)stream, part),
                      fn);
}

int corr_build_region(int algo, const float *fmap1_rows, int NQ, const float *fmap2_rows, int y0, int y1, int B,
                      int D, int H, int W, int levels, float *const *pyr, void *workspace, size_t workspace_bytes,
                      int flags, void *stream) {
    static const char *fn = "corr_build_region";
    g_err[0] = 0;
    if (algo != CORR_BUILD_BF16X6)
        return fail(CORR_EUNSUPPORTED, "%s: only CORR_BUILD_BF16X6 builds by target region (got %d)", fn, algo);
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc) return rc;
    if (D < 1) return fail(CORR_EINVAL, "%s: D must be >= 1 (got %d)", fn, D);
    if (levels > 4) return fail(CORR_EUNSUPPORTED, "%s: levels <= 4 (got %d)", fn, levels);
    if (y0 < 0 || y0 >= y1 || y1 > H || y0 % 8 || (y1 % 8 && y1 != H))
        return fail(CORR_EINVAL, "%s: need 0 <= y0 < y1 <= H, y0 %% 8 == 0, y1 %% 8 == 0 or y1 == H (got %d, %d, H %d)",
                    fn, y0, y1, H);
    if ((rc = check_ptr(fn, fmap1_rows, "fmap1")) || (rc = check_ptr(fn, fmap2_rows, "fmap2_rows"))) return rc;
    if ((uintptr_t)workspace % 256) return fail(CORR_EINVAL, "%s: workspace is not 256-byte aligned", fn);
    const size_t need = build_bf16_workspace(B, D, NQ, H, W);
    if (workspace_bytes < need || !workspace)
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    LevelPtrs lp{};
    if ((rc = check_pyramid(fn, pyr, levels, "pyr", lp.p))) return rc;
    return hip_status(launch_build_bf16_region(fmap1_rows, NQ, fmap2_rows, y0, y1, B, D, H, W, levels, lp, workspace,
                                               (flags & CORR_REGION_PACK_QUERIES) != 0, (hipStream_t)stream),
                      fn);
}

int corr_build(const float *fmap1, const float *fmap2, int B, int D, int H, int W, int levels,
               float *const *pyr, void *stream) {
    return corr_build_rows(fmap1, H * W, fmap2, B, D, H, W, levels, pyr, stream);
}

int corr_lookup_rows(const float *const *pyr, const float *coords_rows, int B, int NQ, int H,
                     int W, int levels, int radius, float *out_rows, void *stream) {
    static const char *fn = "corr_lookup";
    g_err[0] = 0;
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc || (rc = check_radius(fn, radius))) return rc;
    if ((rc = check_ptr(fn, coords_rows, "coords")) || (rc = check_ptr(fn, out_rows, "out"))) return rc;
    ConstLevelPtrs lp{};
    if ((rc = check_pyramid(fn, pyr, levels, "pyr", lp.p))) return rc;
    return hip_status(launch_lookup(lp, coords_rows, B, NQ, H, W, levels, radius, out_rows, (hipStream_t)stream),
                      fn);
}

int corr_lookup(const float *const *pyr, const float *coords, int B, int H, int W, int levels,
                int radius, float *out, void *stream) {
    return corr_lookup_rows(pyr, coords, B, H * W, H, W, levels, radius, out, stream);
}

int corr_lookup_bwd_rows(const float *coords_rows, const float *grad_out_rows, int B, int NQ,
                         int H, int W, int levels, int radius, float *const *grad_pyr,
                         void *stream) {
    static const char *fn = "corr_lookup_bwd";
    g_err[0] = 0;
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc || (rc = check_radius(fn, radius))) return rc;
    if ((rc = check_ptr(fn, coords_rows, "coords")) || (rc = check_ptr(fn, grad_out_rows, "grad_out")))
        return rc;
    LevelPtrs lp{};
    if ((rc = check_levels(fn, grad_pyr, levels, "grad_pyr", lp.p))) return rc;
    return hip_status(
        launch_lookup_bwd(coords_rows, grad_out_rows, B, NQ, H, W, levels, radius, lp, (hipStream_t)stream), fn);
}

int corr_lookup_bwd(const float *coords, const float *grad_out, int B, int H, int W, int levels,
                    int radius, float *const *grad_pyr, void *stream) {
    return corr_lookup_bwd_rows(coords, grad_out, B, H * W, H, W, levels, radius, grad_pyr, stream);
}

int corr_pool_bwd(float *const *grad_pyr, int BN, int H, int W, int levels, void *stream) {
    static const char *fn = "corr_pool_bwd";
    g_err[0] = 0;
    int rc = check_dims(fn, 1, 1, H, W, levels);
    if (rc) return rc;
    if (BN < 1) return fail(CORR_EINVAL, "%s: BN must be >= 1", fn);
    LevelPtrs lp{};
    if ((rc = check_levels(fn, grad_pyr, levels, "grad_pyr", lp.p))) return rc;
    return hip_status(launch_pool_bwd(lp, BN, H, W, levels, (hipStream_t)stream), fn);
}

size_t corr_build_bwd_rows_workspace(int B, int D, int NQ, int H, int W) {
    if (B < 1 || D < 1 || NQ < 1 || H < 1 || W < 1) return 0;
    return build_bwd_workspace(B, D, NQ, H, W);
}

size_t corr_build_bwd_workspace(int B, int D, int H, int W) {
    return corr_build_bwd_rows_workspace(B, D, H * W, H, W);
}

int corr_build_bwd_rows(const float *grad_c, const float *fmap1_rows, int NQ, const float *fmap2,
                        int B, int D, int H, int W, float *dfmap1_rows, float *dfmap2,
                        void *workspace, size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_build_bwd";
    g_err[0] = 0;
    int rc = check_dims(fn, B, NQ, H, W, 1);
    if (rc) return rc;
    if (D < 1) return fail(CORR_EINVAL, "%s: D must be >= 1 (got %d)", fn, D);
    if ((rc = check_ptr(fn, grad_c, "grad_c")) || (rc = check_ptr(fn, fmap1_rows, "fmap1")) ||
        (rc = check_ptr(fn, fmap2, "fmap2")) || (rc = check_ptr(fn, dfmap1_rows, "dfmap1")) ||
        (rc = check_ptr(fn, dfmap2, "dfmap2")))
        return rc;
    const size_t need = build_bwd_workspace(B, D, NQ, H, W);
    if (workspace_bytes < need || (need && !workspace))
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    return hip_status(launch_build_bwd(grad_c, fmap1_rows, NQ, fmap2, B, D, H, W, dfmap1_rows, dfmap2,
                                       (float *)workspace, (hipStream_t)stream),
                      fn);
}

size_t corr_build_bwd_ex_workspace(int algo, int B, int D, int NQ, int H, int W) {
    if (B < 1 || D < 1 || NQ < 1 || H < 1 || W < 1) return 0;
    if (algo == CORR_BUILD_FP32) return build_bwd_workspace(B, D, NQ, H, W);
    if (algo == CORR_BUILD_F16X3 || algo == CORR_BUILD_BF16X6) return build_bwd_split_workspace(B, D, NQ, H, W);
    return (size_t)-1;
}

int corr_build_bwd_ex(int algo, const float *grad_c, const float *fmap1_rows, int NQ, const float *fmap2, int B,
                      int D, int H, int W, float *dfmap1_rows, float *dfmap2, void *workspace,
                      size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_build_bwd_ex";
    if (algo == CORR_BUILD_FP32)
        return corr_build_bwd_rows(grad_c, fmap1_rows, NQ, fmap2, B, D, H, W, dfmap1_rows, dfmap2, workspace,
                                   workspace_bytes, stream);
    g_err[0] = 0;
    if (algo != CORR_BUILD_F16X3 && algo != CORR_BUILD_BF16X6)
        return fail(CORR_EUNSUPPORTED, "%s: unknown algorithm %d", fn, algo);
    int rc = check_dims(fn, B, NQ, H, W, 1);
    if (rc) return rc;
    if (D < 1) return fail(CORR_EINVAL, "%s: D must be >= 1 (got %d)", fn, D);
    if ((rc = check_ptr(fn, grad_c, "grad_c")) || (rc = check_ptr(fn, fmap1_rows, "fmap1")) ||
        (rc = check_ptr(fn, fmap2, "fmap2")) || (rc = check_ptr(fn, dfmap1_rows, "dfmap1")) ||
        (rc = check_ptr(fn, dfmap2, "dfmap2")))
        return rc;
    const size_t need = build_bwd_split_workspace(B, D, NQ, H, W);
    if (workspace_bytes < need || !workspace)
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    return hip_status(launch_build_bwd_split(grad_c, fmap1_rows, NQ, fmap2, B, D, H, W, dfmap1_rows, dfmap2,
                                             workspace, (hipStream_t)stream, algo == CORR_BUILD_BF16X6),
                      fn);
}

int corr_lookup_bwd_multi(const float *const *coords_rows, const float *const *grad_out_rows, int T, int B, int NQ,
                          int H, int W, int levels, int radius, float *const *grad_pyr, void *stream) {
    static const char *fn = "corr_lookup_bwd_multi";
    g_err[0] = 0;
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc || (rc = check_radius(fn, radius))) return rc;
    if (T < 0) return fail(CORR_EINVAL, "%s: T must be >= 0 (got %d)", fn, T);
    if (T > 0 && (!coords_rows || !grad_out_rows)) return fail(CORR_EINVAL, "%s: coords / grad_out arrays are NULL", fn);
    for (int t = 0; t < T; ++t)
        if ((rc = check_ptr(fn, coords_rows[t], "coords[t]")) || (rc = check_ptr(fn, grad_out_rows[t], "grad_out[t]")))
            return rc;
    LevelPtrs lp{};
    if ((rc = check_levels(fn, grad_pyr, levels, "grad_pyr", lp.p))) return rc;
    return hip_status(launch_lookup_bwd_multi(coords_rows, grad_out_rows, T, B, NQ, H, W, levels, radius, lp,
                                              (hipStream_t)stream),
                      fn);
}

int corr_pool_fold(float *const *grad_pyr, int B, int NQ, int H, int W, int levels, void *stream) {
    static const char *fn = "corr_pool_fold";
    g_err[0] = 0;
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc) return rc;
    LevelPtrs lp{};
    if ((rc = check_levels(fn, grad_pyr, levels, "grad_pyr", lp.p))) return rc;
    return hip_status(launch_pool_fold(lp, B, NQ, H, W, levels, nullptr, 1, (hipStream_t)stream), fn);
}

size_t corr_backward_workspace(int algo, int B, int D, int NQ, int H, int W, int radius) {
    if (B < 1 || D < 1 || NQ < 1 || H < 1 || W < 1 || radius < 0) return 0;
    return backward_workspace(algo & ~CORR_BACKWARD_EXACT_FOLD, B, D, NQ, H, W, radius);
}

int corr_backward(int algo, const float *const *coords_rows, const float *const *grad_out_rows, int T,
                  const float *fmap1_rows, int NQ, const float *fmap2, int B, int D, int H, int W, int levels,
                  int radius, float *const *grad_pyr, float *dfmap1_rows, float *dfmap2, void *workspace,
                  size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_backward";
    g_err[0] = 0;
    const int base = algo & ~CORR_BACKWARD_EXACT_FOLD;
    if (base != CORR_BUILD_FP32 && base != CORR_BUILD_F16X3 && base != CORR_BUILD_BF16X6)
        return fail(CORR_EUNSUPPORTED, "%s: unknown algorithm %d", fn, algo);
    int rc = check_dims(fn, B, NQ, H, W, levels);
    if (rc || (rc = check_radius(fn, radius))) return rc;
    if (D < 1) return fail(CORR_EINVAL, "%s: D must be >= 1 (got %d)", fn, D);
    if (T < 0) return fail(CORR_EINVAL, "%s: T must be >= 0 (got %d)", fn, T);
    if (T > 0 && (!coords_rows || !grad_out_rows)) return fail(CORR_EINVAL, "%s: coords / grad_out arrays are NULL", fn);
    for (int t = 0; t < T; ++t)
        if ((rc = check_ptr(fn, coords_rows[t], "coords[t]")) || (rc = check_ptr(fn, grad_out_rows[t], "grad_out[t]")))
            return rc;
    if ((rc = check_ptr(fn, fmap1_rows, "fmap1")) || (rc = check_ptr(fn, fmap2, "fmap2")) ||
        (rc = check_ptr(fn, dfmap1_rows, "dfmap1")) || (rc = check_ptr(fn, dfmap2, "dfmap2")))
        return rc;
    const size_t need = corr_backward_workspace(base, B, D, NQ, H, W, radius);
    if (workspace_bytes < need || (need && !workspace))
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    LevelPtrs lp{};
    if ((rc = check_levels(fn, grad_pyr, levels, "grad_pyr", lp.p))) return rc;
    return hip_status(launch_backward(algo, coords_rows, grad_out_rows, T, fmap1_rows, NQ, fmap2, B, D, H, W, levels,
                                      radius, lp, dfmap1_rows, dfmap2, workspace, (hipStream_t)stream),
                      fn);
}

size_t corr_lookup_conv_weights_bytes(void) { return lookup_conv_weights_bytes(); }

int corr_lookup_conv_weights(const float *weight, int out_channels, int in_channels, void *packed, void *stream) {
    static const char *fn = "corr_lookup_conv_weights";
    g_err[0] = 0;
    int rc;
    if ((rc = check_ptr(fn, weight, "weight")) || (rc = check_ptr(fn, packed, "packed"))) return rc;
    if (out_channels != 256 || in_channels < 1 || in_channels > 4 * 81)
        return fail(CORR_EUNSUPPORTED, "%s: built for 256 output and <= 324 input channels (got %d, %d)", fn,
                    out_channels, in_channels);
    return hip_status(launch_lookup_conv_weights(weight, out_channels, in_channels, packed, (hipStream_t)stream), fn);
}

int corr_lookup_conv(const float *const *pyr, const float *coords, int B, int H, int W, int levels, int radius,
                     const void *packed_weight, const float *bias, int relu, float *out, void *stream) {
    static const char *fn = "corr_lookup_conv";
    g_err[0] = 0;
    int rc = check_dims(fn, B, H * W, H, W, levels);
    if (rc) return rc;
    if (radius != 4 || levels > 4)
        return fail(CORR_EUNSUPPORTED, "%s: built for radius 4 and <= 4 levels (got %d, %d)", fn, radius, levels);
    ConstLevelPtrs lp{};
    if ((rc = check_pyramid(fn, pyr, levels, "pyr", lp.p))) return rc;
    if ((rc = check_ptr(fn, coords, "coords")) || (rc = check_ptr(fn, packed_weight, "packed_weight")) ||
        (rc = check_ptr(fn, bias, "bias")) || (rc = check_ptr(fn, out, "out")))
        return rc;
    return hip_status(launch_lookup_conv(lp, coords, B, H * W, H, W, levels, radius, packed_weight, bias, relu, out,
                                         (hipStream_t)stream),
                      fn);
}

size_t corr_lookup_conv_bwd_workspace(int B, int H, int W, int levels) {
    if (B < 1 || H < 1 || W < 1 || levels < 1 || levels > 4) return 0;
    return lookup_conv_bwd_workspace(B, H * W, levels);
}

int corr_lookup_conv_bwd(const float *const *pyr, const float *coords, int B, int H, int W, int levels, int radius,
                         const void *packed_weight, const float *out, int relu, const float *grad_out,
                         float *grad_weight, float *grad_bias, float *grad_lookup, void *workspace,
                         size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_lookup_conv_bwd";
    g_err[0] = 0;
    int rc = check_dims(fn, B, H * W, H, W, levels);
    if (rc) return rc;
    if (radius != 4 || levels > 4)
        return fail(CORR_EUNSUPPORTED, "%s: built for radius 4 and <= 4 levels (got %d, %d)", fn, radius, levels);
    ConstLevelPtrs lp{};
    if ((rc = check_pyramid(fn, pyr, levels, "pyr", lp.p))) return rc;
    if ((rc = check_ptr(fn, coords, "coords")) || (rc = check_ptr(fn, packed_weight, "packed_weight")) ||
        (rc = check_ptr(fn, grad_out, "grad_out")))
        return rc;
    if (relu && (rc = check_ptr(fn, out, "out"))) return rc;
    if (!grad_weight && !grad_bias && !grad_lookup) return CORR_OK;
    if (grad_weight || grad_bias) {
        const size_t need = lookup_conv_bwd_workspace(B, H * W, levels);
        if (!workspace || workspace_bytes < need)
            return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
        if ((uintptr_t)workspace % 16)
            return fail(CORR_EINVAL, "%s: workspace must be 16-byte aligned", fn);
    }
    if ((H * W) % 4 == 0 && ((uintptr_t)grad_out % 16 || (relu && (uintptr_t)out % 16)))
        return fail(CORR_EINVAL, "%s: grad_out and out must be 16-byte aligned when H*W %% 4 == 0", fn);
    return hip_status(launch_lookup_conv_bwd(lp, coords, B, H * W, H, W, levels, radius, packed_weight, out, relu,
                                             grad_out, grad_weight, grad_bias, grad_lookup, workspace,
                                             (hipStream_t)stream),
                      fn);
}

int corr_convex_upsample(const float *flow, const float *mask, int N, int h, int w, float *out, void *stream) {
    static const char *fn = "corr_convex_upsample";
    g_err[0] = 0;
    if (N < 1 || h < 1 || w < 1)
        return fail(CORR_EINVAL, "%s: N, h, w must be >= 1 (got %d, %d, %d)", fn, N, h, w);
    int rc;
    if ((rc = check_ptr(fn, flow, "flow")) || (rc = check_ptr(fn, mask, "mask")) || (rc = check_ptr(fn, out, "out")))
        return rc;
    return hip_status(launch_convex_upsample(flow, mask, N, h, w, out, (hipStream_t)stream), fn);
}

size_t corr_convex_upsample_bwd_workspace(int N, int h, int w) {
    if (N < 1 || h < 1 || w < 1) return 0;
    return convex_upsample_bwd_workspace(N, h, w);
}

int corr_convex_upsample_bwd(const float *flow, const float *mask, const float *grad_out, int N, int h, int w,
                             float *dflow, float *dmask, void *workspace, size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_convex_upsample_bwd";
    g_err[0] = 0;
    if (N < 1 || h < 1 || w < 1)
        return fail(CORR_EINVAL, "%s: N, h, w must be >= 1 (got %d, %d, %d)", fn, N, h, w);
    int rc;
    if ((rc = check_ptr(fn, flow, "flow")) || (rc = check_ptr(fn, mask, "mask")) ||
        (rc = check_ptr(fn, grad_out, "grad_out")) || (rc = check_ptr(fn, dflow, "dflow")) ||
        (rc = check_ptr(fn, dmask, "dmask")) || (rc = check_ptr(fn, workspace, "workspace")))
        return rc;
    const size_t need = convex_upsample_bwd_workspace(N, h, w);
    if (workspace_bytes < need)
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes, %zu needed", fn, workspace_bytes, need);
    return hip_status(launch_convex_upsample_bwd(flow, mask, grad_out, N, h, w, dflow, dmask, workspace,
                                                 (hipStream_t)stream),
                      fn);
}

size_t corr_voxel_grid_workspace(int n_events, int C, int H, int W) {
    if (n_events < 0 || C < 1 || H < 1 || W < 1) return 0;
    return voxel_workspace(n_events, C, H, W);
}

int corr_voxel_grid(const float *x, const float *y, const float *t, const float *p, int n_events, int C, int H,
                    int W, int normalize, float *out, void *workspace, size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_voxel_grid";
    g_err[0] = 0;
    if (n_events < 0 || C < 1 || H < 1 || W < 1)
        return fail(CORR_EINVAL, "%s: need n_events >= 0 and C, H, W >= 1 (got %d, %d, %d, %d)", fn, n_events, C,
                    H, W);
    if ((long long)n_events * 4 >= (1ll << 31) || (long long)C * H * W >= (1ll << 31))
        return fail(CORR_EINVAL, "%s: problem too large", fn);
    int rc;
    if ((rc = check_ptr(fn, out, "out"))) return rc;
    if (n_events > 0 && ((rc = check_ptr(fn, x, "x")) || (rc = check_ptr(fn, y, "y")) ||
                         (rc = check_ptr(fn, t, "t")) || (rc = check_ptr(fn, p, "p"))))
        return rc;
    const size_t need = voxel_workspace(n_events, C, H, W);
    if (workspace_bytes < need || !workspace)
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    return hip_status(launch_voxel_grid(x, y, t, p, n_events, C, H, W, normalize, out, workspace,
                                        (hipStream_t)stream),
                      fn);
}

size_t corr_voxel_grid_tbilinear_workspace(int n_events, int C, int H, int W) {
    if (n_events < 0 || C < 1 || H < 1 || W < 1) return 0;
    return voxel_tbilinear_workspace(n_events, C, H, W);
}

int corr_voxel_grid_tbilinear(const double *events, int n_events, int C, int H, int W, int normalize, float *out,
                              void *workspace, size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_voxel_grid_tbilinear";
    g_err[0] = 0;
    if (n_events < 0 || C < 1 || H < 1 || W < 1)
        return fail(CORR_EINVAL, "%s: need n_events >= 0 and C, H, W >= 1 (got %d, %d, %d, %d)", fn, n_events, C,
                    H, W);
    if ((long long)n_events * 2 >= (1ll << 31) || (long long)C * H * W >= (1ll << 31))
        return fail(CORR_EINVAL, "%s: problem too large", fn);
    int rc;
    if ((rc = check_ptr(fn, out, "out"))) return rc;
    if (n_events > 0) {
        if ((rc = check_ptr(fn, events, "events"))) return rc;
        if ((uintptr_t)events % 8) return fail(CORR_EINVAL, "%s: events is not 8-byte aligned", fn);
    }
    const size_t need = voxel_tbilinear_workspace(n_events, C, H, W);
    if (workspace_bytes < need || !workspace)
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    return hip_status(
        launch_voxel_grid_tbilinear(events, n_events, C, H, W, normalize, out, workspace, (hipStream_t)stream), fn);
}

size_t corr_forward_splat_workspace(int B, int H, int W) {
    if (B < 1 || H < 1 || W < 1) return 0;
    return splat_workspace(B, H, W);
}

int corr_forward_splat(const float *flow, int B, int H, int W, float *out, void *workspace,
                       size_t workspace_bytes, void *stream) {
    static const char *fn = "corr_forward_splat";
    g_err[0] = 0;
    if (B < 1 || H < 1 || W < 1)
        return fail(CORR_EINVAL, "%s: B, H, W must be >= 1 (got %d, %d, %d)", fn, B, H, W);
    if ((long long)H * W * 4 >= (1ll << 31))
        return fail(CORR_EINVAL, "%s: %dx%d is too large", fn, H, W);
    int rc;
    if ((rc = check_ptr(fn, flow, "flow")) || (rc = check_ptr(fn, out, "out"))) return rc;
    const size_t need = splat_workspace(B, H, W);
    if (workspace_bytes < need || !workspace)
        return fail(CORR_EINVAL, "%s: workspace of %zu bytes needed, got %zu", fn, need, workspace_bytes);
    return hip_status(launch_forward_splat(flow, B, H, W, out, workspace, (hipStream_t)stream), fn);
}

int corr_build_bwd(const float *grad_c, const float *fmap1, const float *fmap2, int B, int D,
                   int H, int W, float *dfmap1, float *dfmap2, void *workspace,
                   size_t workspace_bytes, void *stream) {
    return corr_build_bwd_rows(grad_c, fmap1, H * W, fmap2, B, D, H, W, dfmap1, dfmap2, workspace,
                               workspace_bytes, stream);
}

}  // extern "C"
