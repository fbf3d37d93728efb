// corr_api.cpp — the extern "C" boundary of libcorr_mi355x.so (declared in
// include/corr_mi355x.h).  Validates arguments, records thread-local errors and forwards to
// the gfx950 launchers.  No allocation, no synchronisation, no global mutable state.
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

static int check_dims(const char *fn, int B, int H, int W, int levels) {
    if (B < 1 || H < 1 || W < 1)
        return fail(CORR_EINVAL, "%s: B, H, W must be >= 1 (got %d, %d, %d)", fn, B, H, W);
    if (levels < 1 || levels > CORR_MAX_LEVELS)
        return fail(CORR_EINVAL, "%s: levels must be in [1, %d] (got %d)", fn, CORR_MAX_LEVELS, levels);
    // avg_pool2d(2, 2) on a 1-pixel dimension raises in the reference (corr.py:26)
    if ((H >> (levels - 1)) < 1 || (W >> (levels - 1)) < 1)
        return fail(CORR_EINVAL, "%s: %dx%d is too small for %d pyramid levels", fn, H, W, levels);
    // the lookup's neighbourhood anchors assume |coordinate floors| of in-map taps < 2^20
    if (H > (1 << 20) || W > (1 << 20))
        return fail(CORR_EINVAL, "%s: H and W must be <= 2^20", fn);
    const long long N = (long long)H * W;
    if (N > (1LL << 30) || (long long)B * N > (1LL << 31) - 1)
        return fail(CORR_EINVAL, "%s: B*H*W too large", fn);
    return CORR_OK;
}

static int check_ptr(const char *fn, const void *p, const char *name) {
    if (!p) return fail(CORR_EINVAL, "%s: %s is NULL", fn, name);
    if ((uintptr_t)p % 4) return fail(CORR_EINVAL, "%s: %s is not 4-byte aligned", fn, name);
    return CORR_OK;
}

}  // namespace corr

using namespace corr;

extern "C" {

int corr_version(void) { return 100; }

const char *corr_last_error(void) { return g_err; }

int corr_build(const float *fmap1, const float *fmap2, int B, int D, int H, int W, int levels,
               float *const *pyr, void *stream) {
    g_err[0] = 0;
    int rc = check_dims("corr_build", B, H, W, levels);
    if (rc) return rc;
    if (D < 1) return fail(CORR_EINVAL, "corr_build: D must be >= 1 (got %d)", D);
    if ((rc = check_ptr("corr_build", fmap1, "fmap1")) || (rc = check_ptr("corr_build", fmap2, "fmap2")))
        return rc;
    if (!pyr) return fail(CORR_EINVAL, "corr_build: pyr is NULL");
    LevelPtrs lp{};
    for (int l = 0; l < levels; ++l) {
        if ((rc = check_ptr("corr_build", pyr[l], "pyr[l]"))) return rc;
        lp.p[l] = pyr[l];
    }
    return hip_status(launch_build(fmap1, fmap2, B, D, H, W, levels, lp, (hipStream_t)stream),
                      "corr_build");
}

int corr_lookup(const float *const *pyr, const float *coords, int B, int H, int W, int levels,
                int radius, float *out, void *stream) {
    g_err[0] = 0;
    int rc = check_dims("corr_lookup", B, H, W, levels);
    if (rc) return rc;
    if (radius < 0 || radius > CORR_MAX_RADIUS)
        return fail(CORR_EINVAL, "corr_lookup: radius must be in [0, %d] (got %d)", CORR_MAX_RADIUS, radius);
    if ((rc = check_ptr("corr_lookup", coords, "coords")) || (rc = check_ptr("corr_lookup", out, "out")))
        return rc;
    if (!pyr) return fail(CORR_EINVAL, "corr_lookup: pyr is NULL");
    ConstLevelPtrs lp{};
    for (int l = 0; l < levels; ++l) {
        if ((rc = check_ptr("corr_lookup", pyr[l], "pyr[l]"))) return rc;
        lp.p[l] = pyr[l];
    }
    return hip_status(launch_lookup(lp, coords, B, H, W, levels, radius, out, (hipStream_t)stream),
                      "corr_lookup");
}

int corr_lookup_bwd(const float *coords, const float *grad_out, int B, int H, int W, int levels,
                    int radius, float *const *grad_pyr, void *stream) {
    g_err[0] = 0;
    int rc = check_dims("corr_lookup_bwd", B, H, W, levels);
    if (rc) return rc;
    if (radius < 0 || radius > CORR_MAX_RADIUS)
        return fail(CORR_EINVAL, "corr_lookup_bwd: radius must be in [0, %d] (got %d)", CORR_MAX_RADIUS, radius);
    if ((rc = check_ptr("corr_lookup_bwd", coords, "coords")) ||
        (rc = check_ptr("corr_lookup_bwd", grad_out, "grad_out")))
        return rc;
    if (!grad_pyr) return fail(CORR_EINVAL, "corr_lookup_bwd: grad_pyr is NULL");
    LevelPtrs lp{};
    for (int l = 0; l < levels; ++l) {
        if ((rc = check_ptr("corr_lookup_bwd", grad_pyr[l], "grad_pyr[l]"))) return rc;
        lp.p[l] = grad_pyr[l];
    }
    return hip_status(launch_lookup_bwd(coords, grad_out, B, H, W, levels, radius, lp, (hipStream_t)stream),
                      "corr_lookup_bwd");
}

int corr_pool_bwd(float *const *grad_pyr, int BN, int H, int W, int levels, void *stream) {
    g_err[0] = 0;
    int rc = check_dims("corr_pool_bwd", 1, H, W, levels);
    if (rc) return rc;
    if (BN < 1) return fail(CORR_EINVAL, "corr_pool_bwd: BN must be >= 1");
    if (!grad_pyr) return fail(CORR_EINVAL, "corr_pool_bwd: grad_pyr is NULL");
    LevelPtrs lp{};
    for (int l = 0; l < levels; ++l) {
        if ((rc = check_ptr("corr_pool_bwd", grad_pyr[l], "grad_pyr[l]"))) return rc;
        lp.p[l] = grad_pyr[l];
    }
    return hip_status(launch_pool_bwd(lp, BN, H, W, levels, (hipStream_t)stream), "corr_pool_bwd");
}

size_t corr_build_bwd_workspace(int B, int D, int H, int W) {
    if (B < 1 || D < 1 || H < 1 || W < 1) return 0;
    return build_bwd_workspace(B, D, H, W);
}

int corr_build_bwd(const float *grad_c, const float *fmap1, const float *fmap2, int B, int D,
                   int H, int W, float *dfmap1, float *dfmap2, void *workspace,
                   size_t workspace_bytes, void *stream) {
    g_err[0] = 0;
    int rc = check_dims("corr_build_bwd", B, H, W, 1);
    if (rc) return rc;
    if (D < 1) return fail(CORR_EINVAL, "corr_build_bwd: D must be >= 1 (got %d)", D);
    if ((rc = check_ptr("corr_build_bwd", grad_c, "grad_c")) ||
        (rc = check_ptr("corr_build_bwd", fmap1, "fmap1")) ||
        (rc = check_ptr("corr_build_bwd", fmap2, "fmap2")) ||
        (rc = check_ptr("corr_build_bwd", dfmap1, "dfmap1")) ||
        (rc = check_ptr("corr_build_bwd", dfmap2, "dfmap2")))
        return rc;
    const size_t need = build_bwd_workspace(B, D, H, W);
    if (workspace_bytes < need || (need && !workspace))
        return fail(CORR_EINVAL, "corr_build_bwd: workspace of %zu bytes needed, got %zu", need,
                    workspace_bytes);
    return hip_status(launch_build_bwd(grad_c, fmap1, fmap2, B, D, H, W, dfmap1, dfmap2,
                                       (float *)workspace, (hipStream_t)stream),
                      "corr_build_bwd");
}

}  // extern "C"
