// siren_capi.hip — the C ABI of libsiren_amd.so (include/siren_amd.h): validation, workspace sizing and
// kernel launches. Single translation unit over the kernel headers.
#include "fused_kernels.hpp"
#include "train_kernels.hpp"
#include "w1_kernel.hpp"
// ==========================================================================================================
// C ABI
// ==========================================================================================================
#include "../../include/siren_amd.h"
#include <cmath>
#include <cstdio>
#include <string>

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int check_cfg(const siren_cfg* cfg, bool fused) {
    if (cfg == nullptr) return fail(SIREN_EINVAL, "cfg is NULL");
    if (cfg->d_in < 1 || cfg->d_out < 1 || cfg->hidden < 1 || cfg->n_hidden < 0)
        return fail(SIREN_EINVAL, "d_in, d_out, hidden must be >= 1 and n_hidden >= 0");
    if (!std::isfinite(cfg->omega_first) || !std::isfinite(cfg->omega_hidden))
        return fail(SIREN_EINVAL, "omega values must be finite");
    if (fused) {
        if (cfg->hidden != siren::H) return fail(SIREN_EUNSUPPORTED, "fused kernels need hidden_features == 256");
        if (cfg->d_in > siren::MAXD) return fail(SIREN_EUNSUPPORTED, "fused kernels need in_features <= 4");
        if (cfg->d_out > siren::MAXO) return fail(SIREN_EUNSUPPORTED, "fused kernels need out_features <= 4");
        if (cfg->n_hidden < 1 || cfg->n_hidden > siren::MAX_LH_FWD)
            return fail(SIREN_EUNSUPPORTED, "fused kernels need 1 <= num_hidden_layers <= 8");
    }
    return SIREN_OK;
}

int hip_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIREN_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return SIREN_OK;
}

int64_t ws_floats(const siren_cfg* cfg) {
    return siren::small_pad(cfg->n_hidden) + 2ll * cfg->n_hidden * siren::NB * siren::SLICE;
}

int64_t param_count(const siren_cfg* cfg) {
    const int64_t H = cfg->hidden;
    return H * cfg->d_in + H + (int64_t)cfg->n_hidden * (H * H + H) + (int64_t)cfg->d_out * H + cfg->d_out;
}

// W2 backward workspace: sin activations and deltas of every sine layer in 16-coordinate tiles, plus S
// param-shaped partial slabs of the split-K weight-gradient reduction.
struct TrainPlan {
    int64_t n_pad, tiles, splits, tps, act_floats, partial_floats, total;
    TrainPlan(const siren_cfg* cfg, int64_t n) {
        n_pad = (n + siren::TILE - 1) / siren::TILE * siren::TILE;
        tiles = n_pad / 16;
        const int64_t want = (512 + cfg->n_hidden - 1) / cfg->n_hidden;  // ~512 wgrad workgroups in total
        splits = tiles < want ? tiles : want;
        if (splits < 1) splits = 1;
        tps = (tiles + splits - 1) / splits;
        splits = (tiles + tps - 1) / tps;
        if (splits < 1) splits = 1;
        act_floats = (int64_t)(cfg->n_hidden + 1) * n_pad * siren::H;
        partial_floats = splits * param_count(cfg);
        total = 2 * act_floats + partial_floats;
    }
};
}  // namespace

extern "C" {

int32_t siren_abi_version(void) { return SIREN_ABI_VERSION; }

const char* siren_last_error(void) { return g_err.c_str(); }

int32_t siren_param_count(const siren_cfg* cfg, int64_t* count) {
    if (int rc = check_cfg(cfg, false)) return rc;
    if (count == nullptr) return fail(SIREN_EINVAL, "count is NULL");
    *count = param_count(cfg);
    return SIREN_OK;
}

int32_t siren_workspace_floats(const siren_cfg* cfg, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (count == nullptr) return fail(SIREN_EINVAL, "count is NULL");
    *count = ws_floats(cfg);
    return SIREN_OK;
}

int32_t siren_pack(const siren_cfg* cfg, const float* params, float* ws, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (params == nullptr || ws == nullptr) return fail(SIREN_EINVAL, "params/ws is NULL");
    const int64_t total = ws_floats(cfg);
    const int threads = 256;
    const int64_t blocks = std::min<int64_t>((total + threads - 1) / threads, 8192);
    hipLaunchKernelGGL(siren::pack_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, params,
                       ws, cfg->d_in, cfg->d_out, cfg->n_hidden, siren::small_pad(cfg->n_hidden), total);
    return hip_status("siren_pack");
}

int32_t siren_forward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || y == nullptr) return fail(SIREN_EINVAL, "ws/x/y is NULL");
    const int64_t blocks = (n + siren::TILE - 1) / siren::TILE;
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    const dim3 grid((unsigned)blocks), block(siren::THREADS);
    if (cfg->outermost_linear && cfg->n_hidden <= 5 && (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0) {
#define SIREN_LAUNCH_FWD(LHV)                                                                                    \
    hipLaunchKernelGGL((siren::w1_kernel<LHV, siren::MODE_FWD>), grid, block, 0, (hipStream_t)stream, ws, x, n,      \
                       (const float*)nullptr, y, (float*)nullptr, cfg->d_in, cfg->d_out, cfg->omega_first,         \
                       cfg->omega_hidden, (float*)nullptr, (float*)nullptr, (int64_t)0)
        switch (cfg->n_hidden) {
            case 1: SIREN_LAUNCH_FWD(1); break;
            case 2: SIREN_LAUNCH_FWD(2); break;
            case 3: SIREN_LAUNCH_FWD(3); break;
            case 4: SIREN_LAUNCH_FWD(4); break;
            default: SIREN_LAUNCH_FWD(5); break;
        }
#undef SIREN_LAUNCH_FWD
        return hip_status("siren_forward");
    }
    hipLaunchKernelGGL((siren::fused_kernel<0, false>), grid, block, 0,
                       (hipStream_t)stream, ws, x, n, nullptr, y, nullptr, cfg->d_in, cfg->d_out, cfg->n_hidden,
                       cfg->omega_first, cfg->omega_hidden, cfg->outermost_linear ? 0 : 1);
    return hip_status("siren_forward");
}

int32_t siren_forward_grad(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy,
                           float* y, float* gx, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (cfg->n_hidden > siren::MAX_LH_GRAD)
        return fail(SIREN_EUNSUPPORTED, "siren_forward_grad needs 1 <= num_hidden_layers <= 3");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || gx == nullptr) return fail(SIREN_EINVAL, "ws/x/gx is NULL");
    const int64_t blocks = (n + siren::TILE - 1) / siren::TILE;
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    const dim3 grid((unsigned)blocks), block(siren::THREADS);
    const int fs = cfg->outermost_linear ? 0 : 1;
    const bool legacy = (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) != 0 || fs;
    if (!legacy) {
#define SIREN_LAUNCH_W1(LHV)                                                                                    \
    hipLaunchKernelGGL((siren::w1_kernel<LHV, siren::MODE_W1>), grid, block, 0, (hipStream_t)stream, ws, x, n, gy, y, gx, \
                       cfg->d_in, cfg->d_out, cfg->omega_first, cfg->omega_hidden, (float*)nullptr, (float*)nullptr, \
                       (int64_t)0)
        switch (cfg->n_hidden) {
            case 1: SIREN_LAUNCH_W1(1); break;
            case 2: SIREN_LAUNCH_W1(2); break;
            default: SIREN_LAUNCH_W1(3); break;
        }
#undef SIREN_LAUNCH_W1
        return hip_status("siren_forward_grad");
    }
#define SIREN_LAUNCH_GRAD(LHV)                                                                                   \
    hipLaunchKernelGGL((siren::fused_kernel<LHV, true>), grid, block, 0, (hipStream_t)stream, ws, x, n, gy, y, gx, \
                       cfg->d_in, cfg->d_out, LHV, cfg->omega_first, cfg->omega_hidden, fs)
    switch (cfg->n_hidden) {
        case 1: SIREN_LAUNCH_GRAD(1); break;
        case 2: SIREN_LAUNCH_GRAD(2); break;
        default: SIREN_LAUNCH_GRAD(3); break;
    }
#undef SIREN_LAUNCH_GRAD
    return hip_status("siren_forward_grad");
}

int32_t siren_train_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    *count = TrainPlan(cfg, n).total;
    return SIREN_OK;
}

int32_t siren_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy,
                       float* tws, void* reserved, float* gx, float* gparams, void* stream) {
    (void)reserved;
    if (int rc = check_cfg(cfg, true)) return rc;
    if (cfg->n_hidden > siren::MAX_LH_GRAD)
        return fail(SIREN_EUNSUPPORTED, "siren_backward needs 1 <= num_hidden_layers <= 3");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (ws == nullptr || gy == nullptr || tws == nullptr || gx == nullptr || gparams == nullptr ||
        (n > 0 && x == nullptr))
        return fail(SIREN_EINVAL, "ws/x/gy/tws/gx/gparams is NULL");
    const TrainPlan plan(cfg, n);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {
        (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_backward");
    }
    float* abuf = tws;
    float* dbuf = tws + plan.act_floats;
    float* partial = tws + 2 * plan.act_floats;
    const dim3 grid((unsigned)(plan.n_pad / siren::TILE)), block(siren::THREADS);
    const int fs = cfg->outermost_linear ? 0 : 1;
    if ((cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0 && !fs) {
#define SIREN_LAUNCH_W1S(LHV)                                                                               \
    hipLaunchKernelGGL((siren::w1_kernel<LHV, siren::MODE_STORE>), grid, block, 0, st, ws, x, n, gy, (float*)nullptr, gx, \
                       cfg->d_in, cfg->d_out, cfg->omega_first, cfg->omega_hidden, abuf, dbuf, plan.n_pad)
        switch (cfg->n_hidden) {
            case 1: SIREN_LAUNCH_W1S(1); break;
            case 2: SIREN_LAUNCH_W1S(2); break;
            default: SIREN_LAUNCH_W1S(3); break;
        }
#undef SIREN_LAUNCH_W1S
    } else {
#define SIREN_LAUNCH_STORE(LHV)                                                                                    \
    hipLaunchKernelGGL((siren::fused_kernel<LHV, true, true>), grid, block, 0, st, ws, x, n, gy, (float*)nullptr, gx, \
                       cfg->d_in, cfg->d_out, LHV, cfg->omega_first, cfg->omega_hidden, fs, abuf, dbuf, plan.n_pad)
    switch (cfg->n_hidden) {
        case 1: SIREN_LAUNCH_STORE(1); break;
        case 2: SIREN_LAUNCH_STORE(2); break;
        default: SIREN_LAUNCH_STORE(3); break;
    }
#undef SIREN_LAUNCH_STORE
    }
    if (int rc = hip_status("siren_backward (fused store)")) return rc;
    hipLaunchKernelGGL(siren::wgrad_kernel, dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden), block, 0, st, abuf,
                       dbuf, plan.n_pad, plan.tps, partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_backward (wgrad)")) return rc;
    hipLaunchKernelGGL(siren::small_kernel, dim3((unsigned)plan.splits), block, 0, st, abuf, dbuf, x, gy, n, plan.n_pad,
                       plan.tps, partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_backward (small)")) return rc;
    const int64_t rblocks = std::min<int64_t>((P + 255) / 256, 4096);
    hipLaunchKernelGGL(siren::reduce_kernel, dim3((unsigned)rblocks), dim3(256), 0, st, partial, plan.splits, P,
                       gparams);
    return hip_status("siren_backward (reduce)");
}

}  // extern "C"
