// siren_capi.hip — the C ABI of libsiren_amd.so (include/siren_amd.h): validation, workspace sizing and
// dispatch to the kernel launchers (launch.h; one translation unit per kernel family).
#include "hess_kernel.hpp"
#include "launch.h"
#include "siren_common.h"
#include "siren_params.h"
// ==========================================================================================================
// C ABI
// ==========================================================================================================
#include "../../include/siren_amd.h"
#include <algorithm>
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
        const bool fused_h = cfg->hidden == siren::H || cfg->hidden == 512;
        const bool layered_h = cfg->hidden % 64 == 0 && cfg->hidden >= 64 && cfg->hidden <= 4096;
        if (!fused_h && !layered_h)
            return fail(SIREN_EUNSUPPORTED, "hidden_features must be 256 / 512 (fused kernels) or a multiple of 64 in "
                                            "[64, 4096] (layered path)");
        if (cfg->d_in > siren::MAXD) return fail(SIREN_EUNSUPPORTED, "fused kernels need in_features <= 4");
        if (cfg->d_out > siren::MAXO) return fail(SIREN_EUNSUPPORTED, "fused kernels need out_features <= 4");
        if (cfg->n_hidden < 1 || cfg->n_hidden > (fused_h ? siren::MAX_LH_FWD : 16))
            return fail(SIREN_EUNSUPPORTED, "need 1 <= num_hidden_layers <= 8 (16 on the layered path)");
        if (!fused_h && !cfg->outermost_linear)
            return fail(SIREN_EUNSUPPORTED, "the layered path (hidden other than 256 / 512) needs a linear output layer");
    }
    return SIREN_OK;
}

int hip_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIREN_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return SIREN_OK;
}

bool wide(const siren_cfg* cfg) { return cfg->hidden == 512; }
// hidden widths the fused kernels do not hold in registers: layer-by-layer over coordinate chunks (layered.hip)
bool layered(const siren_cfg* cfg) { return cfg->hidden != siren::H && cfg->hidden != 512; }
int layered_unsupported(const char* what) {
    return fail(SIREN_EUNSUPPORTED, std::string(what) + " covers hidden 256 / 512 (the layered path of other widths "
                                                        "runs W0, W1 and W2: siren_forward / _forward_grad / _backward)");
}

// packed workspace: small block + forward slices + transposed slices (16 x hidden floats each); at hidden 256 a
// second, phase-scaled copy follows for w1_kernel (pack_kernel: weights and biases times w / 2 pi, so its
// accumulators are phases in revolutions and each sin/cos epilogue saves ~4 VALU — siren_common.h sincos_rev)
int64_t small_pad(const siren_cfg* cfg) { return siren::SmallLayout(cfg->hidden).pad(cfg->n_hidden); }
int64_t ws_base(const siren_cfg* cfg) {
    const int64_t h = cfg->hidden;
    return small_pad(cfg) + 2ll * cfg->n_hidden * (h / 16) * (16 * h);
}
int64_t ws_floats(const siren_cfg* cfg) {
    if (layered(cfg)) return siren::layered_ws_floats(cfg->d_in, cfg->hidden, cfg->n_hidden, cfg->d_out);
    return wide(cfg) ? ws_base(cfg) : 2 * ws_base(cfg);
}
// the phase-scaled image needs w0, w != 0 (its reverse multipliers are w0 / s and 2 pi with s = w / 2 pi)
bool w1_ok(const siren_cfg* cfg) {
    return !wide(cfg) && !layered(cfg) && cfg->omega_first != 0.f && cfg->omega_hidden != 0.f;
}
// hidden 256 with 4..5 hidden layers (FCBlock builds any depth, modules.py:65-80): cos(w z_l) of every layer no longer
// fits the register file, so W1 / W2 / the kept W3 run the stored split through HBM (MODE_FWDS + MODE_REV,
// tu_w1deep.hip) and W3 the serial kernel's layer loops
bool deep(const siren_cfg* cfg) {
    return w1_ok(cfg) && cfg->outermost_linear && (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0 &&
           cfg->n_hidden > siren::MAX_LH_GRAD && cfg->n_hidden <= siren::MAX_LH_DEEP;
}
// scr: the caller's chunk scratch (layered_scratch); with LAY_TWS it follows the stored a_l / cos_l rows in tws
int64_t layered_scratch(const siren_cfg* cfg, int64_t n, bool stored) {
    return siren::layered_scratch_floats(cfg->d_in, cfg->hidden, cfg->n_hidden, cfg->d_out, n, stored);
}
int layered_call(int mode, const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy, float* y,
                 float* gx, float* gp, float* tws, float* scr, void* stream, const char* what) {
    if (n > 0 && scr == nullptr)
        return fail(SIREN_EINVAL, std::string(what) + ": the layered path (hidden other than 256 / 512) needs the "
                                  "caller's chunk scratch (tws; see the entry point's *_ws_floats query)");
    const siren::LayeredPlan plan(cfg->d_in, cfg->hidden, cfg->n_hidden, cfg->d_out, n);
    std::string err;
    if (siren::layered_run(mode, plan, ws, cfg->omega_first, cfg->omega_hidden, x, n, gy, y, gx, gp, tws, scr,
                           (hipStream_t)stream, err) != 0)
        return fail(SIREN_EHIP, std::string(what) + ": " + err);
    return hip_status(what);
}
const float* w1_ws(const siren_cfg* cfg, const float* ws) { return ws + ws_base(cfg); }
constexpr float kInv2Pi = 0.159154943091895336f;

// Persistent grid for W1 / STORE (one workgroup per CU): each walks tiles blockIdx.x, + gridDim.x, ... with its
// weight ring streaming across tile boundaries (+1 % on W1, profiles/r01_ab_w1_persist.log). The forward-only
// modes (2 workgroups per CU) measured slower persistent and keep one workgroup per tile.
// SIREN_FLAG_NO_PERSIST: one workgroup per tile (A/B).
// W1 instantiation: the specialised d_out == 1 / ones-cotangent bodies for d_in 2 and 3 at 3 hidden layers
// (image fit, SDF), the general body otherwise
int w1_mode(const siren_cfg* cfg, const float* gy) {
    if (cfg->n_hidden == 3 && cfg->d_out == 1 && gy == nullptr && (cfg->d_in == 2 || cfg->d_in == 3))
        return siren::MODE_W1 | siren::MODE_O1S | siren::MODE_D(cfg->d_in);
    return siren::MODE_W1;
}

int cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (cus[dev] == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cus[dev] = v;
    }
    return cus[dev];
}

dim3 tile_grid(const siren_cfg* cfg, int64_t tiles, int per_cu) {
    if ((cfg->reserved & SIREN_FLAG_NO_PERSIST) != 0) return dim3((unsigned)tiles);
    const int64_t g = (int64_t)cu_count() * per_cu;
    return dim3((unsigned)(tiles < g ? tiles : g));
}

int64_t param_count(const siren_cfg* cfg) {
    const int64_t H = cfg->hidden;
    return H * cfg->d_in + H + (int64_t)cfg->n_hidden * (H * H + H) + (int64_t)cfg->d_out * H + cfg->d_out;
}

// Split-K factor of the weight-gradient kernel: its grid is (S, L, (H/256)^2) workgroups at one per CU, so S is
// chosen to fill whole rounds of the 256 CUs (a grid of 257 would run a second round for one workgroup).
// Round 3 A/B (profiles/r03g_wgrad_rounds.log): one round of ~256 workgroups beats two rounds of ~512 by 2 % on the
// image-fit step and 0.5 % on the Poisson / video steps (half the per-workgroup prologue / slab epilogue and slabs to
// reduce); grouped launches over batched weights keep two rounds (their per-element splits are few already).
int64_t wgrad_splits(const siren_cfg* cfg, int64_t target = 256) {
    const int64_t per_split = (int64_t)cfg->n_hidden * (cfg->hidden / 256) * (cfg->hidden / 256);
    const int64_t s = target / per_split;
    return s > 0 ? s : 1;
}

// Grouped launches (grid (S, L, batch)): about two rounds of workgroups, rounded up to whole rounds of the 256 CUs where
// a split count within 2x of that gives one (32 elements x 3 layers: 5 splits = 480 workgroups ran 1.9 rounds, the
// last one 88 % idle; 8 splits = 768 = 3 full rounds). SIREN_WGRAD_GROUPED_SPLITS overrides (A/B).
int64_t grouped_wgrad_splits(const siren_cfg* cfg, int64_t batch) {
    const int64_t want = std::max<int64_t>(1, wgrad_splits(cfg, 512) / batch);
    if (const char* e = getenv("SIREN_WGRAD_GROUPED_SPLITS")) {
        const long v = atol(e);
        if (v > 0) return v;
    }
    const int64_t per = (int64_t)cfg->n_hidden * (cfg->hidden / 256) * (cfg->hidden / 256) * batch;
    for (int64_t s = want; s <= 2 * want; ++s)
        if ((s * per) % 256 == 0) return s;
    return want;
}

// Edge-layer split (edge_kernel): the first / output layers' gradients reduce the coordinate tiles over their own,
// finer split into compact slabs [W0 | b0 | Wout | bout] (E floats each), about two CU rounds of workgroups over
// (split, 256-neuron block, element); edge_reduce_kernel sums them into the parameter order. (Tied to the wgrad
// split, hidden 512 ran 42 workgroups at 1.6 TB/s.)
struct EdgeSplit {
    int64_t splits, tps, E, floats;
    EdgeSplit(const siren_cfg* cfg, int64_t ntiles, int64_t batch = 1) {
        const int64_t hb = std::max(1, cfg->hidden / 256);
        const int64_t want = std::max<int64_t>(1, 512 / hb / std::max<int64_t>(1, batch));
        splits = std::max<int64_t>(1, std::min(ntiles, want));
        tps = std::max<int64_t>(1, (ntiles + splits - 1) / splits);
        splits = std::max<int64_t>(1, (ntiles + tps - 1) / tps);
        const siren::ParamOffsets off(cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden);
        E = off.hidden0 + (int64_t)cfg->d_out * (cfg->hidden + 1);
        floats = splits * E;
    }
    dim3 grid(const siren_cfg* cfg, int64_t batch = 1) const {
        return dim3((unsigned)splits, (unsigned)std::max(1, cfg->hidden / 256), (unsigned)batch);
    }
};

// W2 backward workspace: sin activations and deltas of every sine layer in 16-coordinate tiles, S
// param-shaped partial slabs of the split-K weight-gradient reduction (+ the edge slabs) and, for hidden 512, the cos
// scratch of the wide kernel (layers 0..L-1).
struct TrainPlan {
    int64_t n_pad, tiles, splits, tps, act_floats, partial_floats, spill_floats, total;
    int64_t eslab_off;  // edge slabs at partial + eslab_off
    EdgeSplit es;
    // batch > 1: a grouped W2 over that many elements shares the CU rounds (fewer splits per element, so the
    // per-split slabs stay a small fraction of the traffic)
    TrainPlan(const siren_cfg* cfg, int64_t n, int64_t batch = 1, int64_t slab_sets = 1)
        : es(cfg, (n + siren::TILE - 1) / siren::TILE * siren::TILE / 16, batch) {
        n_pad = (n + siren::TILE - 1) / siren::TILE * siren::TILE;
        tiles = n_pad / 16;
        const int64_t want = batch > 1 ? grouped_wgrad_splits(cfg, batch) : wgrad_splits(cfg);
        splits = tiles < want ? tiles : want;
        if (splits < 1) splits = 1;
        tps = std::max<int64_t>(1, (tiles + splits - 1) / splits);  // n == 0: no tiles, one empty split
        splits = std::max<int64_t>(1, (tiles + tps - 1) / tps);
        if (splits < 1) splits = 1;
        act_floats = (int64_t)(cfg->n_hidden + 1) * n_pad * cfg->hidden;
        eslab_off = slab_sets * splits * param_count(cfg);
        partial_floats = eslab_off + es.floats;
        spill_floats = wide(cfg) ? (int64_t)cfg->n_hidden * n_pad * cfg->hidden : 0;
        total = 2 * act_floats + partial_floats + spill_floats;
    }
};
// hidden layers: the split-K slabs (S, + S2 for W3's second set); edge layers: the compact edge slabs
int finish_grads(const siren_cfg* cfg, hipStream_t st, const float* partial, int64_t S, int64_t S2, const float* eslab,
                 const EdgeSplit& es, float* gparams, const char* what, int64_t batch = 1, int64_t bpart = 0) {
    const siren::ParamOffsets off(cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden);
    const int64_t P = param_count(cfg);
    const int64_t cap = batch > 1 ? 1024 : 4096;
    const int64_t rblocks = std::max<int64_t>(1, std::min<int64_t>((off.wout - off.hidden0 + 255) / 256, cap));
    siren::launch_reduce(dim3((unsigned)rblocks, (unsigned)batch), st, partial, S, P, gparams, S2, off.hidden0,
                         off.wout, bpart, off.hidden0, off.wout);
    const int64_t eblocks = std::max<int64_t>(1, (es.E + 15) / 16);  // 16 columns per workgroup
    siren::launch_edge_reduce(dim3((unsigned)eblocks, (unsigned)batch), st, eslab, es.splits, es.E, off.hidden0,
                              off.wout, gparams, P, bpart);
    return hip_status(what);
}
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
    if (layered(cfg)) {  // ws = [parameters as they are][W_l^T] and nothing else (immutable since ABI 5: the chunk
                          // scratch is every layered entry point's caller-owned tws, layered_ws_floats)
        siren::layered_pack(siren::LayeredPlan(cfg->d_in, cfg->hidden, cfg->n_hidden, cfg->d_out, -1), params, ws,
                            (hipStream_t)stream);
        return hip_status("siren_pack");
    }
    siren::launch_pack(params, ws, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden, small_pad(cfg), ws_floats(cfg),
                       wide(cfg) ? 0 : ws_base(cfg), cfg->omega_first * kInv2Pi, cfg->omega_hidden * kInv2Pi,
                       (hipStream_t)stream);
    return hip_status("siren_pack");
}

int32_t siren_forward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    *count = layered(cfg) ? layered_scratch(cfg, n, false) : 0;
    return SIREN_OK;
}

int32_t siren_forward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, void* stream) {
    return siren_forward_ex(cfg, ws, x, n, y, nullptr, stream);
}

int32_t siren_forward_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, float* tws,
                         void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || y == nullptr) return fail(SIREN_EINVAL, "ws/x/y is NULL");
    const int64_t blocks = (n + siren::TILE - 1) / siren::TILE;
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    const dim3 grid((unsigned)blocks);
    if (layered(cfg)) return layered_call(siren::LAY_FWD | siren::LAY_Y, cfg, ws, x, n, nullptr, y, nullptr, nullptr,
                                          nullptr, tws, stream, "siren_forward");
    siren::FusedArgs fa{ws, x, n, nullptr, y, nullptr, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first,
                        cfg->omega_hidden, cfg->outermost_linear ? 0 : 1, nullptr, nullptr, 0};
    if (wide(cfg))
        siren::launch_wide(siren::MODE_FWD, grid, (hipStream_t)stream, fa, nullptr);
    else if (cfg->outermost_linear && cfg->n_hidden <= 5 && (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0 &&
             w1_ok(cfg)) {
        fa.ws = w1_ws(cfg, ws);
        siren::launch_w0(grid, (hipStream_t)stream, fa);  // 2 WGs/CU: persistence measured slower
    } else
        siren::launch_legacy_fwd(grid, (hipStream_t)stream, fa);
    return hip_status("siren_forward");
}

// hidden 512: the cos(w z_l) scratch of layers 0..L-1 (lane-major, n padded to whole tiles); hidden 256 keeps cos in
// registers and needs none
int32_t siren_forward_grad_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    const int64_t n_pad = (n + siren::TILE - 1) / siren::TILE * siren::TILE;
    *count = wide(cfg)      ? (int64_t)cfg->n_hidden * n_pad * cfg->hidden
             : deep(cfg)    ? (int64_t)(cfg->n_hidden + 1) * n_pad * siren::H  // lane-major cos of layers 0..L
             : layered(cfg) ? layered_scratch(cfg, n, false)                   // the layered path's chunk scratch
                            : 0;
    return SIREN_OK;
}

int32_t siren_forward_grad(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy,
                           float* y, float* gx, float* tws, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (cfg->n_hidden > siren::MAX_LH_GRAD && !wide(cfg) && !layered(cfg) && !deep(cfg))
        return fail(SIREN_EUNSUPPORTED, "siren_forward_grad needs 1 <= num_hidden_layers <= 5 at hidden 256 (linear "
                                        "output, nonzero omegas beyond 3)");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || gx == nullptr) return fail(SIREN_EINVAL, "ws/x/gx is NULL");
    if (deep(cfg)) {
        // forward half (y + the lane-major cos of every layer into tws; no a_l tiles), then the reverse GEMMs from
        // that cos with the output cotangent gy (no delta tiles)
        if (tws == nullptr)
            return fail(SIREN_EINVAL, "siren_forward_grad at 4..5 hidden layers needs tws (siren_forward_grad_ws_floats)");
        const int64_t blocks = (n + siren::TILE - 1) / siren::TILE;
        if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
        const int64_t n_pad = blocks * siren::TILE;
        siren::FusedArgs ff{w1_ws(cfg, ws), x, n, nullptr, y, nullptr, cfg->d_in, cfg->d_out, cfg->n_hidden,
                            cfg->omega_first, cfg->omega_hidden, 0, nullptr, tws, n_pad};
        siren::launch_w0s(dim3((unsigned)blocks), (hipStream_t)stream, ff);
        siren::FusedArgs fr{w1_ws(cfg, ws), x, n, gy, nullptr, gx, cfg->d_in, cfg->d_out, cfg->n_hidden,
                            cfg->omega_first, cfg->omega_hidden, 0, tws, nullptr, n_pad};
        siren::launch_w1(siren::MODE_REV, tile_grid(cfg, blocks, 1), (hipStream_t)stream, fr);
        return hip_status("siren_forward_grad (4..5 hidden layers)");
    }
    if (layered(cfg))
        return layered_call(siren::LAY_FWD | siren::LAY_Y | siren::LAY_GX, cfg, ws, x, n, gy, y, gx, nullptr, nullptr,
                            tws, stream, "siren_forward_grad");
    const int64_t blocks = (n + siren::TILE - 1) / siren::TILE;
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    const dim3 grid((unsigned)blocks);
    const int fs = cfg->outermost_linear ? 0 : 1;
    siren::FusedArgs fa{ws, x, n, gy, y, gx, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first,
                        cfg->omega_hidden, fs, nullptr, nullptr, 0};
    if (wide(cfg)) {
        // cos scratch of layers 0..L-1 in the caller's workspace (siren_forward_grad_ws_floats)
        if (tws == nullptr) return fail(SIREN_EINVAL, "siren_forward_grad at hidden 512 needs tws (siren_forward_grad_ws_floats)");
        fa.n_pad = blocks * siren::TILE;  // per-layer scratch stride
        siren::launch_wide(siren::MODE_W1, grid, (hipStream_t)stream, fa, tws);
    } else if ((cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) != 0 || fs || !w1_ok(cfg)) {
        siren::launch_legacy_grad(false, grid, (hipStream_t)stream, fa);
    } else {
        fa.ws = w1_ws(cfg, ws);
        siren::launch_w1(w1_mode(cfg, gy), tile_grid(cfg, blocks, 1), (hipStream_t)stream, fa);
    }
    return hip_status("siren_forward_grad");
}

// ---- split-bf16 W1 (w1x_kernel.hpp): workspace [unscaled small block | phase-scaled small block | bf16 stream] ----
static int split_ok(const siren_cfg* cfg) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (cfg->hidden != siren::H || cfg->n_hidden != 3 || cfg->d_out != 1 || (cfg->d_in != 2 && cfg->d_in != 3) ||
        !cfg->outermost_linear || cfg->omega_first == 0.f || cfg->omega_hidden == 0.f)
        return fail(SIREN_EUNSUPPORTED, "the split-bf16 W1 covers hidden 256, 3 hidden layers, in_features 2 / 3, "
                                        "out_features 1, linear output, nonzero omegas");
    return SIREN_OK;
}

int32_t siren_split_ws_floats(const siren_cfg* cfg, int64_t* count) {
    if (int rc = split_ok(cfg)) return rc;
    if (count == nullptr) return fail(SIREN_EINVAL, "count is NULL");
    *count = 2 * small_pad(cfg) + siren::split_stream_words(cfg->n_hidden);
    return SIREN_OK;
}

int32_t siren_pack_split(const siren_cfg* cfg, const float* params, float* wsx, void* stream) {
    if (int rc = split_ok(cfg)) return rc;
    if (params == nullptr || wsx == nullptr) return fail(SIREN_EINVAL, "params/wsx is NULL");
    const int64_t spad = small_pad(cfg);
    // small blocks: pack_kernel over [0, 2 spad) with the scaled copy starting at spad (the stream part is empty)
    siren::launch_pack(params, wsx, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden, spad, 2 * spad, spad,
                       cfg->omega_first * kInv2Pi, cfg->omega_hidden * kInv2Pi, (hipStream_t)stream);
    siren::launch_pack_split(params, (unsigned*)(wsx + 2 * spad), cfg->d_in, cfg->d_out, cfg->n_hidden,
                             cfg->omega_hidden * kInv2Pi, (hipStream_t)stream);
    return hip_status("siren_pack_split");
}

int32_t siren_forward_grad_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, float* y,
                                 float* gx, void* stream) {
    if (int rc = split_ok(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (wsx == nullptr || x == nullptr || gx == nullptr) return fail(SIREN_EINVAL, "wsx/x/gx is NULL");
    const int64_t blocks = (n + siren::TILE - 1) / siren::TILE;
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    const int64_t spad = small_pad(cfg);
    siren::launch_w1x(tile_grid(cfg, blocks, 1), (hipStream_t)stream, wsx + spad, (const unsigned*)(wsx + 2 * spad), x,
                      n, y, gx, cfg->d_in, cfg->omega_first, cfg->omega_hidden);
    return hip_status("siren_forward_grad_split");
}

int32_t siren_forward_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, float* y, void* stream) {
    if (int rc = split_ok(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (wsx == nullptr || x == nullptr || y == nullptr) return fail(SIREN_EINVAL, "wsx/x/y is NULL");
    const int64_t tile = siren::split_fwd_tile();
    const int64_t blocks = (n + tile - 1) / tile;
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    const int64_t spad = small_pad(cfg);
    siren::launch_w0x(tile_grid(cfg, blocks, 1), (hipStream_t)stream, wsx + spad, (const unsigned*)(wsx + 2 * spad), x,
                      n, y, cfg->d_in, cfg->omega_first, cfg->omega_hidden);
    return hip_status("siren_forward_split");
}

int32_t siren_backward_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, const float* gy,
                             float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = split_ok(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (gparams == nullptr) return fail(SIREN_EINVAL, "gparams is NULL");
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {  // empty tensors may carry NULL data pointers: only gparams is written
        (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_backward_split");
    }
    if (wsx == nullptr || x == nullptr || gy == nullptr || tws == nullptr) return fail(SIREN_EINVAL, "wsx/x/gy/tws is NULL");
    const TrainPlan plan(cfg, n);
    if (plan.n_pad / siren::TILE > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    float* abuf = tws;
    float* dbuf = tws + plan.act_floats;
    float* partial = tws + 2 * plan.act_floats;
    const int64_t spad = small_pad(cfg);
    siren::launch_w1x_store(tile_grid(cfg, plan.n_pad / siren::TILE, 1), st, wsx + spad,
                            (const unsigned*)(wsx + 2 * spad), x, n, gy, nullptr, gx, abuf, dbuf, plan.n_pad,
                            cfg->d_in, cfg->omega_first, cfg->omega_hidden);
    if (int rc = hip_status("siren_backward_split (split store)")) return rc;
    // the bf16 wgrad takes whole tile pairs: tps rounded up to even (fewer splits, within the planned slabs)
    const int64_t tpx = plan.tps + (plan.tps & 1), sx = (plan.tiles + tpx - 1) / tpx;
    siren::launch_wgradx(dim3((unsigned)sx, (unsigned)cfg->n_hidden), st, abuf, dbuf, plan.n_pad, tpx, partial, P,
                         cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_backward_split (wgrad)")) return rc;
    siren::launch_small(plan.es.grid(cfg), st, abuf, dbuf, x, gy, n, plan.n_pad, plan.es.tps, partial + plan.eslab_off,
                        plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden);
    if (int rc = hip_status("siren_backward_split (small)")) return rc;
    return finish_grads(cfg, st, partial, sx, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_backward_split (reduce)");
}

// ---- the stored split of the bf16x6 W2 unit: the forward keeps a_l tiles and cos(w z_l), the backward is reverse-only ----
// workspace: [a_l tiles][delta_l tiles][partial slabs][lane-major cos, L + 1 layers], on n rounded up to 128 (the
// split forward's tile)
static int64_t split_n(int64_t n) { return (std::max<int64_t>(n, 1) + 127) / 128 * 128; }

int32_t siren_train_split_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = split_ok(cfg)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    const TrainPlan plan(cfg, split_n(n));
    *count = plan.total + (int64_t)(cfg->n_hidden + 1) * plan.n_pad * cfg->hidden;
    return SIREN_OK;
}

int32_t siren_forward_store_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, float* y,
                                  float* tws, void* stream) {
    if (int rc = split_ok(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (wsx == nullptr || x == nullptr || tws == nullptr) return fail(SIREN_EINVAL, "wsx/x/tws is NULL");
    const TrainPlan plan(cfg, split_n(n));
    if (plan.n_pad / 128 > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    const int64_t spad = small_pad(cfg);
    siren::launch_w0xs(tile_grid(cfg, plan.n_pad / 128, 1), (hipStream_t)stream, wsx + spad,
                       (const unsigned*)(wsx + 2 * spad), x, n, y, tws, tws + plan.total, plan.n_pad, cfg->d_in,
                       cfg->omega_first, cfg->omega_hidden);
    return hip_status("siren_forward_store_split");
}

int32_t siren_backward_stored_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, const float* gy,
                                    float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = split_ok(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (gparams == nullptr) return fail(SIREN_EINVAL, "gparams is NULL");
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {  // empty tensors may carry NULL data pointers: only gparams is written
        (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_backward_stored_split");
    }
    if (wsx == nullptr || x == nullptr || gy == nullptr || tws == nullptr) return fail(SIREN_EINVAL, "wsx/x/gy/tws is NULL");
    const TrainPlan plan(cfg, split_n(n));
    float* abuf = tws;
    float* dbuf = tws + plan.act_floats;
    float* partial = tws + 2 * plan.act_floats;
    const int64_t spad = small_pad(cfg);
    siren::launch_w1xr(tile_grid(cfg, plan.n_pad / siren::split_rev_tile(), 1), st, wsx + spad, (const unsigned*)(wsx + 2 * spad),
                       x, n, gy, gx, tws + plan.total, dbuf, plan.n_pad, cfg->d_in, cfg->omega_first,
                       cfg->omega_hidden);
    if (int rc = hip_status("siren_backward_stored_split (split reverse)")) return rc;
    const int64_t tpx = plan.tps + (plan.tps & 1), sx = (plan.tiles + tpx - 1) / tpx;
    siren::launch_wgradx(dim3((unsigned)sx, (unsigned)cfg->n_hidden), st, abuf, dbuf, plan.n_pad, tpx, partial, P,
                         cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_backward_stored_split (wgrad)")) return rc;
    siren::launch_small(plan.es.grid(cfg), st, abuf, dbuf, x, gy, n, plan.n_pad, plan.es.tps, partial + plan.eslab_off,
                        plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden);
    if (int rc = hip_status("siren_backward_stored_split (small)")) return rc;
    return finish_grads(cfg, st, partial, sx, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_backward_stored_split (reduce)");
}

// diagnostics: while set, W3 launches record s_memtime phase stamps (w3_kernel.hpp) into stamps[256][16]
static unsigned long long* g_w3_prof = nullptr;
int32_t siren_w3_phase_profile(uint64_t* stamps) {
    g_w3_prof = (unsigned long long*)stamps;
    return SIREN_OK;
}

int32_t siren_w1_phase_profile(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, float* gx,
                               uint64_t* stamps, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (cfg->n_hidden != 3 || !w1_ok(cfg) || !cfg->outermost_linear)
        return fail(SIREN_EUNSUPPORTED, "siren_w1_phase_profile covers the hidden-256, 3-hidden-layer W1 kernel");
    if (ws == nullptr || x == nullptr || y == nullptr || gx == nullptr || stamps == nullptr || n <= 0)
        return fail(SIREN_EINVAL, "NULL pointer or n <= 0");
    const int64_t blocks = (n + siren::TILE - 1) / siren::TILE;
    siren::FusedArgs fa{w1_ws(cfg, ws), x, n, nullptr, y, gx, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first,
                        cfg->omega_hidden, 0, (float*)stamps, nullptr, blocks * siren::TILE};
    siren::launch_w1(w1_mode(cfg, nullptr) | siren::MODE_PROF, tile_grid(cfg, blocks, 1), (hipStream_t)stream, fa);
    return hip_status("siren_w1_phase_profile");
}

int32_t siren_forward_laplace(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, float* gx,
                              float* lap, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!w1_ok(cfg) || cfg->d_in > 2 || !cfg->outermost_linear || cfg->n_hidden > 5)
        return fail(SIREN_EUNSUPPORTED, "siren_forward_laplace covers hidden 256, in_features <= 2, linear output, "
                                        "1..5 hidden layers, nonzero omegas");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || lap == nullptr) return fail(SIREN_EINVAL, "ws/x/lap is NULL");
    const int64_t blocks = (n + 15) / 16;  // 4 coordinates x 4 jet streams per wave
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    siren::launch_w4(dim3((unsigned)blocks), (hipStream_t)stream, w1_ws(cfg, ws), x, n, y, gx, lap, cfg->d_in, cfg->d_out,
                     cfg->n_hidden, cfg->omega_first, cfg->omega_hidden);
    return hip_status("siren_forward_laplace");
}

int32_t siren_train_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    if (layered(cfg)) {
        *count = layered_scratch(cfg, n, false);  // the layered path's chunk scratch
    } else {
        const TrainPlan plan(cfg, n);
        *count = plan.total + (deep(cfg) ? plan.act_floats : 0);  // deep: + the stored split's lane-major cos
    }
    return SIREN_OK;
}

int32_t siren_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy,
                       float* tws, void* reserved, float* gx, float* gparams, void* stream) {
    (void)reserved;
    if (int rc = check_cfg(cfg, true)) return rc;
    if (cfg->n_hidden > siren::MAX_LH_GRAD && !wide(cfg) && !layered(cfg) && !deep(cfg))
        return fail(SIREN_EUNSUPPORTED, "siren_backward needs 1 <= num_hidden_layers <= 5 at hidden 256 (linear "
                                        "output, nonzero omegas beyond 3)");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (deep(cfg)) {  // the stored split in one call: forward half into tws, then the reverse-only backward
        if (n == 0) {  // empty tensors may carry NULL data pointers: only gparams is written
            if (gparams == nullptr) return fail(SIREN_EINVAL, "gparams is NULL");
            (void)hipMemsetAsync(gparams, 0, param_count(cfg) * sizeof(float), (hipStream_t)stream);
            return hip_status("siren_backward");
        }
        if (int rc = siren_forward_store(cfg, ws, x, n, nullptr, tws, stream)) return rc;
        return siren_backward_stored(cfg, ws, x, n, gy, tws, gx, gparams, stream);
    }
    if (layered(cfg)) {  // tws is the chunk scratch
        if (n == 0) {  // empty tensors may carry NULL data pointers: only gparams is written
            if (gparams == nullptr) return fail(SIREN_EINVAL, "gparams is NULL");
            (void)hipMemsetAsync(gparams, 0, param_count(cfg) * sizeof(float), (hipStream_t)stream);
            return hip_status("siren_backward");
        }
        if (ws == nullptr || x == nullptr || gy == nullptr || gx == nullptr || gparams == nullptr)
            return fail(SIREN_EINVAL, "ws/x/gy/gx/gparams is NULL");
        return layered_call(siren::LAY_FWD | siren::LAY_GX | siren::LAY_THETA, cfg, ws, x, n, gy, nullptr, gx,
                            gparams, nullptr, tws, stream, "siren_backward");
    }
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
    float* spill = partial + plan.partial_floats;
    const dim3 grid((unsigned)(plan.n_pad / siren::TILE)), block(siren::THREADS);
    const int fs = cfg->outermost_linear ? 0 : 1;
    siren::FusedArgs fa{ws, x, n, gy, nullptr, gx, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first,
                        cfg->omega_hidden, fs, abuf, dbuf, plan.n_pad};
    if (wide(cfg))
        siren::launch_wide(siren::MODE_STORE, grid, st, fa, spill);
    else if ((cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0 && !fs && w1_ok(cfg)) {
        fa.ws = w1_ws(cfg, ws);
        siren::launch_w1(siren::MODE_STORE, tile_grid(cfg, plan.n_pad / siren::TILE, 1), st, fa);
    } else
        siren::launch_legacy_grad(true, grid, st, fa);
    if (int rc = hip_status("siren_backward (fused store)")) return rc;
    const unsigned quads = (unsigned)((cfg->hidden / 256) * (cfg->hidden / 256));
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden, quads), st, abuf, dbuf, plan.n_pad,
                        plan.tps, partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, cfg->hidden);
    if (int rc = hip_status("siren_backward (wgrad)")) return rc;
    siren::launch_small(plan.es.grid(cfg), st, abuf, dbuf, x, gy, n, plan.n_pad, plan.es.tps, partial + plan.eslab_off,
                        plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden);
    if (int rc = hip_status("siren_backward (small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_backward (reduce)");
}

// ---- stored-forward W2 split: the training forward keeps a_l and cos(w z_l) so the backward is reverse-only ----
bool stored_ok(const siren_cfg* cfg) {
    if (!cfg->outermost_linear || (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) != 0) return false;
    return wide(cfg) || layered(cfg) || (w1_ok(cfg) && cfg->n_hidden <= siren::MAX_LH_DEEP);
}
// stored-split workspace: [a_l tiles][delta_l tiles][partial slabs][hidden 512: cos scratch of L + 1 layers]
// [hidden 256: lane-major cos of L + 1 layers]; layered path: [a_0..a_L][cos_0..cos_L], n x H rows each
float* stored_cos(const siren_cfg* cfg, const TrainPlan& plan, float* tws) {
    return wide(cfg) ? tws + 2 * plan.act_floats + plan.partial_floats : tws + plan.total;
}

int32_t siren_train_stored_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!stored_ok(cfg))
        return fail(SIREN_EUNSUPPORTED, "the stored-forward W2 split needs a linear output layer (hidden 256: 1..5 "
                                        "hidden layers)");
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    if (layered(cfg)) {  // [a_0..a_L][cos_0..cos_L] n-row buffers, then the chunk scratch
        *count = siren::layered_stored_floats(cfg->hidden, cfg->n_hidden, n) + layered_scratch(cfg, n, true);
        return SIREN_OK;
    }
    const TrainPlan plan(cfg, n);
    // hidden 256: + the lane-major cos buffer (L + 1 layers, the size of the a_l tiles); hidden 512: the cos
    // scratch grows from L to L + 1 layers
    *count = plan.total + (wide(cfg) ? plan.n_pad * cfg->hidden : plan.act_floats);
    return SIREN_OK;
}

int32_t siren_forward_store(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, float* tws,
                            void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!stored_ok(cfg))
        return fail(SIREN_EUNSUPPORTED, "the stored-forward W2 split covers hidden 256, linear output, 1..5 hidden layers");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    // y may be NULL (siren_backward's internal forward half at 4..5 hidden layers needs no output)
    if (ws == nullptr || x == nullptr || tws == nullptr || (y == nullptr && (wide(cfg) || layered(cfg))))
        return fail(SIREN_EINVAL, "ws/x/y/tws is NULL");
    if (layered(cfg))
        return layered_call(siren::LAY_FWD | siren::LAY_Y | siren::LAY_TWS, cfg, ws, x, n, nullptr, y, nullptr,
                            nullptr, tws, tws + siren::layered_stored_floats(cfg->hidden, cfg->n_hidden, n), stream,
                            "siren_forward_store");
    const TrainPlan plan(cfg, n);
    float* abuf = tws;
    float* cbuf = stored_cos(cfg, plan, tws);
    const dim3 grid((unsigned)(plan.n_pad / siren::TILE));
    if (wide(cfg)) {
        siren::FusedArgs fa{ws, x, n, nullptr, y, nullptr, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first,
                            cfg->omega_hidden, 0, abuf, nullptr, plan.n_pad};
        if ((cfg->reserved & SIREN_FLAG_WIDE_SERIAL) != 0 ||
            !siren::launch_widei(siren::MODE_FWDS, grid, (hipStream_t)stream, fa, cbuf))
            siren::launch_wide(siren::MODE_FWDS, grid, (hipStream_t)stream, fa, cbuf);
        return hip_status("siren_forward_store");
    }
    siren::FusedArgs fa{w1_ws(cfg, ws), x, n, nullptr, y, nullptr, cfg->d_in, cfg->d_out, cfg->n_hidden,
                        cfg->omega_first, cfg->omega_hidden, 0, abuf, cbuf, plan.n_pad};
    siren::launch_w0s(grid, (hipStream_t)stream, fa);
    return hip_status("siren_forward_store");
}

int32_t siren_backward_stored(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy,
                              float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!stored_ok(cfg))
        return fail(SIREN_EUNSUPPORTED, "the stored-forward W2 split covers hidden 256, linear output, 1..5 hidden layers");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0 && layered(cfg)) {  // empty tensors may carry NULL data pointers: only gparams is written
        if (gparams == nullptr) return fail(SIREN_EINVAL, "gparams is NULL");
        (void)hipMemsetAsync(gparams, 0, param_count(cfg) * sizeof(float), (hipStream_t)stream);
        return hip_status("siren_backward_stored");
    }
    if (ws == nullptr || gy == nullptr || tws == nullptr || gx == nullptr || gparams == nullptr ||
        (n > 0 && x == nullptr))
        return fail(SIREN_EINVAL, "ws/x/gy/tws/gx/gparams is NULL");
    if (layered(cfg))
        return layered_call(siren::LAY_GX | siren::LAY_THETA | siren::LAY_TWS, cfg, ws, x, n, gy, nullptr, gx, gparams,
                            tws, tws + siren::layered_stored_floats(cfg->hidden, cfg->n_hidden, n), stream,
                            "siren_backward_stored");
    const TrainPlan plan(cfg, n);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {
        (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_backward_stored");
    }
    float* abuf = tws;
    float* dbuf = tws + plan.act_floats;
    float* partial = tws + 2 * plan.act_floats;
    float* cbuf = stored_cos(cfg, plan, tws);
    if (wide(cfg)) {
        siren::FusedArgs fa{ws, x, n, gy, nullptr, gx, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first,
                            cfg->omega_hidden, 0, nullptr, dbuf, plan.n_pad};
        const dim3 rgrid((unsigned)(plan.n_pad / siren::TILE));
        if ((cfg->reserved & SIREN_FLAG_WIDE_SERIAL) != 0 || !siren::launch_widei(siren::MODE_REV, rgrid, st, fa, cbuf))
            siren::launch_wide(siren::MODE_REV, rgrid, st, fa, cbuf);
    } else {
        siren::FusedArgs fa{w1_ws(cfg, ws), x, n, gy, nullptr, gx, cfg->d_in, cfg->d_out, cfg->n_hidden,
                            cfg->omega_first, cfg->omega_hidden, 0, cbuf, dbuf, plan.n_pad};
        siren::launch_w1(siren::MODE_REV, tile_grid(cfg, plan.n_pad / siren::TILE, 1), st, fa);
    }
    if (int rc = hip_status("siren_backward_stored (reverse)")) return rc;
    const unsigned quads = (unsigned)((cfg->hidden / 256) * (cfg->hidden / 256));
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden, quads), st, abuf, dbuf, plan.n_pad,
                        plan.tps, partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, cfg->hidden);
    if (int rc = hip_status("siren_backward_stored (wgrad)")) return rc;
    siren::launch_small(plan.es.grid(cfg), st, abuf, dbuf, x, gy, n, plan.n_pad, plan.es.tps, partial + plan.eslab_off,
                        plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden);
    if (int rc = hip_status("siren_backward_stored (small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_backward_stored (reduce)");
}

// ---- W4s: backward of the fused Laplacian (laplace_mse training) ------------------------------------------
namespace {
// the Laplacian's jet kernels (W4s) run on the phase-scaled image whenever it exists (jet_kernel.hpp PH: sincos in
// revolutions, 3 VALU fewer per element of the forward jet); zero omegas keep the unscaled image
const float* jet_ws(const siren_cfg* cfg, const float* ws) { return w1_ok(cfg) ? w1_ws(cfg, ws) : ws; }

int check_jet(const siren_cfg* cfg) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (wide(cfg) || layered(cfg) || cfg->d_in > 2 || !cfg->outermost_linear || cfg->n_hidden > 5)
        return fail(SIREN_EUNSUPPORTED,
                    "the fused Laplacian covers hidden 256, in_features <= 2, linear output, 1..5 hidden layers");
    return SIREN_OK;
}

// jet tiles are 16 columns = 4 coordinates x 4 streams: a-jets, zb-jets and z-jets of every layer + S slabs
// q8: the Hessian node's kept backward (qf_kernel.hpp): n_pad a multiple of 32 (8 coordinates per wave), the edge
// kernel's tiles are Q8 tile pairs (8 coordinates); otherwise W4 jet tiles of 4 coordinates, n_pad a multiple of 16
struct JetPlan {
    int64_t n_pad, cols, tiles, splits, tps, buf_floats, partial_floats, total, eslab_off;
    EdgeSplit es;
    static int64_t pad(int64_t n, bool q8) { return q8 ? (n + 31) / 32 * 32 : (n + 15) / 16 * 16; }
    JetPlan(const siren_cfg* cfg, int64_t n, bool q8 = false) : es(cfg, pad(n, q8) / (q8 ? 8 : 4)) {
        n_pad = pad(n, q8);
        cols = 4 * n_pad;
        tiles = cols / 16;
        const int64_t want = wgrad_splits(cfg);
        splits = tiles < want ? tiles : want;
        if (splits < 1) splits = 1;
        tps = std::max<int64_t>(1, (tiles + splits - 1) / splits);  // n == 0: no tiles, one empty split
        splits = std::max<int64_t>(1, (tiles + tps - 1) / tps);
        if (splits < 1) splits = 1;
        buf_floats = (int64_t)(cfg->n_hidden + 1) * cols * siren::H;
        eslab_off = splits * param_count(cfg);
        partial_floats = eslab_off + es.floats;
        total = 3 * buf_floats + partial_floats;
    }
};
}  // namespace

int32_t siren_laplace_backward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_jet(cfg)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    *count = JetPlan(cfg, n).total;
    return SIREN_OK;
}

int32_t siren_laplace_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* glap,
                               float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = check_jet(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (ws == nullptr || tws == nullptr || gx == nullptr || gparams == nullptr ||
        (n > 0 && (x == nullptr || glap == nullptr)))
        return fail(SIREN_EINVAL, "ws/x/glap/tws/gx/gparams is NULL");
    const JetPlan plan(cfg, n);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {
        (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_laplace_backward");
    }
    float* abuf = tws;
    float* dbuf = abuf + plan.buf_floats;
    float* spill = dbuf + plan.buf_floats;
    float* partial = spill + plan.buf_floats;
    siren::launch_jet_store(dim3((unsigned)(plan.n_pad / 16)), st, jet_ws(cfg, ws), x, n, glap, gx, cfg->d_in,
                            cfg->d_out, cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, spill, abuf, dbuf,
                            plan.n_pad, w1_ok(cfg));
    if (int rc = hip_status("siren_laplace_backward (jet store)")) return rc;
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden), st, abuf, dbuf, plan.cols, plan.tps,
                        partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, siren::H, 1);
    if (int rc = hip_status("siren_laplace_backward (wgrad)")) return rc;
    siren::launch_small_jet(plan.es.grid(cfg), st, abuf, dbuf, x, glap, n, plan.n_pad, plan.es.tps,
                            partial + plan.eslab_off, plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_laplace_backward (small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_laplace_backward (reduce)");
}

// ---- split W4 / W4s for laplace_mse training: the forward jet keeps its stores, the backward is reverse-only ----
int32_t siren_forward_laplace_store(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y,
                                    float* gx, float* lap, float* tws, void* stream) {
    if (int rc = check_jet(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || lap == nullptr || tws == nullptr) return fail(SIREN_EINVAL, "ws/x/lap/tws is NULL");
    const JetPlan plan(cfg, n);
    float* abuf = tws;
    float* dbuf = abuf + plan.buf_floats;
    float* spill = dbuf + plan.buf_floats;
    if (w1_ok(cfg))  // the W4 kernel with the stores (interleaved epilogues, phase-scaled image)
        siren::launch_w4s(dim3((unsigned)(plan.n_pad / 16)), (hipStream_t)stream, w1_ws(cfg, ws), x, n, y, gx, lap, abuf,
                          spill, plan.n_pad, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first, cfg->omega_hidden);
    else
        siren::launch_jet_phase(1, dim3((unsigned)(plan.n_pad / 16)), (hipStream_t)stream, ws, x, n, nullptr, gx,
                                cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, spill, abuf,
                                dbuf, plan.n_pad, y, lap, false);
    return hip_status("siren_forward_laplace_store");
}

int32_t siren_laplace_backward_stored(const siren_cfg* cfg, const float* ws, const float* x, int64_t n,
                                      const float* glap, float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = check_jet(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (ws == nullptr || tws == nullptr || gx == nullptr || gparams == nullptr ||
        (n > 0 && (x == nullptr || glap == nullptr)))
        return fail(SIREN_EINVAL, "ws/x/glap/tws/gx/gparams is NULL");
    const JetPlan plan(cfg, n);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {
        (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_laplace_backward_stored");
    }
    float* abuf = tws;
    float* dbuf = abuf + plan.buf_floats;
    float* spill = dbuf + plan.buf_floats;
    float* partial = spill + plan.buf_floats;
    siren::launch_jet_phase(2, dim3((unsigned)(plan.n_pad / 16)), st, jet_ws(cfg, ws), x, n, glap, gx, cfg->d_in,
                            cfg->d_out, cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, spill, abuf, dbuf,
                            plan.n_pad, nullptr, nullptr, w1_ok(cfg));
    if (int rc = hip_status("siren_laplace_backward_stored (jet reverse)")) return rc;
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden), st, abuf, dbuf, plan.cols, plan.tps,
                        partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, siren::H, 1);
    if (int rc = hip_status("siren_laplace_backward_stored (wgrad)")) return rc;
    siren::launch_small_jet(plan.es.grid(cfg), st, abuf, dbuf, x, glap, n, plan.n_pad, plan.es.tps,
                            partial + plan.eslab_off, plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_laplace_backward_stored (small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_laplace_backward_stored (reduce)");
}

// hidden 512: the two-stream jet (wide_jet_kernel.hpp): a-, zb- and z-jets of L + 1 layers over 2 n_pad columns
// (n_pad: 32 coordinates per workgroup), the split-K slabs and the edge slabs
namespace {
// ns = 2 (W3: 32 coordinates per workgroup) or 4 (the mixed jet of the third-order adjoint: 16)
struct W3WidePlan {
    int64_t n_pad, cols, tiles, splits, tps, buf_floats, eslab_off, partial_floats, total;
    EdgeSplit es;
    W3WidePlan(const siren_cfg* cfg, int64_t n, int ns = 2)
        : es(cfg, (n + 64 / ns - 1) / (64 / ns) * (64 / ns) * ns / 16) {
        n_pad = (n + 64 / ns - 1) / (64 / ns) * (64 / ns);
        cols = ns * n_pad;
        tiles = cols / 16;
        const int64_t want = wgrad_splits(cfg);
        splits = std::max<int64_t>(1, std::min(tiles, want));
        tps = std::max<int64_t>(1, (tiles + splits - 1) / splits);
        splits = std::max<int64_t>(1, (tiles + tps - 1) / tps);
        buf_floats = (int64_t)(cfg->n_hidden + 1) * cols * cfg->hidden;
        eslab_off = splits * param_count(cfg);
        partial_floats = eslab_off + es.floats;
        total = 3 * buf_floats + partial_floats;
    }
};
}  // namespace

// ---- third-order adjoint: the backward of a Hessian-vector-product node (jet_kernel.hpp MIX) -----------------
namespace {
int check_mix(const siren_cfg* cfg) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (layered(cfg)) return layered_unsupported("siren_hvp_backward");
    if (!cfg->outermost_linear || (!wide(cfg) && cfg->n_hidden > 5))
        return fail(SIREN_EUNSUPPORTED, "siren_hvp_backward covers a linear output layer (hidden 256: 1..5 hidden layers)");
    return SIREN_OK;
}
}  // namespace

int32_t siren_hvp_backward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_mix(cfg)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    *count = wide(cfg) ? W3WidePlan(cfg, n, 4).total : JetPlan(cfg, n).total;
    return SIREN_OK;
}

// hidden 512: the four-stream mixed jet of wide_jet_kernel<4> (16 coordinates per workgroup), wgrad over 4 n_pad
// columns (value-column bias), EDGE_MIX at h = 512
static int32_t hvp_backward_wide(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                                 const float* u, const float* g, float* tws, float* gx, float* gparams, float* gv,
                                 float* gu, void* stream) {
    const W3WidePlan plan(cfg, n, 4);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    float* abuf = tws;
    float* dbuf = abuf + plan.buf_floats;
    float* spill = dbuf + plan.buf_floats;
    float* partial = spill + plan.buf_floats;
    siren::launch_wide_mix(dim3((unsigned)(plan.n_pad / 16)), st, ws, x, v, g, u, n, cfg->d_in, cfg->d_out,
                           cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, gx, gv, gu, spill, abuf, dbuf, plan.n_pad);
    if (int rc = hip_status("siren_hvp_backward (hidden 512 mixed jet)")) return rc;
    if (gparams == nullptr) return SIREN_OK;
    const unsigned quads = (unsigned)((cfg->hidden / 256) * (cfg->hidden / 256));
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden, quads), st, abuf, dbuf, plan.cols,
                        plan.tps, partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, cfg->hidden, 1);
    if (int rc = hip_status("siren_hvp_backward (hidden 512 wgrad)")) return rc;
    siren::launch_small_mix(plan.es.grid(cfg), st, abuf, dbuf, x, v, g, u, n, plan.n_pad, plan.es.tps,
                            partial + plan.eslab_off, plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden);
    if (int rc = hip_status("siren_hvp_backward (hidden 512 small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_hvp_backward (hidden 512 reduce)");
}

int32_t siren_hvp_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                           const float* u, const float* g, float* tws, float* gx, float* gparams, float* gv,
                           float* gu, void* stream) {
    if (int rc = check_mix(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    const JetPlan plan(cfg, n);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {  // empty batch: zero parameter gradient, nothing else to write (buffers may be empty / NULL)
        if (gparams != nullptr) (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_hvp_backward");
    }
    if (ws == nullptr || tws == nullptr || gx == nullptr || x == nullptr || v == nullptr || g == nullptr)
        return fail(SIREN_EINVAL, "ws/x/v/g/tws/gx is NULL");
    if (wide(cfg)) return hvp_backward_wide(cfg, ws, x, n, v, u, g, tws, gx, gparams, gv, gu, stream);
    float* abuf = tws;
    float* dbuf = abuf + plan.buf_floats;
    float* spill = dbuf + plan.buf_floats;
    float* partial = spill + plan.buf_floats;
    siren::launch_jet_mix(dim3((unsigned)(plan.n_pad / 16)), st, ws, x, n, v, g, u, gx, gv, gu, cfg->d_in, cfg->d_out,
                          cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, spill, abuf, dbuf, plan.n_pad);
    if (int rc = hip_status("siren_hvp_backward (mixed jet)")) return rc;
    if (gparams == nullptr) return SIREN_OK;
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden), st, abuf, dbuf, plan.cols, plan.tps,
                        partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, siren::H, 1);
    if (int rc = hip_status("siren_hvp_backward (wgrad)")) return rc;
    siren::launch_small_mix(plan.es.grid(cfg), st, abuf, dbuf, x, v, g, u, n, plan.n_pad, plan.es.tps,
                            partial + plan.eslab_off, plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden, siren::H);
    if (int rc = hip_status("siren_hvp_backward (small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_hvp_backward (reduce)");
}

// ---- the backward of a Hessian node Hm = sum_j u_j H_j (n, d, d): the quadratic-form jet (jet_kernel.hpp QG) ------
namespace {
int check_quad(const siren_cfg* cfg) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (wide(cfg) || layered(cfg) || !cfg->outermost_linear || cfg->n_hidden > 5 || cfg->d_in > 2)
        return fail(SIREN_EUNSUPPORTED, "siren_hessian_backward covers hidden 256, 1..5 hidden layers, in_features "
                                        "<= 2, linear output");
    return SIREN_OK;
}
}  // namespace

int32_t siren_hessian_backward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count) {
    if (int rc = check_quad(cfg)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    *count = std::max(JetPlan(cfg, n).total, JetPlan(cfg, n, true).total);  // recomputing / kept (Q8) backward
    return SIREN_OK;
}

// ---- the Hessian node's forward: Hm (n, d, d) = sum_j u_j H_j in one 6-stream forward jet (hess_kernel.hpp) -----
int32_t siren_hessian_ws_floats(const siren_cfg* cfg, int64_t n, int32_t keep, int64_t* count) {
    if (int rc = check_quad(cfg)) return rc;
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    *count = keep ? siren::hess_groups(n) * 8 * (int64_t)cfg->n_hidden * 6 * siren::H : 0;  // layers 1..L
    return SIREN_OK;
}

int32_t siren_hessian(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* u, float* kept,
                      float* hm, void* stream) {
    return siren_hessian_ex(cfg, ws, x, n, u, kept, hm, nullptr, nullptr, stream);
}

int32_t siren_hessian_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* u, float* kept,
                         float* hm, float* y, float* gx, void* stream) {
    if (int rc = check_quad(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (n == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || hm == nullptr) return fail(SIREN_EINVAL, "ws/x/hm is NULL");
    if (n > (int64_t)0x7fffffff * 8) return fail(SIREN_EINVAL, "n exceeds the grid");
    siren::launch_hess(dim3((unsigned)(siren::hess_groups(n) / siren::WAVES)), (hipStream_t)stream, ws, x, n, u,
                       cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, hm, kept, y, gx);
    return hip_status("siren_hessian");
}

int32_t siren_hessian_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* G,
                               const float* u, float* tws, float* gx, float* gparams, float* gu, void* stream) {
    return siren_hessian_backward_kept(cfg, ws, x, n, G, u, nullptr, tws, gx, gparams, gu, stream);
}

int32_t siren_hessian_backward_kept(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* G,
                                    const float* u, const float* kept, float* tws, float* gx, float* gparams,
                                    float* gu, void* stream) {
    if (int rc = check_quad(cfg)) return rc;
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    const JetPlan plan(cfg, n);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {
        if (gparams != nullptr) (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_hessian_backward");
    }
    if (ws == nullptr || tws == nullptr || gx == nullptr || x == nullptr || G == nullptr)
        return fail(SIREN_EINVAL, "ws/x/G/tws/gx is NULL");
    if (kept != nullptr) {
        // reverse-only quadratic-form jet on the node's own 8-coordinate layout (qf_kernel.hpp), then the MFMA wgrad
        // over the Q8 tile pairs (value-column bias: jet_bias 3) and EDGE_Q8
        if (n > (int64_t)0x7fffffff * 8) return fail(SIREN_EINVAL, "n exceeds the grid");
        const JetPlan qp(cfg, n, true);
        float* qa = tws;
        float* qd = qa + qp.buf_floats;
        float* qpart = qd + qp.buf_floats;
        if ((cfg->reserved & SIREN_FLAG_QF_SERIAL) != 0)
            siren::launch_qf_rev(siren::hess_groups(n), st, ws, x, n, G, u, kept, gx, gu, cfg->d_in, cfg->d_out,
                                 cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, qa, qd, qp.n_pad);
        else
            siren::launch_qfi_rev(siren::hess_groups(n), st, ws, x, n, G, u, kept, gx, gu, cfg->d_in, cfg->d_out,
                                  cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, qa, qd, qp.n_pad);
        if (int rc = hip_status("siren_hessian_backward (kept quadratic-form jet)")) return rc;
        if (gparams == nullptr) return SIREN_OK;
        siren::launch_wgrad(dim3((unsigned)qp.splits, (unsigned)cfg->n_hidden), st, qa, qd, qp.cols, qp.tps, qpart, P,
                            cfg->d_in, cfg->d_out, cfg->n_hidden, 1, siren::H, 3);
        if (int rc = hip_status("siren_hessian_backward (wgrad)")) return rc;
        siren::launch_small_q8(qp.es.grid(cfg), st, qa, qd, x, u, n, qp.n_pad, qp.es.tps, qpart + qp.eslab_off,
                               qp.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden);
        if (int rc = hip_status("siren_hessian_backward (small)")) return rc;
        return finish_grads(cfg, st, qpart, qp.splits, 0, qpart + qp.eslab_off, qp.es, gparams,
                            "siren_hessian_backward (reduce)");
    }
    float* abuf = tws;
    float* dbuf = abuf + plan.buf_floats;
    float* spill = dbuf + plan.buf_floats;
    float* partial = spill + plan.buf_floats;
    siren::launch_jet_quad(dim3((unsigned)(plan.n_pad / 16)), st, ws, x, n, G, u, gx, gu, cfg->d_in, cfg->d_out,
                           cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, spill, abuf, dbuf, plan.n_pad);
    if (int rc = hip_status("siren_hessian_backward (quadratic-form jet)")) return rc;
    if (gparams == nullptr) return SIREN_OK;
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden), st, abuf, dbuf, plan.cols, plan.tps,
                        partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, siren::H, 1);
    if (int rc = hip_status("siren_hessian_backward (wgrad)")) return rc;
    // EDGE_MIX with v = e_1, g = e_2 (NULL tangents): dW0[:, k] = sum zb_0,value x_k + zb_0,tangent k
    siren::launch_small_mix(plan.es.grid(cfg), st, abuf, dbuf, x, nullptr, nullptr, u, n, plan.n_pad, plan.es.tps,
                            partial + plan.eslab_off, plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden, siren::H);
    if (int rc = hip_status("siren_hessian_backward (small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_hessian_backward (reduce)");
}

// ---- W3: second-order adjoint (Hessian-vector product + mixed theta gradient), d_out == 1 ---------------
namespace {
struct W3Plan {
    int64_t n_pad, tiles, splits, tps, spill_floats, buf_floats, partial_floats, total, eslab_off;
    EdgeSplit es;
    // batch > 1: a grouped launch over batched weights (per-element layout strides: spill_floats, buf_floats,
    // partial_floats; fewer splits per element, as TrainPlan)
    W3Plan(const siren_cfg* cfg, int64_t n, bool theta, int64_t batch = 1)
        : es(cfg, (n + siren::TILE - 1) / siren::TILE * siren::TILE / 16, batch) {
        const TrainPlan tp(cfg, n, batch);
        n_pad = tp.n_pad;
        tiles = tp.tiles;
        splits = tp.splits;
        tps = tp.tps;
        spill_floats = n_pad * (int64_t)(cfg->n_hidden + 1) * 3 * siren::H;
        buf_floats = theta ? (int64_t)(cfg->n_hidden + 1) * n_pad * siren::H : 0;
        eslab_off = 2 * splits * param_count(cfg);
        partial_floats = theta ? eslab_off + es.floats : 0;
        total = spill_floats + 4 * buf_floats + partial_floats;
    }
};
}  // namespace


int32_t siren_second_order_ws_floats(const siren_cfg* cfg, int64_t n, int32_t want_theta, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (layered(cfg)) return layered_unsupported("siren_second_order");
    if (count == nullptr || n < 0) return fail(SIREN_EINVAL, "count is NULL or n < 0");
    *count = wide(cfg) ? W3WidePlan(cfg, n).total : W3Plan(cfg, n, want_theta != 0).total;
    return SIREN_OK;
}

int32_t siren_second_order(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                           float* tws, float* gx, float* gparams, void* stream) {
    return siren_second_order_seeded(cfg, ws, x, n, v, nullptr, tws, gx, gparams, stream);
}

int32_t siren_second_order_seeded(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                                  const float* gy, float* tws, float* gx, float* gparams, void* stream) {
    return siren_second_order_ex(cfg, ws, x, n, v, nullptr, gy, tws, gx, gparams, nullptr, stream);
}

// hidden 512: one two-stream jet launch (forward + reverse), then the split-K wgrad over 2 n_pad columns, the
// EDGE_J2 edge layers and the slab reductions
static int32_t second_order_wide(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                                 const float* u, const float* gy, float* tws, float* gx, float* gparams, float* ydot,
                                 void* stream) {
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    const W3WidePlan plan(cfg, n);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    const bool theta = gparams != nullptr;
    if (n == 0) {
        if (theta) (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_second_order (hidden 512)");
    }
    if (ws == nullptr || tws == nullptr || gx == nullptr || x == nullptr || v == nullptr)
        return fail(SIREN_EINVAL, "ws/x/v/tws/gx is NULL");
    float* abuf = tws;
    float* dbuf = abuf + plan.buf_floats;
    float* spill = dbuf + plan.buf_floats;
    float* partial = spill + plan.buf_floats;
    siren::launch_wide_jet2(dim3((unsigned)(plan.n_pad / 32)), st, ws, x, v, gy, u, n, cfg->d_in, cfg->d_out,
                            cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, gx, ydot, spill, abuf, dbuf, plan.n_pad);
    if (int rc = hip_status("siren_second_order (hidden 512 jet)")) return rc;
    if (!theta) return SIREN_OK;
    const unsigned quads = (unsigned)((cfg->hidden / 256) * (cfg->hidden / 256));
    siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden, quads), st, abuf, dbuf, plan.cols,
                        plan.tps, partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1, cfg->hidden, 2);
    if (int rc = hip_status("siren_second_order (hidden 512 wgrad)")) return rc;
    siren::launch_small_j2(plan.es.grid(cfg), st, abuf, dbuf, x, v, gy, u, n, plan.n_pad, plan.es.tps,
                           partial + plan.eslab_off, plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_second_order (hidden 512 small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                        "siren_second_order (hidden 512 reduce)");
}

static int32_t second_order_impl(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                          const float* u, const float* gy, float* tws, float* gx, float* gparams, float* ydot,
                          float* kept, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!cfg->outermost_linear)
        return fail(SIREN_EUNSUPPORTED, "siren_second_order needs a linear output layer");
    if (layered(cfg)) return layered_unsupported("siren_second_order");
    if (wide(cfg)) {
        if (kept != nullptr) return fail(SIREN_EUNSUPPORTED, "the kept-forward W3 covers hidden 256");
        return second_order_wide(cfg, ws, x, n, v, u, gy, tws, gx, gparams, ydot, stream);
    }
    if (cfg->n_hidden > siren::MAX_LH_GRAD && !deep(cfg))
        return fail(SIREN_EUNSUPPORTED, "siren_second_order needs 1 <= num_hidden_layers <= 5 at hidden 256 (nonzero "
                                        "omegas beyond 3)");
    if (n < 0) return fail(SIREN_EINVAL, "n < 0");
    if (ws == nullptr || tws == nullptr || gx == nullptr || (n > 0 && (x == nullptr || v == nullptr)))
        return fail(SIREN_EINVAL, "ws/x/v/tws/gx is NULL");
    const bool theta = gparams != nullptr;
    const W3Plan plan(cfg, n, theta);
    const hipStream_t st = (hipStream_t)stream;
    const int64_t P = param_count(cfg);
    if (n == 0) {
        if (theta) (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
        return hip_status("siren_second_order");
    }
    float* spill = tws;
    float* A = spill + plan.spill_floats;
    float* At = A + plan.buf_floats;
    float* D = At + plan.buf_floats;
    float* Dt = D + plan.buf_floats;
    float* partial = Dt + plan.buf_floats;
    const float *kA = nullptr, *kC = nullptr;
    if (kept != nullptr) {  // the stored jet forward's a_l tiles double as A
        const TrainPlan tp(cfg, n);
        kA = kept;
        kC = stored_cos(cfg, tp, kept);
        A = kept;
    }
    const dim3 grid((unsigned)(plan.n_pad / siren::TILE));
    siren::launch_w3(theta, grid, st, ws, x, v, gy, u, ydot, cfg->d_out, n, gx, spill, A, At, D, Dt, plan.n_pad,
                     cfg->d_in, cfg->n_hidden, cfg->omega_first, cfg->omega_hidden, kA, kC, g_w3_prof, 0, 0, 0,
                     (cfg->reserved & SIREN_FLAG_W3_SERIAL) != 0);
    if (int rc = hip_status("siren_second_order (w3)")) return rc;
    if (!theta) return SIREN_OK;
    const dim3 wgrid((unsigned)plan.splits, (unsigned)cfg->n_hidden);
    siren::launch_wgrad(wgrid, st, A, D, plan.n_pad, plan.tps, partial, P, cfg->d_in, cfg->d_out, cfg->n_hidden, 1,
                        siren::H);
    siren::launch_wgrad(wgrid, st, At, Dt, plan.n_pad, plan.tps, partial + plan.splits * P, P, cfg->d_in, cfg->d_out,
                        cfg->n_hidden, 0, siren::H);
    if (int rc = hip_status("siren_second_order (wgrad)")) return rc;
    const float* a_last = A + (int64_t)cfg->n_hidden * plan.n_pad * siren::H;  // a_L rows (first-order seed)
    siren::launch_small_w3(plan.es.grid(cfg), st, At, D, Dt, a_last, x, v, gy, u, n, plan.n_pad, plan.es.tps,
                           partial + plan.eslab_off, plan.es.E, cfg->d_in, cfg->d_out, cfg->n_hidden);
    if (int rc = hip_status("siren_second_order (small)")) return rc;
    return finish_grads(cfg, st, partial, plan.splits, plan.splits, partial + plan.eslab_off, plan.es, gparams,
                        "siren_second_order (reduce)");
}

int32_t siren_second_order_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                              const float* u, const float* gy, float* tws, float* gx, float* gparams, float* ydot,
                              void* stream) {
    return second_order_impl(cfg, ws, x, n, v, u, gy, tws, gx, gparams, ydot, nullptr, stream);
}

int32_t siren_second_order_kept(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                                const float* gy, float* kept, float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!stored_ok(cfg) || wide(cfg) || layered(cfg))
        return fail(SIREN_EUNSUPPORTED, "siren_second_order_kept covers hidden 256");
    if (kept == nullptr) return fail(SIREN_EINVAL, "kept is NULL");
    return second_order_impl(cfg, ws, x, n, v, nullptr, gy, tws, gx, gparams, nullptr, kept, stream);
}

int32_t siren_forward_grad_store(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y,
                                 float* gx, float* tws, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (wide(cfg) || layered(cfg)) return fail(SIREN_EUNSUPPORTED, "siren_forward_grad_store covers hidden 256");
    if (int rc = siren_forward_store(cfg, ws, x, n, y, tws, stream)) return rc;
    if (n == 0) return SIREN_OK;
    if (gx == nullptr) return fail(SIREN_EINVAL, "gx is NULL");
    const TrainPlan plan(cfg, n);
    // dPhi/dx (gy = ones) by the reverse GEMMs from the stored cos; no delta tiles
    siren::FusedArgs fa{w1_ws(cfg, ws), x, n, nullptr, nullptr, gx, cfg->d_in, cfg->d_out, cfg->n_hidden,
                        cfg->omega_first, cfg->omega_hidden, 0, stored_cos(cfg, plan, tws), nullptr, plan.n_pad};
    siren::launch_w1(siren::MODE_REV, tile_grid(cfg, plan.n_pad / siren::TILE, 1), (hipStream_t)stream, fa);
    return hip_status("siren_forward_grad_store");
}

// ---- per-step kernels -------------------------------------------------------------------
int32_t siren_sample_sdf(const float* pc_coords, const float* pc_normals, int64_t m, int64_t k, uint64_t seed,
                         uint64_t step, float* coords, float* normals, float* sdf, void* stream) {
    if (m <= 0 || k < 0) return fail(SIREN_EINVAL, "siren_sample_sdf: need m > 0 and k >= 0");
    if (k == 0) return SIREN_OK;
    if (pc_coords == nullptr || pc_normals == nullptr || coords == nullptr || normals == nullptr || sdf == nullptr)
        return fail(SIREN_EINVAL, "siren_sample_sdf: NULL pointer");
    siren::launch_sample_sdf((hipStream_t)stream, pc_coords, pc_normals, m, k, seed, step, coords, normals, sdf);
    return hip_status("siren_sample_sdf");
}

// ---- device marching cubes (sdf_meshing.py:97-102 replacement) ----
static int mc_check(int64_t X, int64_t Y, int64_t Z, bool& empty) {
    if (X < 0 || Y < 0 || Z < 0) return fail(SIREN_EINVAL, "volume dimensions must be >= 0");
    empty = X < 2 || Y < 2 || Z < 2;
    if (!empty && (X * Y * Z >= (int64_t(1) << 32) || X > 65535 || Y > 65535))
        return fail(SIREN_EUNSUPPORTED, "marching cubes needs X*Y*Z < 2^32 and X, Y <= 65535");
    return SIREN_OK;
}

int32_t siren_mc_ws_bytes(int64_t X, int64_t Y, int64_t Z, int64_t* bytes) {
    bool empty = false;
    if (int rc = mc_check(X, Y, Z, empty)) return rc;
    if (bytes == nullptr) return fail(SIREN_EINVAL, "bytes is NULL");
    *bytes = empty ? 0 : 4 * siren::mc_ws_words(X, Y, Z);
    return SIREN_OK;
}

int32_t siren_mc_count(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, void* ws, int64_t* n_verts,
                       int64_t* n_faces, void* stream) {
    bool empty = false;
    if (int rc = mc_check(X, Y, Z, empty)) return rc;
    if (n_verts == nullptr || n_faces == nullptr) return fail(SIREN_EINVAL, "n_verts/n_faces is NULL");
    *n_verts = *n_faces = 0;
    if (empty) return SIREN_OK;
    if (vol == nullptr || ws == nullptr) return fail(SIREN_EINVAL, "vol/ws is NULL");
    if (!std::isfinite(level)) return fail(SIREN_EINVAL, "level must be finite");
    const hipStream_t st = (hipStream_t)stream;
    uint32_t* w = (uint32_t*)ws;
    siren::mc_count(vol, X, Y, Z, level, w, st);
    if (int rc = hip_status("siren_mc_count")) return rc;
    uint32_t tv = 0, tf = 0;
    if (hipMemcpyAsync(&tv, siren::mc_totals(w, X, Y, Z, 0), 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&tf, siren::mc_totals(w, X, Y, Z, 1), 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail(SIREN_EHIP, "siren_mc_count: reading the totals failed");
    if (tv >= (1u << 31) || tf >= (1u << 31))  // saturated by the scan: int32 face indices would wrap
        return fail(SIREN_EUNSUPPORTED, "siren_mc_count: the surface has >= 2^31 vertices or triangles; mesh the "
                                        "volume in pieces");
    *n_verts = tv;
    *n_faces = tf;
    return SIREN_OK;
}

int32_t siren_mc_emit(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, const float* spacing3,
                      const void* ws, float* verts, int32_t* faces, void* stream) {
    bool empty = false;
    if (int rc = mc_check(X, Y, Z, empty)) return rc;
    if (empty) return SIREN_OK;
    if (vol == nullptr || ws == nullptr || spacing3 == nullptr) return fail(SIREN_EINVAL, "vol/ws/spacing is NULL");
    if (verts == nullptr || faces == nullptr) return fail(SIREN_EINVAL, "verts/faces is NULL");
    siren::mc_emit(vol, X, Y, Z, level, spacing3, (const uint32_t*)ws, verts, faces, (hipStream_t)stream);
    return hip_status("siren_mc_emit");
}

int32_t siren_adam_scratch_floats(int64_t* count) {
    if (count == nullptr) return fail(SIREN_EINVAL, "count is NULL");
    *count = siren::STEP_BLOCKS + 4;
    return SIREN_OK;
}

int32_t siren_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
                        float beta1, float beta2, float eps, int64_t step, float max_norm, float* scratch,
                        void* stream) {
    if (n < 0 || step < 1) return fail(SIREN_EINVAL, "siren_adam_step: need n >= 0 and step >= 1");
    if (n == 0) return SIREN_OK;
    if (params == nullptr || grads == nullptr || exp_avg == nullptr || exp_avg_sq == nullptr ||
        (max_norm > 0.f && scratch == nullptr))
        return fail(SIREN_EINVAL, "siren_adam_step: NULL pointer");
    const uintptr_t al = (uintptr_t)params | (uintptr_t)grads | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq;
    if ((al & 15) != 0) return fail(SIREN_EINVAL, "siren_adam_step: buffers must be 16-byte aligned");
    // bias corrections in double on the host (torch computes 1 - beta ** step in Python floats)
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step), bc2 = 1.0 - std::pow((double)beta2, (double)step);
    siren::launch_adam((hipStream_t)stream, params, grads, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, (float)bc1,
                       (float)bc2, max_norm, scratch);
    return hip_status("siren_adam_step");
}

// ---- batched (hypernetwork) weights: BatchLinear with W (B, out, in) (modules.py:16-25, meta_modules.py:41-53) ----
// Element b uses params + b * param_count, ws + b * ws_floats, x + b * n * d_in, y + b * n * d_out, ...
// W0 / W1 on hidden 256 (the w1_kernel family) run as ONE grouped launch (grid.y = batch element); other
// configurations and the W2 backward run the single-network entry points element by element on the stream.
bool grouped_ok(const siren_cfg* cfg) {
    return w1_ok(cfg) && cfg->outermost_linear && (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0;
}

int32_t siren_pack_batched(const siren_cfg* cfg, const float* params, int64_t batch, float* ws, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "batch must be in [0, 65535]");
    if (batch == 0) return SIREN_OK;
    if (params == nullptr || ws == nullptr) return fail(SIREN_EINVAL, "params/ws is NULL");
    if (layered(cfg)) {
        for (int64_t b = 0; b < batch; ++b)
            if (int rc = siren_pack(cfg, params + b * param_count(cfg), ws + b * ws_floats(cfg), stream)) return rc;
        return SIREN_OK;
    }
    // every batched entry point reads only the phase-scaled copy when the W1-family kernels cover the network
    // (linear output, hidden 256, no legacy flag): the unscaled half is not written (half the per-step pack)
    const bool scaled_only = w1_ok(cfg) && cfg->outermost_linear && (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0;
    siren::launch_pack(params, ws, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden, small_pad(cfg), ws_floats(cfg),
                       wide(cfg) ? 0 : ws_base(cfg), cfg->omega_first * kInv2Pi, cfg->omega_hidden * kInv2Pi,
                       (hipStream_t)stream, (int)batch, param_count(cfg), scaled_only ? ws_base(cfg) : 0);
    return hip_status("siren_pack_batched");
}

int32_t siren_pack_batched_ex(const siren_cfg* cfg, const float* params, int64_t batch, float* ws, int32_t full,
                              void* stream) {
    if (!full) return siren_pack_batched(cfg, params, batch, ws, stream);
    if (int rc = check_cfg(cfg, true)) return rc;
    if (batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "batch must be in [0, 65535]");
    if (batch == 0) return SIREN_OK;
    if (params == nullptr || ws == nullptr) return fail(SIREN_EINVAL, "params/ws is NULL");
    if (layered(cfg)) return siren_pack_batched(cfg, params, batch, ws, stream);
    siren::launch_pack(params, ws, cfg->d_in, cfg->d_out, cfg->n_hidden, cfg->hidden, small_pad(cfg), ws_floats(cfg),
                       wide(cfg) ? 0 : ws_base(cfg), cfg->omega_first * kInv2Pi, cfg->omega_hidden * kInv2Pi,
                       (hipStream_t)stream, (int)batch, param_count(cfg), 0);
    return hip_status("siren_pack_batched_ex");
}

// second / third order over batched weights (the create_graph branch of a hypernetwork's hypo network): element b's
// fully packed workspace (siren_pack_batched_ex full = 1) through the single-network entry points, tws reused element
// after element (stream order)
// grouped W3 (hidden 256, 1..3 hidden layers, elements below ~2 CU rounds of tiles): ONE W3 launch (grid.y = element),
// two grouped wgrad launches, one edge and one reduction launch over all elements; workspace per element = the W3Plan
// of the grouped split ([spill][A][At][D][Dt][partial slabs], each block holding every element's part)
bool grouped_w3(const siren_cfg* cfg, int64_t n) {
    return !wide(cfg) && !layered(cfg) && cfg->outermost_linear && cfg->n_hidden <= siren::MAX_LH_GRAD &&
           (cfg->reserved & SIREN_FLAG_LEGACY_KERNEL) == 0 && (n + siren::TILE - 1) / siren::TILE < 2 * cu_count();
}

int32_t siren_second_order_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int32_t want_theta,
                                             int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (batch < 0) return fail(SIREN_EINVAL, "batch < 0");
    if (batch > 1 && n > 0 && grouped_w3(cfg, n)) {
        if (count == nullptr) return fail(SIREN_EINVAL, "count is NULL");
        *count = batch * W3Plan(cfg, n, want_theta != 0, batch).total;
        return SIREN_OK;
    }
    return siren_second_order_ws_floats(cfg, n, want_theta, count);
}

int32_t siren_second_order_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                   const float* v, const float* u, const float* gy, float* tws, float* gx,
                                   float* gparams, float* ydot, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (n < 0 || batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "need n >= 0 and 0 <= batch <= 65535");
    const int64_t W = ws_floats(cfg), P = param_count(cfg);
    const int d = cfg->d_in, o = cfg->d_out;
    if (batch > 0 && ws == nullptr) return fail(SIREN_EINVAL, "ws is NULL");
    if (batch > 1 && n > 0 && grouped_w3(cfg, n)) {
        if (x == nullptr || v == nullptr || tws == nullptr || gx == nullptr)
            return fail(SIREN_EINVAL, "x/v/tws/gx is NULL");
        const bool theta = gparams != nullptr;
        const W3Plan plan(cfg, n, theta, batch);
        const hipStream_t st = (hipStream_t)stream;
        float* spill = tws;
        float* A = spill + batch * plan.spill_floats;
        float* At = A + batch * plan.buf_floats;
        float* D = At + batch * plan.buf_floats;
        float* Dt = D + batch * plan.buf_floats;
        float* partial = Dt + batch * plan.buf_floats;
        siren::launch_w3(theta, dim3((unsigned)(plan.n_pad / siren::TILE), (unsigned)batch), st, ws, x, v, gy, u, ydot,
                         o, n, gx, spill, A, At, D, Dt, plan.n_pad, d, cfg->n_hidden, cfg->omega_first,
                         cfg->omega_hidden, nullptr, nullptr, nullptr, W, plan.spill_floats, plan.buf_floats,
                         (cfg->reserved & SIREN_FLAG_W3_SERIAL) != 0);
        if (int rc = hip_status("siren_second_order_batched (grouped w3)")) return rc;
        if (!theta) return SIREN_OK;
        const dim3 wgrid((unsigned)plan.splits, (unsigned)cfg->n_hidden, (unsigned)batch);
        siren::launch_wgrad(wgrid, st, A, D, plan.n_pad, plan.tps, partial, P, d, o, cfg->n_hidden, 1, siren::H, 0,
                            plan.buf_floats, plan.partial_floats);
        siren::launch_wgrad(wgrid, st, At, Dt, plan.n_pad, plan.tps, partial + plan.splits * P, P, d, o,
                            cfg->n_hidden, 0, siren::H, 0, plan.buf_floats, plan.partial_floats);
        if (int rc = hip_status("siren_second_order_batched (grouped wgrad)")) return rc;
        const float* a_last = A + (int64_t)cfg->n_hidden * plan.n_pad * siren::H;
        siren::launch_small_w3(plan.es.grid(cfg, batch), st, At, D, Dt, a_last, x, v, gy, u, n, plan.n_pad,
                               plan.es.tps, partial + plan.eslab_off, plan.es.E, d, o, cfg->n_hidden, plan.buf_floats,
                               plan.partial_floats);
        if (int rc = hip_status("siren_second_order_batched (grouped small)")) return rc;
        return finish_grads(cfg, st, partial, plan.splits, plan.splits, partial + plan.eslab_off, plan.es, gparams,
                            "siren_second_order_batched (grouped reduce)", batch, plan.partial_floats);
    }
    for (int64_t b = 0; b < batch; ++b)
        if (int rc = siren_second_order_ex(cfg, ws + b * W, x ? x + b * n * d : nullptr, n, v ? v + b * n * d : nullptr,
                                           u ? u + b * n * o : nullptr, gy ? gy + b * n * o : nullptr, tws,
                                           gx ? gx + b * n * d : nullptr, gparams ? gparams + b * P : nullptr,
                                           ydot ? ydot + b * n * o : nullptr, stream))
            return rc;
    return SIREN_OK;
}

int32_t siren_hvp_backward_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int64_t* count) {
    if (batch < 0) return fail(SIREN_EINVAL, "batch < 0");
    return siren_hvp_backward_ws_floats(cfg, n, count);
}

int32_t siren_hvp_backward_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                   const float* v, const float* u, const float* g, float* tws, float* gx,
                                   float* gparams, float* gv, float* gu, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (n < 0 || batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "need n >= 0 and 0 <= batch <= 65535");
    const int64_t W = ws_floats(cfg), P = param_count(cfg);
    const int d = cfg->d_in, o = cfg->d_out;
    if (batch > 0 && ws == nullptr) return fail(SIREN_EINVAL, "ws is NULL");
    for (int64_t b = 0; b < batch; ++b)
        if (int rc = siren_hvp_backward(cfg, ws + b * W, x ? x + b * n * d : nullptr, n, v ? v + b * n * d : nullptr,
                                        u ? u + b * n * o : nullptr, g ? g + b * n * d : nullptr, tws,
                                        gx ? gx + b * n * d : nullptr, gparams ? gparams + b * P : nullptr,
                                        gv ? gv + b * n * d : nullptr, gu ? gu + b * n * o : nullptr, stream))
            return rc;
    return SIREN_OK;
}

int32_t siren_forward_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                              float* y, void* stream) {
    return siren_forward_batched_ex(cfg, ws, x, n, batch, y, nullptr, stream);
}

int32_t siren_forward_batched_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                 float* y, float* tws, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (n < 0 || batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "need n >= 0 and 0 <= batch <= 65535");
    if (n == 0 || batch == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || y == nullptr) return fail(SIREN_EINVAL, "ws/x/y is NULL");
    const int64_t W = ws_floats(cfg), blocks = (n + siren::TILE - 1) / siren::TILE;
    // elements that fill the chip on their own run one by one: concurrent elements would stream several weight
    // sets through each XCD's L2 (measured 7 % slower at 8 x 2^16, profiles/r01_batched.log)
    const int64_t cus = cu_count();
    if (!(grouped_ok(cfg) && cfg->n_hidden <= 5) || blocks >= 4 * cus) {
        for (int64_t b = 0; b < batch; ++b)
            if (int rc = siren_forward_ex(cfg, ws + b * W, x + b * n * cfg->d_in, n, y + b * n * cfg->d_out, tws, stream))
                return rc;
        return SIREN_OK;
    }
    if (blocks > 0x7fffffffll) return fail(SIREN_EINVAL, "n too large");
    siren::FusedArgs fa{w1_ws(cfg, ws), x, n, nullptr, y, nullptr, cfg->d_in, cfg->d_out, cfg->n_hidden,
                        cfg->omega_first, cfg->omega_hidden, 0, nullptr, nullptr, 0, W};
    siren::launch_w0(dim3((unsigned)blocks, (unsigned)batch), (hipStream_t)stream, fa);
    return hip_status("siren_forward_batched");
}

int32_t siren_forward_grad_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                   const float* gy, float* y, float* gx, float* tws, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (n < 0 || batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "need n >= 0 and 0 <= batch <= 65535");
    if (n == 0 || batch == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || gx == nullptr) return fail(SIREN_EINVAL, "ws/x/gx is NULL");
    const int64_t W = ws_floats(cfg), blocks = (n + siren::TILE - 1) / siren::TILE;
    const int d = cfg->d_in, o = cfg->d_out;
    const int64_t cus = cu_count();
    if (!(grouped_ok(cfg) && cfg->n_hidden <= siren::MAX_LH_GRAD) || blocks >= 2 * cus) {
        for (int64_t b = 0; b < batch; ++b)
            if (int rc = siren_forward_grad(cfg, ws + b * W, x + b * n * d, n, gy ? gy + b * n * o : nullptr,
                                            y ? y + b * n * o : nullptr, gx + b * n * d, tws, stream))
                return rc;
        return SIREN_OK;
    }
    siren::FusedArgs fa{w1_ws(cfg, ws), x, n, gy, y, gx, d, o, cfg->n_hidden, cfg->omega_first, cfg->omega_hidden,
                        0, nullptr, nullptr, 0, W};
    // persistent grid split across the batch: about one workgroup per CU in total
    const dim3 g1 = tile_grid(cfg, blocks * batch, 1);  // min(all tiles, CUs)
    const int64_t per = std::max<int64_t>(1, ((int64_t)g1.x + batch - 1) / batch);
    const int64_t gxs = (cfg->reserved & SIREN_FLAG_NO_PERSIST) != 0 ? blocks : std::min(blocks, per);
    siren::launch_w1(w1_mode(cfg, gy), dim3((unsigned)gxs, (unsigned)batch), (hipStream_t)stream, fa);
    return hip_status("siren_forward_grad_batched");
}

// grouped W2 (hidden 256, elements below ~2 CU rounds of tiles): ONE STORE launch (grid.y = element), one wgrad
// launch (grid.z = element), one edge launch and one reduction over all elements; workspace per element =
// siren_train_ws_floats(cfg, n) (siren_train_batched_ws_floats)
bool grouped_w2(const siren_cfg* cfg, int64_t n) {
    return grouped_ok(cfg) && cfg->n_hidden <= siren::MAX_LH_GRAD && (n + siren::TILE - 1) / siren::TILE < 2 * cu_count();
}

int32_t siren_train_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (count == nullptr || n < 0 || batch < 0) return fail(SIREN_EINVAL, "count is NULL or n / batch < 0");
    if (!grouped_w2(cfg, n)) return siren_train_ws_floats(cfg, n, count);  // element by element: one reused
    *count = batch * TrainPlan(cfg, n, batch).total;
    return SIREN_OK;
}

int32_t siren_backward_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                               const float* gy, float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (n < 0 || batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "need n >= 0 and 0 <= batch <= 65535");
    if (batch > 0 && (ws == nullptr || gy == nullptr || gparams == nullptr || tws == nullptr || gx == nullptr ||
                      (n > 0 && x == nullptr)))
        return fail(SIREN_EINVAL, "ws/x/gy/tws/gx/gparams is NULL");
    const int64_t W = ws_floats(cfg), P = param_count(cfg);
    const int d = cfg->d_in, o = cfg->d_out;
    if (batch > 0 && n > 0 && grouped_w2(cfg, n)) {
        const TrainPlan plan(cfg, n, batch);
        const hipStream_t st = (hipStream_t)stream;
        // [a tiles of every element][delta tiles of every element][partial slabs of every element]: element b's
        // tiles at + b * act_floats (the STORE kernel's grid.y offset), its slabs at + b * partial_floats
        const int64_t bact = plan.act_floats, bpart = plan.partial_floats;
        float* abuf = tws;
        float* dbuf = tws + batch * bact;
        float* partial = tws + 2 * batch * bact;
        siren::FusedArgs fa{w1_ws(cfg, ws), x, n, gy, nullptr, gx, d, o, cfg->n_hidden, cfg->omega_first,
                            cfg->omega_hidden, 0, abuf, dbuf, plan.n_pad, W};
        const int64_t tiles = plan.n_pad / siren::TILE;
        const int64_t per = std::max<int64_t>(1, ((int64_t)cu_count() + batch - 1) / batch);
        siren::launch_w1(siren::MODE_STORE, dim3((unsigned)std::min(tiles, per), (unsigned)batch), st, fa);
        if (int rc = hip_status("siren_backward_batched (grouped store)")) return rc;
        siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden, (unsigned)batch), st, abuf, dbuf,
                            plan.n_pad, plan.tps, partial, P, d, o, cfg->n_hidden, 1, cfg->hidden, 0, bact, bpart);
        if (int rc = hip_status("siren_backward_batched (grouped wgrad)")) return rc;
        siren::launch_small(plan.es.grid(cfg, batch), st, abuf, dbuf, x, gy, n, plan.n_pad, plan.es.tps,
                            partial + plan.eslab_off, plan.es.E, d, o, cfg->n_hidden, cfg->hidden, bact, bpart);
        if (int rc = hip_status("siren_backward_batched (grouped small)")) return rc;
        return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                            "siren_backward_batched (grouped reduce)", batch, bpart);
    }
    for (int64_t b = 0; b < batch; ++b)
        if (int rc = siren_backward(cfg, ws + b * W, x + b * n * d, n, gy + b * n * o, tws, nullptr,
                                    gx ? gx + b * n * d : nullptr, gparams + b * P, stream))
            return rc;
    return SIREN_OK;
}

// ---- stored-forward W2 split over batched weights: the training forward (SirenBatchedFunction) keeps every
// element's a_l tiles and cos, so the hypernetwork's backward is reverse-only. Grouped (hidden 256, elements below
// ~2 CU rounds): [a tiles of every element][delta tiles][partial slabs][lane-major cos]; otherwise element b owns the
// single-network layout at tws + b * siren_train_stored_ws_floats(cfg, n).
int32_t siren_train_stored_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int64_t* count) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!stored_ok(cfg)) return fail(SIREN_EUNSUPPORTED, "the stored-forward W2 split needs a linear output layer");
    if (count == nullptr || n < 0 || batch < 0) return fail(SIREN_EINVAL, "count is NULL or n / batch < 0");
    if (grouped_w2(cfg, n)) {
        const TrainPlan plan(cfg, n, batch);
        *count = batch * (plan.total + plan.act_floats);
        return SIREN_OK;
    }
    int64_t per = 0;
    if (int rc = siren_train_stored_ws_floats(cfg, n, &per)) return rc;
    *count = batch * per;
    return SIREN_OK;
}

int32_t siren_forward_store_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                    float* y, float* tws, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!stored_ok(cfg)) return fail(SIREN_EUNSUPPORTED, "the stored-forward W2 split needs a linear output layer");
    if (n < 0 || batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "need n >= 0 and 0 <= batch <= 65535");
    if (n == 0 || batch == 0) return SIREN_OK;
    if (ws == nullptr || x == nullptr || y == nullptr || tws == nullptr) return fail(SIREN_EINVAL, "ws/x/y/tws is NULL");
    const int64_t W = ws_floats(cfg);
    const int d = cfg->d_in, o = cfg->d_out;
    if (grouped_w2(cfg, n)) {
        const TrainPlan plan(cfg, n, batch);
        float* abuf = tws;
        float* cbuf = tws + 2 * batch * plan.act_floats + batch * plan.partial_floats;
        siren::FusedArgs fa{w1_ws(cfg, ws), x, n, nullptr, y, nullptr, d, o, cfg->n_hidden, cfg->omega_first,
                            cfg->omega_hidden, 0, abuf, cbuf, plan.n_pad, W};
        // one workgroup per tile (a persistent grid of ~2 workgroups per CU measured 1 % slower at 32 x 4096,
        // tools/profile_paths.py hypernet vs hypernet_np)
        siren::launch_w0s(dim3((unsigned)(plan.n_pad / siren::TILE), (unsigned)batch), (hipStream_t)stream, fa);
        return hip_status("siren_forward_store_batched (grouped)");
    }
    int64_t per = 0;
    if (int rc = siren_train_stored_ws_floats(cfg, n, &per)) return rc;
    for (int64_t b = 0; b < batch; ++b)
        if (int rc = siren_forward_store(cfg, ws + b * W, x + b * n * d, n, y + b * n * o, tws + b * per, stream))
            return rc;
    return SIREN_OK;
}

int32_t siren_backward_stored_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                      const float* gy, float* tws, float* gx, float* gparams, void* stream) {
    if (int rc = check_cfg(cfg, true)) return rc;
    if (!stored_ok(cfg)) return fail(SIREN_EUNSUPPORTED, "the stored-forward W2 split needs a linear output layer");
    if (n < 0 || batch < 0 || batch > 65535) return fail(SIREN_EINVAL, "need n >= 0 and 0 <= batch <= 65535");
    if (batch > 0 && (ws == nullptr || gy == nullptr || gparams == nullptr || tws == nullptr || gx == nullptr ||
                      (n > 0 && x == nullptr)))
        return fail(SIREN_EINVAL, "ws/x/gy/tws/gx/gparams is NULL");
    const int64_t W = ws_floats(cfg), P = param_count(cfg);
    const int d = cfg->d_in, o = cfg->d_out;
    if (batch > 0 && n > 0 && grouped_w2(cfg, n)) {
        const TrainPlan plan(cfg, n, batch);
        const hipStream_t st = (hipStream_t)stream;
        const int64_t bact = plan.act_floats, bpart = plan.partial_floats;
        float* abuf = tws;
        float* dbuf = tws + batch * bact;
        float* partial = tws + 2 * batch * bact;
        float* cbuf = partial + batch * bpart;
        siren::FusedArgs fa{w1_ws(cfg, ws), x, n, gy, nullptr, gx, d, o, cfg->n_hidden, cfg->omega_first,
                            cfg->omega_hidden, 0, cbuf, dbuf, plan.n_pad, W};
        const int64_t tiles = plan.n_pad / siren::TILE;
        const int64_t per = std::max<int64_t>(1, ((int64_t)cu_count() + batch - 1) / batch);
        siren::launch_w1(siren::MODE_REV, dim3((unsigned)std::min(tiles, per), (unsigned)batch), st, fa);
        if (int rc = hip_status("siren_backward_stored_batched (grouped reverse)")) return rc;
        siren::launch_wgrad(dim3((unsigned)plan.splits, (unsigned)cfg->n_hidden, (unsigned)batch), st, abuf, dbuf,
                            plan.n_pad, plan.tps, partial, P, d, o, cfg->n_hidden, 1, cfg->hidden, 0, bact, bpart);
        if (int rc = hip_status("siren_backward_stored_batched (grouped wgrad)")) return rc;
        siren::launch_small(plan.es.grid(cfg, batch), st, abuf, dbuf, x, gy, n, plan.n_pad, plan.es.tps,
                            partial + plan.eslab_off, plan.es.E, d, o, cfg->n_hidden, cfg->hidden, bact, bpart);
        if (int rc = hip_status("siren_backward_stored_batched (grouped small)")) return rc;
        return finish_grads(cfg, st, partial, plan.splits, 0, partial + plan.eslab_off, plan.es, gparams,
                            "siren_backward_stored_batched (grouped reduce)", batch, bpart);
    }
    int64_t per = 0;
    if (int rc = siren_train_stored_ws_floats(cfg, n, &per)) return rc;
    for (int64_t b = 0; b < batch; ++b)
        if (int rc = siren_backward_stored(cfg, ws + b * W, x + b * n * d, n, gy + b * n * o, tws + b * per,
                                           gx + b * n * d, gparams + b * P, stream))
            return rc;
    return SIREN_OK;
}

}  // extern "C"
