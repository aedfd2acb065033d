// launch.h — host-side launchers of the kernel families (one translation unit each, compiled in parallel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace siren {

struct FusedArgs {
    const float* ws;
    const float* x;
    int64_t n;
    const float* gy;
    float* y;
    float* gx;
    int d, o, lh;
    float w0, w;
    int final_sine;
    float* abuf;
    float* dbuf;
    int64_t n_pad;
    int64_t ws_bstride = 0;  // w1_kernel grouped launch: packed-workspace stride between batch elements (grid.y)
};

// tu_legacy.hip
void launch_pack(const float* p, float* ws, int d, int o, int lh, int h, int64_t spad, int64_t total, int64_t base,
                 float s0, float s, hipStream_t st, int batch = 1, int64_t p_bstride = 0, int64_t begin = 0);
void launch_legacy_fwd(dim3 grid, hipStream_t st, const FusedArgs& a);
void launch_legacy_grad(bool store, dim3 grid, hipStream_t st, const FusedArgs& a);
// tu_w1.hip: mode 0 = W1, 1 = STORE (W2 stage 1), MODE_REV (stored-forward W2 reverse); tu_w0.hip: forward only,
// launch_w0s = MODE_FWDS
void launch_w1(int mode, dim3 grid, hipStream_t st, const FusedArgs& a);
void launch_w0(dim3 grid, hipStream_t st, const FusedArgs& a);
// tu_w1deep.hip: MODE_FWDS / MODE_REV of the W1 kernel at 4..5 hidden layers (hidden 256)
void launch_w1_deep(int mode, dim3 grid, hipStream_t st, const FusedArgs& a);
void launch_w0s(dim3 grid, hipStream_t st, const FusedArgs& a);
// tu_w1nt.hip: MODE_FWDS without a_l tiles (a.abuf == NULL) / MODE_REV without delta tiles (a.dbuf == NULL), 1..5
// hidden layers; launch_w0s and launch_w1(MODE_REV) route here when the tile pointer is NULL
void launch_w1_notile(int mode, dim3 grid, hipStream_t st, const FusedArgs& a);
// tu_w1x.hip: split-bf16 W1 (bf16x6 products on the bf16 matrix pipe; 3 hidden layers, d_in 2 / 3, d_out 1,
// gy = ones); the stream holds split_stream_words(lh) 32-bit words
int64_t split_stream_words(int lh);
void launch_pack_split(const float* p, unsigned* stream, int d, int o, int lh, float s, hipStream_t st);
void launch_w1x(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                float* y, float* gx, int d, float w0, float w);
// the W2 stage of the bf16x6 training leg (forward recompute + reverse from gy (n), a_l / delta_l tiles into abuf / dbuf
// of L + 1 layers of n_pad H floats; gx nullable)
void launch_w1x_store(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x,
                      int64_t n, const float* gy, float* y, float* gx, float* abuf, float* dbuf, int64_t n_pad, int d,
                      float w0, float w);
// the stored split of that stage (X_FWDS: 8 waves, 128-coordinate tiles, a_l tiles + lane-major cos; X_REV: the
// reverse from them, delta_l tiles); n_pad a multiple of 128
void launch_w0xs(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                 float* y, float* abuf, float* cbuf, int64_t n_pad, int d, float w0, float w);
void launch_w1xr(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                 const float* gy, float* gx, const float* cbuf, float* dbuf, int64_t n_pad, int d, float w0, float w);
// its hidden-layer weight gradient on the bf16 pipe (wgradx_kernel.hpp): grid (S, LH), tps even, slabs as launch_wgrad
void launch_wgradx(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, int64_t n_pad, int64_t tps,
                   float* partial, int64_t P, int d, int o, int lh);
// the forward-only split W0 (8 waves, 128 coordinates per workgroup tile)
int split_fwd_tile();
int split_rev_tile();  // the X_REV tile: 16 coordinates per wave
void launch_w0x(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                float* y, int d, float w0, float w);
// tu_w4.hip: JET mode (16 coordinates per workgroup); lap (n) = sum_j Laplacian(y_j), gx (n, d) = sum_j grad y_j
void launch_w4(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, float* y, float* gx, float* lap,
               int d, int o, int lh, float w0, float w);
// W4s split, forward half (MODE_JETS): W4 + the a-jet tiles and the z-jet scratch of jet_store_kernel<JET_REV, PH>
void launch_w4s(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, float* y, float* gx, float* lap,
                float* abuf, float* spill, int64_t n_pad, int d, int o, int lh, float w0, float w);
// tu_jet.hip: W4s (backward of the fused Laplacian), tiles of 16 columns = 4 coordinates x 4 jet streams
void launch_jet_store(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* glap,
                      float* gx, int d, int o, int lh, float w0, float w, float* spill, float* abuf, float* dbuf,
                      int64_t n_pad, bool ph);
void launch_jet_phase(int phase, dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n,
                      const float* glap, float* gx, int d, int o, int lh, float w0, float w, float* spill, float* abuf,
                      float* dbuf, int64_t n_pad, float* y, float* lap, bool ph);
void launch_small_jet(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x,
                      const float* glap, int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E, int d,
                      int o, int lh);
// tu_jet.hip: the third-order adjoint (mixed jet along per-coordinate tangents v, g; output weighting u nullable)
void launch_jet_mix(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* v,
                    const float* g, const float* u, float* gx, float* gv, float* gu, int d, int o, int lh, float w0,
                    float w, float* spill, float* abuf, float* dbuf, int64_t n_pad);
void launch_jet_quad(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* G,
                     const float* u, float* gx, float* gu, int d, int o, int lh, float w0, float w, float* spill,
                     float* abuf, float* dbuf, int64_t n_pad);
// tu_hess.hip: the Hessian node's forward, Hm (n, d, d) = sum_j u_j H_j (d <= 2) in one 6-stream forward jet sweep
// (grid = hess_groups(n) / 4 workgroups); kept (nullable) receives the per-layer jets for launch_qf_rev; y (n, o) /
// gx (n, d) nullable: the value and the seed-weighted gradient from the same sweep
void launch_hess(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* u, int d, int o,
                 int lh, float w0, float w, float* hm, float* kept, float* y, float* gx);
// the kept Hessian-node backward on Q8 tile pairs (qf_kernel.hpp; grid = hess_groups(n) / 4, n_pad = hess_groups(n) * 8):
// abuf / dbuf (L + 1) layers x 4 n_pad columns x 256 floats
void launch_qf_rev(int64_t ngroups, hipStream_t st, const float* ws, const float* x, int64_t n, const float* G,
                   const float* u, const float* kept, float* gx, float* gu, int d, int o, int lh, float w0, float w,
                   float* abuf, float* dbuf, int64_t n_pad);
// tu_qfi.hip: the same backward with its epilogues interleaved into the reverse GEMMs (qfi_kernel.hpp), lh 1..5; same
// arguments, grid and tile layout (results bitwise those of launch_qf_rev)
void launch_qfi_rev(int64_t ngroups, hipStream_t st, const float* ws, const float* x, int64_t n, const float* G,
                    const float* u, const float* kept, float* gx, float* gu, int d, int o, int lh, float w0, float w,
                    float* abuf, float* dbuf, int64_t n_pad);
// its edge layers (EDGE_Q8): rows zb_0 (dbuf layer 0) and the a_L jet (abuf layer L) over n_pad / 8 tile pairs
void launch_small_q8(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* u,
                     int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E, int d, int o, int lh);
void launch_small_mix(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* v,
                      const float* g, const float* u, int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E,
                      int d, int o, int lh, int h);
// tu_wide.hip: hidden width 512 (mode as siren_common.h MODE_*); spill = cos scratch for MODE_W1 / MODE_STORE
void launch_wide(int mode, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill);
// tu_widei.hip: the stored-forward split at hidden 512 with interleaved epilogues (widei_kernel.hpp), MODE_FWDS /
// MODE_REV, 1..5 hidden layers; arguments as launch_wide. Returns false (nothing launched) outside that range.
bool launch_widei(int mode, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill);
// tu_wide_jet.hip: second order at hidden 512 (two-stream jet: 8 coordinates x (value, tangent) per wave, 32 per
// workgroup); abuf / dbuf / spill: (L + 1) layers x 2 n_pad columns x 512 floats each
void launch_wide_jet2(dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy,
                      const float* u, int64_t n, int d, int o, int lh, float w0, float w, float* gx, float* ydot,
                      float* spill, float* abuf, float* dbuf, int64_t n_pad);
void launch_wide_mix(dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* g,
                     const float* u, int64_t n, int d, int o, int lh, float w0, float w, float* gx, float* gv,
                     float* gu, float* spill, float* abuf, float* dbuf, int64_t n_pad);
void launch_small_j2(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* v,
                     const float* gy, const float* u, int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E,
                     int d, int o, int lh);
// tu_w3.hip (launch_small_w3 lives in tu_train.hip with the other edge-layer reductions)
// ws_bs != 0: grouped over batched weights (grid.y = element; per-element strides of ws, the spill and A / At / D / Dt)
void launch_w3(bool theta, dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy,
               const float* u, float* ydot, int o, int64_t n, float* gx, float* spill, float* A, float* At, float* D,
               float* Dt, int64_t n_pad, int d, int lh, float w0, float w, const float* kA = nullptr,
               const float* kC = nullptr, unsigned long long* prof = nullptr, int64_t ws_bs = 0, int64_t spill_bs = 0,
               int64_t buf_bs = 0, bool serial = false);
// tu_w3i_*.hip: the interleaved W3 (w3i_kernel.hpp), one translation unit per (THETA, KEPT); launch_w3 dispatches to
// them unless serial (SIREN_FLAG_W3_SERIAL A/B, or a phase profile, which only w3_kernel records)
#define SIREN_W3I_DECL(TK)                                                                                             \
    void launch_w3i_##TK(dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy, \
                         const float* u, float* ydot, int o, int64_t n, float* gx, float* spill, float* A, float* At, \
                         float* D, float* Dt, int64_t n_pad, int d, int lh, float w0, float w, const float* kA,         \
                         const float* kC, int64_t ws_bs, int64_t spill_bs, int64_t buf_bs);
SIREN_W3I_DECL(tt)
SIREN_W3I_DECL(tf)
SIREN_W3I_DECL(ft)
SIREN_W3I_DECL(ff)
#undef SIREN_W3I_DECL
void launch_small_w3(dim3 grid, hipStream_t st, const float* At, const float* D, const float* Dt, const float* AL,
                     const float* x, const float* v, const float* gy, const float* u, int64_t n, int64_t n_pad, int64_t tps,
                     float* eslab, int64_t E, int d, int o, int lh, int64_t bstride_act = 0, int64_t bstride_e = 0);
// tu_train.hip
// bstride_act / bstride_part: grouped W2 over batched weights (grid.z of wgrad, grid.y of small / reduce = element)
void launch_wgrad(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, int64_t n_pad, int64_t tps,
                  float* partial, int64_t P, int d, int o, int lh, int with_bias, int h, int jet_bias = 0,
                  int64_t bstride_act = 0, int64_t bstride_part = 0);
// edge-layer launchers (launch_small*): grid (edge splits, hidden / 256, batch), tps = the edge split's tiles,
// eslab / E = the compact edge slabs (siren_capi.hip EdgeSplit), bstride_e = their stride between batch elements
void launch_small(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* gy,
                  int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E, int d, int o, int lh, int h,
                  int64_t bstride_act = 0, int64_t bstride_e = 0);
void launch_reduce(dim3 grid, hipStream_t st, const float* partial, int64_t S, int64_t P, float* gp, int64_t S2,
                   int64_t lo, int64_t hi, int64_t bstride_part = 0, int64_t begin = 0, int64_t end = -1);
void launch_edge_reduce(dim3 grid, hipStream_t st, const float* eslab, int64_t SE, int64_t E, int64_t hidden0,
                        int64_t wout, float* gp, int64_t P, int64_t bstride_e);

// layered.hip: hidden widths other than 256 / 512, layer by layer over coordinate chunks (rocBLAS GEMMs + fused
// epilogues); the packed workspace = [params][W_l^T] (immutable), the chunk scratch is the caller's
constexpr int64_t LAYERED_CHUNK = 16384;
constexpr int LAYERED_RPB = 64;  // rows per workgroup of the bias-reducing epilogues (slab rows = chunk / 64)
enum LayeredMode : int {
    LAY_FWD = 1,    // run the forward sweep
    LAY_Y = 2,      // write y
    LAY_GX = 4,     // vjp_x: gx = sum_j gy_j dPhi_j/dx
    LAY_THETA = 8,  // parameter gradients
    LAY_TWS = 16,   // a_l / cos_l of every layer live in the caller's n x H buffers (stored-forward split)
};
struct LayeredPlan {
    int d, H, lh, o;
    int64_t P, P_pad, chunk, buf, R, wt, scratch, scratch_stored;
    LayeredPlan(int d_, int H_, int lh_, int o_, int64_t n);
};
int64_t layered_ws_floats(int d, int H, int lh, int o);
// chunk scratch of a call over n coordinates (stored: the stored split keeps a_l / cos_l in the caller's n-row buffers)
int64_t layered_scratch_floats(int d, int H, int lh, int o, int64_t n, bool stored);
void layered_pack(const LayeredPlan& plan, const float* params, float* ws, hipStream_t st);
inline int64_t layered_stored_floats(int H, int lh, int64_t n) { return 2 * (int64_t)(lh + 1) * n * H; }
int layered_run(int mode, const LayeredPlan& plan, const float* ws, float w0, float w, const float* x, int64_t n,
                const float* gy, float* y, float* gx, float* gparams, float* tws, float* scr, hipStream_t st,
                std::string& err);

// marching.hip: device marching cubes over an (X, Y, Z) volume; ws in uint32 words
int64_t mc_ws_words(int64_t X, int64_t Y, int64_t Z);
void mc_count(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, uint32_t* ws, hipStream_t st);
const uint32_t* mc_totals(const uint32_t* ws, int64_t X, int64_t Y, int64_t Z, int which);
void mc_emit(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, const float* spacing, const uint32_t* ws,
             float* verts, int32_t* faces, hipStream_t st);

constexpr int STEP_BLOCKS = 1024;  // partial sums of the clip-norm pass (4 workgroups per CU)
// tu_step.hip: device point-cloud sampling (dataio.py:420-442), clip_grad_norm_ + Adam over the flat bucket
void launch_sample_sdf(hipStream_t st, const float* pc, const float* pn, int64_t m, int64_t k, uint64_t seed,
                       uint64_t step, float* coords, float* normals, float* sdf);
void launch_adam(hipStream_t st, float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                 float eps, float bc1, float bc2, float max_norm, float* scratch);

}  // namespace siren
