/*
 * siren_amd.h — C ABI of the MI355X-native SIREN engine (libsiren_amd.so).
 *
 * This is the drop-in boundary for the reference's hot path: the SIREN MLP
 *   z_0 = x W_0^T + b_0,  a_l = sin(w * z_l),  z_l = a_{l-1} W_l^T + b_l,  y = a_L W_out^T + b_out
 * and its coordinate derivatives. In the reference (xvdp/siren, a pure-PyTorch code base with no native
 * code of its own) the path is:
 *   modules.py:16-25   BatchLinear.forward  (matmul, in-place bias add)      -> siren_forward*
 *   modules.py:32-34   Sine.forward         (torch.sin(30 * input))          -> fused epilogue
 *   modules.py:89-94   FCBlock.forward / modules.py:143-160 SingleBVPNet.forward
 *   diff_operators.py:39-43 gradient (torch.autograd.grad, grad_outputs=ones) -> siren_forward_grad (gy = NULL)
 *   autograd backward of the stack (training.py:95-96)                       -> siren_forward_grad (gy given)
 *                                                                               + siren_backward (theta-gradients)
 * There is no reference C ABI to mirror; the reference-side binding is the ctypes module
 * siren_amd/_lib.py.
 *
 * Conventions
 *  - Every entry point returns 0 on success, otherwise a SIREN_E* code; siren_last_error() then returns a
 *    thread-local message. No C++ exception crosses this ABI.
 *  - All buffers are device pointers owned by the caller (PyTorch caching allocator). The fused kernels (hidden
 *    256 / 512) never allocate device memory. The one exception is the layered path of other hidden widths: its
 *    layer GEMMs go through a library-owned rocBLAS handle per device (created on first use), and rocBLAS manages
 *    that handle's own device memory (its internal state and GEMM workspace). fp32, contiguous, row-major:
 *      x (n, d_in); y (n, d_out); gy (n, d_out); gx (n, d_in).
 *  - params is ONE flat fp32 buffer in nn.Linear / state_dict order:
 *      W_0 (H, d_in), b_0 (H), [W_l (H, H), b_l (H)] for l = 1..n_hidden, W_out (d_out, H), b_out (d_out)
 *    i.e. exactly torch.cat([p.flatten() for p in SingleBVPNet.parameters()]).
 *  - Work is enqueued on `stream` (a hipStream_t; pass torch.cuda.current_stream().cuda_stream). Nothing
 *    synchronises the host.
 *  - Weights change every optimizer step, so they are re-packed into the caller's workspace by
 *    siren_pack() once per step (a ~1 us kernel) before any compute entry point is used.
 */
#ifndef SIREN_AMD_H
#define SIREN_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIREN_ABI_VERSION 7

enum {
    SIREN_OK = 0,
    SIREN_EINVAL = 1,       /* bad pointer / size / config value                        */
    SIREN_EUNSUPPORTED = 2, /* valid SIREN config outside what the fused kernels cover  */
    SIREN_EHIP = 3          /* a HIP runtime error (launch failure, ...)               */
};

/* cfg.reserved flags (benchmarking only): run the round-1 kernel whose sin/cos epilogues are not
 * interleaved with the MFMA stream, for in-process A/B timing. */
#define SIREN_FLAG_LEGACY_KERNEL 1
/* cfg.reserved flag (benchmarking only): one workgroup per coordinate tile instead of the persistent grid. */
#define SIREN_FLAG_NO_PERSIST 2
/* cfg.reserved flag (benchmarking only): the round-2 second-order kernel whose epilogues run between the GEMMs
 * (w3_kernel) instead of the interleaved one (w3i_kernel). Same results. */
#define SIREN_FLAG_W3_SERIAL 4
/* cfg.reserved flag (benchmarking only): the round-4 kept Hessian-node backward whose epilogues run between the
 * reverse GEMMs (qf_rev_kernel) instead of the interleaved one (qfi_rev_kernel). Same results. */
#define SIREN_FLAG_QF_SERIAL 8
/* cfg.reserved flag (benchmarking only): the hidden-512 stored-forward split on the round-2 kernel whose epilogues
 * run between the GEMMs (wide_kernel) instead of the interleaved one (widei_kernel). Same results. */
#define SIREN_FLAG_WIDE_SERIAL 16

/* Network description. Mirrors SingleBVPNet(out_features, type='sine', in_features, mode='mlp',
 * hidden_features, num_hidden_layers) (modules.py:122-123) and the notebook Siren(in_features,
 * hidden_features, hidden_layers, out_features, outermost_linear, first_omega_0, hidden_omega_0). */
typedef struct siren_cfg {
    int32_t d_in;             /* in_features, 1..4                                         */
    int32_t hidden;           /* hidden_features: 256 or 512 in the fused kernels          */
    int32_t n_hidden;         /* num_hidden_layers: H->H layers between first and last    */
    int32_t d_out;            /* out_features, 1..4                                        */
    float omega_first;        /* w of the first sine layer (30; Sine hard-codes 30)        */
    float omega_hidden;       /* w of the hidden sine layers (30)                          */
    int32_t outermost_linear; /* 1: last layer linear (SingleBVPNet); 0: sin(w*z) as well  */
    int32_t reserved;         /* flags: 0 for normal use; SIREN_FLAG_LEGACY_KERNEL = A/B   */
} siren_cfg;

/* Library ABI version (== SIREN_ABI_VERSION). */
int32_t siren_abi_version(void);

/* Message for the last failing call on this thread ("" if none). */
const char* siren_last_error(void);

/* Number of fp32 values in the flat parameter buffer. */
int32_t siren_param_count(const siren_cfg* cfg, int64_t* count);

/* Number of fp32 values of packed-weight workspace that siren_pack() fills. ws is immutable between packs: no entry
 * point writes it, so one ws may serve calls on several streams. Hidden widths other than 256 / 512 (the layered
 * path: rocBLAS layer GEMMs + HIP epilogues over 16384-coordinate chunks) hold the parameters and W_l^T; their chunk
 * scratch is the caller's tws of each entry point (siren_forward_ws_floats, siren_forward_grad_ws_floats,
 * siren_train_ws_floats, siren_train_stored_ws_floats). */
int32_t siren_workspace_floats(const siren_cfg* cfg, int64_t* count);

/* Repack params into the kernels' LDS-slice layout (workspace ws, siren_workspace_floats() floats). */
int32_t siren_pack(const siren_cfg* cfg, const float* params, float* ws, void* stream);

/* W0 (forward value): y = Phi(x). Replaces SingleBVPNet.forward's model_out (modules.py:143-160).
 * Hidden widths other than 256 / 512 (the layered path) need the caller's chunk scratch: siren_forward_ex with
 * tws of siren_forward_ws_floats(cfg, n) floats (0 elsewhere; siren_forward = siren_forward_ex with tws NULL, which
 * fails with SIREN_EINVAL on a layered network). ABI 5: the packed workspace ws is never written by any call. */
int32_t siren_forward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y,
                      void* stream);
int32_t siren_forward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);
int32_t siren_forward_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, float* tws,
                         void* stream);

/* W1 (forward + coordinate vector-Jacobian product) in ONE launch:
 *   y  = Phi(x)                       (skipped when y == NULL)
 *   gx = sum_j gy_j * dPhi_j/dx       (gy == NULL means gy = ones: diff_operators.gradient, d.o.py:39-43)
 * hidden 256: n_hidden 1..3 keeps cos(w z_l) of every layer in registers (ONE launch; tws may be NULL); 4..5 (linear
 * output, nonzero omegas) runs the stored split's forward half (y + lane-major cos of every layer into tws) and its
 * reverse half (two launches); hidden 512: 1..8 (cos is spilled to tws). tws: siren_forward_grad_ws_floats(cfg, n)
 * floats (0 for hidden 256 with 1..3 hidden layers). */
int32_t siren_forward_grad_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);
int32_t siren_forward_grad(const siren_cfg* cfg, const float* ws, const float* x, int64_t n,
                           const float* gy, float* y, float* gx, float* tws, void* stream);

/* W4 (the fused Laplacian) in ONE launch, forward-mode Taylor jet:
 *   y   (n, d_out)  = Phi(x)                       (skipped when y == NULL)
 *   gx  (n, d_in)   = sum_j dPhi_j/dx              (diff_operators.gradient; skipped when gx == NULL)
 *   lap (n)         = sum_j sum_i d2Phi_j/dx_i2    (diff_operators.laplace, diff_operators.py:27-36)
 * hidden 256, d_in <= 2, linear output layer, n_hidden 1..5. Replaces the d + 1 autograd sweeps that
 * laplace() records (gradient, then one create_graph grad per input dimension). */
int32_t siren_forward_laplace(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y,
                              float* gx, float* lap, void* stream);

/* fp32 values of backward workspace siren_backward() needs for n coordinates (sin activations and deltas of
 * every sine layer, plus the split-K partial gradient slabs; hidden 256 with 4..5 hidden layers: + the stored split's
 * cos buffer, siren_backward then runs siren_forward_store + siren_backward_stored internally). */
int32_t siren_train_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);

/* W2 backward for one coordinate batch: given gy = dL/dy (n, d_out), writes
 *   gx (n, d_in)             = dL/dx                       (model_in.grad, training.py:96)
 *   gparams (param_count)    = dL/dtheta in flat param order (BatchLinear weight/bias .grad)
 * Stages: the fused forward + reverse kernel in store mode, the split-K MFMA weight-gradient kernel and a
 * deterministic slab reduction (no atomics: bitwise reproducible). `reserved` must be NULL.
 * Replaces autograd's MmBackward/SinBackward/MulBackward chain of train_loss.backward() (training.py:95-96). */
int32_t siren_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy,
                       float* tws, void* reserved, float* gx, float* gparams, void* stream);

/* fp32 values of workspace siren_laplace_backward() needs for n coordinates (a-, z- and cotangent jets of every
 * sine layer as 16-column tiles, plus the split-K partial slabs). */
int32_t siren_laplace_backward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);

/* W4s, the backward of the fused Laplacian (laplace_mse training, loss_functions.py:104-109): with glap (n) the
 * cotangent of lap = siren_forward_laplace's output,
 *   gx (n, d_in)          = d/dx sum_c glap_c lap(x_c)
 *   gparams (param_count) = d/dtheta sum_c glap_c lap(x_c)
 * The reverse of the forward-mode jet (same 4 coordinates x 4 streams MFMA columns), then the split-K MFMA
 * weight-gradient kernel over K = 4n columns and a deterministic slab reduction. Same coverage as
 * siren_forward_laplace. Replaces autograd's third-order sweep through laplace()'s graph (training.py:95-96). */
int32_t siren_laplace_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n,
                               const float* glap, float* tws, float* gx, float* gparams, void* stream);

/* fp32 values of workspace siren_second_order() needs (per-layer spill, and with want_theta the tangent /
 * primal activations and adjoints of every layer plus 2*S partial slabs). */
int32_t siren_second_order_ws_floats(const siren_cfg* cfg, int64_t n, int32_t want_theta, int64_t* count);

/* W3, second-order adjoint for hidden 256, d_out <= 4, linear output (the backward of the dPhi/dx graph node that gradients_mse / sdf /
 * divergence differentiate, diff_operators.py:27-43, loss_functions.py:84-89, 214-238): with v (n, d_in) the
 * cotangent of J = dPhi/dx,
 *   gx (n, d_in)          = H(x) v                      (Hessian-vector product)
 *   gparams (param_count) = d/dtheta sum_c <v_c, J(x_c)> (skipped when gparams == NULL)
 * (J = sum_j dPhi_j/dx, what diff_operators.gradient records for a vector output; see siren_second_order_ex)
 * Forward primal+tangent sweep and reverse sweep in one kernel (per-layer state spilled to tws), then the split-K
 * MFMA weight-gradient kernel over K = 2n and a deterministic slab reduction. */
int32_t siren_second_order(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                           float* tws, float* gx, float* gparams, void* stream);

/* W3 with a first-order seed: the gradient of sum_c gy_c y_c + <v_c, J(x_c)> in ONE sweep (gy (n) nullable; NULL is
 * siren_second_order). This is the backward autograd runs when a loss uses both the value and the gradient of the
 * network (loss_functions.py:214-238 sdf: sdf/inter terms on model_out, normal/eikonal terms on gradient()), which
 * the reference evaluates as two separate backward sweeps through training.py:96. Same workspace as
 * siren_second_order. */
int32_t siren_second_order_seeded(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                                  const float* gy, float* tws, float* gx, float* gparams, void* stream);

/* W3 for vector outputs (diff_operators.jacobian / hessian, diff_operators.py:5-24, 46-59; the helmholtz_pml /
 * wave_pml losses, loss_functions.py:112-211): the backward of the vjp node gx = J^T u, with per-coordinate output
 * weighting u (n, d_out) (NULL = ones), first-order seed gy (n, d_out) (NULL = none) and v (n, d_in) the cotangent
 * of gx:
 *   gx (n, d_in)          = d/dx     F,   F = sum_c gy_c . y_c + <v_c, J(x_c)^T u_c>
 *   gparams (param_count) = d/dtheta F    (skipped when gparams == NULL)
 *   ydot (n, d_out)       = J(x_c) v_c = dF/du_c (skipped when ydot == NULL)
 * One W3 sweep; siren_second_order / _seeded are this entry with u = ydot = NULL. Same workspace. */
int32_t siren_second_order_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                              const float* u, const float* gy, float* tws, float* gx, float* gparams, float* ydot,
                              void* stream);

/* Third-order adjoint: the backward of the Hessian-vector-product node h = sum_j u_j H_j(x) v (the node that
 * diff_operators.divergence(gradient(y, x), x) records per input dimension, diff_operators.py:27-36, and that the
 * second jacobian() of helmholtz_pml / wave_pml records, loss_functions.py:112-211). With g (n, d_in) the cotangent
 * of h, S = sum_c <g_c, h_c> = sum_c sum_j u_cj D2 Phi_j(x_c)[v_c, g_c]:
 *   gx (n, d_in)          = dS/dx
 *   gparams (param_count) = dS/dtheta                       (skipped when NULL)
 *   gv (n, d_in)          = dS/dv = sum_j u_j H_j g           (skipped when NULL)
 *   gu (n, d_out)         = dS/du_j = g^T H_j v              (skipped when NULL)
 * v (n, d_in), u (n, d_out) (NULL = ones). One forward-mode jet along (v, g) + its reverse (4 coordinates x 4 streams
 * per MFMA tile), then the split-K MFMA weight-gradient over 4n columns and a deterministic slab reduction. Hidden
 * 256, linear output, 1..5 hidden layers, d_in / d_out <= 4. tws: siren_hvp_backward_ws_floats(cfg, n) floats. */
int32_t siren_hvp_backward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);
int32_t siren_hvp_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                           const float* u, const float* g, float* tws, float* gx, float* gparams, float* gv,
                           float* gu, void* stream);

/* The backward of a Hessian node Hm (n, d_in, d_in) = sum_j u_j H_j(x) (u (n, d_out), NULL = ones): the node that
 * every divergence() / hessian() column of one gradient node reads (diff_operators.py:5-36), so autograd sums the
 * cotangents of all those columns into ONE G (n, d_in, d_in) and the whole third-order backward of laplace_mse through
 * the reference's divergence(gradient()) (loss_functions.py:104-109) is one call. With S = sum_c <G_c, Hm_c>
 * = sum_c sum_j u_cj D2 Phi_j(x_c)[Q_c], Q = sym(G):
 *   gx (n, d_in)          = dS/dx
 *   gparams (param_count) = dS/dtheta                      (skipped when NULL)
 *   gu (n, d_out)         = dS/du_j = D2 Phi_j[Q]          (skipped when NULL)
 * One forward-mode jet (value, d/dx_1, d/dx_2, the second-order stream along Q) + its reverse (4 coordinates x 4
 * streams per MFMA tile), the split-K MFMA weight gradient over 4n columns and a deterministic slab reduction. Hidden
 * 256, linear output, 1..5 hidden layers, d_in <= 2. tws: siren_hessian_backward_ws_floats(cfg, n) floats. */
int32_t siren_hessian_backward_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);
int32_t siren_hessian_backward(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* G,
                               const float* u, float* tws, float* gx, float* gparams, float* gu, void* stream);

/* The Hessian node's forward, Hm (n, d_in, d_in) = sum_j u_j H_j(x) (u (n, d_out), NULL = ones) — what each
 * divergence() / hessian() column of the reference reads (diff_operators.py:5-36: autograd.grad of one gradient
 * column per input dimension) — in ONE forward-mode second-order jet sweep over the coordinate axes (value, 2
 * tangents, 3 second-order streams; 8 coordinates x 6 streams in three MFMA tiles, no reverse sweep). kept (nullable,
 * siren_hessian_ws_floats(cfg, n, 1, &count) floats; caller-owned, 0 floats with keep = 0) receives the per-layer
 * jets of hidden layers 1..L (layer 0 is rebuilt from x): siren_hessian_backward_kept with the same kept then skips
 * the forward GEMMs of its quadratic-form jet. Same
 * coverage as siren_hessian_backward. */
int32_t siren_hessian_ws_floats(const siren_cfg* cfg, int64_t n, int32_t keep, int64_t* count);
int32_t siren_hessian(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* u, float* kept,
                      float* hm, void* stream);
/* siren_hessian that also returns, from the same sweep (its value and first-order streams), y (n, d_out) = Phi(x)
 * and gx (n, d_in) = sum_j u_j dPhi_j/dx — what siren_forward_grad gives — each nullable (ABI 6). A training step of
 * the reference's laplace_mse recipe (model(x), gradient(), divergence()) then needs one forward sweep, not two. */
int32_t siren_hessian_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* u, float* kept,
                         float* hm, float* y, float* gx, void* stream);
/* siren_hessian_backward reading its forward jets from a siren_hessian kept buffer of the same (ws, x, n) (kept
 * NULL: recompute, = siren_hessian_backward). */
int32_t siren_hessian_backward_kept(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* G,
                                    const float* u, const float* kept, float* tws, float* gx, float* gparams,
                                    float* gu, void* stream);

/* Split-bf16 W1 (precision mode "bf16x6"): siren_forward_grad with gy = ones for the headline network (hidden 256,
 * 3 hidden layers, d_in 2 / 3, d_out 1, linear output) with the layer GEMMs on the bf16 matrix pipe. Every fp32
 * weight and activation is split exactly into three bf16 pieces (hi + mid + lo) and each K-step sums the six products
 * down to 2^-16 of the leading one, accumulated in fp32: the error against the fp64 reference is that of the fp32
 * kernel. siren_pack_split fills wsx (siren_split_ws_floats floats) from the flat parameters, once
 * per weight update; siren_forward_grad_split replaces siren_forward_grad(cfg, ws, x, n, NULL, y, gx, NULL, stream)
 * (diff_operators.gradient, diff_operators.py:39-43; y nullable). */
int32_t siren_split_ws_floats(const siren_cfg* cfg, int64_t* count);
int32_t siren_pack_split(const siren_cfg* cfg, const float* params, float* wsx, void* stream);
int32_t siren_forward_grad_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, float* y,
                                 float* gx, void* stream);
/* The forward-only W0 (model_out, SingleBVPNet.forward modules.py:143-160) on the same split image: the forward GEMMs
 * only, two waves per SIMD sharing one weight ring (dense evaluation: sdf_meshing.create_mesh, summaries). */
int32_t siren_forward_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, float* y, void* stream);
/* The training backward of the bf16x6 leg (precision='bf16x6' under a parameter-gradient graph: the image-fit W2 unit
 * with siren_forward_split as its forward): the split-bf16 kernel recomputes the forward, runs the reverse seeded with
 * gy (n) and writes a_l / delta_l tiles, then the fp32 split-K MFMA wgrad, edge layers and slab reduction of
 * siren_backward. Replaces siren_backward(cfg, ws, x, n, gy, tws, NULL, gx, gparams, stream) for the networks
 * siren_forward_grad_split covers; gx (n, d_in) nullable; tws: siren_train_ws_floats(cfg, n) floats. */
int32_t siren_backward_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, const float* gy,
                             float* tws, float* gx, float* gparams, void* stream);
/* The stored-forward form of the same unit (what SirenSplitFunction runs): siren_forward_store_split is
 * siren_forward_split plus the a_l tiles and cos(w z_l) into tws; siren_backward_stored_split runs the reverse GEMMs
 * only from them (delta_l tiles), then the bf16x6 wgrad, edge layers and slab reduction. tws:
 * siren_train_split_ws_floats(cfg, n) floats, passed unchanged from the forward to the backward. */
int32_t siren_train_split_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);
int32_t siren_forward_store_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, float* y,
                                  float* tws, void* stream);
int32_t siren_backward_stored_split(const siren_cfg* cfg, const float* wsx, const float* x, int64_t n, const float* gy,
                                    float* tws, float* gx, float* gparams, void* stream);

/* Diagnostics: the W1 kernel (hidden 256, 3 hidden layers) with s_memtime stamps. stamps receives
 * 256 workgroups x 4 tiles x 4 waves x 8 events (uint64; event 0 tile start, 1..6 after GEMM 0..5, 7 tile end);
 * unrecorded entries are left untouched. y / gx as siren_forward_grad with gy = ones. */
int32_t siren_w1_phase_profile(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, float* gx,
                               uint64_t* stamps, void* stream);
/* Diagnostics: while stamps is non-NULL, every W3 (siren_second_order*) launch records s_memtime stamps of wave 0 of
 * workgroups 0..255 after each phase (start, layer 0, forward GEMM / epilogue per layer, seed, reverse GEMM / epilogue
 * per layer, end) into stamps[256][16] (device memory); NULL switches it off. */
int32_t siren_w3_phase_profile(uint64_t* stamps);

/* ---- per-step kernels around the network ---------------------------------------------
 * Device-side dataio.PointCloud.__getitem__ (dataio.py:420-442): from a resident point cloud pc_coords /
 * pc_normals (m, 3), write 2k samples: rows [0, k) = k on-surface points drawn uniformly with replacement (coords,
 * normals, sdf 0), rows [k, 2k) = k off-surface points uniform in [-1, 1)^3 (normals -1, sdf -1). coords, normals
 * (2k, 3), sdf (2k, 1). A counter RNG of (seed, step, row) (step_kernels.hpp) replaces np.random: reproducible
 * for a given (seed, step), nothing crosses PCIe (training.py:53-54). */
int32_t siren_sample_sdf(const float* pc_coords, const float* pc_normals, int64_t m, int64_t k, uint64_t seed,
                         uint64_t step, float* coords, float* normals, float* sdf, void* stream);

/* fp32 values of device scratch siren_adam_step needs when clipping (per-block norm partials + the norm). */
int32_t siren_adam_scratch_floats(int64_t* count);

/* torch.nn.utils.clip_grad_norm_(max_norm) + torch.optim.Adam.step (training.py:17, 98-104; amsgrad off, no weight
 * decay) over ONE flat fp32 bucket of n parameters: c = min(1, max_norm / (||g|| + 1e-6)) (no clip when
 * max_norm <= 0), m = b1 m + (1 - b1) c g, v = b2 v + (1 - b2) (c g)^2, p -= lr / (1 - b1^step) * m /
 * (sqrt(v / (1 - b2^step)) + eps). step >= 1 is Adam's step count after this update. The global norm stays on the
 * device (scratch[1024] receives it); buffers 16-byte aligned. */
int32_t siren_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
                        float beta1, float beta2, float eps, int64_t step, float max_norm, float* scratch,
                        void* stream);

/* ---- surface extraction: device marching cubes ------------------------------------------
 * Replaces skimage.measure.marching_cubes_lewiner in convert_sdf_samples_to_ply (sdf_meshing.py:97-102) on the
 * (X, Y, Z) fp32 volume create_mesh evaluated (row-major, axis 0 slowest; sdf_meshing.py:24-59). Cube-case
 * marching cubes (table derived by tools/gen_mc_table.py: inside = value < level, inside corners separated on
 * ambiguous faces, no triangle chord along a cube face), vertices welded per grid edge at the linear zero crossing,
 * in index units * spacing, faces wound so normals point towards increasing value. Two calls: siren_mc_count
 * (classification + scans; synchronises the stream to return the sizes), then siren_mc_emit into caller buffers
 * verts (n_verts, 3) fp32 and faces (n_faces, 3) int32; spacing3 is a HOST pointer to 3 floats. ws:
 * siren_mc_ws_bytes, 4-byte aligned, kept between the two calls. X * Y * Z < 2^32, X, Y <= 65535, fewer than 2^31
 * vertices and triangles (siren_mc_count returns SIREN_EUNSUPPORTED otherwise); volumes
 * with an axis < 2 give an empty mesh. */
int32_t siren_mc_ws_bytes(int64_t X, int64_t Y, int64_t Z, int64_t* bytes);
int32_t siren_mc_count(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, void* ws, int64_t* n_verts,
                       int64_t* n_faces, void* stream);
int32_t siren_mc_emit(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, const float* spacing3,
                      const void* ws, float* verts, int32_t* faces, void* stream);

/* ---- batched (hypernetwork) weights ----------------------------------------------------
 * BatchLinear with per-element weights W (B, out, in), b (B, out) (modules.py:16-25; HyperNetwork.forward,
 * meta_modules.py:41-53) applied to coords (B, n, d_in). Element b reads params + b * param_count (state-dict
 * order, as siren_pack), ws + b * workspace_floats, x + b * n * d_in, and writes y + b * n * d_out, gx + b * n * d_in,
 * gparams + b * param_count. batch <= 65535. */
/* siren_pack_batched fills what the first-order batched entry points read: for a linear-output hidden-256 network
 * only the phase-scaled half of each element's workspace. siren_pack_batched_ex with full = 1 writes every element's
 * whole image (what siren_pack writes): required by siren_second_order_batched / siren_hvp_backward_batched and by
 * any single-network entry point handed one element's workspace; full = 0 is siren_pack_batched. */
int32_t siren_pack_batched(const siren_cfg* cfg, const float* params, int64_t batch, float* ws, void* stream);
int32_t siren_pack_batched_ex(const siren_cfg* cfg, const float* params, int64_t batch, float* ws, int32_t full,
                              void* stream);
/* Second and third order over batched weights: the backward of a hypernetwork hypo-network's gradient node
 * (gradients_mse / divergence(gradient()) on SingleBVPNet(params=...), loss_functions.py:84-109 through
 * meta_modules.py:81-92). Element b runs siren_second_order_ex / siren_hvp_backward on ws + b * workspace_floats
 * (packed with full = 1), x / v / g / gx / gv + b * n * d_in, u / gy / ydot / gu + b * n * d_out,
 * gparams + b * param_count (nullable outputs as there). tws: the *_batched_ws_floats count, reused element after
 * element in stream order. */
int32_t siren_second_order_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int32_t want_theta,
                                             int64_t* count);
int32_t siren_second_order_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                   const float* v, const float* u, const float* gy, float* tws, float* gx,
                                   float* gparams, float* ydot, void* stream);
int32_t siren_hvp_backward_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int64_t* count);
int32_t siren_hvp_backward_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                   const float* v, const float* u, const float* g, float* tws, float* gx,
                                   float* gparams, float* gv, float* gu, void* stream);
/* W0 for every element in ONE grouped launch (grid.y = element) at hidden 256, linear output, 1..5 hidden layers;
 * other configurations run siren_forward element by element. */
int32_t siren_forward_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                              float* y, void* stream);
/* the same with the per-element workspace of siren_forward_ex (siren_forward_ws_floats(cfg, n); reused element
 * after element; needed at layered widths only) */
int32_t siren_forward_batched_ex(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                 float* y, float* tws, void* stream);
/* W1 (y, J^T gy) for every element in ONE grouped launch (hidden 256, linear output, 1..3 hidden layers; the
 * persistent grid is split across the elements); gy (B, n, d_out) nullable = ones. tws: the per-element workspace of
 * siren_forward_grad (siren_forward_grad_ws_floats(cfg, n); reused element after element, NULL at hidden 256). */
int32_t siren_forward_grad_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                   const float* gy, float* y, float* gx, float* tws, void* stream);
/* W2 per element (the hypernetwork needs each element's theta-gradient). Hidden 256 with elements below two CU
 * rounds of tiles: ONE grouped launch per stage (fused store, wgrad, edge layers, slab reduction; grid over the
 * elements); otherwise siren_backward element by element. tws: siren_train_batched_ws_floats(cfg, n, batch). */
int32_t siren_train_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int64_t* count);
int32_t siren_backward_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                               const float* gy, float* tws, float* gx, float* gparams, void* stream);

/* Stored-forward W2 split over batched weights (SirenBatchedFunction's training forward under a hypernetwork): the
 * forward keeps every element's a_l tiles and cos(w z_l), the backward (the hypernetwork's theta-gradients) is the
 * reverse sweep only. Hidden 256 with elements below two CU rounds: ONE grouped launch per stage; otherwise the
 * single-network entry points element by element. tws: siren_train_stored_batched_ws_floats(cfg, n, batch) floats,
 * kept from the forward to the backward. */
int32_t siren_train_stored_batched_ws_floats(const siren_cfg* cfg, int64_t n, int64_t batch, int64_t* count);
int32_t siren_forward_store_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                    float* y, float* tws, void* stream);
int32_t siren_backward_stored_batched(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, int64_t batch,
                                      const float* gy, float* tws, float* gx, float* gparams, void* stream);

/* ---- stored-forward W2 split (linear output; hidden 256: 1..5 hidden layers, hidden 512: 1..8) --------------
 * The training forward (model(model_input), training.py:72) keeps what the backward needs, so
 * train_loss.backward() (training.py:96) runs the L reverse GEMMs only instead of recomputing the forward:
 *   siren_forward_store : W0 (y, nullable at hidden 256) + a_l tiles and cos(w z_l) of every sine layer into tws
 *   siren_backward_stored: reverse sweep from the stored cos + split-K MFMA wgrad + edge layers + slab reduction,
 *                          same outputs as siren_backward (gx, gparams); tws must hold siren_forward_store's output
 * tws: siren_train_stored_ws_floats(cfg, n) floats (siren_train_ws_floats + the cos buffer). */
int32_t siren_train_stored_ws_floats(const siren_cfg* cfg, int64_t n, int64_t* count);
int32_t siren_forward_store(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y, float* tws,
                            void* stream);
int32_t siren_backward_stored(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* gy,
                              float* tws, float* gx, float* gparams, void* stream);

/* Stored jet forward for gradient losses (hidden 256): y and J = sum_j dPhi_j/dx (siren_forward_grad's outputs with
 * gy = ones) as siren_forward_store + a reverse-only sweep from the stored cos, leaving a_l / cos in tws
 * (siren_train_stored_ws_floats) for siren_second_order_kept. */
int32_t siren_forward_grad_store(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y,
                                 float* gx, float* tws, void* stream);
/* siren_second_order_seeded from a stored forward (kept = siren_forward_grad_store's / siren_forward_store's tws):
 * the hidden layers run the tangent GEMMs only (the primal a_l and cos come from kept). tws as siren_second_order. */
int32_t siren_second_order_kept(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, const float* v,
                                const float* gy, float* kept, float* tws, float* gx, float* gparams, void* stream);

/* Split W4 / W4s (laplace_mse training): siren_forward_laplace's outputs (y / gx / lap, y and gx nullable) from the
 * forward jet sweep that also keeps the a-jets and z-jets in tws (siren_laplace_backward_ws_floats), then
 * siren_laplace_backward's outputs from the seed + reverse sweep over those stores (no forward recompute). */
int32_t siren_forward_laplace_store(const siren_cfg* cfg, const float* ws, const float* x, int64_t n, float* y,
                                    float* gx, float* lap, float* tws, void* stream);
int32_t siren_laplace_backward_stored(const siren_cfg* cfg, const float* ws, const float* x, int64_t n,
                                      const float* glap, float* tws, float* gx, float* gparams, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SIREN_AMD_H */
