"""Autograd Functions that put the HIP kernels under the reference's autograd contract.

The reference never calls its model's derivatives directly: losses call torch.autograd.grad(model_out,
model_in, ones, create_graph=True) (diff_operators.py:42, :35) and training calls train_loss.backward()
(training.py:96). So the fused kernels sit behind torch.autograd.Function nodes:

  SirenFunction      y = Phi(x; theta)                        forward: W0 kernel
    .backward(gy)    no create_graph: gx via the W1 kernel, (gx, gtheta) via the W2 pipeline (fused reverse
                     sweep + split-K MFMA weight-gradient + slab reduction)
                     create_graph:    differentiable gx through a SirenVJP node
  SirenJetFunction   (y, J = dPhi/dx) from ONE W1 launch as ONE two-output node ("jet" mode, d_out == 1); its
    .backward(gy, gJ) gets the value and gradient cotangents together: the seeded W3 kernel returns the gradient
                     of sum gy*y + <gJ, J> in one sweep (sdf training); create_graph: gy*J + SirenHVP(gJ)
  SirenVJP           gx = J^T gy computed by the W1 kernel as a graph node
  SirenLaplace       the fused Laplacian (W4 jet kernel) and its W4s backward

Which gradients autograd actually wants is read from the engine (torch._C._will_engine_execute_node on the
next nodes), because ctx.needs_input_grad is static: autograd.grad(y, [x]) must not pay for weight gradients.

Second-order adjoints (SirenJetFunction/SirenVJP.backward: gradients_mse / sdf training, the Laplacian's
Hessian-vector products) run on the W3 kernel (siren_second_order[_seeded]) for hidden 256 and
d_out <= 4 (vector outputs through an output weighting u: jacobian / hessian, helmholtz_pml / wave_pml).
laplace_mse training runs the W4s kernels (SirenLaplace). Only theta-gradients under create_graph (meta-learning),
third derivatives through a SirenHVP node (an unfused divergence(), the PML losses' training backward) and second
order at hidden 512 are recomputed through siren_amd._torch_path with device torch ops.
"""
import torch

from . import _torch_path


# SirenFunction under a parameter-gradient graph stores the forward for a reverse-only backward;
# False keeps the recompute-in-backward pipeline (A/B timing, tests)
STORED_FORWARD = True


def _will_execute(ctx, i):
    """Does the autograd engine need the gradient of tensor input i (in forward-argument order of tensors)?"""
    try:
        node = ctx.next_functions[i][0]
    except (AttributeError, IndexError):
        return True
    if node is None:
        return False
    try:
        return bool(torch._C._will_engine_execute_node(node))
    except Exception:  # private API absent/changed: compute everything the inputs allow
        return True


class JetState:
    """Per-module switch for jet mode ('auto' turns it on after the first create_graph x-gradient request). hessian:
    a Hessian node was built from this module's jet node (divergence() / hessian() of its gradient: the reference's
    laplace_mse recipe); from then on the jet forward is the Hessian node's own sweep (siren_hessian_ex: y, dPhi/dx,
    the Hessian and its kept jets at once) and the node reuses it instead of running a second forward."""

    # The speculative modes are tracked per call site, keyed by the flattened coordinate shape (n, d): a module called
    # twice per step on batches of different sizes (e.g. a training and a validation batch) whose Hessian / Laplacian
    # is requested of one call only keeps speculating for that call and not for the other (one shared cell made the
    # unconsumed call switch the mode off and the consuming call's request switch it on again every step, so each
    # step paid one wasted sweep). Calls of the SAME shape share a key (the cell then tracks the most recent one).
    # A module called once per step on batches whose size changes every step (ragged point counts) never meets its
    # recorded key again, so it does not speculate: it runs the plain forward plus the Hessian / Laplacian sweep (the
    # same results, one more launch per step). Telling that call apart from a second call site of another shape needs
    # a step boundary the module does not see (a shape-agnostic fallback made two call sites of different shapes
    # take the record from each other every step).
    MAX_KEYS = 16  # distinct call shapes tracked per module (the oldest is dropped beyond that, with its cell)

    def __init__(self, mode='auto'):
        self.mode = mode
        self.active = mode is True
        self._hessian = {}  # key -> a Hessian node was built from this call's jet node
        self._laplace = {}  # key -> likewise for the fused diff_operators.laplace of the value node (W4 jet sweep)
        self._unused = {}   # key -> [bool]: the last speculative sweep's results were not (yet) consumed

    @staticmethod
    def key(x):
        return tuple(x.shape)

    def hessian(self, key):
        return self._hessian.get(key, False)

    def laplace(self, key):
        return self._laplace.get(key, False)

    def speculate(self, key):
        """Called by a forward about to run a speculative sweep for call key: if the previous one of this key was never
        consumed (the loss stopped asking for the Hessian / Laplacian), switch the key's modes off — a later request
        turns them on again. Returns the flag cell for this forward's node (set to False when its results are
        consumed)."""
        cell = self._unused.pop(key, None)
        if cell is not None and cell[0]:
            self._hessian.pop(key, None)
            self._laplace.pop(key, None)
            return None
        cell = [True]
        self._unused[key] = cell
        return cell

    def _remember(self, table, key):
        table[key] = True
        while len(table) > self.MAX_KEYS:
            old = next(iter(table))
            table.pop(old)
            if old not in self._hessian and old not in self._laplace:
                self._unused.pop(old, None)

    def observe_x_gradient_request(self):
        if self.mode == 'auto':
            self.active = True

    def observe_hessian_request(self, key):
        if self.mode in ('auto', True):
            self._remember(self._hessian, key)

    def observe_laplace_request(self, key):
        if self.mode in ('auto', True):
            self._remember(self._laplace, key)


class SirenFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, jet, x, flat, store=False):
        ws = engine.pack(flat)
        ctx.tws, ctx.pre_laplace = None, None
        # (jet is None unless a graph is being recorded — modules._fused_apply — so a no_grad evaluation after
        # laplace training, e.g. summaries or create_mesh, keeps the plain forward)
        key = JetState.key(x)
        ctx.spec = (jet.speculate(key) if (jet is not None and jet.laplace(key) and engine.laplace_supported)
                    else None)
        if ctx.spec is not None:
            # this module's output went to diff_operators.laplace last time (laplace_mse): the value comes from the
            # W4 jet sweep that laplace() needs anyway, and its Laplacian (+ kept jet stores) wait on this node for
            # fused_laplace — one forward sweep instead of a stored W1 forward AND the jet
            if store and STORED_FORWARD:
                lap, ltws, y = engine.forward_laplace_store(ws, x, want_y=True)
            else:
                y, _, lap = engine.forward_laplace(ws, x)
                ltws = None
            ctx.pre_laplace = (lap, ltws)
        elif store and engine.stored_for(x.shape[0]) and STORED_FORWARD:
            # training forward: keep a_l / cos(w z_l) so the weight-gradient backward is reverse-only
            y, ctx.tws = engine.forward_store(ws, x)
        else:
            y = engine.forward(ws, x)
        ctx.engine, ctx.jet, ctx.ws = engine, jet, ws
        ctx.save_for_backward(x, flat)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, flat = ctx.saved_tensors
        engine, ws = ctx.engine, ctx.ws
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 0)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 1)
        gx = gp = None
        gy = gy.contiguous()
        if not torch.is_grad_enabled():
            if need_p:
                if ctx.tws is not None:
                    gx, gp = engine.backward_stored(ws, x, gy, ctx.tws)
                else:
                    gx, gp = engine.backward_params(ws, x, gy)
                if not need_x:
                    gx = None
            elif need_x:
                _, gx = engine.forward_grad(ws, x, gy, want_y=False)
            return None, None, gx, gp, None
        # create_graph=True: results must be differentiable functions of (x, theta, gy)
        if need_x:
            if ctx.jet is not None and not need_p:
                ctx.jet.observe_x_gradient_request()
            gx = SirenVJP.apply(engine, ws, x, flat, gy)
        if need_p:
            gp = _torch_path.vjp_params(engine.cfg, x, flat, gy, create_graph=True)
        return None, None, gx, gp, None


class SirenSplitFunction(torch.autograd.Function):
    """precision 'bf16x6' under a parameter-gradient graph (the image-fit training step): the stored
    split on the split-bf16 kernels — the forward (siren_forward_store_split) keeps a_l and cos(w z_l), the parameter
    backward (siren_backward_stored_split) runs the reverse GEMMs only and reduces the θ-gradients with the bf16x6
    wgrad. An x-only or create_graph backward runs on the fp32 kernels (the split kernels are first order)."""

    @staticmethod
    def forward(ctx, engine, jet, x, flat):
        wsx = engine.pack_split(flat)
        # the stored split: the forward keeps a_l / cos(w z_l), the parameter backward is reverse-only
        y, ctx.tws = engine.forward_store_split(wsx, x)
        # the fp32 image is packed only when a derivative of y needs it (diff_operators.gradient / laplace through
        # siren_node_of, an x-only or create_graph backward: the fp32 kernels, _node_ws); the parameter backward of the
        # image-fit step never does
        ctx.engine, ctx.jet, ctx.wsx, ctx.ws = engine, jet, wsx, None
        ctx.save_for_backward(x, flat)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, flat = ctx.saved_tensors
        engine = ctx.engine
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 0)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 1)
        gx = gp = None
        gy = gy.contiguous()
        if not torch.is_grad_enabled():
            if need_p:
                gx, gp = engine.backward_stored_split(ctx.wsx, x, gy, ctx.tws, want_gx=need_x)
            elif need_x:
                _, gx = engine.forward_grad(_node_ws(ctx), x, gy, want_y=False)
            return None, None, gx, gp
        ws = _node_ws(ctx)
        if need_x:
            if ctx.jet is not None and not need_p:
                ctx.jet.observe_x_gradient_request()
            gx = SirenVJP.apply(engine, ws, x, flat, gy)
        if need_p:
            gp = _torch_path.vjp_params(engine.cfg, x, flat, gy, create_graph=True)
        return None, None, gx, gp


class SirenJetFunction(torch.autograd.Function):
    """(y, J) = (Phi(x; theta), dPhi/dx) for d_out == 1 from ONE W1 launch, as ONE graph node with two outputs.

    The module returns y; J stays an output of the node and is what diff_operators.gradient's create_graph
    backward hands out (gx = gy * J). Because y and J belong to the same node, a loss that uses both the value and
    the gradient (sdf: loss_functions.py:214-238) reaches this node's backward ONCE with (gy, gJ), and the seeded
    W3 kernel returns the gradient of sum gy*y + <gJ, J> in a single sweep (siren_second_order_seeded) instead of
    the reference's two separate backward passes (a first-order one for the value terms and a second-order one
    for the gradient terms)."""

    @staticmethod
    def forward(ctx, engine, x, flat, store=False, split=False, jet=None):
        ws = engine.pack(flat)
        ctx.tws = None
        ctx.jet, ctx.pre_hessian = jet, None
        pre = None
        key = JetState.key(x)
        ctx.spec = (jet.speculate(key) if (jet is not None and jet.hessian(key) and not split and
                                           engine.hessian_backward_supported) else None)
        if ctx.spec is not None:
            pre = SirenHessian.forward_sweep(engine, ws, x, None, want_yg=True)
        if pre is not None:
            # the Hessian node of this module's gradient will be requested again (it was last step): run its sweep
            # now — y and dPhi/dx come from the same jet — and hand (Hm, kept) to that node (_hessian_product)
            hm, kept, y, J = pre
            ctx.pre_hessian = (hm, kept)
        elif split and engine.split_supported:
            # precision 'bf16x6': the split-bf16 W1 kernel (fp32-level error); a backward recomputes from the fp32 ws
            y, J = engine.forward_grad_split(engine.pack_split(flat), x)
        elif store and engine.stored_supported and engine.cfg.hidden == 256 and STORED_FORWARD:
            # training: keep a_l / cos so the backward (seeded W3) skips the primal forward GEMMs
            y, J, ctx.tws = engine.forward_grad_store(ws, x)
        else:
            y, J = engine.forward_grad(ws, x)
        ctx.engine, ctx.ws = engine, ws
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, flat, J)
        return y, J

    @staticmethod
    def backward(ctx, gy, gJ):
        x, flat, J = ctx.saved_tensors
        engine, ws = ctx.engine, ctx.ws
        # tensor inputs in order: x (0), flat (1)
        need_x = ctx.needs_input_grad[1] and _will_execute(ctx, 0)
        need_p = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
        if (gy is None and gJ is None) or not (need_x or need_p):
            return None, None, None, None, None, None
        gy = gy.contiguous() if gy is not None else None
        gJ = gJ.contiguous() if gJ is not None else None
        gx = gp = None
        if not torch.is_grad_enabled():
            if gJ is None:  # first order only
                if need_p:
                    if ctx.tws is not None:
                        gx, gp = engine.backward_stored(ws, x, gy, ctx.tws)
                    else:
                        gx, gp = engine.backward_params(ws, x, gy)
                else:
                    gx = gy * J
            elif engine.second_order_supported:
                gx, gp = engine.second_order(ws, x, gJ, want_theta=need_p, gy=gy, kept=ctx.tws)
            else:
                gx, gp = _torch_path.jacobian_vjp(engine.cfg, x, flat, gJ, create_graph=False)
                if gy is not None:
                    gx = gx + gy * J
                    if need_p:
                        gp = gp + engine.backward_params(ws, x, gy)[1]
            return None, (gx if need_x else None), (gp if need_p else None), None, None, None
        # create_graph=True: differentiable in (x, theta, gy, gJ); J here is this node's own output 1
        if need_x:
            gx = gy * J if gy is not None else None
            if gJ is not None:
                h = _hessian_product(ctx, engine, ws, x, flat, gJ)
                if h is not None:
                    pass
                elif engine.second_order_supported:
                    h = SirenHVP.apply(engine, ws, x, flat, gJ)
                else:
                    h, _ = _torch_path.jacobian_vjp(engine.cfg, x, flat, gJ, create_graph=True)
                gx = h if gx is None else gx + h
        if need_p:
            if gy is not None:
                gp = _torch_path.vjp_params(engine.cfg, x, flat, gy, create_graph=True)
            if gJ is not None:
                _, gpj = _torch_path.jacobian_vjp(engine.cfg, x, flat, gJ, create_graph=True)
                gp = gpj if gp is None else gp + gpj
        return None, gx, gp, None, None, None


class SirenHVP(torch.autograd.Function):
    """d/dx <v, J(x)^T u> = sum_j u_j H_j(x) v as a graph node (u (n, d_out), None = ones: H v for d_out == 1):
    forward = W3 kernel (x part only, siren_second_order_ex). Its backward is a third derivative — laplace_mse through
    the reference's divergence(gradient()) (diff_operators.py:27-36, one such node per input dimension) and the
    helmholtz_pml / wave_pml training backward (loss_functions.py:112-211) — and runs on the mixed-jet kernel
    (siren_hvp_backward: d/d(x, theta, v, u) of <g, h> in one forward+reverse jet sweep + MFMA wgrad). Only a
    differentiable backward (create_graph over it, a fourth derivative) recomputes with device torch ops."""

    @staticmethod
    def forward(ctx, engine, ws, x, flat, v, u=None):
        gx, _ = engine.second_order(ws, x, v.contiguous(), want_theta=False, u=u)
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat, v, u)
        return gx

    @staticmethod
    def backward(ctx, g):
        x, flat, v, u = ctx.saved_tensors
        eng = ctx.engine
        if eng.hvp_backward_supported and not torch.is_grad_enabled():
            # tensor inputs in order: ws (0), x (1), flat (2), v (3), u (4, when given)
            need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
            need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 2)
            need_v = ctx.needs_input_grad[4] and _will_execute(ctx, 3)
            need_u = u is not None and ctx.needs_input_grad[5] and _will_execute(ctx, 4)
            if not (need_x or need_p or need_v or need_u):
                return None, None, None, None, None, None
            gx, gp, gv, gu = eng.hvp_backward(ctx.ws, x, v, g.contiguous(), u, want_theta=need_p, want_v=need_v,
                                              want_u=need_u)
            return None, None, (gx if need_x else None), gp, gv, gu
        rx, rp, rv, ru = _torch_path.hvp_vjp(eng.cfg, x, flat, v, g, create_graph=torch.is_grad_enabled(), u=u)
        return None, None, rx, rp, rv, ru


class SirenHessian(torch.autograd.Function):
    """Hm (n, d, d), Hm[c, :, i] = sum_j u_j H_j(x_c) e_i (u (n, d_out), None = ones) as ONE graph node per gradient
    node. Every create_graph x-derivative of that gradient node — each divergence() term of the reference's
    laplace = divergence(gradient()) (diff_operators.py:27-36), each hessian() column (:5-24) — is the cheap torch
    product Hm v, so autograd SUMS all their cotangents into one G (n, d, d) and calls this backward ONCE: one
    quadratic-form jet sweep + one MFMA wgrad (siren_hessian_backward) for the whole third-order term, where one
    SirenHVP node per dimension cost d mixed-jet sweeps and d wgrads. Forward: one forward-mode second-order jet
    (siren_hessian) that keeps its per-layer jets (KEEP_MAX_BYTES) for the backward, which then runs the reverse
    GEMMs only."""

    KEEP_MAX_BYTES = 16 << 30  # kept jets: 4 n_hidden 6 256 bytes per point (6 KiB / layer)
    KEEP_FREE_FRACTION = 0.5   # ... and at most this share of the device's free memory at forward time

    @staticmethod
    def _keep_budget(x):
        try:
            free, _ = torch.cuda.mem_get_info(x.device)
        except (RuntimeError, AssertionError):
            free = 0
        return min(SirenHessian.KEEP_MAX_BYTES, int(free * SirenHessian.KEEP_FREE_FRACTION))

    @staticmethod
    def forward_sweep(engine, ws, x, u, want_yg=False):
        """The node's forward kernel: (hm, kept | None) — or (hm, kept | None, y, g) with want_yg — keeping the jets
        when they fit the budget (else the backward recomputes its forward jet)."""
        per_point = 4 * engine.cfg.n_hidden * 6 * 256  # layers 1..L (layer 0 is rebuilt from x)
        if x.shape[0] * per_point <= SirenHessian._keep_budget(x):
            try:
                return engine.hessian(ws, x, u, keep=True, want_yg=want_yg)
            except torch.cuda.OutOfMemoryError:
                pass
        res = engine.hessian(ws, x, u, want_yg=want_yg)
        return res if want_yg else (res, None)

    @staticmethod
    def forward(ctx, engine, ws, x, flat, u=None, pre=None):
        # pre: (hm, kept) of this very (ws, x), run by the jet node's forward (JetState.hessian)
        hm, ctx.kept = pre if pre is not None else SirenHessian.forward_sweep(engine, ws, x, u)
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat, u)
        return hm

    @staticmethod
    def backward(ctx, G):
        x, flat, u = ctx.saved_tensors
        eng = ctx.engine
        # tensor inputs in order: ws (0), x (1), flat (2), u (3, when given)
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 2)
        need_u = u is not None and ctx.needs_input_grad[4] and _will_execute(ctx, 3)
        if not (need_x or need_p or need_u):
            return None, None, None, None, None, None
        if not torch.is_grad_enabled():
            gx, gp, gu = eng.hessian_backward(ctx.ws, x, G.contiguous(), u, want_theta=need_p, want_u=need_u,
                                              kept=ctx.kept)
            ctx.kept = None
            return None, None, (gx if need_x else None), gp, gu, None
        ctx.kept = None  # the differentiable recompute below does not read the kept jets
        rx, rp, ru = _torch_path.hessian_vjp(eng.cfg, x, flat, G, create_graph=True, u=u)
        return None, None, rx, rp, ru, None


def _hessian_product(ctx, engine, ws, x, flat, v, u=None):
    """sum_j u_j H_j v through the gradient node's shared SirenHessian node (built on the first request, kept on the
    gradient node's ctx: later requests of the same node reuse it), or None when the kernels do not cover it."""
    if not engine.hessian_backward_supported:
        return None
    hm = getattr(ctx, 'hessian_node', None)
    if hm is None:
        pre = getattr(ctx, 'pre_hessian', None) if u is None else None
        hm = SirenHessian.apply(engine, ws, x, flat, u, pre)
        ctx.hessian_node = hm
        ctx.pre_hessian = None
        if pre is not None and getattr(ctx, 'spec', None) is not None:
            ctx.spec[0] = False  # the speculative sweep was used
        jet = getattr(ctx, 'jet', None)
        if u is None and jet is not None:
            jet.observe_hessian_request(JetState.key(x))
    # elementwise (n, d, d) products: a batched GEMM of n 2x2 matrices runs ~100x slower on the BLAS path
    return (hm * v.unsqueeze(-2)).sum(-1)


class SirenVJP(torch.autograd.Function):
    """gx = J^T gy = sum_j gy_j dPhi_j/dx as a graph node; forward is the fused W1 kernel. Its backward is the W3
    kernel with output weighting u = gy and v = ggx (siren_second_order_ex), which also returns ggy = J ggx in the
    same sweep; under create_graph, an x-only request becomes a differentiable SirenHVP node (the second
    jacobian() of helmholtz_pml / wave_pml, hessian())."""

    @staticmethod
    def forward(ctx, engine, ws, x, flat, gy):
        _, gx = engine.forward_grad(ws, x, gy, want_y=False)
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat, gy)
        return gx

    @staticmethod
    def backward(ctx, ggx):
        x, flat, gy = ctx.saved_tensors
        eng = ctx.engine
        # tensor inputs in order: ws (0), x (1), flat (2), gy (3)
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 2)
        need_gy = ctx.needs_input_grad[4] and _will_execute(ctx, 3)
        if not (need_x or need_p or need_gy):
            return None, None, None, None, None
        ggx = ggx.contiguous()
        if not eng.second_order_supported or (torch.is_grad_enabled() and (need_p or need_gy)):
            gx, gp, ggy = _torch_path.vjp_vjp(eng.cfg, x, flat, gy, ggx, create_graph=torch.is_grad_enabled())
            return None, None, gx, gp, ggy
        if torch.is_grad_enabled():  # x only, differentiable
            h = _hessian_product(ctx, eng, ctx.ws, x, flat, ggx, gy)
            if h is None:
                h = SirenHVP.apply(eng, ctx.ws, x, flat, ggx, gy)
            return None, None, h, None, None
        res = eng.second_order(ctx.ws, x, ggx, want_theta=need_p, u=gy, want_ydot=need_gy)
        gx, gp = res[0], res[1]
        ggy = res[2] if need_gy else None
        return None, None, (gx if need_x else None), gp, ggy


class SirenBatchedFunction(torch.autograd.Function):
    """y (B, n, d_out) = Phi(x_b; theta_b) for per-element weights theta (B, P) — BatchLinear with batched W
    (modules.py:16-25) under a HyperNetwork (meta_modules.py:41-53, 81-92). Forward: one grouped W0 launch over the
    batch (siren_forward_batched); under a parameter-gradient graph the grouped stored forward (FWDS: a_l / cos kept,
    siren_forward_store_batched). Backward: gx from one grouped W1 launch; theta-gradients (what flows back into the
    hypernetwork) from the grouped reverse-only W2 (siren_backward_stored_batched), or the recompute W2
    (siren_backward_batched) when nothing was stored. Under create_graph gx becomes ONE SirenBatchedVJP node (grouped W1
    forward, per-element W3 backward on a fully packed image); theta-gradients under create_graph (meta-learning only)
    recompute with device torch ops."""

    @staticmethod
    def forward(ctx, engine, x, flat, store=False):
        ws = engine.pack_batched(flat)
        ctx.tws = None
        if store and engine.stored_for(x.shape[1], x.shape[0]) and STORED_FORWARD:
            # training under a hypernetwork: keep every element's a_l / cos, the backward is reverse-only
            y, ctx.tws = engine.forward_store_batched(ws, x)
        else:
            y = engine.forward_batched(ws, x)
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, flat = ctx.saved_tensors
        engine, ws = ctx.engine, ctx.ws
        need_x = ctx.needs_input_grad[1] and _will_execute(ctx, 0)
        need_p = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
        gy = gy.contiguous()
        gx = gp = None
        if not torch.is_grad_enabled():
            if need_p:
                if ctx.tws is not None:
                    gx, gp = engine.backward_stored_batched(ws, x, gy, ctx.tws)
                else:
                    gx, gp = engine.backward_params_batched(ws, x, gy)
            elif need_x:
                _, gx = engine.forward_grad_batched(ws, x, gy, want_y=False)
            return None, (gx if need_x else None), gp, None
        # create_graph: differentiable in (x, theta, gy). The second / third-order kernels read every element's
        # whole packed image, which the forward's first-order pack does not write (siren_pack_batched): repack full
        if need_x:
            gx = SirenBatchedVJP.apply(engine, engine.pack_batched(flat, full=True), x, flat, gy)
        if need_p:  # theta-gradients under create_graph (meta-learning; no reference caller): device torch
            gp = torch.stack([_torch_path.vjp_params(engine.cfg, x[b], flat[b], gy[b], create_graph=True)
                              for b in range(x.shape[0])])
        return None, gx, gp, None


def _stack_or_none(parts):
    return None if parts[0] is None else torch.stack(parts)


class SirenBatchedVJP(torch.autograd.Function):
    """gx (B, n, d_in) = J_b^T gy_b for batched (hypernetwork) weights as ONE graph node: forward = one grouped W1
    launch (siren_forward_grad_batched). Its backward is the W3 sweep of every element (siren_second_order_batched:
    H v, the theta-gradient w.r.t. the predicted weights and J v) — what gradients_mse / sdf on a hypo network need;
    under create_graph an x-only request becomes a SirenBatchedHVP node (divergence(gradient()), laplace_mse).
    ws must be pack_batched(full=True)."""

    @staticmethod
    def forward(ctx, engine, ws, x, flat, gy):
        _, gx = engine.forward_grad_batched(ws, x, gy, want_y=False)
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat, gy)
        return gx

    @staticmethod
    def backward(ctx, ggx):
        x, flat, gy = ctx.saved_tensors
        eng = ctx.engine
        # tensor inputs in order: ws (0), x (1), flat (2), gy (3)
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 2)
        need_gy = ctx.needs_input_grad[4] and _will_execute(ctx, 3)
        if not (need_x or need_p or need_gy):
            return None, None, None, None, None
        ggx = ggx.contiguous()
        if not eng.second_order_supported or (torch.is_grad_enabled() and (need_p or need_gy)):
            parts = [_torch_path.vjp_vjp(eng.cfg, x[b], flat[b], gy[b], ggx[b], create_graph=torch.is_grad_enabled())
                     for b in range(x.shape[0])]
            return (None, None) + tuple(_stack_or_none([p[i] for p in parts]) for i in range(3))
        if torch.is_grad_enabled():  # x only, differentiable
            return None, None, SirenBatchedHVP.apply(eng, ctx.ws, x, flat, ggx, gy), None, None
        res = eng.second_order_batched(ctx.ws, x, ggx, want_theta=need_p, u=gy, want_ydot=need_gy)
        gx, gp = res[0], res[1]
        ggy = res[2] if need_gy else None
        return None, None, (gx if need_x else None), gp, ggy


class SirenBatchedHVP(torch.autograd.Function):
    """h_b = sum_j u_bj H_bj(x) v_b for batched weights as ONE graph node (the per-dimension node of divergence() on a
    hypo network's gradient): forward = W3 per element (x part only); backward = the mixed-jet third-order adjoint
    per element (siren_hvp_backward_batched). ws must be pack_batched(full=True)."""

    @staticmethod
    def forward(ctx, engine, ws, x, flat, v, u=None):
        gx, _ = engine.second_order_batched(ws, x, v.contiguous(), want_theta=False, u=u)
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat, v, u)
        return gx

    @staticmethod
    def backward(ctx, g):
        x, flat, v, u = ctx.saved_tensors
        eng = ctx.engine
        if eng.hvp_backward_supported and not torch.is_grad_enabled():
            # tensor inputs in order: ws (0), x (1), flat (2), v (3), u (4, when given)
            need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
            need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 2)
            need_v = ctx.needs_input_grad[4] and _will_execute(ctx, 3)
            need_u = u is not None and ctx.needs_input_grad[5] and _will_execute(ctx, 4)
            if not (need_x or need_p or need_v or need_u):
                return None, None, None, None, None, None
            gx, gp, gv, gu = eng.hvp_backward_batched(ctx.ws, x, v, g.contiguous(), u, want_theta=need_p,
                                                      want_v=need_v, want_u=need_u)
            return None, None, (gx if need_x else None), gp, gv, gu
        parts = [_torch_path.hvp_vjp(eng.cfg, x[b], flat[b], v[b], g[b], create_graph=torch.is_grad_enabled(),
                                     u=None if u is None else u[b]) for b in range(x.shape[0])]
        return (None, None) + tuple(_stack_or_none([p[i] for p in parts]) for i in range(4))


class SirenLaplace(torch.autograd.Function):
    """Laplacian sum_j sum_i d2 Phi_j/dx_i2 (n, 1) as ONE graph node: forward = the W4 jet kernel
    (siren_forward_laplace: y, grad and Laplacian in one forward-mode sweep). diff_operators.laplace routes here
    when its y comes straight from a SirenFunction node of x. Backward (laplace_mse training, a third derivative)
    = the W4s kernels (siren_laplace_backward: reverse of the jet + MFMA wgrad over 4N columns); only a
    differentiable backward (create_graph over it, a fourth derivative) recomputes with device torch ops."""

    @staticmethod
    def forward(ctx, engine, ws, x, flat, store=False, pre=None):
        ctx.tws = None
        if pre is not None:  # (lap, kept stores | None) run by the value node's forward (JetState.laplace)
            lap, ctx.tws = pre
        elif store and STORED_FORWARD:  # training: keep the jet stores, the backward is reverse-only
            lap, ctx.tws = engine.forward_laplace_store(ws, x)
        else:
            _, _, lap = engine.forward_laplace(ws, x)
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat)
        return lap

    @staticmethod
    def backward(ctx, glap):
        x, flat = ctx.saved_tensors
        # tensor inputs in order: ws (0), x (1), flat (2)
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 2)
        if not (need_x or need_p):
            return None, None, None, None, None, None
        if not torch.is_grad_enabled():
            if ctx.tws is not None:
                gx, gp = ctx.engine.laplace_backward_stored(ctx.ws, x, glap, ctx.tws)
            else:
                gx, gp = ctx.engine.laplace_backward(ctx.ws, x, glap)
            return None, None, (gx if need_x else None), (gp if need_p else None), None, None
        gx, gp = _torch_path.laplace_vjp(ctx.engine.cfg, x, flat, glap.contiguous(),
                                         create_graph=torch.is_grad_enabled())
        return None, None, (gx if need_x else None), (gp if need_p else None), None, None


_VIEW_NODES = ('ViewBackward0', 'ReshapeAliasBackward0', 'UnsafeViewBackward0')


def _node_ws(node):
    """The packed fp32 workspace of a SirenFunction / SirenJetFunction / SirenSplitFunction node (the split node packs
    it on first use and keeps it)."""
    if node.ws is None:
        node.ws = node.engine.pack(node.saved_tensors[1])
    return node.ws


def siren_node_of(y, x):
    """The SirenFunction / SirenJetFunction node that produced y (its value output, through views only) from a view
    of x, else None."""
    node = getattr(y, 'grad_fn', None)
    out_nr = getattr(y, 'output_nr', 0)
    for _ in range(4):
        if node is None:
            return None
        name = type(node).__name__
        if name in ('SirenFunctionBackward', 'SirenJetFunctionBackward', 'SirenSplitFunctionBackward'):
            break
        if name not in _VIEW_NODES:
            return None
        node, out_nr = node.next_functions[0]
    else:
        return None
    if out_nr != 0:  # the jet node's second output is dPhi/dx, not the network value
        return None
    if not hasattr(node, 'engine') or not hasattr(node, 'ws'):
        return None
    xs = node.saved_tensors[0]
    if xs.data_ptr() != x.data_ptr() or xs.numel() != x.numel() or x.shape[-1] != xs.shape[-1]:
        return None
    if not (xs is x or xs._base is x or (x._base is not None and xs._base is x._base)):
        return None
    return node


def fused_laplace(y, x):
    """diff_operators.laplace(y, x) in one W4 launch when y = SingleBVPNet/FCBlock output of x; else None."""
    node = siren_node_of(y, x)
    if node is None or not node.engine.laplace_supported:
        return None
    xs, flat = node.saved_tensors[:2]
    store = torch.is_grad_enabled() and flat.requires_grad
    pre = getattr(node, 'pre_laplace', None)
    if pre is not None and store and pre[1] is None:
        pre = None  # computed without the jet stores (no parameter graph then); this call wants them
    lap = SirenLaplace.apply(node.engine, _node_ws(node), xs, flat, store, pre)
    if hasattr(node, 'pre_laplace'):
        node.pre_laplace = None
    if getattr(node, 'spec', None) is not None:
        # a Laplacian was requested of this node: the speculation was right even when its sweep ran without the jet
        # stores this call needs (recomputed above) — the next forward must not read it as unconsumed
        node.spec[0] = False
    jet = getattr(node, 'jet', None)
    if jet is not None:
        jet.observe_laplace_request(JetState.key(xs))
    return lap.view(*y.shape[:-1], 1)
