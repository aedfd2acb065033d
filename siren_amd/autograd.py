"""Autograd Functions that put the HIP kernels under the reference's autograd contract.

The reference never calls its model's derivatives directly: losses call torch.autograd.grad(model_out,
model_in, ones, create_graph=True) (diff_operators.py:42, :35) and training calls train_loss.backward()
(training.py:96). So the fused kernels sit behind torch.autograd.Function nodes:

  SirenFunction      y = Phi(x; theta)                        forward: W0 kernel, or the W1 kernel in "jet"
                                                              mode (y and dPhi/dx in ONE launch, d_out == 1)
    .backward(gy)    no create_graph: gx via the W1 kernel (or gy*J from jet mode), (gx, gtheta) via the
                     W2 pipeline (fused reverse sweep + split-K MFMA weight-gradient + slab reduction)
                     create_graph:    differentiable gx through SirenJacobian / SirenVJP nodes
  SirenJacobian      J (jet-mode dPhi/dx, already computed by the forward launch) as a graph node
  SirenVJP           gx = J^T gy computed by the W1 kernel as a graph node

Which gradients autograd actually wants is read from the engine (torch._C._will_engine_execute_node on the
next nodes), because ctx.needs_input_grad is static: autograd.grad(y, [x]) must not pay for weight gradients.

Second-order adjoints (SirenJacobian/SirenVJP.backward: gradients_mse / sdf training, the Laplacian's
Hessian-vector products) run on the W3 kernel (siren_second_order) for hidden 256 and d_out == 1.
Third-order adjoints (SirenHVP.backward: laplace_mse training, W4s), second order at hidden 512 and vector
outputs under create_graph are recomputed through siren_amd._torch_path on the device.
"""
import torch

from . import _torch_path


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
    """Per-module switch for jet mode ('auto' turns it on after the first create_graph x-gradient request)."""

    def __init__(self, mode='auto'):
        self.mode = mode
        self.active = mode is True

    def observe_x_gradient_request(self):
        if self.mode == 'auto':
            self.active = True


class SirenFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, jet, x, flat):
        ws = engine.pack(flat)
        J = None
        use_jet = (jet is not None and jet.active and engine.cfg.d_out == 1 and engine.grad_supported
                   and x.requires_grad)
        if use_jet:
            y, J = engine.forward_grad(ws, x)
        else:
            y = engine.forward(ws, x)
        ctx.engine, ctx.jet, ctx.ws, ctx.J = engine, jet, ws, J
        ctx.save_for_backward(x, flat)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, flat = ctx.saved_tensors
        engine, ws, J = ctx.engine, ctx.ws, ctx.J
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 0)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 1)
        gx = gp = None
        gy = gy.contiguous()
        if not torch.is_grad_enabled():
            if need_p:
                gx, gp = engine.backward_params(ws, x, gy)
                if not need_x:
                    gx = None
            elif need_x:
                if J is not None:
                    gx = gy * J
                else:
                    _, gx = engine.forward_grad(ws, x, gy, want_y=False)
            return None, None, gx, gp
        # create_graph=True: results must be differentiable functions of (x, theta, gy)
        if need_x:
            if ctx.jet is not None and not need_p:
                ctx.jet.observe_x_gradient_request()
            if J is not None:
                gx = gy * SirenJacobian.apply(engine, [J], x, flat, ws)
            else:
                gx = SirenVJP.apply(engine, ws, x, flat, gy)
        if need_p:
            gp = _torch_path.vjp_params(engine.cfg, x, flat, gy, create_graph=True)
        return None, None, gx, gp


class SirenJacobian(torch.autograd.Function):
    """J(x; theta) = dPhi/dx (d_out == 1) as a graph node; the value comes from the jet-mode forward launch.

    backward(gJ) is the second-order adjoint: (H gJ, d/dtheta <gJ, J>) from the W3 kernel
    (siren_second_order). Under create_graph (laplace/divergence, third-order losses) the Hessian-vector product
    becomes a SirenHVP node whose forward is the same kernel."""

    @staticmethod
    def forward(ctx, engine, holder, x, flat, ws):
        ctx.engine, ctx.ws = engine, ws
        ctx.save_for_backward(x, flat)
        return holder[0].clone()  # a fresh output tensor per node (J may feed several gradient() calls)

    @staticmethod
    def backward(ctx, gJ):
        x, flat = ctx.saved_tensors
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 0)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 1)
        gJ = gJ.contiguous()
        if not ctx.engine.second_order_supported:  # hidden 512: no W3 kernel yet
            gx, gp = _torch_path.jacobian_vjp(ctx.engine.cfg, x, flat, gJ, create_graph=torch.is_grad_enabled())
            return None, None, (gx if need_x else None), (gp if need_p else None), None
        if not torch.is_grad_enabled():
            gx, gp = ctx.engine.second_order(ctx.ws, x, gJ, want_theta=need_p)
            return None, None, (gx if need_x else None), gp, None
        gx = SirenHVP.apply(ctx.engine, ctx.ws, x, flat, gJ) if need_x else None
        gp = None
        if need_p:
            _, gp = _torch_path.jacobian_vjp(ctx.engine.cfg, x, flat, gJ, create_graph=True)
        return None, None, gx, gp, None


class SirenHVP(torch.autograd.Function):
    """H(x; theta) v (d_out == 1) as a graph node: forward = W3 kernel (x part only); its own backward (a third
    derivative: laplace_mse training) is recomputed with device torch ops."""

    @staticmethod
    def forward(ctx, engine, ws, x, flat, v):
        gx, _ = engine.second_order(ws, x, v.contiguous(), want_theta=False)
        ctx.engine = engine
        ctx.save_for_backward(x, flat, v)
        return gx

    @staticmethod
    def backward(ctx, g):
        x, flat, v = ctx.saved_tensors
        rx, rp, rv = _torch_path.hvp_vjp(ctx.engine.cfg, x, flat, v, g, create_graph=torch.is_grad_enabled())
        return None, None, rx, rp, rv


class SirenVJP(torch.autograd.Function):
    """gx = sum_j gy_j dPhi_j/dx as a graph node; forward is the fused W1 kernel. For d_out == 1 its backward is
    the W3 kernel with v = gy * ggx (plus <ggx, J> for gy, from the W1 kernel)."""

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
        w3_ok = eng.second_order_supported
        if torch.is_grad_enabled() or not w3_ok:
            gx, gp, ggy = _torch_path.vjp_vjp(eng.cfg, x, flat, gy, ggx, create_graph=torch.is_grad_enabled())
            return None, None, gx, gp, ggy
        # tensor inputs in order: ws (0), x (1), flat (2), gy (3)
        need_x = ctx.needs_input_grad[2] and _will_execute(ctx, 1)
        need_p = ctx.needs_input_grad[3] and _will_execute(ctx, 2)
        need_gy = ctx.needs_input_grad[4] and _will_execute(ctx, 3)
        ggx = ggx.contiguous()
        gx = gp = ggy = None
        if need_x or need_p:
            gx, gp = eng.second_order(ctx.ws, x, (gy * ggx).contiguous(), want_theta=need_p)
        if need_gy:
            _, J = eng.forward_grad(ctx.ws, x, want_y=False)
            ggy = (J * ggx).sum(-1, keepdim=True)
        return None, None, (gx if need_x else None), gp, ggy


class SirenLaplace(torch.autograd.Function):
    """Laplacian sum_j sum_i d2 Phi_j/dx_i2 (n, 1) as ONE graph node: forward = the W4 jet kernel
    (siren_forward_laplace: y, grad and Laplacian in one forward-mode sweep). diff_operators.laplace routes here
    when its y comes straight from a SirenFunction node of x. Backward (laplace_mse training, a third derivative)
    = the W4s kernels (siren_laplace_backward: reverse of the jet + MFMA wgrad over 4N columns); only a
    differentiable backward (create_graph over it, a fourth derivative) recomputes with device torch ops."""

    @staticmethod
    def forward(ctx, engine, ws, x, flat):
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
            return None, None, None, None
        if not torch.is_grad_enabled():
            gx, gp = ctx.engine.laplace_backward(ctx.ws, x, glap)
            return None, None, (gx if need_x else None), (gp if need_p else None)
        gx, gp = _torch_path.laplace_vjp(ctx.engine.cfg, x, flat, glap.contiguous(),
                                         create_graph=torch.is_grad_enabled())
        return None, None, (gx if need_x else None), (gp if need_p else None)


_VIEW_NODES = ('ViewBackward0', 'ReshapeAliasBackward0', 'UnsafeViewBackward0')


def siren_node_of(y, x):
    """The SirenFunction node that produced y (through views only) from a view of x, else None."""
    node = getattr(y, 'grad_fn', None)
    for _ in range(4):
        if node is None:
            return None
        name = type(node).__name__
        if name == 'SirenFunctionBackward':
            break
        if name not in _VIEW_NODES:
            return None
        node = node.next_functions[0][0]
    else:
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
    xs, flat = node.saved_tensors
    lap = SirenLaplace.apply(node.engine, node.ws, xs, flat)
    return lap.view(*y.shape[:-1], 1)
