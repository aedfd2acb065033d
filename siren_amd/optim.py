"""FusedAdam: clip_grad_norm_ + torch.optim.Adam.step (training.py:17, 98-104) as two HIP launches over ONE flat
parameter bucket (siren_adam_step, step_kernels.hpp), with the global gradient norm kept on the device.

The parameters are re-seated as views of a flat fp32 buffer (state-dict order), and their .grad as views of a
flat gradient buffer that zero_grad() clears in place, so autograd accumulates straight into the bucket and the
step reads it without a gather. Semantics: torch.optim.Adam (amsgrad off, weight_decay 0, maximize off) after
torch.nn.utils.clip_grad_norm_(params, max_norm) when max_norm is set.
"""
import ctypes

import torch

from . import _lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class FusedAdam:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, max_norm=None):
        self.params = [p for p in params]
        if not self.params:
            raise ValueError('FusedAdam got an empty parameter list')
        dev = self.params[0].device
        if dev.type != 'cuda' or any(p.device != dev or p.dtype != torch.float32 for p in self.params):
            raise RuntimeError('FusedAdam needs fp32 parameters on one ROCm device')
        self.lib = _lib.load()
        self.lr, self.betas, self.eps, self.max_norm = float(lr), tuple(betas), float(eps), max_norm
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, device=dev)
        # the gradient bucket + one slot for the coordinate count of a count-weighted all-reduce (allreduce_grad)
        self.bucket = torch.zeros(n + 1, device=dev)
        self.grad = self.bucket[:n]
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_adam_scratch_floats(ctypes.byref(cnt)), 'siren_adam_scratch_floats')
        self.scratch = torch.zeros(cnt.value, device=dev)
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                self.flat[off:off + k].copy_(p.reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                off += k
        self._bind_grads()
        self.step_count = 0

    def _bind_grads(self):
        off = 0
        for p in self.params:
            k = p.numel()
            p.grad = self.grad[off:off + k].view_as(p)
            off += k

    def zero_grad(self, set_to_none=False):
        self.grad.zero_()
        self._bind_grads()

    def _gather_grads(self):
        """Copy any .grad that autograd replaced (e.g. after set_to_none) back into the bucket."""
        off = 0
        for p in self.params:
            k = p.numel()
            g = p.grad
            view = self.grad[off:off + k]
            if g is None:
                view.zero_()
            elif g.data_ptr() != view.data_ptr():
                view.copy_(g.reshape(-1))
            off += k
        self._bind_grads()

    @torch.no_grad()
    def allreduce_grad(self, world, count=None):
        """Data parallel: reduce the flat gradient bucket over ranks with ONE all-reduce (RCCL over xGMI), in place.
        count=None averages (equal shards); count = this rank's coordinate count weights the ranks' mean-loss
        gradients by their shares (sum_r n_r g_r / sum_r n_r, distributed.allreduce_gradients), the count riding
        in the bucket's last slot so it stays one collective and no host sync."""
        import torch.distributed as dist
        self._gather_grads()
        if count is None:
            dist.all_reduce(self.grad, op=dist.ReduceOp.SUM)
            self.grad.div_(world)
            return
        self.grad.mul_(float(count))
        self.bucket[-1] = float(count)
        dist.all_reduce(self.bucket, op=dist.ReduceOp.SUM)
        self.grad.div_(self.bucket[-1:].clamp_min(1.))

    @torch.no_grad()
    def step(self):
        self._gather_grads()
        self.step_count += 1
        mx = float(self.max_norm) if self.max_norm else 0.
        st = ctypes.c_void_p(torch.cuda.current_stream(self.flat.device).cuda_stream)
        _lib.check(self.lib.siren_adam_step(_ptr(self.flat), _ptr(self.grad), _ptr(self.exp_avg),
                                            _ptr(self.exp_avg_sq), self.flat.numel(), self.lr, self.betas[0],
                                            self.betas[1], self.eps, self.step_count, mx, _ptr(self.scratch), st),
                   'siren_adam_step')

    def grad_norm(self):
        """The pre-clip global gradient norm of the last clipped step (device tensor; no host sync)."""
        return self.scratch[1024]
