"""Training loop with the reference's semantics (training.py:14-129), device-agnostic and DP-aware.

Same steps per iteration: forward (training.py:72), sum of loss means (73-84), zero_grad + backward (95-96),
optional grad-norm clip (98-102), Adam step (104), checkpoints (44-48, 89-91, 126-129). Differences, all
harness plumbing: no interactive overwrite prompt (training.py:25-28), TensorBoard is optional (a no-op
writer when absent), and under torch.distributed the flat weight-gradient bucket is all-reduced BEFORE the
clip so every rank clips the same global gradient.
"""
import os
import time

import numpy as np
import torch

from . import distributed


class _NullWriter:
    def add_scalar(self, *a, **k):
        pass


def _host(losses):
    return torch.stack([torch.as_tensor(v).float().cpu() for v in losses]).numpy() if losses else np.zeros(0)


def _writer(summaries_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(summaries_dir)
    except Exception:
        return _NullWriter()


def _coord_count(model_input):
    """Coordinates in this rank's batch (B * N of model_input['coords'] (B, N, d))."""
    c = model_input['coords']
    return c.numel() // max(1, c.shape[-1])


def train(model, train_dataloader, epochs, lr, steps_til_summary, epochs_til_checkpoint, model_dir, loss_fn,
          summary_fn=None, val_dataloader=None, double_precision=False, clip_grad=False, use_lbfgs=False,
          loss_schedules=None, device='cuda', log=print, writer=None, fused_adam=False):
    if double_precision:
        raise NotImplementedError('siren_amd computes in fp32 (the reference default)')
    if use_lbfgs:
        optim = torch.optim.LBFGS(lr=lr, params=model.parameters(), max_iter=50000, max_eval=50000,
                                  history_size=50, line_search_fn='strong_wolfe')
    elif fused_adam:  # clip + Adam in two HIP launches over one flat bucket, norm kept on the device (optim.py)
        from .optim import FusedAdam
        optim = FusedAdam(model.parameters(), lr=lr, max_norm=(1. if clip_grad is True else clip_grad) or None)
    else:
        optim = torch.optim.Adam(lr=lr, params=model.parameters())
    checkpoints_dir = os.path.join(model_dir, 'checkpoints')
    os.makedirs(checkpoints_dir, exist_ok=True)
    writer = writer or _writer(os.path.join(model_dir, 'summaries'))
    world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0

    def step_losses(model_input, gt, total_steps):
        model_output = model(model_input)
        losses = loss_fn(model_output, gt)
        train_loss = 0.
        for name, loss in losses.items():
            single = loss.mean()
            if loss_schedules is not None and name in loss_schedules:
                single = single * loss_schedules[name](total_steps)
            writer.add_scalar(name, single, total_steps)
            train_loss = train_loss + single
        return model_output, train_loss

    total_steps, train_losses = 0, []
    for epoch in range(epochs):
        if not epoch % epochs_til_checkpoint and epoch and rank == 0:
            torch.save(model.state_dict(), os.path.join(checkpoints_dir, 'model_epoch_%04d.pth' % epoch))
            np.savetxt(os.path.join(checkpoints_dir, 'train_losses_epoch_%04d.txt' % epoch), _host(train_losses))
        for model_input, gt in train_dataloader:
            start = time.time()
            model_input = {k: v.to(device) for k, v in model_input.items()}
            gt = {k: v.to(device) for k, v in gt.items()}
            if use_lbfgs:
                def closure():
                    optim.zero_grad()
                    _, loss = step_losses(model_input, gt, total_steps)
                    count = _coord_count(model_input) if world > 1 else None
                    if count != 0:
                        loss.backward()
                    if world == 1:
                        return loss
                    # the line search must see the GLOBAL loss on every rank (the gradient already is global), or
                    # the ranks' strong-Wolfe searches take different steps and the replicas drift apart
                    return distributed.allreduce_gradients(list(model.parameters()), world, count, loss=loss)
                optim.step(closure)
            model_output, train_loss = step_losses(model_input, gt, total_steps)
            train_losses.append(train_loss.detach())  # device scalar: no per-step host sync (training.py:86)
            writer.add_scalar('total_train_loss', train_loss, total_steps)
            if not total_steps % steps_til_summary and rank == 0:
                torch.save(model.state_dict(), os.path.join(checkpoints_dir, 'model_current.pth'))
                if summary_fn is not None:
                    summary_fn(model, model_input, gt, model_output, writer, total_steps)
            if not use_lbfgs:
                optim.zero_grad()
                # under DP each rank's mean-loss gradient is weighted by its coordinate count in the reduction (exact
                # full-batch gradient for unequal shards); an empty shard contributes zeros, never its NaN mean
                count = _coord_count(model_input) if world > 1 else None
                if count != 0:
                    train_loss.backward()
                if fused_adam and world > 1:
                    optim.allreduce_grad(world, count)  # the bucket itself is the all-reduce buffer: no gather / scatter
                else:
                    distributed.allreduce_gradients(list(model.parameters()), world, count)
                if clip_grad and not fused_adam:
                    max_norm = 1. if isinstance(clip_grad, bool) else clip_grad
                    torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
                optim.step()
            if not total_steps % steps_til_summary and rank == 0:
                log('Epoch %d, Total loss %0.6f, iteration time %0.6f' % (epoch, float(train_losses[-1]),
                                                                           time.time() - start))
            total_steps += 1
    if rank == 0:
        torch.save(model.state_dict(), os.path.join(checkpoints_dir, 'model_final.pth'))
        np.savetxt(os.path.join(checkpoints_dir, 'train_losses_final.txt'), _host(train_losses))
    return [float(v) for v in _host(train_losses)]
