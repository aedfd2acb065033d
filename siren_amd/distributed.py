"""Data parallelism over the coordinate batch: one process per GPU, torch.distributed over RCCL
("nccl" backend on ROCm; "gloo" for the CPU tests).

Every coordinate's value and derivatives depend only on that coordinate and the replicated weights, and every
hot-path loss is a mean over coordinates, so with equal shards the global loss gradient is the average of the
per-rank gradients. The only collective on the data path is ONE all-reduce of the flat weight-gradient bucket
per step (0.79 MB for 5x256 d2; 3.2 MB for 5x512): a ring all-reduce over xGMI is latency-bound at that size,
so the whole model's gradients travel as a single bucket rather than per-parameter calls.
"""
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get('WORLD_SIZE', '1')), int(os.environ.get('RANK', '0')), \
        int(os.environ.get('LOCAL_RANK', '0'))


def init(backend=None):
    """Initialise the default process group from torchrun's environment (MASTER_ADDR=127.0.0.1 etc.)."""
    world, rank, local = env_world()
    if world <= 1 or dist.is_initialized():
        return world, rank, local
    if backend is None:
        backend = 'nccl' if torch.cuda.is_available() else 'gloo'
    if backend == 'nccl':
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend)
    return world, rank, local


def shard(n, world, rank, align=64):
    """[start, stop) of rank's share of n coordinates: boundaries at the multiples of `align` (the kernels' coordinate
    tile) nearest below the even split, the last rank ending at n, so the shares differ by less than `align` (ranks
    may be empty when n < world * align). Unequal shares are made exact by allreduce_gradients(count=...), which
    weights each rank's mean-loss gradient by its coordinate count."""
    def bound(r):
        return n if r >= world else (r * n // world) // align * align
    return bound(rank), bound(rank + 1)


def broadcast_parameters(module, src=0):
    if not (dist.is_available() and dist.is_initialized()):
        return
    with torch.no_grad():
        flat = torch.cat([p.detach().reshape(-1) for p in module.parameters()])
        dist.broadcast(flat, src)
        off = 0
        for p in module.parameters():
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()


def allreduce_gradients(params, world=None, count=None, loss=None):
    """Reduce .grad of `params` over ranks with ONE all-reduce of a flat bucket (in place).

    count=None: plain average (equal shards). count = this rank's coordinate count: the bucket carries count * grad
    plus the count itself, so the result is sum_r n_r g_r / sum_r n_r — the full-batch gradient of a mean-over-
    coordinates loss for any split, including empty shards (count 0 contributes nothing; its NaN mean-loss gradient
    must not have been back-propagated, see training.train).
    loss = this rank's (mean) loss: it rides in the same bucket with the same weighting and the global loss is
    returned (a detached scalar; an empty shard's NaN loss counts as 0) — what an LBFGS closure must return so every
    rank's line search sees the same function. Without a process group the local loss (or None) is returned."""
    if not (dist.is_available() and dist.is_initialized()):
        return loss
    world = world or dist.get_world_size()
    if count is not None:
        # every rank sends the full bucket of TRAINABLE parameters (so every rank must train the same set, for the
        # buckets to line up), an empty shard's unset grads as zeros; frozen parameters keep grad None, which
        # torch.optim skips (a zero grad would still receive weight decay / momentum)
        params = [p for p in params if p.requires_grad]
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
    else:
        params = [p for p in params if p.grad is not None]
    if not params and loss is None:
        return None
    dev = params[0].grad if params else torch.as_tensor(loss)
    extra = []
    if loss is not None:
        lv = torch.as_tensor(loss).detach().reshape(1).to(dev.device, torch.float32)
        extra.append(torch.zeros_like(lv) if count == 0 else lv)
    if count is not None:
        extra.append(dev.new_full((1,), float(count)))
    flat = torch.cat([p.grad.reshape(-1) for p in params] + extra)
    body = flat[:flat.numel() - (1 if count is not None else 0)]  # gradients (+ loss): the count-weighted part
    if count is not None:
        body.mul_(float(count))
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    if count is not None:
        body.div_(flat[-1:].clamp_min(1.))
    else:
        body.div_(world)
    off = 0
    for p in params:
        n = p.numel()
        p.grad.copy_(flat[off:off + n].view_as(p.grad))
        off += n
    return flat[off].clone() if loss is not None else None
