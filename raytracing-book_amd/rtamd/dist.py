"""One process per GPU: interleaved row stripes + one collective gather.

A pixel's sample stream depends only on (pixel, per-frame u_rand_factor,
scene) (random.glsl:2-7, compute.glsl:346), so any row partition renders
bit-identically to one GPU.  Rank k owns the stripes s with s % world == k
(SURVEY §8e).  During rendering there is no inter-GPU traffic; at the end each
rank contributes its stripe-compacted, equally padded [padded_rows, W, 4]
RGBA32F block to one all_gather (RCCL over xGMI with backend "nccl", gloo on
CPU) and the blocks are de-interleaved into the full image.
"""
import numpy as np
import torch
import torch.distributed as dist

from .render import deinterleave, local_rows, padded_local_rows


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* if set."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend, device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    return rank, world, local_rank


def gather_image(local_block, height, world, stripe_rows):
    """All-gather the [padded_rows, W, 4] blocks and de-interleave (rank 0 and others)."""
    if world == 1:
        rows = local_rows(height, 0, 1, stripe_rows)
        return local_block[:rows].cpu().numpy()
    padded = padded_local_rows(height, world, stripe_rows)
    assert local_block.shape[0] == padded
    if dist.get_backend() == "nccl":
        out = torch.empty((world,) + tuple(local_block.shape), dtype=local_block.dtype, device=local_block.device)
        dist.all_gather_into_tensor(out, local_block.contiguous())
        g = out.cpu().numpy()
    else:
        blk = local_block.detach().cpu().contiguous()   # gloo gathers host tensors
        parts = [torch.empty_like(blk) for _ in range(world)]
        dist.all_gather(parts, blk)
        g = np.stack([p.cpu().numpy() for p in parts])
    return deinterleave(g, height, world, stripe_rows)
