"""One process per GPU: interleaved row stripes + one collective gather.

A pixel's sample stream depends only on (pixel, per-frame u_rand_factor,
scene) (random.glsl:2-7, compute.glsl:346), so any row partition renders
bit-identically to one GPU.  Rank k owns the stripes s with s % world == k
(SURVEY §8e).  During rendering there is no inter-GPU traffic; at the end each
rank contributes its stripe-compacted, equally padded [padded_rows, W, 4]
RGBA32F block to one gather to rank 0 (RCCL over xGMI with backend "nccl",
gloo on CPU), and rank 0 de-interleaves the blocks into the full image.
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
    """Gather the ranks' [padded_rows, W, 4] blocks to rank 0 and de-interleave.

    Returns the [H, W, 4] image on rank 0 and None on every other rank: only
    rank 0 receives the blocks (one gather, not an all-gather) and only rank 0
    copies them to the host."""
    if world == 1:
        rows = local_rows(height, 0, 1, stripe_rows)
        return local_block[:rows].cpu().numpy()
    padded = padded_local_rows(height, world, stripe_rows)
    assert local_block.shape[0] == padded
    rank = dist.get_rank()
    blk = local_block.contiguous()
    if dist.get_backend() != "nccl":
        blk = blk.detach().cpu()   # gloo gathers host tensors
    if rank == 0:
        parts = [torch.empty_like(blk) for _ in range(world)]
        dist.gather(blk, gather_list=parts, dst=0)
        g = torch.stack(parts).cpu().numpy()
        return deinterleave(g, height, world, stripe_rows)
    dist.gather(blk, dst=0)
    return None


def _agree(ok, what):
    """Every rank learns whether every rank got through `what` (MIN all-reduce): a failure on
    one rank raises on all of them, so none is left blocked in the next RCCL call."""
    dev = "cpu"
    if dist.get_backend() == "nccl":
        dev = f"cuda:{torch.cuda.current_device()}"
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if float(t.item()) < 1.0:
        raise RuntimeError(f"native gather: {what} failed on some rank")


def native_gather(ctx, rank, world, timeout_ms=None):
    """The gather through the C ABI (rt_comm_init + rt_gather_image: RCCL sends to rank 0,
    de-interleave kernel there): rank 0 makes the communicator id, torch.distributed
    hands it to the other ranks and agrees, between the steps, that every rank got
    through the last one.  Returns the [H, W, 4] image on rank 0, None elsewhere.

    The agreements bound what one rank's failure can do to the others:
    rt_comm_init's argument checks are made on every rank before any rank enters
    ncclCommInitRank (a collective), and every rank's render is synchronised (rt_sync,
    which reports a device fault) before any rank enters the Send / Recv group.

    `timeout_ms` bounds rt_comm_init and rt_gather_image on every rank
    (rt_comm_set_timeout): a peer that never joins or never posts its half of the exchange
    makes the call raise RTError(RT_ERR_TIMEOUT) with the communicator aborted, not block."""
    from . import render
    if world == 1:
        return ctx.read_image()
    # rank 0 always takes part in the broadcast, id or not, so a failure to make the id (RCCL
    # not loadable) raises on every rank instead of leaving the others waiting for it
    uid, err = None, None
    if rank == 0:
        try:
            uid = render.comm_unique_id()
        except Exception as e:  # noqa: BLE001 -- reported on every rank below
            err = repr(e)
    box = [(uid, err)]
    dist.broadcast_object_list(box, src=0)
    uid, err = box[0]
    if uid is None:
        raise RuntimeError(f"rank 0 could not make an RCCL communicator id: {err}")
    # rt_comm_init's own preconditions (rt_capi.hip: a 1-device context partitioned as (rank, world))
    _agree(len(getattr(ctx, "devices", (0,))) == 1 and getattr(ctx, "rank", rank) == rank
           and getattr(ctx, "world", world) == world, "the rt_comm_init preconditions")
    ok = True
    try:
        if timeout_ms is not None:
            ctx.comm_set_timeout(timeout_ms)
        ctx.comm_init(uid, rank, world)
    except Exception:  # noqa: BLE001 -- every rank raises in _agree
        ok = False
    _agree(ok, "rt_comm_init")
    ok = True
    try:
        ctx.sync()
    except Exception:  # noqa: BLE001
        ok = False
    _agree(ok, "rt_sync before the gather")
    return ctx.gather_image()
