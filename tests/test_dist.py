"""Multi-process stripe partition + gather on CPU (gloo, world_size 2 and 3).

Each rank renders only the stripes it owns (here with the oracle, standing in
for the device render, since there is no GPU), compacts them into the
[padded_rows, W, 4] block layout rt.h produces for a partitioned context, and
calls rtamd.dist.gather_image — the same function bench.py uses over RCCL.
Rank 0 checks the gathered image bit for bit against a single-process render.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle
import rtamd
from rtamd import dist as rdist
from helpers import bit_equal

H, W, STRIPE = 29, 12, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        r, w, _ = rdist.init_from_env(backend="gloo")
        assert (r, w) == (rank, world)
        sc = rtamd.Scene(8, W, H, seed=1)
        o = pyoracle.OracleScene(sc, max_depth=4, spp=4)
        rf = rtamd.frame_rand_factors(1, 0, 2)
        part = pyoracle.render(o, rf, rank=rank, world=world, stripe_rows=STRIPE, nthreads=2)
        rows = rtamd.stripe_rows_of(H, rank, world, STRIPE)
        block = torch.zeros((rtamd.padded_local_rows(H, world, STRIPE), W, 4), dtype=torch.float32)
        block[:len(rows)] = torch.from_numpy(part[rows])
        img = rdist.gather_image(block, H, world, STRIPE)
        if rank == 0:
            full = pyoracle.render(o, rf, nthreads=2)
            q.put(("ok", bool(bit_equal(img, full))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report, never hang the parent
        q.put(("error", f"rank {rank}: {e!r}"))


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_stripe_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not q.empty():
        msgs.append(q.get())
    assert ("ok", True) in msgs, msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_gather_single_rank_is_identity():
    block = torch.from_numpy(np.random.default_rng(0).random((16, 5, 4), dtype=np.float32))
    img = rdist.gather_image(block, 13, 1, 16)
    assert img.shape == (13, 5, 4) and np.array_equal(img, block[:13].numpy())
