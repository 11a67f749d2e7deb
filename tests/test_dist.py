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


class _FakeCtx:
    """Stands in for rtamd.RenderContext in the native gather's host logic (no GPU here)."""

    def __init__(self, rank, image=None, world=2, fail_init=False):
        self.rank, self.image, self.uid, self.calls = rank, image, None, []
        self.world, self.devices, self.fail_init = world, (0,), fail_init

    def sync(self):
        self.calls.append("sync")

    def read_image(self):
        self.calls.append("read_image")
        return self.image

    def comm_init(self, uid, rank, world):
        self.calls.append(("comm_init", rank, world))
        if self.fail_init:
            raise OSError("rt_comm_init: ncclCommInitRank failed")
        self.uid = bytes(uid)

    def gather_image(self):
        self.calls.append("gather_image")
        return self.image if self.rank == 0 else None


def test_native_gather_world1_is_read_image():
    """at world 1 the C-ABI gather (bench.py's gather path) is rt_read_image."""
    img = np.random.default_rng(1).random((7, 5, 4), dtype=np.float32)
    c = _FakeCtx(0, img, world=1)
    out = rdist.native_gather(c, 0, 1)
    assert out is img and c.calls == ["read_image"]


def _native_worker(rank, world, port, q, fail=False, fail_init_rank=None):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        rdist.init_from_env(backend="gloo")
        import rtamd.render as R

        def fake_uid():
            assert rank == 0, "only rank 0 makes the communicator id"
            if fail:
                raise OSError("librccl.so.1: cannot open shared object file")
            return bytes(range(7, 7 + 128))
        R.comm_unique_id = fake_uid
        c = _FakeCtx(rank, np.full((3, 2, 4), 5.0, np.float32) if rank == 0 else None, world=world,
                     fail_init=rank == fail_init_rank)
        try:
            out = rdist.native_gather(c, rank, world)
            q.put((rank, c.uid, c.calls, None if out is None else out.shape))
        except RuntimeError as e:
            q.put((rank, "raised", c.calls, str(e)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report, never hang the parent
        q.put(("error", f"rank {rank}: {e!r}"))


def test_native_gather_hands_rank0_id_to_every_rank():
    """The native gather's host side at world 2 (gloo): rank 0 makes the RCCL id, torch.distributed
    broadcasts it, every rank runs rt_comm_init(id, rank, world) then rt_gather_image; only rank 0
    returns an image."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not q.empty():
        msgs.append(q.get())
    assert len(msgs) == world and all(m[0] != "error" for m in msgs), msgs
    by_rank = {m[0]: m for m in msgs}
    uid = bytes(range(7, 7 + 128))
    for r in range(world):
        _, got, calls, shape = by_rank[r]
        assert got == uid and calls == [("comm_init", r, world), "sync", "gather_image"], (r, calls)
        assert shape == ((3, 2, 4) if r == 0 else None)


def test_native_gather_id_failure_raises_on_every_rank():
    """If rank 0 cannot make the RCCL id, every rank raises (none waits for a broadcast that
    never comes); bench.py then falls back to the torch gather on all ranks."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_worker, args=(r, world, port, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not q.empty():
        msgs.append(q.get())
    assert sorted(m[0] for m in msgs) == [0, 1], msgs
    for m in msgs:
        assert m[1] == "raised" and m[2] == [] and "cannot open" in m[3], m


def test_native_gather_one_rank_comm_init_failure_raises_on_every_rank():
    """if only rank 1 fails in rt_comm_init, rank 0 must not go on into rt_gather_image
    (its Recv would wait for a Send that never comes): every rank raises, none calls gather_image,
    and bench.py falls back to the torch gather on all ranks."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_worker, args=(r, world, port, q, False, 1)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not q.empty():
        msgs.append(q.get())
    assert sorted(m[0] for m in msgs) == [0, 1], msgs
    for m in msgs:
        assert m[1] == "raised" and "gather_image" not in m[2] and "rt_comm_init" in m[3], m


def test_bench_cpu_threads_follow_the_quota():
    """the CPU baseline uses the job's CPUs (cgroup quota, else affinity), not nproc."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.cpu_threads({"nproc": 256, "affinity_cpus": 256, "cgroup_cpu_quota": 16.0}) == 16
    assert bench.cpu_threads({"nproc": 256, "affinity_cpus": 8, "cgroup_cpu_quota": 16.0}) == 8
    assert bench.cpu_threads({"nproc": 256, "affinity_cpus": 12, "cgroup_cpu_quota": None}) == 12
    assert bench.cpu_threads({"nproc": 4, "affinity_cpus": 4, "cgroup_cpu_quota": 0.4}) == 1
    # one CPU per physical core of the affinity set for the pinned run
    cores = bench.physical_core_cpus(sorted(os.sched_getaffinity(0)))
    assert cores and len(set(cores)) == len(cores) and set(cores) <= set(os.sched_getaffinity(0))


def test_gather_single_rank_is_identity():
    block = torch.from_numpy(np.random.default_rng(0).random((16, 5, 4), dtype=np.float32))
    img = rdist.gather_image(block, 13, 1, 16)
    assert img.shape == (13, 5, 4) and np.array_equal(img, block[:13].numpy())


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


class _BlockingCtx(_FakeCtx):
    """A context whose rt_gather_image never returns (a peer that never posts its half)."""

    def gather_image(self):
        import threading
        self.calls.append("gather_image")
        threading.Event().wait()


def _hang_worker(rank, world, port, path, block):
    try:
        import types
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        rdist.init_from_env(backend="gloo")
        import rtamd.render as R
        R.comm_unique_id = lambda: bytes(range(128))
        bench = _bench_module()
        img = np.zeros((4, 3, 4), np.float32)
        cls = _BlockingCtx if block else _FakeCtx
        ctx = cls(rank, img if rank == 0 else None, world=world)
        ctx.comm_set_timeout = lambda ms: ctx.calls.append(("timeout", ms))
        out = {"metric": "m", "value": 6803.59, "unit": "Msamples/s", "n_gpus": world}
        args = types.SimpleNamespace(comm_timeout_ms=1000, height=4, stripe_rows=8, png=None, fast_bvh=False,
                                     gather_deadline=3.0)
        with open(f"{path}.{rank}", "w") as f:
            guard = bench.LineGuard(out, rank, args.gather_deadline, stream=f)
            extra = bench.finish(args, None, ctx, None, rank, world, 0, None, 0)
            guard.emit(extra)
            dist.barrier()
            dist.destroy_process_group()
            guard.close()
    except Exception as e:  # noqa: BLE001 -- reported through the file
        with open(f"{path}.{rank}.err", "w") as f:
            f.write(repr(e))
        os._exit(3)


def _run_hang(tmp_path, block):
    import json
    import time
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    path = str(tmp_path / "line")
    t = time.perf_counter()
    procs = [ctx.Process(target=_hang_worker, args=(r, world, port, path, block)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    took = time.perf_counter() - t
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = [open(f"{path}.{r}.err").read() for r in range(world) if os.path.exists(f"{path}.{r}.err")]
    assert not errs, errs
    lines = [json.loads(x) for x in open(f"{path}.0").read().splitlines() if x.strip()]
    rest = open(f"{path}.1").read()
    return lines, rest, [p.exitcode for p in procs], took


def test_bench_line_survives_a_gather_that_never_returns(tmp_path):
    """rank 0's rt_gather_image blocks forever (its peer never posts).  The
    bench's watchdog (LineGuard) still prints exactly one line with the timed value and
    gather_path "timeout", and every rank leaves with status 0 well before any outer limit."""
    lines, rest, codes, took = _run_hang(tmp_path, True)
    assert len(lines) == 1, lines
    assert lines[0]["value"] == 6803.59 and lines[0]["gather_path"] == "timeout", lines[0]
    assert rest == "" and codes == [0, 0], (rest, codes)
    assert took < 60, took


def test_bench_line_once_when_the_gather_completes(tmp_path):
    """The same harness with a gather that completes: one line, the native path's fields, no
    watchdog line after it (close() stops the timer)."""
    lines, rest, codes, _ = _run_hang(tmp_path, False)
    assert len(lines) == 1, lines
    ln = lines[0]
    assert ln["value"] == 6803.59 and ln["gather_path"].startswith("rt_gather_image"), ln
    assert ln["gather_native_error"] is None and ln["nan_pixels"] == 0, ln
    assert rest == "" and codes == [0, 0], (rest, codes)


def test_native_gather_sets_the_deadline_before_comm_init():
    """native_gather hands timeout_ms to rt_comm_set_timeout before rt_comm_init (world 1 has no
    communicator and reads the image)."""
    c = _FakeCtx(0, np.zeros((2, 2, 4), np.float32), world=1)
    assert rdist.native_gather(c, 0, 1, timeout_ms=5) is c.image and c.calls == ["read_image"]
