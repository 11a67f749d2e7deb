"""GPU tests of the rt.h boundary beyond the per-scene parity cases.

All through the C ABI on cuda:0, each compared bit for bit (NaN positions
equal) against the committed golden fixtures or the CPU oracle:
golden vectors, stripe partitions (one process per rank, several contexts on
one GPU), ragged/tiny sizes, max_depth edge values, >512 frames per call,
image write/read and resume, caller-bound device image + caller stream, every
kernel variant, the multi-device host gather, the RaytraceExecutor mirror, and
the ABI's error behaviour.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import rtamd
from helpers import bit_equal, gpu_image, mismatch_report, oracle_image

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden_cases():
    with open(os.path.join(GOLDEN, "index.json")) as f:
        return sorted(json.load(f).items(), key=lambda kv: int(kv[0]))


@pytest.mark.parametrize("sid,case", _golden_cases(), ids=lambda v: v if isinstance(v, str) else "")
def test_golden_fixtures(gpu, sid, case):
    """Device render == the committed oracle fixture (no oracle call at run time)."""
    s = rtamd.Scene(int(sid), case["width"], case["height"], seed=case["seed"])
    g = np.load(os.path.join(GOLDEN, case["file"]))
    out = gpu_image(s, case["frames"], max_depth=case["depth"], spp=case["spp"], seed=case["seed"])
    assert bit_equal(out, g["image"]), mismatch_report(out, g["image"])


@pytest.mark.parametrize("world,stripe", [(2, 16), (3, 4), (8, 1), (5, 64)])
def test_stripe_partition_contexts(gpu, world, stripe):
    """rt_set_partition: each rank's context renders only its stripes, stripe-compacted;
    de-interleaved they equal the unpartitioned render."""
    H, W = 45, 33
    s = rtamd.Scene(8, W, H, seed=1)
    full = gpu_image(s, 4)
    padded = rtamd.padded_local_rows(H, world, stripe)
    blocks = np.zeros((world, padded, W, 4), np.float32)
    for r in range(world):
        ctx = rtamd.RenderContext(devices=(0,), rank=r, world=world, stripe_rows=stripe)
        ctx.upload_scene(s)
        ctx.set_params(max_depth=5, spp=4)
        ctx.resize(W, H)
        ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
        loc = ctx.read_image()
        assert loc.shape[0] == rtamd.local_rows(H, r, world, stripe)
        blocks[r, :loc.shape[0]] = loc
        ctx.close()
    img = rtamd.deinterleave(blocks, H, world, stripe)
    assert bit_equal(img, full), mismatch_report(img, full)


@pytest.mark.parametrize("devices", [(0, 0), (0, 0, 0)])
def test_multi_device_context_device_gather(gpu, devices):
    """A context over several device slots (here device 0 repeated) splits rows in stripes;
    rt_read_image gathers the blocks on device 0 (peer copies: RCCL allows one rank per
    device) and de-interleaves them there; equals the single-slot render."""
    s = rtamd.Scene(6, 40, 37, seed=1)
    a = gpu_image(s, 4)
    ctx = rtamd.RenderContext(devices=devices)
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=4)
    ctx.resize(40, 37)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
    b = ctx.read_image()
    assert ctx.gather_path() == "peer"
    ctx.close()
    assert bit_equal(a, b), mismatch_report(a, b)


def test_process_communicator_gather(gpu):
    """rt_comm_unique_id / rt_comm_init / rt_gather_image: the RCCL path a one-process-per-GPU
    host takes without any Python harness, here as a world-1 communicator on one GPU (the
    N-rank sends are unmeasured on this one-GPU box)."""
    s = rtamd.Scene(8, 48, 27, seed=1)
    ref = oracle_image(s, 3)
    ctx = rtamd.RenderContext()
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=3)
    ctx.resize(48, 27)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 3))
    with pytest.raises(rtamd.RTError, match="rt_comm_init"):
        ctx.gather_image()
    ctx.comm_init(rtamd.comm_unique_id(), 0, 1)
    out = ctx.gather_image()
    assert ctx.gather_path() == "rccl"
    ctx.close()
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_process_communicator_times_out_without_its_peer(gpu):
    """rank 0 of a world-2 communicator whose rank 1 never joins.  With a
    2 s deadline (rt_comm_set_timeout) rt_comm_init returns RT_ERR_TIMEOUT with the
    communicator aborted, instead of blocking in ncclCommInitRank; the context still renders
    and reads its stripes, and a gather asks for rt_comm_init again."""
    import time
    s = rtamd.Scene(8, 48, 27, seed=1)
    ctx = rtamd.RenderContext(rank=0, world=2, stripe_rows=8)
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=2)
    ctx.resize(48, 27)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 2))
    ctx.comm_set_timeout(2000)
    t = time.perf_counter()
    with pytest.raises(rtamd.RTError, match="no completion within 2000 ms") as e:
        ctx.comm_init(rtamd.comm_unique_id(), 0, 2)
    took = time.perf_counter() - t
    assert e.value.code == -6 and took < 30, (e.value, took)
    with pytest.raises(rtamd.RTError, match="rt_comm_init"):
        ctx.gather_image()
    ctx.comm_abort()   # idempotent
    blk = ctx.read_image()
    ref = oracle_image(s, 2)
    rows = rtamd.stripe_rows_of(27, 0, 2, 8)
    ctx.close()
    assert bit_equal(blk, ref[rows]), mismatch_report(blk, ref[rows])


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (65, 9), (3, 70), (129, 1)])
def test_ragged_sizes(gpu, w, h):
    """Sizes that are not multiples of the 8x8 wave tile."""
    s = rtamd.Scene(8, w, h, seed=1)
    ref = oracle_image(s, 3)
    out = gpu_image(s, 3)
    assert bit_equal(out, ref), mismatch_report(out, ref)


@pytest.mark.parametrize("depth", [0, 1, 2, 50])
def test_max_depth_edges(gpu, depth):
    s = rtamd.Scene(7, 24, 24, seed=1)
    ref = oracle_image(s, 3, max_depth=depth)
    out = gpu_image(s, 3, max_depth=depth)
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_more_frames_than_one_launch(gpu):
    """1100 frames in one rt_render call (> RT_MAX_FRAMES_PER_LAUNCH = 512): three equal
    launches of 367 / 367 / 366 frames."""
    s = rtamd.Scene(3, 8, 8, seed=1)
    ref = oracle_image(s, 1100, spp=1100)
    out = gpu_image(s, 1100, spp=1100)
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_write_image_and_resume(gpu):
    """rt_write_image + continue == uninterrupted progressive render (resume from a checkpoint)."""
    s = rtamd.Scene(4, 20, 16, seed=1)
    full = gpu_image(s, 6, spp=6)
    ctx = rtamd.RenderContext()
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=6)
    ctx.resize(20, 16)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 3))
    half = ctx.read_image()
    ctx.close()
    ctx = rtamd.RenderContext()
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=6)
    ctx.resize(20, 16)
    ctx.write_image(half)
    assert bit_equal(ctx.read_image(), half)
    ctx.render(4, rtamd.frame_rand_factors(1, 3, 3))
    out = ctx.read_image()
    ctx.close()
    assert bit_equal(out, full), mismatch_report(out, full)


def test_bound_torch_image_and_stream(gpu):
    """rt_bind_device_image + rt_set_stream: the kernel accumulates into a torch tensor on
    torch's stream (the path bench.py times)."""
    import torch
    s = rtamd.Scene(8, 48, 27, seed=1)
    ref = oracle_image(s, 4)
    img = torch.zeros((27, 48, 4), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.Stream(device=0)
    ctx = rtamd.RenderContext()
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=4)
    ctx.set_stream(stream.cuda_stream)
    ctx.resize(48, 27)                                    # sizes the image the bound buffer must hold
    ctx.bind_device_image(img.data_ptr(), img.numel() * 4)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
    stream.synchronize()
    out = img.cpu().numpy()
    ctx.close()
    assert bit_equal(out, ref), mismatch_report(out, ref)


VARIANTS = [0, 37, 30, 61]   # streamed batched pooled samples (default), one pixel per lane (round-1 default), threaded meta walk, exact near-first walk


# work splits (rt_capi.hip rt_render; rt_debug.h RT_OPTION_*): one unit per tile with all
# frames (folded per wave), ordered frame chunks handed over between waves, staged chunks
# (the default)
SPLITS = {
    "direct": {"chunk_target": 0},
    "ordered1": {"stage_tiles": 0, "chunk_target": 1},
    "ordered16": {"stage_tiles": 0, "chunk_target": 16},
    "ordered_max": {"stage_tiles": 0, "chunk_target": 100000},
    "staged": {},
    "staged_max": {"staged_chunk_target": 100000},
}


@pytest.mark.parametrize("sid", [8, 6, 7])
@pytest.mark.parametrize("split", list(SPLITS))
def test_all_kernel_variants_identical(gpu, split, sid):
    """The release kernel under every work split (SPLITS), and every structure of the A/B
    build (RT_OPTION_KERNEL_VARIANT, librtamd_ab.so) render the same bits; scenes 8
    (canonical boxes, media, Perlin, image texture), 6 and 7 (rotated boxes: the general
    box test)."""
    s = rtamd.Scene(sid, 40, 24, seed=1)
    ref = oracle_image(s, 6)
    out = gpu_image(s, 6, options=SPLITS[split])
    assert bit_equal(out, ref), f"release, split {split}: {mismatch_report(out, ref)}"
    for v in VARIANTS:
        out = gpu_image(s, 6, options=dict(SPLITS[split], kernel_variant=v), ab=True)
        assert bit_equal(out, ref), f"A/B variant {v}, split {split}: {mismatch_report(out, ref)}"


@pytest.mark.parametrize("split", ["ordered_max", "staged_max"])
def test_chunk_chain_small_image(gpu, split):
    """Few tiles, many chunks: each of the 15 tiles' 600 frames in one-frame chunks over
    2 launches (300 + 300 frames): ordered, every chunk waits for the previous one (the
    hand-off is on the critical path; render_stream folds two units per wave in claim
    order); staged, every chunk's colours folded by fold_kernel."""
    s = rtamd.Scene(8, 40, 24, seed=1)
    ref = oracle_image(s, 600, spp=600)
    out = gpu_image(s, 600, spp=600, options=SPLITS[split])
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_stats_build_renders_same_bits(gpu):
    """The diagnostic build (rt_debug_enable_stats, A/B library) changes timing only; the
    release library has no stats kernels."""
    s = rtamd.Scene(8, 40, 24, seed=1)
    ref = oracle_image(s, 2)
    rel = rtamd.RenderContext()
    assert rtamd.amd().rt_debug_enable_stats(rel._h, 1) == -3
    rel.close()
    L = rtamd.amd_ab()
    ctx = rtamd.RenderContext(ab=True)
    assert L.rt_debug_enable_stats(ctx._h, 1) == 0
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=2)
    ctx.resize(40, 24)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 2))
    out = ctx.read_image()
    stats = (ctypes.c_ulonglong * 64)()
    assert L.rt_debug_read_stats(ctx._h, stats, 64) == 0
    ctx.close()
    assert bit_equal(out, ref), mismatch_report(out, ref)
    assert any(stats[k] for k in range(64))


def test_executor_mirror(gpu):
    """RaytraceExecutor: setSamplePerPixel, raytrace until sampleComplete, listeners fire once."""
    s = rtamd.Scene(6, 16, 16, seed=9)
    ctx = rtamd.RenderContext()
    ctx.upload_scene(s)
    ctx.resize(16, 16)
    ex = rtamd.RaytraceExecutor(ctx, seed=9)
    fired = []
    ex.addCompleteListener(lambda: fired.append(ex.getNumSamples()))
    ex.setSamplePerPixel(10)
    while not ex.sampleComplete():
        ex.raytrace(4)
    assert ex.getNumSamples() == 10 and fired == [10] and ex.getFinishTime() >= 0
    out = ctx.read_image()
    ctx.close()
    ref = oracle_image(s, 10, spp=10, seed=9)
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_error_behaviour(gpu):
    L = rtamd.amd()
    ctx = rtamd.RenderContext()
    h = ctx._h
    rf = rtamd.frame_rand_factors(1, 0, 1)
    fp = rf.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert L.rt_render(h, 1, 1, fp) == -3                    # RT_ERR_STATE: nothing uploaded / no image
    assert b"rt_resize" in L.rt_last_error(h) or b"BVH" in L.rt_last_error(h)
    assert L.rt_upload_buffer(h, 0, b"\0" * 47, 47) == -1    # not a multiple of the 48-byte sphere record
    assert L.rt_upload_buffer(h, 6, b"", 0) == -1            # no binding 6
    assert L.rt_upload_texture(h, 8, 1, 1, 1, b"\0\0\0") == -4    # RT_ERR_LIMIT: slots 0..7
    s = rtamd.Scene(6, 8, 8, seed=1)
    ctx.upload_scene(s)
    ctx.resize(8, 8)
    assert L.rt_render(h, 0, 1, fp) == -1                    # frames are 1-based (frame_count = ++numSamples)
    assert L.rt_render(h, 1, 1, None) == -1
    with pytest.raises(rtamd.RTError, match="bad image size"):
        ctx.resize(-1, 8)
    ctx.close()


def test_context_teardown_frees_device_memory(gpu):
    """rt_destroy frees everything a context allocated (the packed Perlin table and the
    sparse staging flags leaked): eight create / upload / staged sparse render / destroy cycles of
    scene 8 (Perlin texture, 640x360x64 frames: 14.7 MB of flags and 236 MB of staged colours per
    context) leave the device's free memory where the first cycle left it."""
    import torch
    s = rtamd.Scene(8, 640, 360, seed=1)

    def cycle():
        ctx = rtamd.RenderContext()
        ctx.upload_scene(s)
        ctx.set_params(max_depth=5, spp=4096)
        ctx.resize(640, 360)
        ctx.render(1, rtamd.frame_rand_factors(1, 0, 64))
        ctx.sync()
        info = ctx.last_launch()
        ctx.close()
        return info

    info = cycle()   # the runtime's first-use allocations
    assert info["staged"] and info["sparse"], info
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(8):
        cycle()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 < (32 << 20), (free0, free1)
