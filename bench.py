#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X path tracer on the Book-2 final scene.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
it is launched under torch.distributed.run, one rank per GPU.  A *step* is one
pass of the hot path over one batch: every pixel of the image advanced by F
progressive frames (F samples per pixel) through rt_render.  With N ranks the
image rows are split into interleaved stripes and each step advances F*N
frames, so every rank does a fixed W x H x F samples per step (weak scaling).
value = all ranks' samples / max-over-ranks wall time of the K timed steps.
Inputs (scene buffers, image) are resident in HBM before the timed region.

Workloads (BASELINE.json configs; --preset, default c3 = the metric's config):
  c2  scene 0 (Book-1 final), 1920x1080, sqrt_spp for 1024 spp
  c3  scene 8 (Book-2 final), 1920x1080, sqrt_spp for 4096 spp   <- headline
  c4  scene 6 (Book-3 Cornell box), 1920x1080, sqrt_spp for 4096 spp
  c5  scene 8, 3840x2160, sqrt_spp for 8192 spp (the 8-GPU config)
max_depth 5 (the reference CLI default, Main.java:37) unless --depth.

The rank-0 JSON line carries
  * roofline: the render kernel against the VALU issue ceiling (bound "valu"):
    achieved = SQ_INSTS_VALU per launch (rocprofv3 PMC, committed in
    profiles/valu.json for this config) / the launch time measured here with
    HIP events on the kernel's stream; peak = 1024 SIMDs x 2.4 GHz / 2 cycles
    per wave64 VALU instruction (MI355X_MICROARCH.md:54,473; the microkernel
    tools/valu_peak.hip measures the 4-waves-per-SIMD ceiling, also reported);
  * cpu_baseline: the CPU oracle (oracle/, a restatement of the reference's
    GLSL; the reference has no CPU path) with one thread per CPU of the job's
    cgroup quota (else its affinity set), 30 s unpinned and 30 s with each thread
    pinned to its own physical core, on a bounded stripe of the same workload,
    plus its single-thread rate, the load average and the C1 CPU config in full;
  * gather_parity (N > 1): rank 0 re-renders each rank's first stripe alone and
    compares it bit for bit with the gathered image.
"""
import argparse
import json
import math
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SIMDS = 1024                   # 256 CUs x 4 SIMD-32
CLOCK_HZ = 2.4e9               # max clock
CYCLES_PER_VALU = 2.0          # wave64 VALU instruction on a SIMD-32 (MI355X_MICROARCH.md:54,473)
VALU_PEAK = SIMDS * CLOCK_HZ / CYCLES_PER_VALU / 1e9   # 1228.8 G wave-instructions/s
METRIC = "Msamples/sec (W×H×spp/s) on Book-2 final scene @1080p, 1/2/4/8 GPUs"

PRESETS = {
    "c2": dict(scene=0, width=1920, height=1080, spp_total=1024, name="C2 scene0 Book-1 final"),
    "c3": dict(scene=8, width=1920, height=1080, spp_total=4096, name="C3 scene8 Book-2 final"),
    "c4": dict(scene=6, width=1920, height=1080, spp_total=4096, name="C4 scene6 Book-3 Cornell box"),
    "c5": dict(scene=8, width=3840, height=2160, spp_total=8192, name="C5 scene8 Book-2 final 4K"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--preset", default="c3", choices=sorted(PRESETS))
    p.add_argument("--scene", type=int, default=None)
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--spp-total", type=int, default=None, help="sqrt_spp uniform (the config's spp)")
    p.add_argument("--frames-per-step", type=int, default=64, help="spp per step per rank")
    p.add_argument("--depth", type=int, default=5)
    p.add_argument("--stripe-rows", type=int, default=8)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=60.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--png", default=None)
    p.add_argument("--comm-timeout-ms", type=int, default=60000,
                   help="deadline of the native RCCL gather's rt_comm_init / rt_gather_image (rt_comm_set_timeout)")
    p.add_argument("--gather-deadline", type=float, default=240.0,
                   help="N > 1: seconds after the timed region by which gather + parity check must finish, "
                        "else the line is printed with the timed value and gather_path 'timeout' (LineGuard)")
    p.add_argument("--fast-bvh", action="store_true",
                   help="the non-parity fast mode (rt_set_bvh_mode RT_BVH_SAH): a separate line, never the headline")
    a = p.parse_args()
    pre = PRESETS[a.preset]
    for k in ("scene", "width", "height", "spp_total"):
        if getattr(a, k) is None:
            setattr(a, k, pre[k])
    a.workload_name = pre["name"] if all(getattr(a, k) == pre[k] for k in ("scene", "width", "height", "spp_total")) \
        else f"scene{a.scene}"
    return a


def config_key(a, frames):
    return f"scene{a.scene}_{a.width}x{a.height}_f{frames}_d{a.depth}" + ("_sah" if a.fast_bvh else "")


def bvh_counts(scene, args):
    """Node visits and prim tests per sample of the reference BVH and of the SAH tree, from the
    oracle's counters (the reference's stack walk over each tree) on a small render of the same
    scene (240x135, 8 frames): what the fast mode removes."""
    import types
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    import rtamd
    sc = rtamd.Scene(args.scene, 240, 135, seed=args.seed)
    rf = rtamd.frame_rand_factors(args.seed, 0, 8)
    out = {"sample": "oracle counters, 240x135, 8 frames, the same scene and depth"}
    for name, b in (("reference", sc.buffers[1]), ("sah", rtamd.sah_bvh(sc))):
        v = types.SimpleNamespace(**{k: getattr(sc, k) for k in ("textures", "camera", "background", "width",
                                                                 "height")})
        v.buffers = dict(sc.buffers)
        v.buffers[1] = b
        _, c = pyoracle.render(pyoracle.OracleScene(v, max_depth=args.depth, spp=args.spp_total), rf,
                               nthreads=min(16, os.cpu_count() or 1), counters=True)
        n = c["samples"]
        out[name] = {"bvh_nodes": len(b) // 32, "node_visits_per_sample": round(c["node_visits"] / n, 2),
                     "prim_tests_per_sample": round((c["sphere_tests"] + c["box_tests"] + c["quad_tests"] +
                                                     c["medium_tests"]) / n, 2)}
    return out


# ---------------------------------------------------------------- CPU baseline
def host_facts():
    model, sockets, cores_per = "unknown", set(), None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k = k.strip()
                if k == "model name" and model == "unknown":
                    model = v.strip()
                elif k == "physical id":
                    sockets.add(v.strip())
                elif k == "cpu cores" and cores_per is None:
                    cores_per = int(v)
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    phys = (len(sockets) or 1) * cores_per if cores_per else None
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "physical_cores": phys,
            "cgroup_cpu_quota": quota}


def cpu_threads(facts):
    """Threads for the CPU baseline: the CPUs this job may actually use.  One per visible CPU
    oversubscribes a cgroup quota (256 threads in a 16-CPU quota measured ~3.5x below 16
    threads), so the quota, rounded, when there is one, else the affinity count."""
    n = facts.get("affinity_cpus") or facts.get("nproc") or 1
    q = facts.get("cgroup_cpu_quota")
    if q:
        n = min(n, max(1, int(round(q))))
    return max(1, int(n))


def physical_core_cpus(cpus):
    """One logical CPU per physical core of `cpus` (the lowest id of each SMT sibling set,
    /sys/devices/system/cpu/cpu*/topology/thread_siblings_list), in id order."""
    cpus = sorted(set(cpus))
    seen, out = set(), []
    for c in cpus:
        try:
            txt = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
            sib = set()
            for part in txt.split(","):
                lo, _, hi = part.partition("-")
                sib.update(range(int(lo), int(hi or lo) + 1))
        except (OSError, ValueError):
            sib = {c}
        key = min(sib)
        if key in seen:
            continue
        seen.add(key)
        out.append(min(sib & set(cpus)) if sib & set(cpus) else c)
    return out


def _oracle_rate(pyoracle, rtamd, osc, W, H, rows_rank, rows_world, stripe, seed, seconds, threads):
    """Frames of the rows of one stripe set, in growing chunks, until `seconds`."""
    image = np.zeros((H, W, 4), np.float32)
    rows = rtamd.local_rows(H, rows_rank, rows_world, stripe)
    nf, chunk, dt = 0, 1, 0.0
    while dt < seconds and nf < 1 << 20:
        rf = rtamd.frame_rand_factors(seed, nf, chunk)
        t = time.perf_counter()
        pyoracle.render(osc, rf, first_frame=nf + 1, image=image, rank=rows_rank, world=rows_world,
                        stripe_rows=stripe, nthreads=threads)
        dt += time.perf_counter() - t
        nf += chunk
        chunk = max(1, min(2 * chunk, int((seconds - dt) / (dt / nf)) if dt < seconds else 1))
    return W * rows * nf, nf, rows, dt


def cpu_baseline(scene, args):
    """CPU oracle (oracle/, the build's scalar restatement of compute.glsl; the
    reference has no CPU path) on this host.  One thread per usable
    CPU (cpu_threads) on the full-width rows of stripe 0 of 8 of the same workload
    (the rate does not depend on spp), twice: threads left to the scheduler, and
    each thread pinned to its own physical core of the affinity set (one CPU per SMT
    pair); `value` is the better of the two.  Also: a 1-thread
    rate (pinned) on the same rows, the load average before and after, the C1 config
    (scene 9, 400x225, 64 spp, depth 8) rendered in full, and the host facts."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    import rtamd
    facts = host_facts()
    threads = cpu_threads(facts)
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count()))
    cores = physical_core_cpus(aff)
    pin = cores[:threads] if len(cores) >= threads else cores + [c for c in aff if c not in cores][:threads - len(cores)]
    load0 = os.getloadavg()
    osc = pyoracle.OracleScene(scene, max_depth=args.depth, spp=args.spp_total)
    W, H = scene.width, scene.height
    half = max(5.0, args.cpu_seconds / 2)

    def run(cpus, nthreads, seconds):
        pyoracle.set_thread_cpus(cpus)
        try:
            return _oracle_rate(pyoracle, rtamd, osc, W, H, 0, 8, args.stripe_rows, args.seed, seconds, nthreads)
        finally:
            pyoracle.set_thread_cpus(None)

    s_u, nf_u, rows, dt_u = run(None, threads, half)
    s_p, nf_p, _, dt_p = run(pin, threads, half)
    # one thread on the same rows (stripe 0 of 8), pinned, so that the rates compare like for like
    s1, nf1, rows1, dt1 = run(pin[:1], 1, min(15.0, args.cpu_seconds))
    load1 = os.getloadavg()
    # C1 (BASELINE.json configs[0]): the CPU reference path's own config, in full (pinned)
    c1 = rtamd.Scene(9, 400, 225, seed=args.seed)
    oc1 = pyoracle.OracleScene(c1, max_depth=8, spp=64)
    rf = rtamd.frame_rand_factors(args.seed, 0, 64)
    pyoracle.set_thread_cpus(pin)
    t = time.perf_counter()
    pyoracle.render(oc1, rf, first_frame=1, nthreads=threads)
    c1_s = time.perf_counter() - t
    pyoracle.set_thread_cpus(None)
    per_thread = s1 / dt1 / 1e6
    r_u, r_p = s_u / dt_u / 1e6, s_p / dt_p / 1e6
    best_pinned = r_p >= r_u
    samples, nf, dt = (s_p, nf_p, dt_p) if best_pinned else (s_u, nf_u, dt_u)
    return {
        "value": round(max(r_u, r_p), 3),
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "threads": threads,
        "threads_rule": "round(cgroup CPU quota), else the affinity CPU count, capped by both",
        "pinning": "pinned" if best_pinned else "unpinned",
        **facts,
        "sample": f"scene {args.scene} {W}x{H} max_depth {args.depth}: rows of stripe 0/8 ({rows} rows x {W}), "
                  f"{nf} frames = {samples} samples in {dt:.1f} s, {threads} threads "
                  f"({'one per physical core, pinned' if best_pinned else 'unpinned'})",
        "unpinned_msamples_s": round(r_u, 3),
        "pinned_msamples_s": round(r_p, 3),
        "pinned_cpus": pin,
        "physical_cores_in_affinity": len(cores),
        "single_thread_msamples_s": round(per_thread, 3),
        "single_thread_sample": f"the same rows, {nf1} frames = {s1} samples in {dt1:.1f} s, 1 thread pinned "
                                f"to CPU {pin[0] if pin else '?'}",
        "single_thread_x_threads_msamples_s": round(per_thread * threads, 3),
        "parallel_efficiency": round(max(r_u, r_p) / (per_thread * threads), 3),
        "parallel_efficiency_unpinned": round(r_u / (per_thread * threads), 3),
        "parallel_efficiency_pinned": round(r_p / (per_thread * threads), 3),
        "loadavg_start": [round(x, 2) for x in load0],
        "loadavg_end": [round(x, 2) for x in load1],
        "extrapolated_not_measured": {
            "physical_cores_x_single_thread_msamples_s": round(per_thread * facts["physical_cores"], 1)
            if facts["physical_cores"] else None,
            "note": "single-thread rate x the host's physical cores: an extrapolation for a host without the "
                    "job's CPU quota, not a measurement"},
        "c1": {"config": "scene 9 (Book-1 three spheres), 400x225, 64 spp, max_depth 8, full render",
               "samples": 400 * 225 * 64, "seconds": round(c1_s, 3),
               "msamples_s": round(400 * 225 * 64 / c1_s / 1e6, 3), "threads": threads, "pinned": True},
    }


# ---------------------------------------------------------------- gather parity
def gather_parity(scene, args, full, world, dev, factors, n_frames):
    """the gathered image checked bit for bit, on rank 0 after the timed
    region.  For every rank k, the first stripe it owns (stripe k, rows [8k, 8k+8)) is
    re-rendered alone -- a 1-device context partitioned as rank k of one rank per stripe,
    so it owns stripe k only -- over the same frames and rand factors, and compared with
    those rows of `full`.  A stripe block received at a wrong offset, a wrong rank's block
    or a wrong de-interleave shows up here; nan_pixels cannot catch it.  Any row partition
    renders the same bits as one GPU (tests/test_gpu_fullsize.py), so a match is exact."""
    import rtamd
    H, W, sr = args.height, args.width, args.stripe_rows
    n_stripes = (H + sr - 1) // sr
    ok, checked = True, []
    for k in range(min(world, n_stripes)):
        c = rtamd.RenderContext(devices=(dev,), rank=k, world=n_stripes, stripe_rows=sr)
        try:
            c.upload_scene(scene)
            c.set_params(max_depth=args.depth, spp=args.spp_total)
            c.resize(W, H)
            c.render(1, factors[:n_frames])
            blk = c.read_image()
        finally:
            c.close()
        ref = full[k * sr:min(H, (k + 1) * sr)]
        same = blk.shape == ref.shape and np.array_equal(np.isnan(blk), np.isnan(ref)) and \
            np.array_equal(blk.view(np.uint32)[~np.isnan(blk)], ref.view(np.uint32)[~np.isnan(ref)])
        ok = ok and bool(same)
        checked.append(k)
    return ok, checked


# ---------------------------------------------------------------- roofline
def roofline(args, frames_per_launch, samples_per_launch, avg_launch_ms):
    """VALU-issue roofline of render_persistent (see module docstring)."""
    def load(name):
        try:
            with open(os.path.join(REPO, "profiles", name)) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}
    key = config_key(args, frames_per_launch)
    profiles = load("valu.json")
    rec = profiles.get(key)
    if not rec:   # N > 1 launches more frames of 1/N of the rows: the 64-frame profile, per sample
        key = config_key(args, 64)
        rec = profiles.get(key)
    if not rec:
        log(f"no committed VALU profile for {key} (profiles/valu.json); roofline omitted")
        return None
    # the committed counts are for rec["samples_per_launch"]; scaled per sample if the launch differs
    per = samples_per_launch / rec["samples_per_launch"]
    insts = rec["SQ_INSTS_VALU"] * per
    t = avg_launch_ms * 1e-3
    achieved = insts / t / 1e9
    peak_meas = load("r02_valu_peak.json").get("wave_inst_per_s_4waves")
    traffic = rec["hbm_bytes_per_launch"] * per if rec.get("hbm_bytes_per_launch") else None
    lane = rec.get("valu_lane_utilization")
    out = {"bound": "valu", "achieved": round(achieved, 1), "peak": VALU_PEAK, "unit": "Gwave-inst/s",
           "frac": round(achieved / VALU_PEAK, 4), "traffic": traffic,
           "kernel": "render_persistent", "avg_launch_ms": round(avg_launch_ms, 3),
           "samples_per_launch": samples_per_launch, "valu_insts_per_launch": insts,
           "valu_lane_utilization": lane,
           "lane_weighted_frac": round(achieved / VALU_PEAK * lane, 4) if lane else None,
           "peak_measured_4waves_per_simd": round(peak_meas / 1e9, 1) if peak_meas else None,
           "frac_of_measured_4wave_peak": round(achieved * 1e9 / peak_meas, 4) if peak_meas else None,
           "dram_gbs": round(traffic / t / 1e9, 1) if traffic else None,
           "dram_frac": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
           "profile": key,
           "note": "achieved = SQ_INSTS_VALU per launch (rocprofv3 PMC, profiles/valu.json) / launch time measured "
                   "live with HIP events; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction; "
                   "lane_weighted_frac counts only the active lanes; traffic = DRAM bytes per launch "
                   "(FETCH_SIZE x2 + WRITE_SIZE), far below HBM: the scene is LDS/L2-resident"}
    return out


# ---------------------------------------------------------------- the line survives the gather
class LineGuard:
    """the timed value cannot be lost to the exchange after the timed region.

    Everything the line needs from the timed region is in `out` before the gather starts.  A
    watchdog (a daemon timer, `deadline_s`) then bounds the gather, its torch fallback and the
    gather parity check together: if they have not finished by then, rank 0 prints the line
    with the timed value and gather_path "timeout", every rank logs it and leaves with status 0
    (`exit_fn`, os._exit: a process blocked inside RCCL or a collective cannot unwind).  The
    product path is bounded itself as well (rt_comm_set_timeout, native_gather's timeout_ms);
    this is the last line of defence.  Exactly one line is printed either way."""

    def __init__(self, out, rank, deadline_s, exit_fn=os._exit, stream=None):
        self.out, self.rank, self.deadline_s, self.exit_fn = out, rank, deadline_s, exit_fn
        self.stream = stream
        self.lock = threading.Lock()
        self.printed = False
        self.timer = None
        if deadline_s and deadline_s > 0:
            self.timer = threading.Timer(deadline_s, self._fire)
            self.timer.daemon = True
            self.timer.start()

    def _print(self, line):
        print(json.dumps(line), file=self.stream or sys.stdout, flush=True)

    def _fire(self):
        with self.lock:
            if not self.printed and self.rank == 0:
                line = dict(self.out)
                line.update(gather_path="timeout", gather_native_error=(
                    f"gather + parity check did not finish within {self.deadline_s:g} s of the timed region; "
                    "the timed value stands"), gather_parity=None)
                self._print(line)
            self.printed = True
        log(f"rank {self.rank}: gather watchdog fired after {self.deadline_s:g} s; leaving")
        self.exit_fn(0)

    def emit(self, extra):
        """Print the line (rank 0) with the post-gather fields, unless the watchdog already did.
        The watchdog keeps running until close(): the final barrier is bounded too."""
        with self.lock:
            if self.printed:
                return
            self.printed = True
            if self.rank == 0:
                line = dict(self.out)
                line.update(extra)
                self._print(line)

    def close(self):
        if self.timer:
            self.timer.cancel()


def main():
    args = parse()
    import torch
    import rtamd
    from rtamd import dist as rdist

    # RT_BENCH_BACKEND=gloo RT_BENCH_DEVICE=0: rehearse the N-rank path with every
    # rank on one GPU (gloo collectives); the driver's real N-GPU runs use RCCL.
    rank, world, local_rank = rdist.init_from_env(os.environ.get("RT_BENCH_BACKEND"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev = int(os.environ.get("RT_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev)
    stream = torch.cuda.Stream(device=dev)

    scene = rtamd.Scene(args.scene, args.width, args.height, seed=args.seed)
    ctx = rtamd.RenderContext(devices=(dev,), rank=rank, world=world, stripe_rows=args.stripe_rows)
    if args.fast_bvh:
        ctx.set_bvh_mode("sah")
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=args.depth, spp=args.spp_total)
    ctx.resize(args.width, args.height)
    padded = ctx.padded_rows
    image = torch.zeros((padded, args.width, 4), dtype=torch.float32, device=f"cuda:{dev}")
    ctx.bind_device_image(image.data_ptr(), image.numel() * 4)
    ctx.set_stream(stream.cuda_stream)

    F = args.frames_per_step * world          # frames per step (weak scaling: fixed samples per rank)
    n_local_px = ctx.local_rows * args.width
    total_steps = args.warmup + args.steps
    factors = rtamd.frame_rand_factors(args.seed, 0, F * total_steps)
    frame = 1

    def step():
        nonlocal frame
        ctx.render(frame, factors[frame - 1:frame - 1 + F])
        frame += F

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        ev = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            step()
            e1.record(stream)
            ev.append((e0, e1))
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in ev]
    launches_per_step = math.ceil(F / 512)   # rt_render: equal launches of at most 512 frames
    avg_launch_ms = float(np.mean(kernel_ms)) / launches_per_step
    t_max = elapsed
    rank_ms = [avg_launch_ms]
    if world > 1:
        on_gpu = torch.distributed.get_backend() == "nccl"
        tdev = f"cuda:{dev}" if on_gpu else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        t_max = float(t.item())
        km = torch.tensor([avg_launch_ms], dtype=torch.float64, device=tdev)
        parts = [torch.zeros_like(km) for _ in range(world)]
        torch.distributed.all_gather(parts, km)
        rank_ms = [float(p.item()) for p in parts]

    samples_total = args.width * args.height * F * args.steps   # all ranks together
    value = samples_total / t_max / 1e6
    frames_per_launch = math.ceil(F / launches_per_step)
    samples_per_launch = n_local_px * frames_per_launch

    # The line's timed fields, complete before anything else runs (LineGuard): the gather below
    # cannot lose them.
    out = {
        "metric": METRIC + (" [fast mode: SAH BVH, non-parity]" if args.fast_bvh else ""),
        "value": round(value, 2),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: seeded scene {args.scene} (seed={args.seed}), built in-process",
        "config": {"workload": f"{args.workload_name}, {args.width}x{args.height}, sqrt_spp for {args.spp_total} spp, "
                               f"{args.frames_per_step} spp/step/rank, max_depth {args.depth}",
                   "preset": args.preset, "scene": args.scene, "width": args.width, "height": args.height,
                   "spp_total": args.spp_total, "spp_per_step": F, "max_depth": args.depth,
                   "stripe_rows": args.stripe_rows, "parallelism": f"row-stripes x{world}"},
        "kernel_ms_per_launch": {"max": round(max(rank_ms), 3), "min": round(min(rank_ms), 3)},
        "roofline": roofline(args, frames_per_launch, samples_per_launch, avg_launch_ms) if rank == 0 else None,
        "cpu_baseline": None,
    }
    if args.fast_bvh:
        out["fast_bvh"] = {"mode": "RT_BVH_SAH (rt_set_bvh_mode): non-parity fast mode, NOT the headline",
                           "parity": "statistical against the reference BVH (tests/test_gpu_fast_bvh.py, the gallery "
                                     "anchors); bit-exact against the oracle walking the same SAH tree",
                           "bvh_mode_ran": ctx.last_launch()["bvh_mode"]}
    if world > 1:
        log(f"rank {rank}: timed region done, {value:.1f} Msamples/s; gathering")
    guard = LineGuard(out, rank, args.gather_deadline if world > 1 else 0)
    extra = finish(args, scene, ctx, image, rank, world, dev, factors, F * total_steps)
    if rank != 0:
        guard.emit({})
        if world > 1:
            torch.distributed.barrier()
            torch.distributed.destroy_process_group()
        guard.close()
        return
    if args.fast_bvh:
        try:
            out["fast_bvh"]["bvh_counts"] = bvh_counts(scene, args)
        except Exception as e:  # noqa: BLE001 -- reported
            out["fast_bvh"]["bvh_counts_error"] = repr(e)
    cpu = None
    # the CPU baseline is an N = 1 figure (rank 0 of a one-GPU run); an N-rank run skips it so
    # the other ranks do not idle in the final barrier for a minute
    if not args.no_cpu_baseline and world == 1:
        try:
            cpu = cpu_baseline(scene, args)
        except Exception as e:  # the baseline is reported, not required
            log("cpu baseline failed:", repr(e))
    extra["cpu_baseline"] = cpu
    if world == 1:
        try:
            extra["camera_move_host_ms"] = camera_move_cost(ctx, scene, factors)
        except Exception as e:  # noqa: BLE001 -- reported, not required
            log("camera move cost failed:", repr(e))
    guard.emit(extra)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    guard.close()


def camera_move_cost(ctx, scene, factors, reps=5):
    """Host time a camera move adds to the next rt_render, after the timed region: the
    walk's node collapse is planned for the camera (rt_capi.hip plan_collapse, a grid of camera rays
    walked on the host, then the links rebuilt and re-uploaded), so an interactive host pays it on
    every move.  Median host time of a one-frame rt_render after a small translation of the camera,
    minus the same call with the camera unchanged (both enqueue only; the device work is not
    waited for).  Any plan is exact, so the image does not depend on it."""
    import torch
    cam = np.array(scene.camera, np.float32).copy()
    def call(moved, k):
        c = cam.copy()
        if moved:
            d = np.float32(0.01 * (k + 1))
            c[4:7] += d    # camera_pos (rt_camera_ubo)
            c[8:11] += d   # up_left: the same view, translated
        ctx.set_camera(c)
        torch.cuda.synchronize()
        t = time.perf_counter()
        ctx.render(1, factors[:1])
        dt = time.perf_counter() - t
        torch.cuda.synchronize()
        return dt
    call(False, 0)
    still = [call(False, 0) for _ in range(reps)]
    moved = [call(True, k) for k in range(reps)]
    ctx.set_camera(cam)
    return {"move_ms": round((float(np.median(moved)) - float(np.median(still))) * 1e3, 3),
            "render_call_still_ms": round(float(np.median(still)) * 1e3, 3),
            "render_call_moved_ms": round(float(np.median(moved)) * 1e3, 3),
            "what": "host time of a one-frame rt_render after a camera translation minus with the camera "
                    "unchanged (the collapse re-plan and link upload; bench.py camera_move_cost)"}


def finish(args, scene, ctx, image, rank, world, dev, factors, n_frames):
    """After the timed region: the gather of the accumulated stripes to rank 0 (reported
    separately, not in value) and, on rank 0, its bit-exact check.  The product's path behind
    the C ABI first (rt_comm_init + rt_gather_image: ncclSend to rank 0, de-interleave kernel
    there; what a Java host calls), bounded by --comm-timeout-ms on every rank; the torch
    gather is the reported fallback if that path fails on any rank (e.g. several ranks on one
    GPU in a rehearsal, or a timeout).  Returns the line's post-gather fields."""
    import torch
    from rtamd import dist as rdist
    full, gather_path, gather_err = None, None, None
    if torch.cuda.is_initialized():   # (a CPU test drives this with stand-in contexts)
        torch.cuda.synchronize()
    tg = time.perf_counter()
    try:
        if os.environ.get("RT_BENCH_GATHER") == "torch":   # escape hatch: the torch gather only
            raise RuntimeError("RT_BENCH_GATHER=torch")
        full = rdist.native_gather(ctx, rank, world, timeout_ms=args.comm_timeout_ms)
        gather_path = "rt_gather_image (RCCL send/recv + device de-interleave)" if world > 1 \
            else "rt_read_image (world 1)"
    except Exception as e:   # noqa: BLE001 -- any failure of the native path falls back
        gather_err = repr(e)[:300]
        log("native gather failed, falling back to torch.distributed.gather:", gather_err)
    ok = torch.tensor([0.0 if full is None and (rank == 0 or gather_err) else 1.0], dtype=torch.float64)
    if world > 1:   # every rank takes the same path
        ok = ok.to(f"cuda:{dev}" if torch.distributed.get_backend() == "nccl" else "cpu")
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
    if float(ok.item()) < 1.0:
        full = rdist.gather_image(image, args.height, world, args.stripe_rows)
        gather_path = "torch.distributed.gather (fallback)"
    if torch.cuda.is_initialized():   # (a CPU test drives this with stand-in contexts)
        torch.cuda.synchronize()
    gather_ms = (time.perf_counter() - tg) * 1e3
    if rank != 0:
        return {}
    if args.png:
        import rtamd
        rtamd.save_png(full, args.png)
    nan_px = int(np.isnan(full[..., :3]).any(axis=-1).sum())
    g_ok, g_stripes = None, []
    if world > 1 and not args.fast_bvh:   # other ranks wait in the final barrier meanwhile
        try:
            g_ok, g_stripes = gather_parity(scene, args, full, world, dev, factors, n_frames)
        except Exception as e:  # noqa: BLE001 -- reported, never fatal
            log("gather parity check failed to run:", repr(e))
    return {"gather_ms": round(gather_ms, 3), "gather_path": gather_path, "gather_native_error": gather_err,
            "gather_parity": g_ok, "gather_parity_stripes": len(g_stripes), "nan_pixels": nan_px}


if __name__ == "__main__":
    main()
