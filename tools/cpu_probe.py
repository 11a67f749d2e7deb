"""Host CPU facts for bench.py's cpu_baseline: CPU model, nproc, the affinity
mask and the cgroup CPU quota, plus the CPU oracle's throughput at a few
thread counts on a fixed workload (scene 8, 1920 px wide rows), so the thread
count the baseline uses is the one that actually gets the host's cores.
Usage: python tools/cpu_probe.py [--seconds S] [--threads 16,32,...]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_quota():
    """CPUs the cgroup quota allows (cpu.max 'quota period'), or None."""
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(p).read().split()[:2]
            if q != "max":
                return float(q) / float(per)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def host_facts():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": cgroup_quota()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--threads", default=None)
    a = ap.parse_args()
    facts = host_facts()
    print(json.dumps(facts), flush=True)
    import numpy as np
    import pyoracle
    import rtamd
    scene = rtamd.Scene(8, 1920, 1080, seed=1)
    osc = pyoracle.OracleScene(scene, max_depth=5, spp=4096)
    counts = [int(t) for t in a.threads.split(",")] if a.threads else sorted(
        {1, 8, 16, 32, 64, facts["affinity_cpus"] or 1, facts["nproc"] or 1})
    for t in counts:
        img = np.zeros((1080, 1920, 4), np.float32)
        nf, dt = 0, 0.0
        while dt < a.seconds:
            rf = rtamd.frame_rand_factors(1, nf, 1)
            t0 = time.perf_counter()
            # rows of stripe 0 of 16 (68 rows x 1920)
            pyoracle.render(osc, rf, first_frame=nf + 1, image=img, rank=0, world=16, stripe_rows=8, nthreads=t)
            dt += time.perf_counter() - t0
            nf += 1
        rows = rtamd.local_rows(1080, 0, 16, 8)
        print(json.dumps({"threads": t, "frames": nf, "seconds": round(dt, 2),
                          "msamples_per_s": round(rows * 1920 * nf / dt / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
