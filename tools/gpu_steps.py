#!/usr/bin/env python3
"""Table-driven runner for one GPU call (replaces the per-call probe_*.sh scripts of rounds 2-4).

    python tools/gpu_steps.py tools/calls/<table>.txt [name ...]

A table has one step per line: ``name  timeout_s  command...`` (lines starting with ``#`` are comments;
``$L`` expands to raytracing-book_amd/lib; leading ``VAR=value`` words set the step's environment).  Each step runs under ``timeout -k 10`` with its
output in gpurun_out/<name>.log; the runner prints the lines of that log that matter (medians,
bit checks, pytest totals, the bench JSON) and stops at the first step that fails, so a fault,
abort or time limit ends the call there.  Given names, only those steps run.
"""
import os
import re
import shlex
import subprocess
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = re.compile(r"median|DIFFER|passed|failed|error|smoke ok|bits|ratio|ms/launch|Msamples|^\{")


def steps(path):
    out = []
    for line in open(path):
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        name, to, cmd = line.split(None, 2)
        out.append((name, int(to), cmd.replace("$L", "raytracing-book_amd/lib")))
    return out


def main():
    table, only = sys.argv[1], set(sys.argv[2:])
    os.chdir(ROOT)
    os.makedirs("gpurun_out", exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    for name, to, cmd in steps(table):
        if only and name not in only:
            continue
        print(f"== {name}", flush=True)
        log = os.path.join("gpurun_out", f"{name}.log")
        argv, senv = shlex.split(cmd), dict(env)
        while argv and re.match(r"^[A-Z_][A-Z0-9_]*=", argv[0]):   # leading VAR=value: the step's env
            k, _, v = argv.pop(0).partition("=")
            senv[k] = v
        with open(log, "w") as f:
            rc = subprocess.call(["timeout", "-k", "10", str(to)] + argv, stdout=f, stderr=subprocess.STDOUT,
                                 env=senv)
        print(f"== {name} rc={rc}", flush=True)
        with open(log, errors="replace") as f:
            lines = f.read().splitlines()
        for ln in [x for x in lines if KEEP.search(x)][-40:]:
            print("   " + ln[:400])
        if lines:
            print("   tail: " + lines[-1][:300], flush=True)
        if rc != 0:
            sys.exit(rc)


if __name__ == "__main__":
    main()
