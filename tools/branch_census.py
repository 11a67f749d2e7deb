"""Branch census of one render kernel: the source lines (rt_kernel.hip, rt_glsl.h, ...) in front
of each exec-mask branch (`s_cbranch_execz` / `s_cbranch_execnz`), from `hipcc -S
-gline-tables-only` (the `.loc` directive last seen before the branch).  Lists where the
compiler kept `if`s as divergent-branch blocks.
usage: python tools/branch_census.py [--opt 47] [--block 1024] [--top 40]
"""
import argparse
import collections
import re
import subprocess

ROOT = __file__.rsplit("/tools/", 1)[0]
PKG = ROOT + "/raytracing-book_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", type=int, default=47, help="the kernel's OPT template argument (47: scene 8's)")
    ap.add_argument("--block", type=int, default=1024)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    asm = "/tmp/rt_kernel_census.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-slp-vectorize", "-gline-tables-only", "-I" + ROOT + "/include", "-I" + PKG + "/csrc",
                    "--cuda-device-only", "-S", "-o", asm, PKG + "/csrc/rt_kernel.hip"], check=True,
                   capture_output=True)
    head = re.compile(r"_ZN12_GLOBAL__N_117render_persistentILi4ELb0ELi%dELi%dEEEvPK14rt_kernel_args:"
                      % (a.block, a.opt))
    files, cur, inside = {}, None, False
    hist = collections.Counter()
    for line in open(asm):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
            continue
        if head.match(line):
            inside = True
            continue
        if inside and line.startswith(".Lfunc_end"):
            break
        if not inside:
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            cur = "%s:%s" % (files.get(m.group(1), m.group(1)), m.group(2))
        elif "s_cbranch_execz" in line or "s_cbranch_execnz" in line:
            hist[cur] += 1
    if not hist:
        raise SystemExit("kernel OPT=%d BLOCK=%d not found" % (a.opt, a.block))
    for k, v in hist.most_common(a.top):
        print("%4d  %s" % (v, k))
    print("total exec branches: %d" % sum(hist.values()))


if __name__ == "__main__":
    main()
