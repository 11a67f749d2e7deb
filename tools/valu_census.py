"""Static VALU census of one render kernel: the vector instructions of the compiled kernel
attributed to the source function they come from (`hipcc -S -gline-tables-only`: the `.loc`
line before each instruction, mapped to the enclosing function of rt_kernel.hip / rt_glsl.h).
Static counts (code size per function after inlining), not executions: a guide to where the
kernel's VALU code lives.  usage: python tools/valu_census.py [--opt 47] [--block 1024]
"""
import argparse
import collections
import re
import subprocess

ROOT = __file__.rsplit("/tools/", 1)[0]
PKG = ROOT + "/raytracing-book_amd"
SRC = {"rt_kernel.hip": PKG + "/csrc/rt_kernel.hip", "rt_kernel_common.h": PKG + "/csrc/rt_kernel_common.h",
       "rt_glsl.h": ROOT + "/include/rt/rt_glsl.h"}
DEF = re.compile(r"^(?:template\s*<[^>]*>\s*)?(?:__device__|__global__|RT_HD|__host__)[^(;]*?\b(\w+)\s*\(")


def function_of_lines(path):
    """line -> enclosing function name (the last definition header at or above the line)."""
    names, cur = {}, "?"
    for i, line in enumerate(open(path), 1):
        m = DEF.match(line)
        if m:
            cur = m.group(1)
        names[i] = cur
    return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", type=int, default=47)
    ap.add_argument("--block", type=int, default=1024)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    asm = "/tmp/rt_kernel_valu_census.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-slp-vectorize", "-gline-tables-only", "-I" + ROOT + "/include", "-I" + PKG + "/csrc",
                    "--cuda-device-only", "-S", "-o", asm, PKG + "/csrc/rt_kernel.hip"], check=True,
                   capture_output=True)
    fmap = {k: function_of_lines(v) for k, v in SRC.items()}
    head = re.compile(r"_ZN12_GLOBAL__N_117render_persistentILi4ELb0ELi%dELi%dEEEvPK14rt_kernel_args:"
                      % (a.block, a.opt))
    files, loc, inside = {}, ("?", 0), False
    per_fn, per_line = collections.Counter(), collections.Counter()
    total = 0
    for line in open(asm):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
            continue
        if head.match(line):
            inside = True
            continue
        if not inside:
            continue
        if line.startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            loc = (files.get(m.group(1), "?"), int(m.group(2)))
            continue
        if re.match(r"\s*v_", line):
            total += 1
            f, ln = loc
            fn = fmap.get(f, {}).get(ln, f) if f in fmap else f
            per_fn[fn] += 1
            per_line[f"{f}:{ln}"] += 1
    print(f"VALU instructions in render_persistent<..., {a.block}, ..., {a.opt}>: {total}")
    for fn, n in per_fn.most_common(a.top):
        print(f"{n:6d}  {fn}")


if __name__ == "__main__":
    main()
