"""Live-VGPR audit of a release render kernel, per source region (VERDICT r5 Weak 3 / Next 1).

Which part of `render_persistent` sets its 128 VGPRs?  The kernel is compiled for gfx950 with the
release flags plus `-gline-tables-only` (the instruction stream is the release one up to a handful
of instructions: the tool reports the difference), disassembled, and every instruction is
attributed to a region through its inline stack (llvm-symbolizer --inlining): the first frame below
`render_stream`, or the line range of `render_stream` itself for the scheduling code.  A backward
liveness analysis over the kernel's control-flow graph (branch targets from the disassembly) gives
the VGPRs live at every instruction, counted on the allocated (physical) registers, AGPRs included.

Limits, stated in the report: an exec-masked write is taken as a full definition (a value a
divergent block overwrites in some lanes is counted dead above that block on its path); a call
(`s_swappc_b64`) is taken as using nothing and defining nothing, so its callee's own registers are
reported apart (from -Rpass-analysis=kernel-resource-usage).

usage: python tools/vgpr_audit.py [--opt 47] [--block 1024] [--out profiles/r06_vgpr_audit.txt]
"""
import argparse
import bisect
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytracing-book_amd")
LLVM = "/opt/rocm/lib/llvm/bin"
HIPFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC",
            "-I" + ROOT + "/include", "-I" + PKG + "/csrc", "--cuda-device-only", "-c"]

REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")
TARGET = re.compile(r"<[^>+]*\+0x([0-9a-f]+)>")
ADDR = re.compile(r"//\s*([0-9A-Fa-f]{8,}):")


def build(tmp, dbg):
    src = os.path.join(PKG, "csrc", "rt_kernel.hip")
    bundle = os.path.join(tmp, "vgpr_audit_%s.o" % ("dbg" if dbg else "rel"))
    cmd = ["/opt/rocm/bin/hipcc"] + HIPFLAGS + (["-gline-tables-only"] if dbg else []) + [
        "-o", bundle, src, "-Rpass-analysis=kernel-resource-usage"]
    rep = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    elf = bundle + ".gfx950"
    subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + bundle,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + elf], check=True)
    return elf, rep


def resources(rep):
    """Function name -> {remark: value} from the resource-usage remarks."""
    out, cur = {}, None
    for line in rep.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return out


def disasm(elf, sym):
    txt = subprocess.run([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", "--disassemble-symbols=" + sym, elf],
                         capture_output=True, text=True, check=True).stdout
    ins = []
    for line in txt.splitlines():
        m = ADDR.search(line)
        if not m or not line.startswith("\t"):
            continue
        body = line.split("//")[0].strip()
        op, _, rest = body.partition(" ")
        t = TARGET.search(line)
        ins.append({"addr": int(m.group(1), 16), "op": op, "args": rest.strip(),
                    "target": int(t.group(1), 16) if t and op.startswith("s_") and "branch" in op else None})
    return ins


def regs(s):
    out = set()
    for m in REG.finditer(s):
        base = 0 if m.group(1) == "v" else 256
        if m.group(2) is not None:
            out.add(base + int(m.group(2)))
        else:
            out.update(range(base + int(m.group(3)), base + int(m.group(4)) + 1))
    return out


def split_ops(args):
    ops, depth, cur = [], 0, ""
    for ch in args:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def def_use(i):
    op, ops = i["op"], split_ops(i["args"])
    if op.startswith("s_") or not ops:
        return set(), set()
    first = regs(ops[0].split()[0]) if ops else set()
    rest = set()
    for o in ops[1:]:
        rest |= regs(o)
    store_like = (op.startswith(("ds_write", "ds_store", "global_store", "flat_store", "scratch_store", "buffer_store"))
                  or (op.startswith(("ds_", "global_atomic", "flat_atomic", "buffer_atomic")) and "rtn" not in op
                      and not op.startswith(("ds_read", "ds_bpermute", "ds_permute", "ds_swizzle"))
                      and " sc0" not in " " + i["args"] and "glc" not in i["args"]))
    if store_like:
        return set(), first | rest
    if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set(), first | rest
    partial = (op.startswith(("v_fmac", "v_mac", "v_pk_fmac", "v_writelane", "v_swap", "v_dot2c"))
               or "UNUSED_PRESERVE" in i["args"] or re.search(r"dst_sel:(?!DWORD)", i["args"]) is not None)
    return first, (first | rest) if partial else rest


def liveness(ins):
    idx = {x["addr"]: k for k, x in enumerate(ins)}
    n = len(ins)
    succ = [[] for _ in range(n)]
    for k, x in enumerate(ins):
        op = x["op"]
        if op in ("s_endpgm", "s_setpc_b64"):
            continue
        if x["target"] is not None and x["target"] + ins[0]["addr"] in idx:
            succ[k].append(idx[x["target"] + ins[0]["addr"]])
        elif x["target"] is not None and x["target"] in idx:
            succ[k].append(idx[x["target"]])
        if op != "s_branch" and k + 1 < n:
            succ[k].append(k + 1)
    du = [def_use(x) for x in ins]
    dmask = [sum(1 << r for r in d) for d, _ in du]
    umask = [sum(1 << r for r in u) for _, u in du]
    live_in = [0] * n
    live_out = [0] * n
    pred = [[] for _ in range(n)]
    for k in range(n):
        for s in succ[k]:
            pred[s].append(k)
    work = collections.deque(range(n - 1, -1, -1))
    inq = [True] * n
    while work:
        k = work.popleft()
        inq[k] = False
        lo = 0
        for s in succ[k]:
            lo |= live_in[s]
        li = umask[k] | (lo & ~dmask[k])
        live_out[k] = lo
        if li != live_in[k]:
            live_in[k] = li
            for p in pred[k]:
                if not inq[p]:
                    inq[p] = True
                    work.append(p)
    return [max(bin(a).count("1"), bin(b).count("1")) for a, b in zip(live_in, live_out)], live_in, live_out


def symbolize(elf, addrs):
    inp = "\n".join("0x%x" % a for a in addrs) + "\n"
    out = subprocess.run([LLVM + "/llvm-symbolizer", "--obj=" + elf, "--inlining", "--functions=short", "-C"],
                         input=inp, capture_output=True, text=True, check=True).stdout
    stacks, cur = [], []
    lines = out.split("\n")
    k = 0
    while k < len(lines):
        if lines[k] == "":
            if cur or k + 1 < len(lines):
                stacks.append(cur)
            cur = []
            k += 1
            continue
        fn, loc = lines[k], lines[k + 1] if k + 1 < len(lines) else "?:0:0"
        f, _, rest = loc.rpartition(":")
        f2, _, ln = f.rpartition(":")
        cur.append((fn, os.path.basename(f2), int(ln) if ln.isdigit() else 0))
        k += 2
    return stacks[:len(addrs)]


# render_stream's own lines (rt_kernel.hip) by scheduling part
def stream_part(path, line, src_lines):
    for name, lo, hi in src_lines:
        if lo <= line <= hi:
            return name
    return "render_stream (other)"


def stream_ranges():
    """Line ranges of render_stream's parts, found from their comments in rt_kernel.hip."""
    src = open(os.path.join(PKG, "csrc", "rt_kernel.hip")).read().splitlines()
    marks = [("watchdog", "a progress watchdog"), ("fold", "fold the units whose samples"),
             ("claim", "claim samples for the FRESH lanes"), ("begin", "a new walk (bounce()"),
             ("rounds", "rounds of node walk + leaf tests"), ("shade-tail", "shade the HIT lanes together"),
             ("pass-tail", "the samples stored in this pass"), ("end", "__global__ void")]
    pos = []
    for name, text in marks:
        for k, l in enumerate(src):
            if text in l:
                pos.append((name, k + 1))
                break
    out = []
    for (name, a), (_, b) in zip(pos, pos[1:]):
        out.append(("sched:" + name, a, b - 1))
    return out


REGION_OF = [
    ("link_walk", "NODE"), ("load_node", "NODE"), ("spine_entry", "BEGIN"),
    ("leaf_prims_t", "LEAF"), ("after_trace", "SHADE"), ("start_path", "START"), ("stage_lds", "STAGE"),
    ("unit_geo", "sched:unit_geo"), ("wait_chunk", "sched:fold"), ("publish_chunk", "sched:fold"),
]


def region(stack, ranges):
    # outermost first
    st = list(reversed(stack))
    for k, (fn, f, ln) in enumerate(st):
        if fn.startswith("render_stream") or "render_stream<" in fn:
            if k + 1 >= len(st):
                return stream_part(f, ln, ranges), None
            nxt = st[k + 1][0]
            for key, reg in REGION_OF:
                if key in nxt:
                    sub = st[k + 2][0].split("(")[0].split("<")[0] if k + 2 < len(st) else "-"
                    return reg, sub
            # an inlined helper called from render_stream's own code: its call line decides
            return stream_part(f, st[k][2] if False else ln, ranges), nxt.split("(")[0]
    fn = st[0][0] if st else "?"
    for key, reg in REGION_OF:
        if any(key in x[0] for x in st):
            return reg, None
    return "kernel:" + fn.split("(")[0].split("<")[0], None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", type=int, default=47)
    ap.add_argument("--block", type=int, default=1024)
    ap.add_argument("--out", default=None)
    ap.add_argument("--tmp", default="/tmp")
    a = ap.parse_args()
    sym = "_ZN12_GLOBAL__N_117render_persistentILi4ELb0ELi%dELi%dEEEvPK14rt_kernel_args" % (a.block, a.opt)
    elf_d, rep_d = build(a.tmp, True)
    elf_r, rep_r = build(a.tmp, False)
    ins = disasm(elf_d, sym)
    ins_r = disasm(elf_r, sym)
    res_r = resources(rep_r)
    ops_d = [x["op"] for x in ins]
    ops_r = [x["op"] for x in ins_r]
    sm = __import__("difflib").SequenceMatcher(a=ops_d, b=ops_r, autojunk=False)
    same = sum(b.size for b in sm.get_matching_blocks())
    counts, live_in, live_out = liveness(ins)
    stacks = symbolize(elf_d, [x["addr"] for x in ins])
    ranges = stream_ranges()
    out = []
    p = out.append
    p("# Live-VGPR audit: render_persistent<4, false, %d, %d> (tools/vgpr_audit.py)" % (a.block, a.opt))
    rr = next((v for k, v in res_r.items() if k == sym), {})
    p("release build: VGPRs %s, AGPRs %s, VGPR spills %s, SGPR spills %s, scratch %s B/lane, occupancy %s waves/SIMD"
      % (rr.get("VGPRs"), rr.get("AGPRs"), rr.get("VGPRs Spill"), rr.get("SGPRs Spill"),
         rr.get("ScratchSize [bytes/lane]"), rr.get("Occupancy [waves/SIMD]")))
    p("instructions: %d in the -gline-tables-only build, %d in the release build, %d matched in order (%.2f%%)"
      % (len(ops_d), len(ops_r), same, 100.0 * same / max(len(ops_r), 1)))
    for k, v in res_r.items():
        if "render_persistent" not in k and "fold" not in k and "deinter" not in k and "eval_builtin" not in k:
            p("callee %s: VGPRs %s, SGPRs %s, scratch %s B/lane" % (k, v.get("VGPRs"), v.get("SGPRs"),
                                                                    v.get("ScratchSize [bytes/lane]")))
    maxreg = 0
    for x in ins:
        for r in regs(x["args"]):
            if r < 256:
                maxreg = max(maxreg, r + 1)
    p("highest VGPR index used + 1: %d" % maxreg)
    by = collections.defaultdict(list)
    sub = collections.defaultdict(list)
    for k, x in enumerate(ins):
        rg, sb = region(stacks[k] if k < len(stacks) else [], ranges)
        by[rg].append(k)
        if sb:
            sub[(rg, sb)].append(k)
    p("")
    p("%-24s %7s %7s %7s %7s %7s" % ("region", "instrs", "max", "p90", "p50", ">=120"))
    def row(name, ks):
        cs = sorted(counts[k] for k in ks)
        q = lambda f: cs[min(len(cs) - 1, int(f * len(cs)))]
        p("%-24s %7d %7d %7d %7d %7d" % (name[:24], len(ks), cs[-1], q(0.9), q(0.5), sum(c >= 120 for c in cs)))
    order = sorted(by, key=lambda r: -max(counts[k] for k in by[r]))
    for r in order:
        row(r, by[r])
    p("")
    p("sub-regions (the first inlined frame below the region's function), by max live VGPRs:")
    for (r, sb), ks in sorted(sub.items(), key=lambda kv: -max(counts[k] for k in kv[1]))[:40]:
        row("  %s/%s" % (r, sb), ks)
    p("")
    # the state a region carries through: VGPRs live at its instructions that the region neither
    # reads nor writes (the path / hit record / schedule state of the lanes), against those it uses
    p("carried-through VGPRs (live at the region's peak instruction, not touched anywhere in the region):")
    for r in order:
        ks = by[r]
        touched = 0
        for k in ks:
            d, u = def_use(ins[k])
            touched |= sum(1 << x for x in d | u)
        kp = max(ks, key=lambda k: counts[k])
        lv = live_in[kp] | live_out[kp]
        p("  %-22s peak %3d: %3d carried through, %3d used by the region; the region touches %3d VGPRs in all"
          % (r[:22], counts[kp], bin(lv & ~touched).count("1"), bin(lv & touched).count("1"), bin(touched).count("1")))
    p("")
    p("SGPR spill traffic (v_writelane / v_readlane), scratch accesses and calls by region:")
    for r in order:
        c = collections.Counter(ins[k]["op"] for k in by[r])
        wl, rl = c["v_writelane_b32"], c["v_readlane_b32"]
        sc = sum(v for o, v in c.items() if o.startswith("scratch_"))
        cl = c["s_swappc_b64"]
        if wl or rl or sc or cl:
            p("  %-22s writelane %3d  readlane %3d  scratch %2d  calls %2d" % (r[:22], wl, rl, sc, cl))
    # the out-of-line callees (perlin turbulence, the medium's boundary): highest VGPR they use
    syms = subprocess.run([LLVM + "/llvm-readelf", "-sW", elf_r], capture_output=True, text=True).stdout
    for line in syms.splitlines():
        f = line.split()
        if (len(f) >= 8 and f[3] == "FUNC" and "render_persistent" not in f[7]
                and not re.search(r"(fold|deinterleave|eval_builtin)_kernel", f[7])):
            cins = disasm(elf_r, f[7])
            mx = max([r + 1 for x in cins for r in regs(x["args"]) if r < 256] or [0])
            p("  callee %s: %d instructions, highest VGPR index + 1 = %d" % (f[7], len(cins), mx))
    p("")
    # what a smaller register budget would cost: the 512-thread instantiation of the same OPT at
    # 5 and 6 waves per SIMD (the kernel's MINW template argument), spills by the compiler's report
    src = open(os.path.join(PKG, "csrc", "rt_kernel.hip")).read()
    for w in (5, 6):
        alt = os.path.join(a.tmp, "vgpr_audit_w%d.hip" % w)
        with open(alt, "w") as f:
            f.write(src.replace("render_persistent<4, false, BLOCK, OPT>", "render_persistent<%d, false, BLOCK, OPT>" % w))
        rep = subprocess.run(["/opt/rocm/bin/hipcc"] + HIPFLAGS + ["-o", alt + ".o", alt,
                              "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
        rw = resources(rep).get(sym.replace("ILi4ELb0ELi%d" % a.block, "ILi%dELb0ELi512" % w), {})
        p("at %d waves per SIMD (512-thread instantiation): VGPRs %s, VGPR spills %s, scratch %s B/lane"
          % (w, rw.get("VGPRs"), rw.get("VGPRs Spill"), rw.get("ScratchSize [bytes/lane]")))
    p("")
    peak = max(counts)
    pk = [k for k in range(len(ins)) if counts[k] >= peak - 2]
    p("instructions within 2 of the peak (%d live): %d; their source lines:" % (peak, len(pk)))
    lines = collections.Counter()
    for k in pk:
        st = stacks[k] if k < len(stacks) else []
        if st:
            fn, f, ln = st[0]
            lines["%s:%d (%s) [%s]" % (f, ln, fn.split("(")[0][:40], region(st, ranges)[0])] += 1
    for l, c in lines.most_common(25):
        p("  %4d  %s" % (c, l))
    txt = "\n".join(out)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
