"""Register / spill / scratch report of the render kernels (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python tools/kernel_resources.py [--ab]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
PKG = ROOT + "/raytracing-book_amd"


def main():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC",
           "-I" + ROOT + "/include", "-I" + PKG + "/csrc", "--cuda-device-only", "-c", "-o", "/tmp/rt_kernel_dev.o",
           PKG + "/csrc/rt_kernel.hip", "-Rpass-analysis=kernel-resource-usage"]
    if "--ab" in sys.argv:
        cmd.insert(1, "-DRT_AB_KNOBS")
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    for r in rows:
        if "render_persistent" not in r["name"] and "fold" not in r["name"]:
            continue
        tpl = re.search(r"ILb(\d)ELi(\d)ELb(\d)ELb(\d)ELi(\d+)ELb(\d)ELi(\d+)E", r["name"])
        tag = ("LINK=%s MINW=%s STATS=%s LDSN=%s BLOCK=%s FAST=%s OPT=%s" % tpl.groups()) if tpl else r["name"]
        print(f"{tag:60s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>3} "
              f"spillV {r.get('VGPRs Spill', '?'):>3} spillS {r.get('SGPRs Spill', '?'):>3} "
              f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
