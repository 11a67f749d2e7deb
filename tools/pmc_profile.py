"""Collect rocprofv3 PMC counters for the render kernel, one counter group per
pass (separate rocprofv3 runs, --kernel-trace only alongside --pmc), and write a
summary JSON.  Run on the GPU box:  python tools/pmc_profile.py --out profiles/pmc_r01.json
HBM traffic per the MI355X guide: FETCH_SIZE under-reports coalesced reads by 2x
on gfx950 and is in KB; we report FETCH_SIZE*1024 (raw) and the x2-corrected
bound, plus WRITE_SIZE*1024."""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GROUPS = [
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM", "SQ_INSTS_LDS"],
    ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"],
    ["SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU_TRANS_F32"],
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
    ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"],
    ["GRBM_GUI_ACTIVE", "GRBM_COUNT"],
    ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_SCRATCH" if False else "SQ_INSTS_FLAT"],
    ["SQ_WAIT_INST_LDS", "SQ_INSTS_BRANCH", "SQ_INST_CYCLES_VMEM", "SQ_ACTIVE_INST_SCA"],
    ["TA_TA_BUSY_sum", "TA_FLAT_READ_WAVEFRONTS_sum", "GRBM_GUI_ACTIVE"],
    ["TD_TD_BUSY", "TD_TC_STALL"],
    ["SQ_ACTIVE_INST_VMEM", "SQ_INST_CYCLES_VMEM_RD", "SQ_BUSY_CU_CYCLES", "SQ_INST_LEVEL_VMEM",
     "SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_TA_CMD_FIFO_FULL"],
    ["TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_RDRET_STALL_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum",
     "TCP_TCP_TA_DATA_STALL_CYCLES_sum"],
    # 14, 15: instruction fetch (SQC instruction cache) and where wave time goes
    ["SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE", "SQC_ICACHE_REQ"],
    ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_IFETCH", "SQ_IFETCH_LEVEL",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA"],
]


def available():
    try:
        out = subprocess.run(["rocprofv3", "-L"], capture_output=True, text=True, timeout=120).stdout
    except Exception:
        return None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "pmc.json"))
    ap.add_argument("--target", default="--scene 8 --frames 64")
    ap.add_argument("--traffic-key", default="scene8_1920x1080_f64_d5")
    ap.add_argument("--traffic-out", default=os.path.join(REPO, "gpurun_out", "traffic.json"))
    ap.add_argument("--groups", default=None, help="comma list of group indices (default all)")
    ap.add_argument("--valu-key", default=None, help="bench.py config key: write the roofline record to --valu-out")
    ap.add_argument("--valu-out", default=os.path.join(REPO, "gpurun_out", "valu.json"))
    ap.add_argument("--samples", type=int, default=1920 * 1080 * 64, help="samples in the profiled launch")
    a = ap.parse_args()
    listing = available() or ""
    res = {}
    os.makedirs(os.path.join(REPO, "gpurun_out", "pmc"), exist_ok=True)
    sel = None if a.groups is None else {int(g) for g in a.groups.split(",")}
    for gi, grp in enumerate(GROUPS):
        if sel is not None and gi not in sel:
            continue
        grp = [c for c in grp if not listing or c in listing]
        if not grp:
            continue
        d = os.path.join(REPO, "gpurun_out", "pmc", f"g{gi}")
        cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--kernel-trace", "--pmc", *grp, "--output-format", "csv",
               "-d", d, "-o", "run", "--", sys.executable, os.path.join(REPO, "tools", "render_once.py"),
               *a.target.split()]
        r = subprocess.run(cmd, capture_output=True, text=True)
        print("group", gi, grp, "rc", r.returncode, flush=True)
        if r.returncode not in (0,):
            print(r.stderr[-2000:], flush=True)
            if r.returncode in (124, 134, 137, 139):
                break
            continue
        # sum a counter over this pass's rows (dimensions / XCDs); a counter that an
        # earlier group already measured keeps that pass's value (never summed across passes)
        got = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if "render_" not in row.get("Kernel_Name", ""):
                        continue
                    name = row.get("Counter_Name")
                    got[name] = got.get(name, 0.0) + float(row.get("Counter_Value", 0))
        for name, val in got.items():
            res.setdefault(name, val)
    # per launch (render_once --launches 1 => one render dispatch per pass)
    if "FETCH_SIZE" in res:
        res["hbm_read_bytes_raw"] = res["FETCH_SIZE"] * 1024
        res["hbm_read_bytes_x2"] = res["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in res:
        res["hbm_write_bytes"] = res["WRITE_SIZE"] * 1024
    if "hbm_read_bytes_x2" in res and "hbm_write_bytes" in res:
        res["hbm_bytes_per_launch"] = res["hbm_read_bytes_x2"] + res["hbm_write_bytes"]
    if "SQ_THREAD_CYCLES_VALU" in res and "SQ_ACTIVE_INST_VALU" in res and res["SQ_ACTIVE_INST_VALU"]:
        res["valu_lane_utilization"] = res["SQ_THREAD_CYCLES_VALU"] / (64.0 * res["SQ_ACTIVE_INST_VALU"])
    if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
        res["tcc_hit_rate"] = res["TCC_HIT_sum"] / max(1.0, res["TCC_HIT_sum"] + res["TCC_MISS_sum"])
    res["target"] = a.target
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))
    if a.valu_key and "SQ_INSTS_VALU" in res:
        # the record bench.py's roofline reads (profiles/valu.json)
        vj = {}
        if os.path.exists(a.valu_out):
            with open(a.valu_out) as f:
                vj = json.load(f)
        rec = {k: res[k] for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VALU_TRANS_F32", "valu_lane_utilization",
                                   "hbm_bytes_per_launch", "hbm_read_bytes_x2", "hbm_write_bytes", "tcc_hit_rate")
               if k in res}
        rec["samples_per_launch"] = a.samples
        rec["target"] = a.target
        rec["method"] = ("rocprofv3 --kernel-trace --pmc, one counter group per pass, one render launch "
                         "(tools/render_once.py); FETCH_SIZE x2 (gfx950) + WRITE_SIZE")
        vj[a.valu_key] = rec
        with open(a.valu_out, "w") as f:
            json.dump(vj, f, indent=1, sort_keys=True)
    if a.traffic_key and "hbm_bytes_per_launch" in res:
        # the entry bench.py reads as roofline.traffic
        tj = {}
        if os.path.exists(a.traffic_out):
            with open(a.traffic_out) as f:
                tj = json.load(f)
        tj[a.traffic_key] = {k: res[k] for k in ("hbm_bytes_per_launch", "hbm_read_bytes_raw", "hbm_read_bytes_x2",
                                                 "hbm_write_bytes") if k in res}
        tj[a.traffic_key]["method"] = ("rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE in separate passes "
                                       "(KB); reads x2 per the gfx950 FETCH_SIZE correction; one launch")
        tj[a.traffic_key]["target"] = a.target
        with open(a.traffic_out, "w") as f:
            json.dump(tj, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
