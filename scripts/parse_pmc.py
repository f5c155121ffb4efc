"""Summarise rocprofv3 PMC passes (scripts/profile_pmc.sh) for the render kernel.

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) KiB -> bytes; FETCH_SIZE is
doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half the bytes of a wide
coalesced read; FETCH_SIZE counts Infinity-Cache hits too).  Writes
profiles/pmc_config<X>.json, which bench.py reads for roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.environ.get("PMC_DIR", os.path.join(ROOT, "gpurun_out"))
sys.path.insert(0, ROOT)
from bench import kernel_source_digest  # noqa: E402


def bench_variant(name):
    """The kernel variant the profiled bench run launched (its JSON line)."""
    for line in reversed(open(os.path.join(OUT, f"pmc_{name}.log")).read().splitlines()):
        if line.startswith("{"):
            m = re.search(r"variant ([^)]+)\)", json.loads(line)["roofline"]["kernel"] or "")
            return m.group(1) if m else None
    return None


def load(name):
    files = glob.glob(os.path.join(OUT, f"pmc_{name}", "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)  # (kernel, counter) -> per-dispatch values
    for f in files:
        per = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if "render_" not in k:
                    continue
                per[(row["Dispatch_Id"], k, row["Counter_Name"])] += float(row["Counter_Value"])
        for (disp, k, c), v in per.items():
            vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items() if v}


def main(config="B"):
    res = {}
    for name in ("fetch", "write", "valu", "salu", "clock", "wait", "l2", "mfma"):
        if os.path.isdir(os.path.join(OUT, f"pmc_{name}")):
            res.update(load(name))
    out = {"config": config, "kernel_variant": bench_variant("fetch"),
           "kernel_source_sha256": kernel_source_digest("bvh" if config.endswith("_bvh") else "brute"), "counters_per_launch": res}
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        out["hbm_bytes_per_launch"] = int((2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024)
    trace = glob.glob(os.path.join(OUT, "pmc_clock", "**", "*kernel_trace.csv"), recursive=True)
    durs = []
    for f in trace:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "render_" in row.get("Kernel_Name", ""):
                    durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    if durs:
        out["kernel_ns_profiled"] = sum(durs) / len(durs)
        if "GRBM_GUI_ACTIVE" in res:
            # the clock the kernel held (MI355X_MICROARCH.md "DVFS give-back": GRBM_GUI_ACTIVE sums the 8
            # XCDs); bench.py prices the matrix roofline at this clock beside the 2.4 GHz spec
            out["clock_ghz"] = res["GRBM_GUI_ACTIVE"] / 8 / out["kernel_ns_profiled"]
    if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
        out["l2_hit_rate"] = res["TCC_HIT_sum"] / max(res["TCC_HIT_sum"] + res["TCC_MISS_sum"], 1.0)
    if "SQ_THREAD_CYCLES_VALU" in res and "SQ_ACTIVE_INST_VALU" in res:
        out["valu_lane_utilisation"] = res["SQ_THREAD_CYCLES_VALU"] / (64.0 * res["SQ_ACTIVE_INST_VALU"])
    if "SQ_ACTIVE_INST_VALU" in res and "SQ_WAVE_CYCLES" in res:
        out["valu_active_frac_of_wave_cycles"] = res["SQ_ACTIVE_INST_VALU"] / res["SQ_WAVE_CYCLES"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in res and "GRBM_GUI_ACTIVE" in res:
        # busy cycles summed over the SIMDs (1,024) vs the kernel's GPU cycles (GRBM_GUI_ACTIVE is per XCD x 8)
        out["mfma_busy_frac"] = res["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * res["GRBM_GUI_ACTIVE"] / 8)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    path = os.path.join(ROOT, "profiles", f"pmc_config{config}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(sys.argv[1:] or ["B"]))
