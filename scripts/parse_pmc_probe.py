"""Summarise scripts/pmc_probe.sh output: per-dispatch averages of every counter
for kernels whose name contains a filter, plus derived ratios.

    python scripts/parse_pmc_probe.py <tag> [kernel-substring]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def main(tag, filt="render_"):
    per_kernel = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(OUT, f"pmcp_{tag}_*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if filt not in k:
                    continue
                per[(row["Dispatch_Id"], k, row["Counter_Name"])] += float(row["Counter_Value"])
        for (_, k, c), v in per.items():
            per_kernel[k.split("(")[0][:90]][c].append(v)
    res = {}
    for k, cs in per_kernel.items():
        c = {n: sum(v) / len(v) for n, v in cs.items()}
        d = {}
        if "SQ_INSTS_VALU" in c and "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
            d["lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / max(c["SQ_ACTIVE_INST_VALU"] * 64, 1)
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
            d["valu_active_per_wave_cycle"] = c["SQ_ACTIVE_INST_VALU"] / max(c["SQ_WAVE_CYCLES"], 1)
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
            d["wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            d["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1)
        res[k] = {"counters": c, "derived": d}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
