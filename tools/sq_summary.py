#!/usr/bin/env python3
"""Summarise a rocprofv3 SQ counter pass (tools/gpu_pmc_sq.sh) per lh_* kernel into
profiles/sq_<config>.json, which bench.py reads for the VALU roofline of the large-m
configs: SQ_INSTS_VALU (wave-level VALU instructions per launch, median over dispatches)
and the wait / busy ratios.  Usage: sq_summary.py COUNTER_CSV CONFIG [OUT_JSON]"""
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """'void lh_inverse_kernel<4>(lh::InverseArgs)' -> 'lh_inverse_kernel'."""
    name = name[5:] if name.startswith("void ") else name
    return name.split("(")[0].split("<")[0]


def main():
    path, cfg = sys.argv[1], sys.argv[2]
    per = {}
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        if not short(name).startswith("lh_"):
            continue
        per.setdefault(name, {}).setdefault((row["Dispatch_Id"]), {})[row["Counter_Name"]] = float(row["Counter_Value"])
    out = {"config": cfg, "source": f"rocprofv3 --pmc SQ_* --kernel-trace of tools/prof_kernels.py {cfg}",
           "note": "SQ_INSTS_VALU counts wave-level VALU instructions; SQ_WAVE_CYCLES / SQ_WAIT_ANY in quad-cycles",
           "kernels": {}}
    for name, disp in per.items():
        agg = {}
        for c in sorted({c for d in disp.values() for c in d}):
            agg[c] = statistics.median(d[c] for d in disp.values() if c in d)
        if agg.get("SQ_WAVE_CYCLES"):
            agg["wait_any_frac"] = round(agg.get("SQ_WAIT_ANY", 0) / agg["SQ_WAVE_CYCLES"], 4)
        agg["dispatches"] = len(disp)
        out["kernels"][short(name)] = agg
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(REPO, "profiles", f"sq_{cfg}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
