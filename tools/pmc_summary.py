#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) per lh_* kernel into
profiles/pmc_<config>.json, which bench.py reads for roofline.traffic.
FETCH_SIZE is doubled: on gfx950 it reports half of the bytes of wide streaming reads
(MI355X_MICROARCH.md, HBM).  Usage: pmc_summary.py OUTDIR CONFIG"""
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def per_kernel(path, counter):
    vals = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter and row["Kernel_Name"].lstrip("void ").startswith("lh_"):
            vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def main():
    out_dir, cfg = sys.argv[1], sys.argv[2]
    import bench
    k, m, nbytes, stripes, erasures = bench.CONFIGS[cfg]
    f = per_kernel(os.path.join(out_dir, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_kernel(os.path.join(out_dir, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    e = min(k, m)  # decode bytes for e = min(k, m); random-erasure configs write fewer blocks
    alg = {"encode": (k + m) * nbytes * stripes, "decode": (k + e) * nbytes * stripes}
    res = {"config": cfg, "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of "
                                    f"tools/prof_kernels.py {cfg}",
           "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of wide reads); WRITE_SIZE KiB x 1024",
           "algorithmic_bytes_per_launch": alg, "kernels": {}}
    for name in sorted(set(f) | set(w)):
        fb, wb = f.get(name, 0.0) * 2048, w.get(name, 0.0) * 1024
        res["kernels"][name] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb}

    def pick(words):
        for name, v in res["kernels"].items():
            if any(wd in name for wd in words):
                return name, v
        return None, None
    for role, words in (("encode", ["lh_jit_encode_win", "lh_jit_encode", "lh_apply_generic"]),
                        ("decode", ["lh_jit_decode_fused", "lh_jit_decode_wide", "lh_jit_decode", "lh_apply_generic"])):
        name, v = pick(words)
        if v:
            res[role] = dict(v, kernel=name, ratio_to_algorithmic=v["hbm_bytes_per_launch"] / alg[role])
    path = os.path.join(REPO, "profiles", f"pmc_{cfg}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
