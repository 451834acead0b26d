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


def short(name):
    """'void lh_inverse_kernel<4>(lh::InverseArgs)' -> 'lh_inverse_kernel'."""
    name = name[5:] if name.startswith("void ") else name
    return name.split("(")[0].split("<")[0]


def per_kernel(path, counter):
    vals = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter and short(row["Kernel_Name"]).startswith("lh_"):
            vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def main():
    out_dir, cfg = sys.argv[1], sys.argv[2]
    import bench
    k, m, nbytes, stripes, erasures = bench.CONFIGS[cfg]
    f = per_kernel(os.path.join(out_dir, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_kernel(os.path.join(out_dir, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    # decode bytes: read k slots, write e blocks per stripe -- e = min(k, m), or for the
    # random-erasure configs the mean e of tools/prof_kernels.py's workload (seed 3)
    if erasures == "random":
        es = [e for e, _ in bench.random_erasures(k, m, stripes, 3)]
        e = sum(es) / len(es)
    else:
        e = min(k, m)
    alg = {"encode": (k + m) * nbytes * stripes, "decode": (k + e) * nbytes * stripes}
    res = {"config": cfg, "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of "
                                    f"tools/prof_kernels.py {cfg}",
           "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of wide reads); WRITE_SIZE KiB x 1024",
           "algorithmic_bytes_per_launch": alg, "kernels": {}}
    for name in sorted(set(f) | set(w)):
        fb, wb = f.get(name, 0.0) * 2048, w.get(name, 0.0) * 1024
        res["kernels"][short(name)] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb}

    # Each phase's traffic: the sum over the kernels one encode_batch / decode_batch launches
    # (the large-m decode is planner + phase A + lh_inverse_kernel).
    import longhair_amd as lh
    for role, names in zip(("encode", "decode"), lh.kernel_names(k, m, nbytes)):
        got = [res["kernels"][n] for n in names if n in res["kernels"]]
        if got:
            tot = {key: sum(v[key] for v in got) for key in ("fetch_bytes", "write_bytes", "hbm_bytes_per_launch")}
            res[role] = dict(tot, kernel="+".join(n for n in names if n in res["kernels"]),
                             ratio_to_algorithmic=tot["hbm_bytes_per_launch"] / alg[role])
    path = os.path.join(REPO, "profiles", f"pmc_{cfg}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
