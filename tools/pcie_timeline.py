#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --memory-copy-trace run of tools/pcie_bench.py:
for each host-batch call (encode, decode; found as the gaps between bursts of activity),
the wall time, the busy time of host-to-device copies, device-to-host copies and kernels
(union of their intervals), and how much of the wall time the host link carried a copy in
each direction.  Usage: pcie_timeline.py PROF_DIR"""
import csv
import glob
import os
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    d = sys.argv[1]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ev = []
    for r in (rows(kt[0]) if kt else []):
        ev.append(("K:" + r.get("Kernel_Name", "?").split("(")[0][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0))
    for r in (rows(mt[0]) if mt else []):
        kind = r.get("Direction") or r.get("Kind") or r.get("Operation") or "?"
        ev.append(("C:" + kind, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r.get("Bytes", 0) or 0)))
    ev.sort(key=lambda x: x[1])
    if not ev:
        print("no events")
        return
    # split into calls: a gap of > 2 ms with nothing running separates two host-batch calls
    calls, cur, end = [], [], None
    for e in ev:
        if end is not None and e[1] - end > 2_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = e[2] if end is None else max(end, e[2])
    calls.append(cur)
    for i, c in enumerate(calls):
        t0, t1 = min(e[1] for e in c), max(e[2] for e in c)
        kinds = sorted({e[0] for e in c})
        line = [f"call {i}: {len(c)} events, wall {(t1 - t0) / 1e6:.2f} ms"]
        for k in kinds:
            iv = [(e[1], e[2]) for e in c if e[0] == k]
            b = sum(e[3] for e in c if e[0] == k)
            line.append(f"  {k}: n={len(iv)} busy {union(iv) / 1e6:.2f} ms ({union(iv) / (t1 - t0):.0%})"
                        + (f", {b / 1e9:.3f} GB, {b / max(1, union(iv)):.1f} GB/s while busy" if b else ""))
        print("\n".join(line))


if __name__ == "__main__":
    main()
