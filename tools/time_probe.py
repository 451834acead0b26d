#!/usr/bin/env python3
"""Timing-only probe (no correctness check, for instrumented variants such as LH_PB_SKIP):
encode_batch / decode_batch time per variant on a bench config.
Usage: python tools/time_probe.py CONFIG 'NAME:ENV=VAL,ENV=VAL' ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import longhair_amd as lh  # noqa: E402

KNOBS = ["LONGHAIR_AMD_JIT_DEFINES", "LONGHAIR_AMD_NO_FUSED_PLAN"]


def main():
    cfg = sys.argv[1]
    k, m, nbytes, stripes, erasures = bench.CONFIGS[cfg]
    torch.cuda.set_device(0)
    assert lh.cauchy_256_init() == 0
    X, D, rows0, idx = bench.make_workload(k, m, nbytes, stripes, seed=5, erasures=erasures)
    R = torch.empty((stripes, m, nbytes), dtype=torch.uint8, device="cuda")
    rows = rows0.clone()
    for spec in sys.argv[2:] or ["base:"]:
        name, _, envs = spec.partition(":")
        for key in KNOBS:
            os.environ.pop(key, None)
        for kv in filter(None, envs.split(";")):
            key, _, val = kv.partition("=")
            os.environ[key] = val
        lh.prepare(k, m, nbytes, stripes)
        enc, dec = [], []
        for _ in range(4):
            a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            lh.encode_batch(X, m, recovery=R)
            b.record()
            rows.copy_(rows0)
            c.record()
            lh.decode_batch(D, rows, m)
            d = torch.cuda.Event(enable_timing=True)
            d.record()
            torch.cuda.synchronize()
            enc.append(a.elapsed_time(b))
            dec.append(c.elapsed_time(d))
        print(f"{cfg} {name:12s} encode {min(enc[1:]):.4f} ms  decode {min(dec[1:]):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
