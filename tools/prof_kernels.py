#!/usr/bin/env python3
"""Profiling driver: the bench workload's encode and decode launched a few times each
(after JIT warm-up) so rocprofv3 can attribute per-dispatch counters to lh_* kernels.
Usage: rocprofv3 --pmc FETCH_SIZE -d OUT -o run --output-format csv -- python3 tools/prof_kernels.py [config]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
import longhair_amd as lh  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "k29m4"
    k, m, nbytes, stripes, erasures = bench.CONFIGS[cfg]
    torch.cuda.set_device(0)
    assert lh.cauchy_256_init() == 0
    lh.prepare(k, m, nbytes, stripes)
    X, D, rows0, rec_index = bench.make_workload(k, m, nbytes, stripes, seed=3, erasures=erasures)
    rec = D[:, k - m:] if rec_index is None else torch.empty((stripes, m, nbytes), dtype=torch.uint8, device="cuda")
    rows = rows0.clone()
    for _ in range(3):
        lh.encode_batch(X, m, recovery=rec)
        if rec_index is not None:
            D.view(-1, nbytes).index_copy_(0, rec_index[0], rec.view(-1, nbytes).index_select(0, rec_index[1]))
        rows.copy_(rows0)
        lh.decode_batch(D, rows, m)
    torch.cuda.synchronize()
    print("prof_kernels done", cfg, lh.batch_path(k, m, nbytes), lh.batch_path(k, m, nbytes, True))


if __name__ == "__main__":
    main()
