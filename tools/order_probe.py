#!/usr/bin/env python3
"""Probe: decode time with the surviving blocks in a shuffled slot order (bench workload)
vs in ascending order, k=29 m=4 1296 B x 65536 stripes (device-resident)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import longhair_amd as lh  # noqa: E402


def timed(fn, reps=10):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    tot = 0.0
    for a, b in evs:
        fn(a, b)
    torch.cuda.synchronize()
    return min(a.elapsed_time(b) for a, b in evs)


def main():
    k, m, nbytes, stripes = 29, 4, 1296, 65536
    torch.cuda.set_device(0)
    assert lh.cauchy_256_init() == 0
    lh.prepare(k, m, nbytes, stripes)
    X, D, rows0, _ = bench.make_workload(k, m, nbytes, stripes, seed=7)
    # in-order variant: survivors sorted by row, recovery at the end
    order = rows0[:, : k - m].long().sort(dim=1)
    D2 = D.clone()
    D2[:, : k - m] = torch.gather(D[:, : k - m], 1, order.indices.unsqueeze(-1).expand(-1, -1, nbytes))
    rows2 = rows0.clone()
    rows2[:, : k - m] = order.values.to(torch.uint8)
    for name, DD, r0 in (("shuffled", D, rows0), ("ascending", D2, rows2)):
        lh.encode_batch(X, m, recovery=DD[:, k - m:])
        rows = r0.clone()

        def run(a, b):
            rows.copy_(r0)
            a.record()
            lh.decode_batch(DD, rows, m)
            b.record()
        ms = timed(run)
        ok = torch.equal(torch.gather(DD, 1, rows.long().argsort(dim=1).unsqueeze(-1).expand(-1, -1, nbytes)), X)
        print(f"{name:10s} decode {ms:.4f} ms  {k * nbytes * stripes / ms / 1e6:.1f} GB/s in  ok={ok}", flush=True)

        def enc(a, b):
            a.record()
            lh.encode_batch(X, m, recovery=DD[:, k - m:])
            b.record()
        print(f"{name:10s} encode {timed(enc):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
