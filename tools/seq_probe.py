#!/usr/bin/env python3
"""Why the bench's per-kernel times exceed tools/tune.py's on the same box: the k29/m4 step
(encode, rows reset, decode) timed with HIP events under several issue patterns -- back to back
as bench.py does, a host sync after every step as tune.py does, a sync plus a 2 ms idle gap,
decodes alone, and a spin kernel (no memory traffic) before or after each decode.
Usage: python tools/seq_probe.py > gpurun_out/seq_probe.txt"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import longhair_amd as lh  # noqa: E402


def main():
    k, m, nbytes, stripes = 29, 4, 1296, 65536
    torch.cuda.set_device(0)
    assert lh.cauchy_256_init() == 0
    lh.prepare(k, m, nbytes, stripes)
    X, D, rows0, _ = bench.make_workload(k, m, nbytes, stripes, seed=1234)
    rec = D[:, k - m:]
    rows = rows0.clone()

    spin = int(os.environ.get("SEQ_SPIN", "200000"))  # torch.cuda._sleep cycles (no memory traffic)

    def step(ev, mode="back-to-back"):
        ev[0].record()
        if mode != "decode-only":
            lh.encode_batch(X, m, recovery=rec)
        ev[1].record()
        rows.copy_(rows0)
        if mode == "spin-before-decode":
            torch.cuda._sleep(spin)
        ev[2].record()
        lh.decode_batch(D, rows, m)
        ev[3].record()
        if mode == "spin-after-decode":
            torch.cuda._sleep(spin)

    for _ in range(3):
        step([torch.cuda.Event(enable_timing=True) for _ in range(4)])
    torch.cuda.synchronize()
    for rnd in range(3):
        for mode in ("back-to-back", "sync", "sync+gap", "decode-only", "spin-before-decode", "spin-after-decode"):
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(20)]
            for ev in evs:
                step(ev, mode)
                if mode.startswith("sync"):
                    torch.cuda.synchronize()
                if mode == "sync+gap":
                    time.sleep(0.002)
            torch.cuda.synchronize()
            enc = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs)
            dec = sum(e[2].elapsed_time(e[3]) for e in evs) / len(evs)
            first = evs[0][2].elapsed_time(evs[0][3])
            per = " ".join(f"{e[2].elapsed_time(e[3]):.3f}" for e in evs)
            print(f"round {rnd} {mode:18s} encode {enc:.4f} decode {dec:.4f} ms (first decode {first:.4f}) [{per}]",
                  flush=True)


if __name__ == "__main__":
    main()
