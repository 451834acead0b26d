#!/usr/bin/env python3
"""Why the bench's per-kernel times exceed tools/tune.py's on the same box: the k29/m4 step
(encode, rows reset, decode) timed with HIP events under several issue patterns -- back to back
as bench.py does, a host sync after every step as tune.py does, a sync plus a 2 ms idle gap,
decodes alone, a spin kernel (no memory traffic) before or after each decode, and the same step
through the pointer-table calls (back to back and synced).
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
    lh.prepare_ptrs(k, m, nbytes)
    s_idx = torch.arange(stripes, device="cuda", dtype=torch.int64).unsqueeze(1)

    def table(t, n):
        return (t.data_ptr() + s_idx * t.stride(0) + torch.arange(n, device="cuda", dtype=torch.int64) * t.stride(1)
                ).contiguous()
    dptr, rptr, bptr = table(X, k), table(rec, m), table(D, k)

    spin = int(os.environ.get("SEQ_SPIN", "200000"))  # torch.cuda._sleep cycles (no memory traffic)

    def step(ev, mode="back-to-back"):
        ptr = mode.startswith("ptr")
        ev[0].record()
        if mode != "decode-only":
            if ptr:
                lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr)
            else:
                lh.encode_batch(X, m, recovery=rec)
        ev[1].record()
        rows.copy_(rows0)
        if mode == "spin-before-decode":
            torch.cuda._sleep(spin)
        ev[2].record()
        if ptr:
            lh.decode_batch_ptrs(k, m, nbytes, bptr, rows)
        else:
            lh.decode_batch(D, rows, m)
        ev[3].record()
        if mode == "spin-after-decode":
            torch.cuda._sleep(spin)

    for _ in range(3):
        step([torch.cuda.Event(enable_timing=True) for _ in range(4)])
    torch.cuda.synchronize()
    for rnd in range(3):
        modes = ("back-to-back", "sync", "sync+gap", "decode-only", "spin-before-decode", "spin-after-decode",
                 "ptr back-to-back", "ptr sync")
        if os.environ.get("SEQ_MODES"):
            modes = os.environ["SEQ_MODES"].split(",")
        for mode in modes:
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(20)]
            for ev in evs:
                step(ev, mode)
                if mode.endswith("sync") or mode.startswith("sync"):
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
