#!/usr/bin/env python3
"""What the bench's cold-start ramp is: the k29/m4 step (encode, rows reset,
decode) timed with HIP events, 20 back-to-back steps per phase, in one process:

  A  first steps after setup (fresh process, fresh buffers)          -- the ramp the bench settles away
  B  the same buffers again, right after A                           -- steady state
  C  after a 2 s idle (host sleep, GPU idle)                         -- clocks dropping while idle?
  D  a second, freshly allocated workload (new buffers, warm GPU)    -- first touch of the buffers?
  E  after a 200 ms spin kernel (GPU busy, no memory traffic)        -- clocks held up by compute?
  F  after 2 s idle, then a 200 ms spin kernel, then the steps       -- does compute warm-up remove C?

Usage: python tools/cold_probe.py > gpurun_out/cold_probe.txt"""
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

    def workload(seed):
        X, D, rows0, _ = bench.make_workload(k, m, nbytes, stripes, seed=seed)
        return X, D, rows0, rows0.clone(), D[:, k - m:]

    def phase(name, w, n=20):
        X, D, rows0, rows, rec = w
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(n)]
        for ev in evs:
            ev[0].record()
            lh.encode_batch(X, m, recovery=rec)
            ev[1].record()
            rows.copy_(rows0)
            ev[2].record()
            lh.decode_batch(D, rows, m)
            ev[3].record()
        torch.cuda.synchronize()
        enc = [ev[0].elapsed_time(ev[1]) for ev in evs]
        dec = [ev[2].elapsed_time(ev[3]) for ev in evs]
        print(f"{name:44s} encode {' '.join('%.3f' % x for x in enc)}", flush=True)
        print(f"{'':44s} decode {' '.join('%.3f' % x for x in dec)}", flush=True)
        return enc, dec

    def spin(ms):
        # torch.cuda._sleep(cycles): a busy kernel without memory traffic (~2.1 GHz assumed)
        torch.cuda._sleep(int(ms * 2.1e6))

    w1 = workload(1234)
    torch.cuda.synchronize()
    phase("A first steps after setup", w1)
    phase("B same buffers, right after A", w1)
    time.sleep(2.0)
    phase("C after 2 s idle", w1)
    w2 = workload(99)
    torch.cuda.synchronize()
    phase("D fresh buffers, warm GPU", w2)
    spin(200)
    phase("E after a 200 ms spin kernel", w2)
    time.sleep(2.0)
    spin(200)
    phase("F 2 s idle, then a 200 ms spin kernel", w2)


if __name__ == "__main__":
    main()
