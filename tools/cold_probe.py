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

import glob  # noqa: E402
import threading  # noqa: E402

# The clock levels the driver reports (sysfs pp_dpm_*: the current level is marked '*'),
# sampled every ~2 ms in a thread, so each phase can be read against the clocks.
DPM = sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_*"))
SAMPLES = []


def sampler(stop):
    while not stop.is_set():
        row = [time.perf_counter()]
        for f in DPM:
            try:
                cur = [ln for ln in open(f).read().splitlines() if ln.rstrip().endswith("*")]
                row.append(cur[0].split(":", 1)[1].strip().rstrip("*").strip() if cur else "?")
            except OSError:
                row.append("-")
        SAMPLES.append(row)
        time.sleep(0.002)


def main():
    k, m, nbytes, stripes = 29, 4, 1296, 65536
    torch.cuda.set_device(0)
    assert lh.cauchy_256_init() == 0
    lh.prepare(k, m, nbytes, stripes)

    def workload(seed):
        X, D, rows0, _ = bench.make_workload(k, m, nbytes, stripes, seed=seed)
        return X, D, rows0, rows0.clone(), D[:, k - m:]

    marks = []

    def phase(name, w, n=20):
        X, D, rows0, rows, rec = w
        marks.append((name, time.perf_counter()))
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
        marks.append((name + " (end)", time.perf_counter()))
        enc = [ev[0].elapsed_time(ev[1]) for ev in evs]
        dec = [ev[2].elapsed_time(ev[3]) for ev in evs]
        print(f"{name:44s} encode {' '.join('%.3f' % x for x in enc)}", flush=True)
        print(f"{'':44s} decode {' '.join('%.3f' % x for x in dec)}", flush=True)
        return enc, dec

    def spin(ms):
        # torch.cuda._sleep(cycles): a busy kernel without memory traffic (~2.1 GHz assumed)
        torch.cuda._sleep(int(ms * 2.1e6))

    stop = threading.Event()
    th = threading.Thread(target=sampler, args=(stop,), daemon=True)
    th.start()
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
    stop.set()
    th.join()
    # clock levels: the distinct values per phase window and the 200 ms before it
    print("# clocks (sysfs " + ", ".join(os.path.basename(f) for f in DPM) + ")", flush=True)
    for i in range(0, len(marks), 2):
        name, t0 = marks[i]
        t1 = marks[i + 1][1]
        def levels(a, b):
            rows = [r[1:] for r in SAMPLES if a <= r[0] <= b]
            return [sorted(set(col)) for col in zip(*rows)] if rows else []
        print(f"{name:44s} before {levels(t0 - 0.2, t0)}  during {levels(t0, t1)}", flush=True)
    if SAMPLES:  # the level sequence of each file over the whole run (changes only)
        for j, f in enumerate(DPM):
            seq, last = [], None
            for r in SAMPLES:
                if r[j + 1] != last:
                    seq.append(f"{r[0] - SAMPLES[0][0]:.3f}s:{r[j + 1]}")
                    last = r[j + 1]
            print(os.path.basename(f), " ".join(seq[:80]), flush=True)


if __name__ == "__main__":
    main()
