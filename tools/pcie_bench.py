#!/usr/bin/env python3
"""PCIe-inclusive rate: stripes start and end in pinned host memory;
cauchy_256_{encode,decode}_host_batch pipelines H2D / kernels / D2H over three streams.
Prints one JSON line per config.  Usage: python tools/pcie_bench.py [config ...]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import longhair_amd as lh  # noqa: E402

CONFIGS = {"k29m4": (29, 4, 1296, 65536), "k200m56": (200, 56, 65536, 64), "k128m32": (128, 32, 8192, 2048)}


SHUFFLE = os.environ.get("PCIE_SHUFFLE") == "1"
CHUNK = int(os.environ.get("PCIE_CHUNK", "0"))  # stripes per pipeline chunk (0: ~64 MiB)


def run(name, reps=3):
    k, m, nbytes, stripes = CONFIGS[name]
    e_cap = min(k, m)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8).pin_memory()
    rec = torch.empty((stripes, m, nbytes), dtype=torch.uint8).pin_memory()
    lh.prepare(k, m, nbytes, 0)
    lh.encode_host_batch(data.numpy(), m, recovery=rec.numpy(), chunk_stripes=CHUNK)  # warm-up (JIT, buffers)
    t0 = time.perf_counter()
    for _ in range(reps):
        lh.encode_host_batch(data.numpy(), m, recovery=rec.numpy(), chunk_stripes=CHUNK)
    enc = (time.perf_counter() - t0) / reps
    # decode scenario: random erasures (e in [1, min(k, m)]), recovery blocks at the end
    rng = np.random.Generator(np.random.PCG64(1))
    blocks = torch.empty_like(data).pin_memory()
    rows = torch.empty((stripes, k), dtype=torch.uint8).pin_memory()
    bn, rn, dn, recn = blocks.numpy(), rows.numpy(), data.numpy(), rec.numpy()
    for s in range(stripes):
        e = int(rng.integers(1, e_cap + 1)) if name == "k200m56" else e_cap
        keep = rng.permutation(k)[: k - e]
        rr = rng.permutation(m)[:e]
        bn[s, : k - e] = dn[s, keep]
        bn[s, k - e:] = recn[s, rr]
        rn[s, : k - e] = keep
        rn[s, k - e:] = k + rr
        if SHUFFLE:  # packets in arrival order: recovery blocks spread over the slots
            p = rng.permutation(k)
            bn[s] = bn[s, p]
            rn[s] = rn[s, p]
    b0, r0 = bn.copy(), rn.copy()
    lh.decode_host_batch(bn, rn, m, chunk_stripes=CHUNK)
    order = np.argsort(rn, axis=1)
    assert np.array_equal(np.take_along_axis(bn, order[:, :, None], axis=1), dn), "decode mismatch"
    tot = 0.0
    for _ in range(reps):
        bn[:] = b0
        rn[:] = r0
        t0 = time.perf_counter()
        lh.decode_host_batch(bn, rn, m, chunk_stripes=CHUNK)
        tot += time.perf_counter() - t0
    dec = tot / reps
    inb = k * nbytes * stripes
    return {"config": name, "k": k, "m": m, "block_bytes": nbytes, "stripes": stripes,
            "encode_GBps_pcie_inclusive": round(inb / enc / 1e9, 2),
            "decode_GBps_pcie_inclusive": round(inb / dec / 1e9, 2),
            "encode_s": round(enc, 5), "decode_s": round(dec, 5),
            "slots": "shuffled" if SHUFFLE else "recovery blocks last", "chunk_stripes": CHUNK or "auto (encode ~64 MiB, decode <= 256 MiB)",
            "writeback": os.environ.get("LONGHAIR_AMD_PIPE_WRITEBACK", "kernel"),
            "note": "pinned host in/out, 3-stream chunked pipeline, input GB/s (1e9)"}


def main():
    torch.cuda.set_device(0)
    assert lh.cauchy_256_init() == 0
    for name in sys.argv[1:] or ["k29m4", "k200m56"]:
        print(json.dumps(run(name)), flush=True)


if __name__ == "__main__":
    main()
