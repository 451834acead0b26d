#!/usr/bin/env python3
"""Generate golden fixtures from the REFERENCE implementation itself.

Runs only in the build container: it loads oracle/_ref/liblonghair_ref.so, which
`make -C oracle ref` compiles from the unmodified /root/reference sources.  Outputs
(committed, data only) go to tests/golden/:

  encode_grid.json   per (k, m, bytes, seed): return code + digest of the m recovery
                     blocks, for every k in [1, 255] x a set of m, plus invalid params.
  encode_full.json   a few tiny cases with full input and output bytes (hex).
  decode_cases.json  decode scenarios (block order, rows) -> return code, final rows and
                     the digest of every block buffer after decode.

Inputs are regenerated from tests/lhutil.fill(seed, n); digests are tests/lhutil.h64.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import lhutil  # noqa: E402

M_SET = [1, 2, 3, 4, 5, 6, 7, 8, 9, 16, 32, 33, 64, 128]


def seed_of(k, m, bytes_, salt=0):
    return (k * 1000003 + m * 1009 + bytes_ * 7 + salt) & 0xFFFFFFFF


def encode_grid(ref):
    cases = []
    for k in range(1, 256):
        ms = sorted(set([m for m in M_SET if k + m <= 256] + [256 - k]))
        for m in ms:
            if m < 1:
                continue
            for bytes_ in ([16] if k > 8 else [8, 16, 24]):
                seed = seed_of(k, m, bytes_)
                data = lhutil.fill(seed, k * bytes_)
                rc, rec = ref.encode(k, m, data, bytes_)
                cases.append([k, m, bytes_, seed, rc, lhutil.h64(rec)])
    # Larger blocks at the BASELINE.json shapes and a few odd sub-block sizes.
    for k, m, bytes_ in [(29, 1, 1296), (29, 2, 1296), (29, 3, 1296), (29, 4, 1296),
                         (29, 5, 1296), (29, 8, 1296), (29, 14, 1296), (128, 32, 8192),
                         (200, 56, 65536), (10, 4, 8), (10, 4, 40), (10, 4, 1288),
                         (17, 6, 520), (64, 64, 2048), (2, 254, 64), (249, 7, 64),
                         (100, 100, 136), (255, 1, 24)]:
        seed = seed_of(k, m, bytes_, 1)
        data = lhutil.fill(seed, k * bytes_)
        rc, rec = ref.encode(k, m, data, bytes_)
        cases.append([k, m, bytes_, seed, rc, lhutil.h64(rec)])
    # Invalid parameters: validation happens only when m > 1, after row 0 is written.
    for k, m, bytes_ in [(200, 57, 16), (250, 7, 16), (29, 4, 12), (29, 4, 1300),
                         (29, 1, 12), (255, 2, 8), (29, 1, 5)]:
        seed = seed_of(k, m, bytes_, 2)
        data = lhutil.fill(seed, k * bytes_)
        rc, rec = ref.encode(k, m, data, bytes_)
        # Only recovery block 0 is defined on failure.
        cases.append([k, m, bytes_, seed, rc, lhutil.h64(rec[:bytes_])])
    return cases


def encode_full(ref):
    out = []
    for k, m, bytes_ in [(1, 3, 8), (2, 2, 8), (3, 2, 16), (4, 2, 16), (4, 4, 24),
                         (5, 3, 32), (6, 6, 40), (7, 5, 48), (8, 8, 64), (3, 1, 8)]:
        seed = seed_of(k, m, bytes_, 3)
        data = lhutil.fill(seed, k * bytes_)
        rc, rec = ref.encode(k, m, data, bytes_)
        out.append({"k": k, "m": m, "bytes": bytes_, "rc": rc, "data": data.tobytes().hex(),
                    "recovery": rec.tobytes().hex()})
    return out


def run_decode(ref, k, m, bytes_, seed, slots, rows):
    data = lhutil.fill(seed, k * bytes_).reshape(k, bytes_) if k else None
    rc, rec = ref.encode(k, m, data, bytes_)
    rec = rec.reshape(m, bytes_) if m else rec
    bufs = []
    for kind, x in slots:
        bufs.append((data[x] if kind == "d" else rec[x]).copy())
    rc_d, new_rows = ref.decode(k, m, bufs, rows, bytes_)
    return rc, rc_d, new_rows, [lhutil.h64(b) for b in bufs]


def decode_cases(ref):
    cases = []

    def add(k, m, bytes_, slots, tag):
        seed = seed_of(k, m, bytes_, 4 + len(cases))
        rows = [x if kind == "d" else k + x for kind, x in slots]
        rc_e, rc_d, new_rows, digests = run_decode(ref, k, m, bytes_, seed, slots, rows)
        cases.append({"tag": tag, "k": k, "m": m, "bytes": bytes_, "seed": seed,
                      "slots": [[kind, x] for kind, x in slots], "rows_in": rows,
                      "rc_encode": rc_e, "rc": rc_d, "rows_out": new_rows, "digests": digests})

    # The reference's own order_test shape (tests/cauchy_256_tests.cpp:122-205).
    add(4, 2, 1296, [("d", 0), ("d", 3), ("r", 0), ("r", 1)], "order_test")
    add(4, 2, 1296, [("d", 2), ("d", 1), ("r", 1), ("r", 0)], "order_test_swapped")
    # The reference sweep's shape: erase blocks 0..e-1, recovery rows k..k+e-1 first.
    for k, m, e in [(29, 4, 1), (29, 4, 2), (29, 4, 3), (29, 4, 4), (10, 8, 8), (3, 250, 3),
                    (128, 32, 32), (200, 56, 56), (2, 2, 2), (255, 1, 1)]:
        bytes_ = 1296 if k <= 29 else 64
        slots = [("r", j) for j in range(e)] + [("d", x) for x in range(e, k)]
        add(k, m, bytes_, slots, "sweep_prefix")
    # Random erasure positions, random recovery rows, shuffled block order.
    rng_cases = [(29, 4, 4, 1296), (29, 4, 3, 1296), (29, 2, 2, 16), (29, 8, 8, 16),
                 (29, 14, 9, 16), (128, 32, 32, 1024), (128, 32, 17, 64),
                 (200, 56, 56, 512), (200, 56, 23, 512), (10, 246, 10, 16),
                 (249, 7, 7, 16), (17, 6, 6, 520), (64, 64, 40, 24), (5, 3, 2, 8),
                 (100, 100, 100, 16), (30, 30, 1, 16), (255, 1, 1, 16), (2, 254, 2, 8)]
    for i, (k, m, e, bytes_) in enumerate(rng_cases):
        for rep in range(3):
            slots, _ = lhutil.erasure_case(1000 + 17 * i + rep, k, m, e)
            add(k, m, bytes_, slots, "random")
    # Nothing erased; k == 1; m == 1 with one erasure; m == 1 with no erasure (quirk).
    add(29, 4, 16, [("d", x) for x in range(29)], "no_erasure")
    add(1, 5, 16, [("r", 3)], "k1")
    add(1, 1, 16, [("d", 0)], "k1_m1")
    add(8, 1, 16, [("d", 0), ("d", 1), ("r", 0), ("d", 3), ("d", 4), ("d", 5), ("d", 6), ("d", 7)],
        "m1_one_erasure")
    add(8, 1, 16, [("d", x) for x in range(8)], "m1_no_erasure_quirk")
    # Invalid parameters with an erasure present -> -1 (rows untouched).
    add(200, 57, 16, [("r", 0)] + [("d", x) for x in range(1, 200)], "invalid_km")
    return cases


def main():
    ref = lhutil.RefLib()
    os.makedirs(lhutil.GOLDEN, exist_ok=True)
    grid = encode_grid(ref)
    json.dump({"spec": "rows: [k, m, bytes, seed, rc, h64(recovery)]", "cases": grid},
              open(os.path.join(lhutil.GOLDEN, "encode_grid.json"), "w"), separators=(",", ":"))
    json.dump(encode_full(ref), open(os.path.join(lhutil.GOLDEN, "encode_full.json"), "w"), indent=0)
    dec = decode_cases(ref)
    json.dump(dec, open(os.path.join(lhutil.GOLDEN, "decode_cases.json"), "w"), separators=(",", ":"))
    print("encode_grid", len(grid), "decode", len(dec))


if __name__ == "__main__":
    main()
