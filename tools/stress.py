#!/usr/bin/env python3
"""Randomised parity stress (not a test: a tool for GPU sessions).  For random shapes --
those with a specialised module in the on-disk cache and, with LONGHAIR_AMD_JIT_COMPILE=0,
the generic kernels for the rest -- encode + decode random stripes (random erasures,
recovery rows and slot order) through the strided batch calls, compare a sample of stripes
with the C oracle, and run the same inputs through the pointer-table calls on scattered
blocks, which must give identical bytes, rows and status.
Usage: python tools/stress.py SECONDS [SEED] [--lds-sample N]   (prints one line per shape, FAIL lines
on mismatch, then a count of the shapes each kernel served)
--lds-sample N: draw the shapes from the first N of tools/precompile.py's seeded sample of
LDS-staged register-network shapes (lds_sample(): encode lh_jit_encode, decode
lh_jit_decode_fused, 16-byte-multiple blocks), whose modules that tool compiles beforehand."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ.setdefault("LONGHAIR_AMD_JIT_COMPILE", "0")

import torch  # noqa: E402

import lhutil  # noqa: E402
import longhair_amd as lh  # noqa: E402


def scatter(blocks, rng):
    """Copy [S, n, B] blocks to random places (random byte offsets) of a pool; return the
    pool, the int64 pointer table and the places."""
    S, n, B = blocks.shape
    stride = B + 16
    order = rng.permutation(S * n)
    offs = rng.integers(0, 16, size=S * n)
    pool = torch.zeros(S * n * stride + 64, dtype=torch.uint8, device="cuda")
    p2 = pool[: S * n * stride].view(S * n, stride)
    flat = blocks.reshape(S * n, B)
    for o in np.unique(offs):
        sel = np.nonzero(offs == o)[0]
        p2[torch.from_numpy(order[sel]).cuda(), int(o):int(o) + B] = flat[torch.from_numpy(sel).cuda()]
    ptrs = torch.from_numpy((order * stride + offs).reshape(S, n).astype(np.int64) + pool.data_ptr()).cuda()
    return pool, ptrs, (p2, order, offs, S, n, B)


def gather(place):
    p2, order, offs, S, n, B = place
    out = torch.empty((S * n, B), dtype=torch.uint8, device="cuda")
    for o in np.unique(offs):
        sel = np.nonzero(offs == o)[0]
        out[torch.from_numpy(sel).cuda()] = p2[torch.from_numpy(order[sel]).cuda(), int(o):int(o) + B]
    return out.view(S, n, B)


COUNTS = {}


def one(rng, oracle, shapes=None):
    if shapes:
        k, m, nbytes = shapes[int(rng.integers(0, len(shapes)))]
    else:
        k = int(rng.choice([2, 3, 5, 8, 12, 17, 29, 40, 64, 100, 128, 200]))
        m = int(rng.choice([1, 2, 3, 4, 6, 8, 12, 16, 20, 32]))
        if k + m > 256:
            m = 256 - k
        nbytes = 8 * int(rng.choice([1, 2, 3, 21, 64, 162, 256, 512, 1024]))
    stripes = int(rng.integers(1, 40))
    g = torch.Generator(device="cuda").manual_seed(int(rng.integers(1 << 30)))
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    rec = lh.encode_batch(data, m)
    enc_trace = lh.last_launch()
    dh, rh = data.cpu().numpy(), rec.cpu().numpy()
    blocks = np.empty((stripes, k, nbytes), dtype=np.uint8)
    rows = np.empty((stripes, k), dtype=np.uint8)
    for s in range(stripes):
        e = int(rng.integers(0, min(k, m) + 1))
        slots, r = lhutil.erasure_case(int(rng.integers(1 << 30)), k, m, e)
        for i, (kind, x) in enumerate(slots):
            blocks[s, i] = dh[s, x] if kind == "d" else rh[s, x]
        rows[s] = r
    sb, sr = torch.from_numpy(blocks).cuda(), torch.from_numpy(rows).cuda()
    sstat = lh.decode_batch(sb, sr, m)
    dec_trace = lh.last_launch()
    torch.cuda.synchronize()
    bad = []
    for s in sorted({0, stripes - 1}):
        rc, exp = oracle.encode(k, m, dh[s], nbytes)
        if exp.tobytes() != rh[s].tobytes():
            bad.append(f"encode stripe {s}")
        bufs = [blocks[s, i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows[s]), nbytes)
        got = sb[s].cpu().numpy()
        if list(sr[s].cpu().numpy()) != exp_rows or any(got[i].tobytes() != bufs[i].tobytes() for i in range(k)):
            bad.append(f"decode stripe {s}")
    # pointer tables on the same inputs
    dpool, dptr, _ = scatter(data, rng)
    rpool, rptr, rplace = scatter(torch.zeros((stripes, m, nbytes), dtype=torch.uint8, device="cuda"), rng)
    lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr)
    if not torch.equal(gather(rplace), rec):
        bad.append("encode_ptrs")
    pool, ptrs, place = scatter(torch.from_numpy(blocks).cuda(), rng)
    pr = torch.from_numpy(rows).cuda()
    pstat = lh.decode_batch_ptrs(k, m, nbytes, ptrs, pr)
    ptr_trace = lh.last_launch()
    torch.cuda.synchronize()
    if not (torch.equal(pstat, sstat) and torch.equal(pr, sr) and torch.equal(gather(place), sb)):
        bad.append("decode_ptrs")
    for name in set(enc_trace) | set(dec_trace) | set(ptr_trace):
        COUNTS[name] = COUNTS.get(name, 0) + 1
    print(f"k={k} m={m} bytes={nbytes} stripes={stripes} enc={'+'.join(enc_trace)} dec={'+'.join(dec_trace)} "
          f"ptr={'+'.join(ptr_trace)} {'FAIL ' + ','.join(bad) if bad else 'ok'}", flush=True)
    return not bad


def main():
    args = list(sys.argv[1:])
    shapes = None
    if "--lds-sample" in args:
        i = args.index("--lds-sample")
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import precompile
        shapes = precompile.lds_sample(int(args[i + 1]))
        del args[i:i + 2]
    secs = float(args[0]) if len(args) > 0 else 60
    seed = int(args[1]) if len(args) > 1 else int(time.time())
    print(f"seed {seed}" + (f", {len(shapes)} LDS-sample shapes" if shapes else ""), flush=True)
    rng = np.random.Generator(np.random.PCG64(seed))
    assert lh.cauchy_256_init() == 0
    oracle = lhutil.Oracle()
    t0, n, fails = time.time(), 0, 0
    while time.time() - t0 < secs:
        n += 1
        fails += 0 if one(rng, oracle, shapes) else 1
    print("kernels (shapes served): " + ", ".join(f"{k} {v}" for k, v in sorted(COUNTS.items(), key=lambda kv: -kv[1])),
          flush=True)
    print(f"{n} shapes, {fails} failed", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
