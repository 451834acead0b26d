#!/usr/bin/env python3
"""Benchmark: GB/s of input data encoded + decoded, device-resident (BASELINE.json metric).

One step = (1) cauchy_256_encode_batch of every stripe's k data blocks, writing the m
recovery blocks straight into the recovery slots of the decode buffer, (2) reset of the
Block.row bytes, (3) cauchy_256_decode_batch of every stripe in place (k - e surviving
originals in a per-stripe shuffled order + e recovery blocks, e = min(k, m) erased
originals chosen per stripe).  Input bytes per step = 2 * k * bytes * stripes.

Default workload: BASELINE.json configs[1] -- k=29, m=4, 1296-byte blocks, 65536 stripes
per GPU (weak scaling across ranks: every rank codes its own 65536 stripes, no collective
on the data path).  N > 1: `python -m torch.distributed.run --nproc-per-node N bench.py`.

Prints one JSON line (rank 0).  See DESIGN.md for the roofline and cpu_baseline definitions.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

CONFIGS = {
    # name: (k, m, bytes, stripes per GPU, erasures per stripe)
    "k29m4": (29, 4, 1296, 65536, "max"),        # BASELINE configs[1] / [3] (per GPU)
    "k128m32": (128, 32, 8192, 8192, "max"),     # BASELINE configs[2]
    "k200m56": (200, 56, 65536, 64, "random"),   # BASELINE configs[4] (device-resident part)
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="k29m4", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=0, help="override stripes per GPU")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU work (thread-seconds) for the baseline")
    return ap.parse_args()


def setup_dist():
    import torch
    import torch.distributed as dist
    from longhair_amd.shard import world_info
    world, rank, local = world_info()
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(world, value):
    from longhair_amd.shard import max_over_ranks as mx
    return value if world == 1 else mx(value, device="cuda")


def make_workload(k, m, nbytes, stripes, seed, erasures="max"):
    """Data X [S, k, bytes] and a decode buffer D [S, k, bytes] whose first slots hold the
    surviving originals of each stripe in a shuffled order and whose last e_s slots
    receive recovery blocks; rows0 = the matching Block.row bytes.

    erasures="max": e = m erased originals per stripe (m <= k), recovery rows 0..m-1 --
    the encode then writes straight into D's recovery slots (rec_index is None).
    erasures="random": e_s uniform in [1, min(k, m)] per stripe, a random subset of the
    recovery rows; rec_index = (dst, src) row indices that copy the needed recovery
    blocks from the encode output R [S, m, bytes] into D each step."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    perm = torch.argsort(torch.rand(stripes, k, device="cuda", generator=g), dim=1)
    D = torch.empty_like(X)
    if erasures == "max":
        e = min(k, m)
        assert e == m, "erasures='max' writes all m recovery rows into the decode buffer"
        keep = perm[:, : k - e]
        D[:, : k - e] = torch.gather(X, 1, keep.unsqueeze(-1).expand(-1, -1, nbytes))
        rows0 = torch.cat([keep, torch.arange(k, k + e, device="cuda").expand(stripes, e)], dim=1)
        return X, D, rows0.to(torch.uint8).contiguous(), None
    rng = torch.Generator().manual_seed(seed)
    rows0 = torch.empty((stripes, k), dtype=torch.long)
    dst, src = [], []
    perm_c = perm.cpu()
    for s in range(stripes):
        e = int(torch.randint(1, min(k, m) + 1, (1,), generator=rng))
        rec_rows = torch.randperm(m, generator=rng)[:e]
        rows0[s, : k - e] = perm_c[s, : k - e]
        rows0[s, k - e:] = k + rec_rows
        for j in range(e):
            dst.append(s * k + k - e + j)
            src.append(s * m + int(rec_rows[j]))
    rows0 = rows0.cuda()
    keep_all = torch.where(rows0 < k, rows0, torch.zeros_like(rows0))
    D.copy_(torch.gather(X, 1, keep_all.unsqueeze(-1).expand(-1, -1, nbytes)))
    idx = (torch.tensor(dst, device="cuda"), torch.tensor(src, device="cuda"))
    return X, D, rows0.to(torch.uint8).contiguous(), idx


def cpu_baseline(k, m, nbytes, target_seconds, stripes=4096):
    """Reference codec (oracle/_ref, compiled from the reference sources) -- or, if that
    build is absent, the oracle restatement -- on the host cores, same step definition,
    a bounded sample of stripes."""
    import numpy as np
    import lhutil
    bench_so = os.path.join(REPO, "oracle", "liblh_cpubench.so")
    if not os.path.exists(bench_so):
        return None
    hb = ctypes.CDLL(bench_so)
    hb.lhb_run.restype = ctypes.c_double
    if os.path.exists(lhutil.REF_SO):
        lib, kind = lhutil.RefLib(), "reference"
        enc, dec = lib.lib.cauchy_256_encode, lib.lib.cauchy_256_decode
    else:
        lib, kind = lhutil.Oracle(), "port"
        enc, dec = lib.lib.lho_encode, lib.lib.lho_decode
    e = min(k, m)
    data = lhutil.fill(99, stripes * k * nbytes)
    rng = np.random.Generator(np.random.PCG64(5))
    erased = np.stack([rng.choice(k, size=e, replace=False) for _ in range(stripes)]).astype(np.uint8)
    threads = max(1, min(16, os.cpu_count() or 1))
    ok = ctypes.c_int(0)
    args = lambda passes: (ctypes.cast(enc, ctypes.c_void_p), ctypes.cast(dec, ctypes.c_void_p),
                           k, m, nbytes, stripes, data.ctypes.data_as(ctypes.c_void_p),
                           erased.ctypes.data_as(ctypes.c_void_p), e, threads, passes, ctypes.byref(ok))
    t1 = hb.lhb_run(*args(1))  # warm-up + correctness pass
    if not ok.value:
        return {"error": "cpu baseline produced wrong data"}
    passes = max(1, int(target_seconds / max(t1 * threads, 1e-6)))
    t = hb.lhb_run(*args(passes))
    gbs = 2.0 * k * nbytes * stripes * passes / t / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": threads, "kind": kind,
            "sample": f"{stripes} stripes x {passes} passes of encode+decode (e={e}), "
                      f"{threads} threads, {t:.1f} s wall, {t * threads:.1f} s CPU",
            "ok": bool(ok.value)}


def main():
    args = parse()
    import torch
    world, rank, local = setup_dist()
    import longhair_amd as lh

    k, m, nbytes, stripes, erasures = CONFIGS[args.config]
    if args.stripes:
        stripes = args.stripes
    assert lh.cauchy_256_init() == 0, lh.lib().cauchy_256_last_error()
    lh.prepare(k, m, nbytes, stripes)
    X, D, rows0, rec_index = make_workload(k, m, nbytes, stripes, seed=1234 + rank, erasures=erasures)
    e_mean = float((rows0 >= k).sum()) / stripes
    if rec_index is None:
        rec_view = D[:, k - m:]     # the encode writes straight into D's recovery slots
    else:
        R = torch.empty((stripes, m, nbytes), dtype=torch.uint8, device="cuda")
        rec_view = R
        Dflat, Rflat = D.view(-1, nbytes), R.view(-1, nbytes)
    rows = rows0.clone()
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        lh.encode_batch(X, m, recovery=rec_view)
        if ev is not None:
            ev[1].record(stream)
        if rec_index is not None:   # deliver the received recovery blocks to their slots
            Dflat.index_copy_(0, rec_index[0], Rflat.index_select(0, rec_index[1]))
        rows.copy_(rows0)
        if ev is not None:
            ev[2].record(stream)
        lh.decode_batch(D, rows, m)
        if ev is not None:
            ev[3].record(stream)

    for _ in range(args.warmup):
        step()
    # Correctness gate on the final warm-up state: decoded slots must equal the data.
    barrier(world)
    if args.warmup:
        order = rows.long().argsort(dim=1)
        restored = torch.gather(D, 1, order.unsqueeze(-1).expand(-1, -1, nbytes))
        assert torch.equal(restored, X), "decode did not restore the data"

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    barrier(world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    barrier(world)
    t1 = time.perf_counter()
    elapsed = max_over_ranks(world, t1 - t0)

    enc_ms = sum(ev[0].elapsed_time(ev[1]) for ev in evs) / args.steps
    dec_ms = sum(ev[2].elapsed_time(ev[3]) for ev in evs) / args.steps
    ms_per_step = elapsed / args.steps * 1e3
    in_bytes = 2.0 * k * nbytes * stripes * world
    value = in_bytes * args.steps / elapsed / 1e9
    enc_alg = float(k + m) * nbytes * stripes           # read k, write m blocks per stripe
    dec_alg = (k + e_mean) * nbytes * stripes           # read k slots, write e blocks
    enc_k, dec_k = lh.kernel_names(k, m, nbytes)
    roof = {
        "encode": {"kernel": "+".join(enc_k), "ms": round(enc_ms, 4),
                   "achieved": round(enc_alg / (enc_ms * 1e-3) / 1e9, 1)},
        "decode": {"kernel": "+".join(dec_k), "ms": round(dec_ms, 4),
                   "achieved": round(dec_alg / (dec_ms * 1e-3) / 1e9, 1)},
    }
    dom = "decode" if dec_ms > enc_ms else "encode"
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", f"pmc_{args.config}.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        traffic = pmc.get(dom, {}).get("hbm_bytes_per_launch")
    out = {
        "metric": "GB/s of input data encoded+decoded, device-resident, per GPU and whole node",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"k={k} m={m} bytes={nbytes}, {stripes} stripes per GPU, encode + "
                               f"decode with {'e=' + str(min(k, m)) if erasures == 'max' else 'random e in [1,' + str(min(k, m)) + ']'}"
                               f" erased originals per stripe (mean {e_mean:.1f})",
                   "k": k, "m": m, "block_bytes": nbytes, "stripes_per_gpu": stripes,
                   "parallelism": f"stripes sharded over {world} rank(s), no collective"},
        "encode_GBps": round(k * nbytes * stripes / (enc_ms * 1e-3) / 1e9, 1),
        "decode_GBps": round(k * nbytes * stripes / (dec_ms * 1e-3) / 1e9, 1),
        "roofline": {"bound": "hbm", "kernel": roof[dom]["kernel"], "achieved": roof[dom]["achieved"],
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(roof[dom]["achieved"] / HBM_PEAK_GBS, 4), "traffic": traffic},
        "kernels": roof,
    }
    if rank == 0 and world == 1 and args.cpu_baseline != "off":
        out["cpu_baseline"] = cpu_baseline(k, m, nbytes, args.cpu_seconds,
                                           stripes=max(2, min(4096, (256 << 20) // (k * nbytes))))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
