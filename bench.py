#!/usr/bin/env python3
"""Benchmark: GB/s of input data encoded + decoded, device-resident (BASELINE.json metric).

One step = (1) cauchy_256_encode_batch of every stripe's k data blocks, writing the m
recovery blocks straight into the recovery slots of the decode buffer, (2) reset of the
Block.row bytes, (3) cauchy_256_decode_batch of every stripe in place (k - e surviving
originals in a per-stripe shuffled order + e recovery blocks, e = min(k, m) erased
originals chosen per stripe).  Input bytes per step = 2 * k * bytes * stripes.

Default workload: BASELINE.json configs[1] -- k=29, m=4, 1296-byte blocks, 65536 stripes
per GPU.  Multi-GPU (one process per GPU, no collective on the data path):

  python bench.py --gpus N                      weak scaling, 65536 stripes per rank
                                                (N = 8 is BASELINE configs[3]: 524288 stripes)
  python bench.py --gpus N --global-stripes G   strong scaling: G stripes split with
                                                longhair_amd.shard.shard_range

With --gpus N > 1 and no torchrun environment, this process starts
`torch.distributed.run --nproc-per-node N` on itself before touching any GPU and exits
with its code; under torchrun (WORLD_SIZE set) it must see WORLD_SIZE == N.
The process group is always gloo: the codec needs no collective (stripes are independent),
so the group only carries the barriers around the timed region and the per-rank timing
reduction -- the same code path with or without a GPU.  `--dry-run` replaces the HIP work
with a CPU stand-in (tests the launcher and the aggregation on a machine without a GPU).

Legs besides the device-resident steps (rank 0 unless noted): the PCIe-inclusive rate from
pinned host memory (every rank at once, `--pcie`, default on), the per-call latency of the
drop-in entry points, and the reference CPU codec on the host cores (`cpu_baseline`) over
the same erasure patterns as the GPU workload.

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
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# Calibrated ceilings of this chip (round 5: tools/ubench_r5.hip, profiles/r5b_ubench_floor.txt,
# one box; the same run reproduces the MI355X_MICROARCH.md float4 copy at 6.60 TB/s against the
# guide's 6.29): one-shot grids (one chunk set per thread), non-temporal loads and stores.
HBM_CEILING_GBS = 7131.3   # read-only stream, dwordx4, non-temporal, one-shot grid
HBM_CEILING_SRC = "profiles/r5b_ubench_floor.txt (read dwordx4 one-shot nt U=8: 2.46 GB read-only)"
# The encode's and decode's own byte mix (2.463 GB read + 0.340 GB written) as a flat stream,
# the fastest of the round-5 shapes (8 waves per block, 512-byte store segments): 0.4592 ms =
# 6.10 TB/s of total traffic, 5.36 TB/s of input.  The fastest 29:4 stream built, not a proven
# bound (its writes cost 2.9 TB/s against the copy's 6.1).
MIX_CEILING_GBS = 6104.4
FLAT_FLOOR_MS = 0.4592
FLAT_FLOOR_SRC = "profiles/r5b_ubench_floor.txt (mix LB=8 SEG=512 BS=256: 29:4 read:write flat stream)"
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (SIMD-32, MI355X_MICROARCH.md 'Wave scheduling'), 2.4 GHz -> wave-instructions / s.
VALU_PEAK_GINSTR = 256 * 4 * 2.4e9 / 2 / 1e9
# Measured v_bitop3_b32 issue rate at 8 waves/SIMD (profiles/r2_ubench_ceiling.txt).
VALU_CEILING_GINSTR = 761.5


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="untimed steps for this long before the warm-up steps, so the GPU's clocks settle "
                         "(reported as settle_steps; 0 = off)")
    ap.add_argument("--config", default="k29m4", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=0, help="override stripes per GPU (weak scaling)")
    ap.add_argument("--global-stripes", type=int, default=0,
                    help="strong scaling: total stripes split over the ranks with shard_range")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="wall-time budget of the CPU baseline leg")
    ap.add_argument("--dropin-calls", type=int, default=-1,
                    help="per-call drop-in latency leg (host pointers, one stripe per call); 0 = off")
    ap.add_argument("--ptr", default="on", choices=["on", "off"],
                    help="also time the step through the pointer-table batch calls (after the timed region)")
    ap.add_argument("--family", default="on", choices=["on", "off"],
                    help="also time the step on the block-size family modules (shapes they serve; untimed region)")
    ap.add_argument("--pcie", default="on", choices=["on", "off"],
                    help="PCIe-inclusive leg: cauchy_256_*_host_batch from pinned host memory on every rank")
    ap.add_argument("--pcie-stripes", type=int, default=0,
                    help="stripes per rank in the PCIe leg (default: the workload, capped at ~640 MB)")
    ap.add_argument("--align", type=int, default=0,
                    help="decode buffer: pad the stripe stride so the recovery slots start on this byte "
                         "boundary (0 = contiguous [S, k, bytes])")
    ap.add_argument("--dry-run", action="store_true", help="no HIP work: CPU stand-in step over gloo")
    ap.add_argument("--share-gpu", action="store_true",
                    help="map rank r to device r %% device_count (runs the N > 1 path on fewer GPUs than ranks: "
                         "a functional check of the control path, not a scaling measurement)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------ launcher
def launch(args):
    """Parent of an N-rank run: start torch.distributed.run with one process per GPU on
    this script and return its exit code.  Runs before anything touches a GPU (the
    children select their devices themselves); the child is a subprocess, never an exec."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def setup_dist(dry, share_gpu=False):
    """One process per GPU.  The group is gloo in every run: no data-path collective exists
    (SURVEY 8e), so it carries only host-side barriers and the timing reduction.
    share_gpu: rank -> device local % device_count (device_count() does not initialise the
    GPU on this image)."""
    import torch
    import torch.distributed as dist
    from longhair_amd.shard import world_info
    world, rank, local = world_info()
    if not dry:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()) if share_gpu else local)
    if world > 1:
        # gloo prints its connection report ("[Gloo] Rank r is connected to ...") on file
        # descriptor 1 from C++; stdout carries only rank 0's JSON line, so fd 1 points at
        # stderr while the group connects.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend="gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    return world, rank, local


def barrier(world, dry):
    """Device idle on every rank, then all ranks meet, then the device again."""
    import torch
    import torch.distributed as dist
    if not dry:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if not dry:
        torch.cuda.synchronize()


def per_rank(world, rank, value, dry=False):
    """Every rank's `value`, in rank order (one gloo all-reduce of a one-hot CPU vector)."""
    if world == 1:
        return [float(value)]
    import torch
    import torch.distributed as dist
    t = torch.zeros(world, dtype=torch.float64)
    t[rank] = float(value)
    dist.all_reduce(t)
    return [float(v) for v in t.tolist()]


# ------------------------------------------------------------------------ workload
def random_erasures(k, m, stripes, seed):
    """erasures="random": per stripe (e, the e recovery rows used), e uniform in
    [1, min(k, m)] -- a CPU generator, so tools can replay a workload's erasure counts."""
    import torch
    rng = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(stripes):
        e = int(torch.randint(1, min(k, m) + 1, (1,), generator=rng))
        out.append((e, torch.randperm(m, generator=rng)[:e]))
    return out


def aligned_layout(k, m, nbytes, align):
    """(offset, stripe stride) of a decode buffer whose every stripe's recovery slots
    k - m .. k - 1 -- the blocks the encode writes and the decode overwrites -- start on an
    `align`-byte boundary: the stride is k * bytes rounded up to a multiple of `align`, the
    buffer starts `offset` bytes into an aligned allocation.  align 0: (0, k * bytes)."""
    if not align or ((k - m) * nbytes % align == 0 and k * nbytes % align == 0):
        return 0, k * nbytes
    return (-(k - m) * nbytes) % align, -(-k * nbytes // align) * align


def decode_buffer(k, m, nbytes, stripes, align):
    """The decode buffer D [S, k, bytes]: contiguous, or laid out by
    aligned_layout.  Returns (D, stripe stride)."""
    import torch
    off, stride = aligned_layout(k, m, nbytes, align)
    if stride == k * nbytes:
        return torch.empty((stripes, k, nbytes), dtype=torch.uint8, device="cuda"), stride
    buf = torch.empty(off + stride * stripes, dtype=torch.uint8, device="cuda")  # 256-B aligned
    return buf[off:].as_strided((stripes, k, nbytes), (stride, nbytes, 1)), stride


def make_workload(k, m, nbytes, stripes, seed, erasures="max", align=0):
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
    D, _ = decode_buffer(k, m, nbytes, stripes, align if erasures == "max" else 0)
    if erasures == "max":
        e = min(k, m)
        assert e == m, "erasures='max' writes all m recovery rows into the decode buffer"
        keep = perm[:, : k - e]
        D[:, : k - e] = torch.gather(X, 1, keep.unsqueeze(-1).expand(-1, -1, nbytes))
        rows0 = torch.cat([keep, torch.arange(k, k + e, device="cuda").expand(stripes, e)], dim=1)
        return X, D, rows0.to(torch.uint8).contiguous(), None
    rows0 = torch.empty((stripes, k), dtype=torch.long)
    dst, src = [], []
    perm_c = perm.cpu()
    for s, (e, rec_rows) in enumerate(random_erasures(k, m, stripes, seed)):
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


# ------------------------------------------------------------------ CPU baseline leg
def effective_cpus():
    """(threads to use, CPUs in our affinity mask, cgroup CPU quota or None): the
    threads are the affinity count capped by the cgroup quota the box grants."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, aff, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def per_call_us(enc, dec, k, m, nbytes, calls, data, blocks_for, rounds=5):
    """Microseconds of one cauchy_256_encode and one cauchy_256_decode call (one stripe, host
    pointers, the reference's call shape): `calls` calls each, in `rounds` rounds;
    encode_us / decode_us = the best round's mean (a host shared with other work preempts
    some rounds -- one 12 ms window measured 12.0 us per decode where the rest of the run
    and other boxes gave 7.3-8.7), *_mean_us = the mean over all calls.  The reference CPU
    codec is timed by this same function.
    blocks_for(i) -> a fresh ctypes Block array (rows reset to the erased state)."""
    import numpy as np
    ptrs = (ctypes.POINTER(ctypes.c_ubyte) * k)()
    for x in range(k):
        ptrs[x] = ctypes.cast(data.ctypes.data + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
    rec = np.zeros(m * nbytes, dtype=np.uint8)
    rp = ctypes.c_void_p(rec.ctypes.data)
    for _ in range(5):
        assert enc(k, m, ptrs, rp, nbytes) == 0
    per = max(1, calls // rounds)
    enc_t = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        for _ in range(per):
            enc(k, m, ptrs, rp, nbytes)
        enc_t.append((time.perf_counter() - t0) / per)
    arrays = [blocks_for(i, rec) for i in range(per * rounds + 5)]
    for i in range(5):
        assert dec(k, m, arrays[i], nbytes) == 0
    dec_t = []
    for r in range(rounds):
        t0 = time.perf_counter()
        for i in range(per):
            dec(k, m, arrays[5 + r * per + i], nbytes)
        dec_t.append((time.perf_counter() - t0) / per)
    return {"encode_us": round(min(enc_t) * 1e6, 2), "decode_us": round(min(dec_t) * 1e6, 2),
            "encode_mean_us": round(sum(enc_t) / rounds * 1e6, 2), "decode_mean_us": round(sum(dec_t) / rounds * 1e6, 2),
            "calls": per * rounds, "rounds": rounds}


def dropin_blocks(k, m, nbytes, data, erased_rows=None):
    """Factory of decode Block arrays: the first min(k, m) originals erased and replaced
    by recovery blocks k.. (each array gets its own recovery copies, so every timed call
    decodes a fresh stripe)."""
    import numpy as np
    import lhutil
    e = min(k, m)
    keep = [x for x in range(k)][e:]
    store = []

    def make(i, rec):
        r = rec.copy()
        store.append(r)
        arr = (lhutil.Block * k)()
        for j, x in enumerate(keep):
            arr[j].data = ctypes.cast(data.ctypes.data + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
            arr[j].row = x
        for j in range(e):
            arr[len(keep) + j].data = ctypes.cast(r.ctypes.data + j * nbytes, ctypes.POINTER(ctypes.c_ubyte))
            arr[len(keep) + j].row = k + j
        return arr
    return make


def erasure_patterns(rows, k):
    """From Block.row bytes [n, k] of decode slots: (erased originals [n, e_max], erasures
    per stripe [n], recovery rows used [n, e_max]) for lhb_run_pattern."""
    import numpy as np
    n = rows.shape[0]
    e_of = (rows >= k).sum(axis=1).astype(np.uint8)
    e_max = max(1, int(e_of.max()))
    erased = np.zeros((n, e_max), dtype=np.uint8)
    rec = np.zeros((n, e_max), dtype=np.uint8)
    for s in range(n):
        miss = np.setdiff1d(np.arange(k), rows[s][rows[s] < k])[: e_of[s]]
        erased[s, : len(miss)] = miss
        rr = np.sort(rows[s][rows[s] >= k]) - k
        rec[s, : len(rr)] = rr
    return erased, e_of, rec, e_max


def cpu_baseline(k, m, nbytes, budget_s, stripes, patterns=None):
    """Reference codec (oracle/_ref, compiled from the reference sources) -- or, if that
    build is absent, the oracle restatement -- on the host cores, same step definition,
    a bounded sample of stripes: all granted cores, then one thread; plus the per-call
    latency of one-stripe encode / decode (the reference API shape).  `patterns`: the
    Block.row bytes of the GPU workload's first decode stripes, so the reference decodes
    the same erasure counts and recovery rows as the line it is reported beside."""
    import numpy as np
    import lhutil
    bench_so = os.path.join(REPO, "oracle", "liblh_cpubench.so")
    if not os.path.exists(bench_so):
        return None
    hb = ctypes.CDLL(bench_so)
    hb.lhb_run_pattern.restype = ctypes.c_double
    if os.path.exists(lhutil.REF_SO):
        lib, kind = lhutil.RefLib(), "reference"
        enc, dec = lib.lib.cauchy_256_encode, lib.lib.cauchy_256_decode
    else:
        lib, kind = lhutil.Oracle(), "port"
        enc, dec = lib.lib.lho_encode, lib.lib.lho_decode
    data = lhutil.fill(99, stripes * k * nbytes)
    if patterns is None:
        e = min(k, m)
        rng = np.random.Generator(np.random.PCG64(5))
        erased = np.stack([rng.choice(k, size=e, replace=False) for _ in range(stripes)]).astype(np.uint8)
        e_of = np.full(stripes, e, dtype=np.uint8)
        rec_rows = np.tile(np.arange(e, dtype=np.uint8), (stripes, 1))
    else:
        idx = np.arange(stripes) % patterns.shape[0]
        erased, e_of, rec_rows, e = erasure_patterns(np.ascontiguousarray(patterns[idx]), k)
    erased, e_of, rec_rows = (np.ascontiguousarray(a) for a in (erased, e_of, rec_rows))
    e_mean = float(e_of.mean())
    threads, aff, quota = effective_cpus()
    ok = ctypes.c_int(0)
    cpu_s = ctypes.c_double(0.0)
    vp = ctypes.c_void_p

    def run(nstripes, nthreads, passes):
        t = hb.lhb_run_pattern(ctypes.cast(enc, vp), ctypes.cast(dec, vp), k, m, nbytes, nstripes,
                               data.ctypes.data_as(vp), erased.ctypes.data_as(vp), e_of.ctypes.data_as(vp),
                               rec_rows.ctypes.data_as(vp), e, nthreads, passes, ctypes.byref(ok),
                               ctypes.byref(cpu_s))
        return t, cpu_s.value, bool(ok.value)

    t1, _, good = run(stripes, threads, 1)  # warm-up + correctness pass
    if not good:
        return {"error": "cpu baseline produced wrong data"}
    passes = max(1, int(0.65 * budget_s / max(t1, 1e-6)))
    t, cs, good = run(stripes, threads, passes)
    gbs = 2.0 * k * nbytes * stripes * passes / t / 1e9
    s1 = max(2, min(stripes, stripes // max(1, threads)))
    t1a, _, _ = run(s1, 1, 1)
    p1 = max(1, int(0.25 * budget_s / max(t1a, 1e-6)))
    tb, cs1, good1 = run(s1, 1, p1)
    gbs1 = 2.0 * k * nbytes * s1 * p1 / tb / 1e9
    out = {"value": round(gbs, 3), "unit": "GB/s", "cores": threads, "kind": kind,
           "sample": f"{stripes} stripes x {passes} passes of encode+decode "
                     f"({'the GPU workload' + chr(39) + 's erasure patterns, ' if patterns is not None else ''}"
                     f"mean e {e_mean:.1f}), {threads} threads: "
                     f"{t:.1f} s wall, {cs:.1f} s CPU measured; 1 thread: {s1} stripes x {p1} passes, "
                     f"{tb:.1f} s wall",
           "value_1thread": round(gbs1, 3), "cpu_seconds": round(cs, 2), "wall_seconds": round(t, 2),
           "cpu_model": cpu_model(), "cores_affinity": aff, "cgroup_cpu_quota": quota,
           "ok": bool(good and good1)}
    calls = max(10, min(2000, int(4e7 / (k * nbytes))))
    d0 = lhutil.fill(7, k * nbytes)
    enc.restype = dec.restype = ctypes.c_int
    out["per_call_us"] = per_call_us(enc, dec, k, m, nbytes, calls, d0, dropin_blocks(k, m, nbytes, d0))
    return out


def device_per_call_us(lib, k, m, nbytes, calls, rounds=5):
    """As per_call_us, with every block in device memory (the drop-in calls then take the
    pointer-table form: one copy of the pointers, the blocks coded where they lie)."""
    import torch
    import lhutil
    data = torch.from_numpy(lhutil.fill(7, k * nbytes)).cuda()
    rec = torch.zeros(m * nbytes, dtype=torch.uint8, device="cuda")
    ptrs = (ctypes.POINTER(ctypes.c_ubyte) * k)()
    for x in range(k):
        ptrs[x] = ctypes.cast(data.data_ptr() + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
    rp = ctypes.c_void_p(rec.data_ptr())
    for _ in range(5):
        assert lib.cauchy_256_encode(k, m, ptrs, rp, nbytes) == 0
    per = max(1, calls // rounds)
    enc_t = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        for _ in range(per):
            lib.cauchy_256_encode(k, m, ptrs, rp, nbytes)
        enc_t.append((time.perf_counter() - t0) / per)
    e = min(k, m)
    n = per * rounds + 5
    recs = rec.repeat(n).view(n, m * nbytes)  # a fresh copy of the recovery blocks per call
    arrays = []
    for i in range(n):
        arr = (lhutil.Block * k)()
        for j, x in enumerate(range(e, k)):
            arr[j].data = ctypes.cast(data.data_ptr() + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
            arr[j].row = x
        for j in range(e):
            arr[k - e + j].data = ctypes.cast(recs[i].data_ptr() + j * nbytes, ctypes.POINTER(ctypes.c_ubyte))
            arr[k - e + j].row = k + j
        arrays.append(arr)
    for i in range(5):
        assert lib.cauchy_256_decode(k, m, arrays[i], nbytes) == 0
    dec_t = []
    for r in range(rounds):
        t0 = time.perf_counter()
        for i in range(per):
            lib.cauchy_256_decode(k, m, arrays[5 + r * per + i], nbytes)
        dec_t.append((time.perf_counter() - t0) / per)
    got = recs[n - 1].view(m, nbytes)[:e].cpu()
    ok = bool(torch.equal(got, data.view(k, nbytes)[:e].cpu()))
    return {"encode_us": round(min(enc_t) * 1e6, 2), "decode_us": round(min(dec_t) * 1e6, 2),
            "encode_mean_us": round(sum(enc_t) / rounds * 1e6, 2), "decode_mean_us": round(sum(dec_t) / rounds * 1e6, 2),
            "calls": per * rounds, "rounds": rounds, "ok": ok}


def dropin_leg(lh, k, m, nbytes, calls):
    """Per-call latency of the product's drop-in cauchy_256_encode / cauchy_256_decode with
    host pointers, one stripe per call (the reference API shape), plus the ctypes call
    overhead of this harness."""
    import numpy as np
    import lhutil
    lib = lh.lib()
    d0 = lhutil.fill(7, k * nbytes)
    # top level: the library's default policy, i.e. what an unchanged reference caller gets
    out = per_call_us(lib.cauchy_256_encode, lib.cauchy_256_decode, k, m, nbytes, calls, d0,
                      dropin_blocks(k, m, nbytes, d0))
    out["policy"] = lh.dispatch_policy()
    out["host_isa"] = lh.host_isa()
    # which engine the default policy used for these calls: the launch trace is empty when a
    # call ran on the host SIMD engine (cauchy_256_last_launch)
    ptrs0 = (ctypes.POINTER(ctypes.c_ubyte) * k)()
    for x in range(k):
        ptrs0[x] = ctypes.cast(d0.ctypes.data + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
    rec0 = np.zeros(m * nbytes, dtype=np.uint8)
    lib.cauchy_256_encode(k, m, ptrs0, ctypes.c_void_p(rec0.ctypes.data), nbytes)
    out["engine"] = (f"host SIMD engine ({out['host_isa']})" if not lh.last_launch()
                     else "GPU (" + "+".join(lh.last_launch()) + ")")
    # the same calls forced onto the GPU (include/cauchy_256_dispatch.h)
    prev = lh.set_dispatch("gpu")
    out["gpu"] = per_call_us(lib.cauchy_256_encode, lib.cauchy_256_decode, k, m, nbytes, calls, d0,
                             dropin_blocks(k, m, nbytes, d0))
    lh.set_dispatch(prev)
    # blocks already in device memory (any policy runs them on the GPU)
    out["gpu_device_blocks"] = device_per_call_us(lib, k, m, nbytes, calls)
    out["gpu_device_blocks"]["kernels"] = lh.last_launch()
    # the recovered blocks of the last decoded array must equal the erased originals
    ref = lhutil.fill(7, k * nbytes).reshape(k, nbytes)
    rec = np.zeros(m * nbytes, dtype=np.uint8)
    ptrs = (ctypes.POINTER(ctypes.c_ubyte) * k)()
    for x in range(k):
        ptrs[x] = ctypes.cast(d0.ctypes.data + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
    assert lib.cauchy_256_encode(k, m, ptrs, ctypes.c_void_p(rec.ctypes.data), nbytes) == 0
    make = dropin_blocks(k, m, nbytes, d0)   # holds the recovery copies the Block array points at
    arr = make(0, rec)
    assert lib.cauchy_256_decode(k, m, arr, nbytes) == 0
    for j in range(k):
        got = np.ctypeslib.as_array(arr[j].data, shape=(nbytes,))
        assert got.tobytes() == ref[arr[j].row].tobytes(), "drop-in decode mismatch"
    noop = lib.cauchy_256_last_error
    t0 = time.perf_counter()
    for _ in range(calls):
        noop()
    out["ctypes_overhead_us"] = round((time.perf_counter() - t0) / calls * 1e6, 2)
    out["dispatch"] = (f"top level: the default policy ({out['policy']}), served by the {out['engine']}; "
                       "out['gpu']: the same calls forced onto the GPU; out['gpu_device_blocks']: the blocks "
                       "in device memory (pointer-table form)")
    return out


def pcie_leg(lh, args, k, m, nbytes, X, D, rows0, rec_view, rec_index, world, rank, reps=3):
    """PCIe-inclusive rate: the workload's first stripes copied to pinned host
    memory, then cauchy_256_encode_host_batch and cauchy_256_decode_host_batch (H2D, kernels
    and D2H pipelined over three streams), every rank at the same time.  Input GB/s per rank
    and for the node (all ranks' input bytes / the slowest rank's time)."""
    import torch
    n = args.pcie_stripes or min(X.shape[0], max(1, (640 << 20) // (k * nbytes)))
    n = min(n, X.shape[0])
    # decode input: the recovery blocks back in their slots (the timed steps decoded them)
    lh.encode_batch(X, m, recovery=rec_view)
    if rec_index is not None:
        D.view(-1, nbytes).index_copy_(0, rec_index[0], rec_view.reshape(-1, nbytes).index_select(0, rec_index[1]))
    torch.cuda.synchronize()
    hx = X[:n].cpu().pin_memory()
    hb0 = D[:n].cpu()
    hb = hb0.clone().pin_memory()
    hr0 = rows0[:n].cpu()
    hr = hr0.clone().pin_memory()
    hrec = torch.empty((n, m, nbytes), dtype=torch.uint8).pin_memory()
    return pcie_timed(lh, k, m, nbytes, hx.numpy(), hb.numpy(), hr.numpy(), hrec.numpy(), hb0.numpy(),
                      hr0.numpy(), world, rank, reps)


def pcie_timed(lh, k, m, nbytes, xn, bn, rn, recn, b0, r0, world, rank, reps=3, dry=False):
    """The timed part of pcie_leg on host arrays (data xn [n, k, B], decode slots bn and rows
    rn, recovery recn; b0 / r0 the slots and rows to restore before each decode), every rank
    at once between barriers, and the cross-rank aggregation: every rank makes the same
    per_rank calls in the same order (tests/test_multiproc.py drives it at world 2 on gloo
    with a stand-in codec)."""
    import numpy as np
    n = xn.shape[0]
    lh.encode_host_batch(xn, m, recovery=recn)           # warm-up: buffers, streams
    lh.decode_host_batch(bn, rn, m)
    order = np.argsort(rn, axis=1)
    ok = bool(np.array_equal(np.take_along_axis(bn, order[:, :, None], axis=1), xn))
    te = td = 0.0
    for _ in range(reps):
        barrier(world, dry)
        t0 = time.perf_counter()
        lh.encode_host_batch(xn, m, recovery=recn)
        te += time.perf_counter() - t0
        bn[:] = b0
        rn[:] = r0
        barrier(world, dry)
        t0 = time.perf_counter()
        lh.decode_host_batch(bn, rn, m)
        td += time.perf_counter() - t0
    te, td = te / reps, td / reps
    inb = float(k * nbytes * n)
    enc_r = per_rank(world, rank, inb / te / 1e9)
    dec_r = per_rank(world, rank, inb / td / 1e9)
    te_max, td_max = max(per_rank(world, rank, te)), max(per_rank(world, rank, td))
    ok_all = min(per_rank(world, rank, 1.0 if ok else 0.0)) == 1.0
    return {"stripes_per_rank": n, "input_MB_per_rank": round(inb / 1e6, 1),
            "encode_GBps_per_rank": [round(v, 2) for v in enc_r],
            "decode_GBps_per_rank": [round(v, 2) for v in dec_r],
            "node_encode_GBps": round(inb * world / te_max / 1e9, 2),
            "node_decode_GBps": round(inb * world / td_max / 1e9, 2),
            "ok": ok_all,
            "what": "input GB/s incl. host-to-device and device-to-host copies: pinned host stripes, "
                    "cauchy_256_{encode,decode}_host_batch, every rank at once, mean of "
                    f"{reps} (decode: the workload's erasure patterns, recovered blocks written back)"}


def ptr_leg(lh, k, m, nbytes, X, D, rows0, rec_view, rec_index=None, reps=5, settle_s=0.25):
    """The same step through the pointer-table calls (cauchy_256_*_batch_ptrs): tables that
    point at the very blocks the strided step uses, so the bytes moved are the same and only
    the addressing differs.  With random erasures (rec_index) the received recovery slots
    point straight at the encode's output blocks, where the strided step copies them into the
    decode buffer first (that copy is outside both timings).  HIP-event times on the launch
    stream, mean of `reps` after untimed passes for `settle_s` (the leg follows the correctness
    gate, after which the first steps run slow: DESIGN.md 6.2.1); the decoded data is checked
    against X afterwards."""
    import torch
    lh.prepare_ptrs(k, m, nbytes)  # the pointer-table modules (cached at build time for the configs)
    stripes = X.shape[0]
    s_idx = torch.arange(stripes, device="cuda", dtype=torch.int64).unsqueeze(1)

    def table(t, n):
        return (t.data_ptr() + s_idx * t.stride(0) + torch.arange(n, device="cuda", dtype=torch.int64) * t.stride(1)
                ).contiguous()
    dptr, rptr, bptr = table(X, k), table(rec_view, m), table(D, k)
    if rec_index is not None:
        bptr.view(-1)[rec_index[0]] = rec_view.data_ptr() + rec_index[1] * nbytes
    rows = rows0.clone()
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    enc = dec = 0.0
    traces = {}
    t_s, warm = time.perf_counter(), 0
    while True:  # untimed passes (at least one) for settle_s
        lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr, stream=stream)
        rows.copy_(rows0)
        lh.decode_batch_ptrs(k, m, nbytes, bptr, rows, stream=stream)
        warm += 1
        if warm % 4 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() - t_s >= settle_s:
                break
    for i in range(reps + 1):
        ev[0].record(stream)
        lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr, stream=stream)
        ev[1].record(stream)
        traces.setdefault("encode", lh.last_launch())
        rows.copy_(rows0)
        ev[2].record(stream)
        lh.decode_batch_ptrs(k, m, nbytes, bptr, rows, stream=stream)
        ev[3].record(stream)
        traces.setdefault("decode", lh.last_launch())
        torch.cuda.synchronize()
        if i:  # the first pass warms up
            enc += ev[0].elapsed_time(ev[1]) / reps
            dec += ev[2].elapsed_time(ev[3]) / reps
    order = rows.long().argsort(dim=1)
    got = D
    if rec_index is not None:
        got = D.clone()
        got.view(-1, nbytes)[rec_index[0]] = rec_view.reshape(-1, nbytes)[rec_index[1]]
    ok = bool(torch.equal(torch.gather(got, 1, order.unsqueeze(-1).expand(-1, -1, nbytes)), X))
    return {"encode_ms": round(enc, 4), "decode_ms": round(dec, 4),
            "encode_GBps": round(k * nbytes * stripes / (enc * 1e-3) / 1e9, 1),
            "decode_GBps": round(k * nbytes * stripes / (dec * 1e-3) / 1e9, 1),
            "encode_kernels": traces["encode"], "decode_kernels": traces["decode"], "ok": ok,
            "what": "the step through cauchy_256_{encode,decode}_batch_ptrs: per-block device pointer tables "
                    "(the reference's data_ptrs[] / Block.data per stripe) over the same buffers, "
                    f"HIP events, mean of {reps} after {warm} untimed passes"}


def family_leg(lh, k, m, nbytes, X, D, rows0, rec_view, reps=5, settle_s=0.25):
    """The same step on the (k, m) block-size family modules (jit_codec.hip LH_FAMILY: the
    block size a kernel argument, one module per (k, m) and role), which serve
    every block size that has no size-specialised module -- the first call at a new size.
    Forced with LONGHAIR_AMD_JIT_DEFINES=LH_FAMILY=1 for the leg only; HIP events on the launch
    stream, mean of `reps` after untimed passes for `settle_s`; the decoded data is checked.
    None when neither family serves the shape."""
    import torch
    enc_ok = lh.lib().cauchy_256_batch_path(k, m, nbytes, 8) == 1
    dec_ok = lh.lib().cauchy_256_batch_path(k, m, nbytes, 9) == 1
    if not (enc_ok or dec_ok):
        return None
    saved = os.environ.get("LONGHAIR_AMD_JIT_DEFINES")
    os.environ["LONGHAIR_AMD_JIT_DEFINES"] = "LH_FAMILY=1"
    try:
        stripes = X.shape[0]
        lh.prepare(k, m, nbytes, stripes)  # the family modules (cached at build time for the BASELINE shapes)
        rows = rows0.clone()
        stream = torch.cuda.current_stream()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        enc = dec = 0.0
        traces = {}
        t_s, warm = time.perf_counter(), 0
        while True:
            lh.encode_batch(X, m, recovery=rec_view, stream=stream)
            rows.copy_(rows0)
            lh.decode_batch(D, rows, m, stream=stream)
            warm += 1
            if warm % 4 == 0:
                torch.cuda.synchronize()
                if time.perf_counter() - t_s >= settle_s:
                    break
        for i in range(reps + 1):
            ev[0].record(stream)
            lh.encode_batch(X, m, recovery=rec_view, stream=stream)
            ev[1].record(stream)
            traces.setdefault("encode", lh.last_launch())
            rows.copy_(rows0)
            ev[2].record(stream)
            lh.decode_batch(D, rows, m, stream=stream)
            ev[3].record(stream)
            traces.setdefault("decode", lh.last_launch())
            torch.cuda.synchronize()
            if i:
                enc += ev[0].elapsed_time(ev[1]) / reps
                dec += ev[2].elapsed_time(ev[3]) / reps
        order = rows.long().argsort(dim=1)
        ok = bool(torch.equal(torch.gather(D, 1, order.unsqueeze(-1).expand(-1, -1, nbytes)), X))
    finally:
        if saved is None:
            os.environ.pop("LONGHAIR_AMD_JIT_DEFINES", None)
        else:
            os.environ["LONGHAIR_AMD_JIT_DEFINES"] = saved
    return {"encode_ms": round(enc, 4), "decode_ms": round(dec, 4),
            "encode_kernels": traces["encode"], "decode_kernels": traces["decode"], "ok": ok,
            "what": "the step on the (k, m) block-size family modules (the block size a kernel argument: what a "
                    "block size without a size-specialised module runs), forced for this leg, HIP events, "
                    f"mean of {reps} after {warm} untimed passes"}


def reflayout_leg(lh, k, m, nbytes, X, rows0, reps=5, settle_s=0.25):
    """The decode on the reference benchmark's block order (tests/cauchy_256_tests.cpp:296-307:
    every surviving original in its own slot, the recovery blocks in the erased originals'
    slots) instead of the bench's shuffled survivors: the same erasures (rows0), the slots in
    row order, so the decode reads each stripe's survivors in memory order.  HIP events, mean
    of `reps` after untimed passes for `settle_s`; the recovery blocks are put back before
    every pass (outside the events) and the decoded stripes are checked against X."""
    import torch
    stripes, e = X.shape[0], m
    stream = torch.cuda.current_stream()
    R = lh.encode_batch(X, m, stream=stream)  # [S, m, bytes]
    keep = rows0[:, : k - e].long()
    present = torch.zeros((stripes, k), dtype=torch.int32, device="cuda").scatter_(1, keep, 1)
    er = torch.argsort(present, dim=1, stable=True)[:, :e]  # erased originals, ascending
    D2 = X.clone()
    rows_ref = torch.arange(k, device="cuda").repeat(stripes, 1).scatter_(
        1, er, (k + torch.arange(e, device="cuda")).repeat(stripes, 1)).to(torch.uint8)
    rows = rows_ref.clone()
    idx = er.unsqueeze(-1).expand(-1, -1, nbytes)

    def reset():
        D2.scatter_(1, idx, R[:, :e])
        rows.copy_(rows_ref)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t_s, warm = time.perf_counter(), 0
    while True:
        reset()
        lh.decode_batch(D2, rows, m, stream=stream)
        warm += 1
        if warm % 4 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() - t_s >= settle_s:
                break
    dec = 0.0
    trace = None
    for i in range(reps + 1):
        reset()
        ev[0].record(stream)
        lh.decode_batch(D2, rows, m, stream=stream)
        ev[1].record(stream)
        trace = trace or lh.last_launch()
        torch.cuda.synchronize()
        if i:
            dec += ev[0].elapsed_time(ev[1]) / reps
    ok = bool(torch.equal(D2, X))
    return {"decode_ms": round(dec, 4), "decode_GBps": round(k * nbytes * stripes / (dec * 1e-3) / 1e9, 1),
            "decode_kernels": trace, "ok": ok,
            "what": "decode_batch on the reference benchmark's block order (survivors in their own slots, "
                    "recovery blocks in the erased slots; same erasures), HIP events, "
                    f"mean of {reps} after {warm} untimed passes"}


def load_profile(name):
    path = os.path.join(REPO, "profiles", name)
    return json.load(open(path)) if os.path.exists(path) else None


# ------------------------------------------------------------------------------ main
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    dry = args.dry_run
    import torch
    world, rank, local = setup_dist(dry, args.share_gpu)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    from longhair_amd.shard import shard_range

    k, m, nbytes, stripes, erasures = CONFIGS[args.config]
    if args.stripes:
        stripes = args.stripes
    scaling = "weak"
    lo = rank * stripes
    if args.global_stripes:
        scaling = "strong"
        lo, hi = shard_range(args.global_stripes, world, rank)
        stripes = hi - lo
    total_stripes = args.global_stripes or stripes * world

    if dry:
        import numpy as np
        buf = np.ones((1 << 20,), dtype=np.uint8)
        out_buf = np.empty_like(buf)
        e_mean = float(min(k, m))

        def step(ev=None):
            np.bitwise_xor(buf, buf, out=out_buf)
    else:
        import longhair_amd as lh
        assert lh.cauchy_256_init() == 0, lh.lib().cauchy_256_last_error()
        lh.prepare(k, m, nbytes, stripes)
        X, D, rows0, rec_index = make_workload(k, m, nbytes, stripes, seed=1234 + lo, erasures=erasures,
                                               align=args.align)
        e_mean = float((rows0 >= k).sum()) / max(1, stripes)
        if rec_index is None:
            rec_view = D[:, k - m:]     # the encode writes straight into D's recovery slots
        else:
            R = torch.empty((stripes, m, nbytes), dtype=torch.uint8, device="cuda")
            rec_view = R
            Dflat, Rflat = D.view(-1, nbytes), R.view(-1, nbytes)
        rows = rows0.clone()
        stream = torch.cuda.current_stream()  # every kernel below is launched on this stream
        traces = {}

        def step(ev=None):
            if ev is not None:
                ev[0].record(stream)
            lh.encode_batch(X, m, recovery=rec_view, stream=stream)
            traces.setdefault("encode", lh.last_launch())
            if ev is not None:
                ev[1].record(stream)
            if rec_index is not None:   # deliver the received recovery blocks to their slots
                Dflat.index_copy_(0, rec_index[0], Rflat.index_select(0, rec_index[1]))
            rows.copy_(rows0)
            if ev is not None:
                ev[2].record(stream)
            lh.decode_batch(D, rows, m, stream=stream)
            traces.setdefault("decode", lh.last_launch())
            if ev is not None:
                ev[3].record(stream)

    # Settle: untimed steps for --settle-ms before the warm-up.  A fresh process's first
    # back-to-back steps run slow and speed up over ~20 ms (profiles/r7e_seq_probe.txt: the
    # k29/m4 decode 0.668 -> 0.553 ms over its first 20 steps, then flat at 0.56 ms in every
    # later round, synced or not), so 3 warm-up steps alone leave the timed steps on that ramp.
    # The first 20 settle steps carry HIP events: the line reports them as cold_start_ms
    # (outside the timed region).
    settle_steps = 0
    cold = []
    if args.settle_ms > 0 and not dry:
        torch.cuda.synchronize()
        t_s = time.perf_counter()
        while True:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if len(cold) < 20 else None
            step(ev)
            if ev is not None:
                cold.append(ev)
            settle_steps += 1
            if settle_steps % 8 == 0:
                torch.cuda.synchronize()
                if time.perf_counter() - t_s >= args.settle_ms / 1e3:
                    break
    for _ in range(args.warmup):
        step()
    barrier(world, dry)

    evs = None if dry else [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    barrier(world, dry)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(None if dry else evs[i])
    barrier(world, dry)
    t1 = time.perf_counter()
    if (args.steps or args.warmup) and not dry:
        # Correctness gate on the last step's state: decoded slots must equal the data.  (After
        # the timed region: run between the warm-up and the timed steps, its 2.5 GB gather left
        # the first timed decodes ~5 % slow, profiles/r7f_bench_k29m4.json.)
        order = rows.long().argsort(dim=1)
        restored = torch.gather(D, 1, order.unsqueeze(-1).expand(-1, -1, nbytes))
        assert torch.equal(restored, X), "decode did not restore the data"
        del restored, order
    elapsed_ranks = per_rank(world, rank, t1 - t0, dry)
    stripes_ranks = per_rank(world, rank, stripes, dry)
    elapsed = max(elapsed_ranks)

    step_bytes = 2.0 * k * nbytes                  # input bytes per stripe per step
    ms_per_step = elapsed / args.steps * 1e3
    value = step_bytes * sum(stripes_ranks) * args.steps / elapsed / 1e9
    per_gpu = [round(step_bytes * s * args.steps / t / 1e9, 2) for s, t in zip(stripes_ranks, elapsed_ranks)]
    workload = (f"k={k} m={m} bytes={nbytes}, "
                + (f"{args.global_stripes} stripes split over {world} GPU(s)" if scaling == "strong"
                   else f"{stripes} stripes per GPU")
                + f", encode + decode with "
                + ("e=" + str(min(k, m)) if erasures == "max" else "random e in [1," + str(min(k, m)) + "]")
                + f" erased originals per stripe (mean {e_mean:.1f})")
    out = {
        "metric": "GB/s of input data encoded+decoded, device-resident, per GPU and whole node",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_steps": settle_steps,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": workload, "k": k, "m": m, "block_bytes": nbytes,
                   "stripes_per_gpu": stripes if scaling == "weak" else None,
                   "global_stripes": total_stripes,
                   "decode_buffer_stripe_stride": None if dry else int(D.stride(0)),
                   "parallelism": f"stripes sharded over {world} rank(s), no collective"},
        "per_gpu_GBps": per_gpu,
        "node_GBps": round(value, 2),
    }
    if dry:
        out["dry_run"] = True
    else:
        enc_ms = sum(ev[0].elapsed_time(ev[1]) for ev in evs) / args.steps
        dec_ms = sum(ev[2].elapsed_time(ev[3]) for ev in evs) / args.steps
        out["step_ms"] = {"encode": [round(ev[0].elapsed_time(ev[1]), 3) for ev in evs],
                          "decode": [round(ev[2].elapsed_time(ev[3]), 3) for ev in evs]}
        if cold:
            out["cold_start_ms"] = {
                "encode": [round(ev[0].elapsed_time(ev[1]), 3) for ev in cold],
                "decode": [round(ev[2].elapsed_time(ev[3]), 3) for ev in cold],
                "note": ("the first settle steps after setup, back to back, HIP events; untimed, outside "
                         "the timed region (DESIGN.md 6.2.1)")}
        enc_alg = float(k + m) * nbytes * stripes           # read k, write m blocks per stripe
        dec_alg = (k + e_mean) * nbytes * stripes           # read k slots, write e blocks
        # the kernels the batch calls really launched (cauchy_256_last_launch)
        enc_k, dec_k = traces.get("encode") or lh.kernel_names(k, m, nbytes)[0], \
            traces.get("decode") or lh.kernel_names(k, m, nbytes)[1]
        roof = {
            "encode": {"kernel": "+".join(enc_k), "ms": round(enc_ms, 4),
                       "achieved": round(enc_alg / (enc_ms * 1e-3) / 1e9, 1)},
            "decode": {"kernel": "+".join(dec_k), "ms": round(dec_ms, 4),
                       "achieved": round(dec_alg / (dec_ms * 1e-3) / 1e9, 1)},
        }
        dom = "decode" if dec_ms > enc_ms else "encode"
        pmc = load_profile(f"pmc_{args.config}.json")
        traffic = pmc.get(dom, {}).get("hbm_bytes_per_launch") if pmc and stripes == CONFIGS[args.config][3] else None
        hbm = {"bound": "hbm", "kernel": roof[dom]["kernel"], "achieved": roof[dom]["achieved"],
               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(roof[dom]["achieved"] / HBM_PEAK_GBS, 4),
               "traffic": traffic, "measured_ceiling": MIX_CEILING_GBS, "ceiling_source": FLAT_FLOOR_SRC,
               "frac_of_measured_ceiling": round(roof[dom]["achieved"] / MIX_CEILING_GBS, 4)}
        out["encode_GBps"] = round(k * nbytes * stripes / (enc_ms * 1e-3) / 1e9, 1)
        out["decode_GBps"] = round(k * nbytes * stripes / (dec_ms * 1e-3) / 1e9, 1)
        out["roofline"] = hbm
        # Large m is VALU-issue-bound: price the dominant kernel against the VALU
        # peak from its committed SQ_INSTS_VALU count per launch (profiles/sq_<config>.json).
        sq = load_profile(f"sq_{args.config}.json")
        if sq and args.config != "k29m4" and stripes == CONFIGS[args.config][3]:
            names = dec_k if dom == "decode" else enc_k
            base = [n.split("<")[0].split("(")[0] for n in names]   # rocprof names: no template args
            counts = [sq.get("kernels", {}).get(n, {}).get("SQ_INSTS_VALU") for n in base]
            if all(counts):
                insts = float(sum(counts))   # every kernel of the phase, over the phase's event time
                ach = insts / (roof[dom]["ms"] * 1e-3) / 1e9
                out["roofline"] = {"bound": "valu", "kernel": roof[dom]["kernel"], "achieved": round(ach, 1),
                                   "peak": round(VALU_PEAK_GINSTR, 1), "unit": "G wave-instr/s",
                                   "frac": round(ach / VALU_PEAK_GINSTR, 4), "traffic": traffic,
                                   "measured_ceiling": VALU_CEILING_GINSTR,
                                   "frac_of_measured_ceiling": round(ach / VALU_CEILING_GINSTR, 4),
                                   "valu_insts_per_launch": insts, "valu_source": f"profiles/sq_{args.config}.json",
                                   "hbm": hbm}
        out["kernels"] = roof
        if args.config == "k29m4":
            # BASELINE north star: >= 70 % of the HBM-read roofline on the k29/m4 encode
            # (input bytes read per second by the encode kernel / HBM peak).
            enc_in = k * nbytes * stripes / (enc_ms * 1e-3) / 1e9
            out["north_star"] = {"kernel": "+".join(enc_k), "input_read_GBps": round(enc_in, 1),
                                 "frac_of_hbm_peak": round(enc_in / HBM_PEAK_GBS, 4), "target": 0.70,
                                 "frac_of_measured_read_ceiling": round(enc_in / HBM_CEILING_GBS, 4)}
            if stripes == CONFIGS[args.config][3]:
                # the same bytes as a flat 29:4 read:write stream, stores interleaved,
                # non-temporal, one-shot grid (tools/ubench_floor.hip): the calibrated floor
                out["north_star"].update({
                    "measured_floor_ms": FLAT_FLOOR_MS, "floor_source": FLAT_FLOOR_SRC,
                    "frac_of_measured_floor": round(FLAT_FLOOR_MS / enc_ms, 4),
                    "floor_frac_of_hbm_peak": round(k * nbytes * stripes / (FLAT_FLOOR_MS * 1e-3) / 1e9
                                                    / HBM_PEAK_GBS, 4)})
    if not dry and args.ptr == "on":
        out["ptr_tables"] = ptr_leg(lh, k, m, nbytes, X, D, rows0, rec_view, rec_index)
    if not dry and rank == 0 and args.family == "on" and rec_index is None:
        out["reference_order"] = reflayout_leg(lh, k, m, nbytes, X, rows0)
        fam = family_leg(lh, k, m, nbytes, X, D, rows0, rec_view)
        if fam is not None:
            out["family"] = fam
    if not dry and args.pcie == "on":
        # every rank at once: the node's host links and memory are shared
        out["pcie"] = pcie_leg(lh, args, k, m, nbytes, X, D, rows0, rec_view, rec_index, world, rank)
    if args.share_gpu and world > 1:
        out["share_gpu"] = (f"{world} ranks on {torch.cuda.device_count() if not dry else 0} device(s): a functional "
                            "check of the N > 1 control path, not a scaling measurement")
    if rank == 0 and not dry:
        calls = args.dropin_calls if args.dropin_calls >= 0 else max(10, min(2000, int(4e7 / (k * nbytes))))
        if calls:
            out["dropin_per_call"] = dropin_leg(lh, k, m, nbytes, calls)
        if args.cpu_baseline != "off":
            n_cpu = min(stripes, max(64, (256 << 20) // (k * nbytes)), 4096)
            out["cpu_baseline"] = cpu_baseline(k, m, nbytes, args.cpu_seconds, stripes=n_cpu,
                                               patterns=rows0[:n_cpu].cpu().numpy())
            if world > 1:
                out["cpu_baseline"]["note"] = (f"rank 0's host, after the {world}-rank timed region "
                                               "(the other ranks idle)")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
