"""N > 1 path on CPU: world_size-2 gloo groups exercise the sharding and the
max-over-ranks aggregation bench.py uses; each rank codes its stripe shard with the
oracle (no GPU here) and the union must equal the single-process result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import lhutil
from longhair_amd.shard import aggregate_rate, max_over_ranks, shard_range


def test_shard_range_partitions():
    for total in (0, 1, 7, 65536, 524288, 1000003):
        for world in (1, 2, 3, 4, 8):
            ranges = [shard_range(total, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k, m, nbytes = 29, 4, 48
    oracle = lhutil.Oracle()
    lo, hi = shard_range(total, world, rank)
    data = lhutil.fill(11, total * k * nbytes).reshape(total, k, nbytes)
    digests = {}
    for s in range(lo, hi):
        rc, rec = oracle.encode(k, m, data[s], nbytes)
        assert rc == 0
        digests[s] = lhutil.h64(rec)
    elapsed = 0.5 + rank  # deterministic stand-in for a rank's timed region
    slowest = max_over_ranks(elapsed)
    rate = aggregate_rate((hi - lo) * k * nbytes, elapsed)
    gathered = [None] * world
    dist.all_gather_object(gathered, digests)
    dist.destroy_process_group()
    q.put((rank, slowest, rate, gathered))


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_encode_matches_single_process(world):
    total = 37
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    oracle = lhutil.Oracle()
    k, m, nbytes = 29, 4, 48
    data = lhutil.fill(11, total * k * nbytes).reshape(total, k, nbytes)
    expect = {s: lhutil.h64(oracle.encode(k, m, data[s], nbytes)[1]) for s in range(total)}
    for rank, slowest, rate, gathered in results:
        assert slowest == 0.5 + (world - 1)
        assert abs(rate - total * k * nbytes / slowest) < 1e-6
        merged = {}
        for d in gathered:
            assert not (set(d) & set(merged))   # shards are disjoint
            merged.update(d)
        assert merged == expect


def _bench(*argv, env=None):
    import json
    import subprocess
    import sys
    e = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(v, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(lhutil.REPO, "bench.py"), *argv], capture_output=True,
                       text=True, timeout=300, env=e, cwd=lhutil.REPO)
    return r, (json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else None)


def test_bench_launcher_weak_world2():
    """`bench.py --gpus 2` starts torch.distributed.run with two ranks itself (dry run: gloo,
    CPU stand-in step) and reports the whole-job rate over both ranks."""
    r, line = _bench("--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["dry_run"]
    assert len(line["per_gpu_GBps"]) == 2
    assert line["config"]["global_stripes"] == 2 * 65536
    # value = all ranks' bytes / slowest rank's time
    per_step = 2 * 29 * 1296 * 65536 * 2 * 3 / 1e9
    assert abs(line["value"] - per_step / (line["ms_per_step"] * 3 / 1e3)) / line["value"] < 0.01


def test_bench_launcher_strong_world2():
    r, line = _bench("--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "0", "--global-stripes", "1001")
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["global_stripes"] == 1001 and line["config"]["stripes_per_gpu"] is None


def test_bench_rejects_world_mismatch():
    """Under a torchrun environment the world size must equal --gpus."""
    r, _ = _bench("--gpus", "2", "--dry-run", "--steps", "1", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_cpu_baseline_uses_the_workload_patterns():
    """bench.py's cpu_baseline decodes the GPU workload's own erasure patterns (per-stripe e
    and recovery rows from the Block.row bytes), so its sample states the same mean e."""
    import numpy as np
    import bench
    if not os.path.exists(os.path.join(lhutil.REPO, "oracle", "liblh_cpubench.so")):
        pytest.skip("oracle/liblh_cpubench.so not built")
    k, m, nbytes = 12, 5, 64
    rng = np.random.Generator(np.random.PCG64(3))
    rows = []
    for s in range(10):
        e = int(rng.integers(1, m + 1))
        keep = rng.permutation(k)[: k - e]
        rr = rng.permutation(m)[:e]
        rows.append(np.concatenate([keep, k + rr]))
    rows = np.array(rows, dtype=np.uint8)
    erased, e_of, rec, e_max = bench.erasure_patterns(rows, k)
    assert list(e_of) == [int((r >= k).sum()) for r in rows]
    for s in range(10):
        assert set(erased[s, : e_of[s]]) == set(range(k)) - set(rows[s][rows[s] < k].tolist())
        assert sorted(rec[s, : e_of[s]] + k) == sorted(rows[s][rows[s] >= k].tolist())
    out = bench.cpu_baseline(k, m, nbytes, 0.3, stripes=10, patterns=rows)
    assert out["ok"], out
    assert f"mean e {e_of.mean():.1f}" in out["sample"]


@pytest.mark.parametrize("k,m,nbytes,align", [(29, 4, 1296, 128), (29, 4, 1296, 64), (17, 6, 520, 128),
                                              (128, 32, 8192, 128), (29, 4, 1296, 0)])
def test_bench_aligned_decode_buffer_layout(k, m, nbytes, align):
    """bench.py --align: every stripe's recovery slots start on an `align`-byte boundary, the
    stripe stride holds the k slots and is a multiple of `align`, the padding stays small."""
    import bench
    off, stride = bench.aligned_layout(k, m, nbytes, align)
    assert stride >= k * nbytes and off >= 0
    if not align:
        assert (off, stride) == (0, k * nbytes)
        return
    assert stride % align == 0 and stride - k * nbytes < align and off < align
    for s in range(5):
        assert (off + s * stride + (k - m) * nbytes) % align == 0


def test_per_call_timing_takes_the_best_round():
    """bench.per_call_us: `calls` calls per engine in `rounds` rounds; encode_us / decode_us
    are the best round's mean (one preempted round must not decide the comparison with the
    reference, which the same function times), *_mean_us the overall mean."""
    import time

    import numpy as np

    import bench
    state = {"n": 0}

    def slow_first_round(*_):
        state["n"] += 1
        if 6 <= state["n"] <= 15:  # the first timed round (after 5 warm-up calls)
            time.sleep(0.002)
        return 0

    out = bench.per_call_us(slow_first_round, lambda *_: 0, 4, 2, 16, 50, np.zeros(64, dtype=np.uint8),
                            lambda i, rec: None)
    assert out["calls"] == 50 and out["rounds"] == 5
    assert out["encode_us"] < 100 and out["encode_mean_us"] > 300  # one round of 10 x 2 ms in 50 calls
    assert out["decode_us"] <= out["decode_mean_us"]


class _StandInCodec:
    """Host-batch entry points of longhair_amd with the same argument shapes: encode is a
    no-op, decode puts each stripe's missing originals into its recovery slots (it is handed
    the originals -- the control path under test does not look at how they were recovered).
    Rank r sleeps r * 10 ms per call, so the slowest rank is known."""

    def __init__(self, X, k, delay):
        self.X, self.k, self.delay = X, k, delay

    def encode_host_batch(self, xn, m, recovery=None):
        import time
        time.sleep(self.delay)

    def decode_host_batch(self, bn, rn, m):
        import time
        time.sleep(self.delay)
        k = self.k
        for s in range(bn.shape[0]):
            missing = sorted(set(range(k)) - set(int(r) for r in rn[s] if r < k))
            for j in [j for j in range(k) if rn[s, j] >= k]:
                x = missing.pop(0)
                bn[s, j] = self.X[s, x]
                rn[s, j] = x


def _pcie_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    k, m, nbytes, n = 6, 3, 65536, 40   # 15.7 MB per rank: rates of a few GB/s at 10-20 ms
    X = lhutil.fill(40 + rank, n * k * nbytes).reshape(n, k, nbytes)
    rows = np.array([[3, 4, 5, 6, 7, 8]] * n, dtype=np.uint8)   # originals 0..2 erased
    slots = X.copy()
    slots[:, :3] = X[:, 3:]
    slots[:, 3:] = 0
    rows[:, :3] = [3, 4, 5]
    rows[:, 3:] = [k, k + 1, k + 2]
    b0, r0 = slots.copy(), rows.copy()
    out = bench.pcie_timed(_StandInCodec(X, k, 0.01 + 0.02 * rank), k, m, nbytes, X, slots, rows,
                           np.zeros((n, m, nbytes), dtype=np.uint8), b0, r0, world, rank, reps=2, dry=True)
    dist.destroy_process_group()
    q.put((rank, out))


def test_pcie_leg_aggregation_world2():
    """bench.pcie_timed (the timed half of the PCIe-inclusive leg) at world 2 on gloo: both
    ranks make the same cross-rank calls, every rank gets both ranks' rates, the node rate is
    all input bytes over the slowest rank's time, and `ok` is the AND over ranks."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pcie_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = results[0], results[1]
    for out in (a, b):
        assert out["ok"] is True
        assert len(out["encode_GBps_per_rank"]) == 2 and len(out["decode_GBps_per_rank"]) == 2
        # rank 1 sleeps 30 ms per call against rank 0's 10: it is the slower one, and the node
        # rate is both ranks' bytes over its time
        assert out["encode_GBps_per_rank"][1] < out["encode_GBps_per_rank"][0]
        assert out["decode_GBps_per_rank"][1] < out["decode_GBps_per_rank"][0]
        assert abs(out["node_encode_GBps"] - 2 * out["encode_GBps_per_rank"][1]) <= 0.02
        assert abs(out["node_decode_GBps"] - 2 * out["decode_GBps_per_rank"][1]) <= 0.02
    assert a["encode_GBps_per_rank"] == b["encode_GBps_per_rank"]
    assert a["node_decode_GBps"] == b["node_decode_GBps"]
