"""GPU parity at the BASELINE.json configurations in their stated form (configs[2], [3],
[4]) and at the fused-decode edge shapes with 64 lanes per stripe.  The HIP codec runs
through the C ABI; the C oracle (pinned to the reference, tests/test_oracle.py) checks
every stripe byte for byte and row for row.  Bit-exact.  Run with `-m gpu` on an MI355X.

Reference semantics: sort_blocks (cauchy_256.cpp:538-570) -- recovery slots in array order
take the missing original rows ascending (generate_bitmatrix, :786)."""
import numpy as np
import pytest

import lhutil

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lh():
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import longhair_amd
    assert longhair_amd.cauchy_256_init() == 0
    return longhair_amd


def _random_e_cases(k, m, stripes, seed):
    """Per stripe: e uniform in [1, min(k, m)], e random erased originals, e random
    recovery rows, shuffled slot order (as bench.py's 'random' workload)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for _ in range(stripes):
        e = int(rng.integers(1, min(k, m) + 1))
        out.append(lhutil.erasure_case(int(rng.integers(0, 2**31)), k, m, e))
    return out


def _received(data, rec, cases):
    """blocks [S, k, B] and rows [S, k] as the receiver holds them."""
    stripes, k, nbytes = data.shape
    blocks = np.empty_like(data)
    rows = np.empty((stripes, k), dtype=np.uint8)
    for s, (slots, rws) in enumerate(cases):
        for i, (kind, x) in enumerate(slots):
            blocks[s, i] = data[s, x] if kind == "d" else rec[s, x]
        rows[s] = rws
    return blocks, rows


def _oracle_decode_all(oracle, k, m, nbytes, blocks, rows):
    exp_b, exp_r = blocks.copy(), rows.copy()
    for s in range(blocks.shape[0]):
        bufs = [exp_b[s, i].copy() for i in range(k)]
        rc, r = oracle.decode(k, m, bufs, list(exp_r[s]), nbytes)
        assert rc == 0
        exp_b[s] = np.stack(bufs)
        exp_r[s] = r
    return exp_b, exp_r


def _device_and_host_decode(lh, k, m, blocks, rows, exp_b, exp_r, chunk=0):
    import torch
    # device-resident batch decode
    d_blocks = torch.from_numpy(blocks).cuda()
    d_rows = torch.from_numpy(rows).cuda()
    status = lh.decode_batch(d_blocks, d_rows, m)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert np.array_equal(d_rows.cpu().numpy(), exp_r)
    got = d_blocks.cpu().numpy()
    for s in range(blocks.shape[0]):
        assert np.array_equal(got[s], exp_b[s]), f"decode_batch stripe {s}"
    del d_blocks
    # pinned host buffers through the overlapped H2D / decode / D2H pipeline
    pb = torch.from_numpy(blocks.copy()).pin_memory()
    pr = torch.from_numpy(rows.copy()).pin_memory()
    status = lh.decode_host_batch(pb.numpy(), pr.numpy(), m, chunk_stripes=chunk)
    assert (status == 0).all()
    assert np.array_equal(pr.numpy(), exp_r)
    hb = pb.numpy()
    for s in range(blocks.shape[0]):
        assert np.array_equal(hb[s], exp_b[s]), f"decode_host_batch stripe {s}"


def test_config4_k200_m56_random_erasures(lh, oracle):
    """BASELINE configs[4]: k=200, m=56, 65536-byte blocks, random e in [1, 56], random
    recovery rows, shuffled slots; decode_batch and the pinned decode_host_batch (two
    stripes per chunk, so the three-stream ring turns over) against the oracle."""
    k, m, nbytes, stripes = 200, 56, 65536, 16
    data = lhutil.fill(4004, stripes * k * nbytes).reshape(stripes, k, nbytes)
    import torch
    rec = lh.encode_batch(torch.from_numpy(data).cuda(), m).cpu().numpy()
    for s in (0, stripes - 1):  # encode spot check (full encode parity: test_gpu_parity.py)
        rc, exp = oracle.encode(k, m, data[s], nbytes)
        assert rc == 0 and rec[s].tobytes() == exp.tobytes()
    cases = _random_e_cases(k, m, stripes, seed=44)
    es = [sum(1 for kind, _ in sl if kind == "r") for sl, _ in cases]
    assert max(es) > 4 and min(es) < max(es)  # a real mix, past the fused e <= 4 path
    blocks, rows = _received(data, rec, cases)
    exp_b, exp_r = _oracle_decode_all(oracle, k, m, nbytes, blocks, rows)
    _device_and_host_decode(lh, k, m, blocks, rows, exp_b, exp_r, chunk=2)
    # the decode restores the data (the oracle agrees with it, checked above)
    order = np.argsort(exp_r, axis=1)
    assert np.array_equal(np.take_along_axis(exp_b, order[:, :, None], axis=1), data)


def test_config2_k128_m32_random_erasures(lh, oracle):
    """BASELINE configs[2] shape: k=128, m=32, 8192-byte blocks, 32 stripes with random e
    in [1, 32] (the multi-stripe planner path), device and pinned host decode."""
    import torch
    k, m, nbytes, stripes = 128, 32, 8192, 32
    data = lhutil.fill(2002, stripes * k * nbytes).reshape(stripes, k, nbytes)
    rec = lh.encode_batch(torch.from_numpy(data).cuda(), m).cpu().numpy()
    for s in range(stripes):
        rc, exp = oracle.encode(k, m, data[s], nbytes)
        assert rc == 0 and rec[s].tobytes() == exp.tobytes(), s
    cases = _random_e_cases(k, m, stripes, seed=22)
    blocks, rows = _received(data, rec, cases)
    exp_b, exp_r = _oracle_decode_all(oracle, k, m, nbytes, blocks, rows)
    _device_and_host_decode(lh, k, m, blocks, rows, exp_b, exp_r, chunk=5)


def test_config2_full_batch_roundtrip(lh, oracle):
    """configs[2] at full size (8192 stripes, e = 32): encode -> erase -> decode restores
    every stripe; oracle spot checks on encode and decode."""
    import torch
    k, m, nbytes, stripes = 128, 32, 8192, 8192
    g = torch.Generator(device="cuda").manual_seed(3)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    rec = lh.encode_batch(data, m)
    perm = torch.argsort(torch.rand(stripes, k, device="cuda", generator=g), dim=1)
    keep = perm[:, : k - m]
    blocks = torch.empty_like(data)
    blocks[:, : k - m] = torch.gather(data, 1, keep.unsqueeze(-1).expand(-1, -1, nbytes))
    blocks[:, k - m:] = rec
    rows = torch.cat([keep, torch.arange(k, k + m, device="cuda").expand(stripes, m)], dim=1).to(torch.uint8)
    spots = [0, 1, 4097, stripes - 1]
    before = {s: (blocks[s].cpu().numpy().copy(), rows[s].cpu().numpy().copy()) for s in spots}
    status = lh.decode_batch(blocks, rows, m)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    order = rows.long().argsort(dim=1)
    assert torch.equal(torch.gather(blocks, 1, order.unsqueeze(-1).expand(-1, -1, nbytes)), data)
    for s in spots:
        rc, exp = oracle.encode(k, m, data[s].cpu().numpy(), nbytes)
        assert rec[s].cpu().numpy().tobytes() == exp.tobytes()
        b0, r0 = before[s]
        bufs = [b0[i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, m, bufs, list(r0), nbytes)
        assert rc == 0 and list(rows[s].cpu().numpy()) == exp_rows
        assert blocks[s].cpu().numpy().tobytes() == np.stack(bufs).tobytes()


def test_config3_eight_shards_equal_one_launch(lh, oracle):
    """BASELINE configs[3]: 524288 stripes of k=29, m=4, 1296 B split evenly across 8
    ranks with shard_range.  The 8 shards run one after another on this GPU (what each
    rank of `bench.py --gpus 8 --global-stripes 524288` codes); their union must equal
    one unsharded launch, every shard's decode must restore its data, and oracle spot
    checks pin a stripe of every shard."""
    import torch
    from longhair_amd.shard import shard_range
    k, m, nbytes, total, world = 29, 4, 1296, 524288, 8
    g = torch.Generator(device="cuda").manual_seed(8)
    data = torch.randint(0, 256, (total, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    full = lh.encode_batch(data, m)
    sharded = torch.empty_like(full)
    for r in range(world):
        lo, hi = shard_range(total, world, r)
        assert hi - lo == total // world
        lh.encode_batch(data[lo:hi], m, recovery=sharded[lo:hi])
    torch.cuda.synchronize()
    assert torch.equal(full, sharded)
    del sharded
    for r in range(world):
        lo, hi = shard_range(total, world, r)
        n = hi - lo
        perm = torch.argsort(torch.rand(n, k, device="cuda", generator=g), dim=1)
        keep = perm[:, : k - m]
        blocks = torch.empty((n, k, nbytes), dtype=torch.uint8, device="cuda")
        blocks[:, : k - m] = torch.gather(data[lo:hi], 1, keep.unsqueeze(-1).expand(-1, -1, nbytes))
        blocks[:, k - m:] = full[lo:hi]
        rows = torch.cat([keep, torch.arange(k, k + m, device="cuda").expand(n, m)], dim=1).to(torch.uint8)
        status = lh.decode_batch(blocks, rows, m)
        torch.cuda.synchronize()
        assert int((status != 0).sum()) == 0, r
        order = rows.long().argsort(dim=1)
        assert torch.equal(torch.gather(blocks, 1, order.unsqueeze(-1).expand(-1, -1, nbytes)), data[lo:hi]), r
        s = lo + (r * 7919) % n
        rc, exp = oracle.encode(k, m, data[s].cpu().numpy(), nbytes)
        assert rc == 0 and full[s].cpu().numpy().tobytes() == exp.tobytes(), r
        del blocks, rows


@pytest.mark.parametrize("k,m,nbytes", [(64, 4, 4096), (64, 3, 4096), (64, 2, 8192)])
def test_fused_decode_64_lane_stripes(lh, oracle, k, m, nbytes):
    """Fused decode shapes whose stripe spans all 64 lanes of a wave (k = 64): original
    row 63 erased and a recovery block in slot 63 (the lane the planner's ballot masks
    must keep), plus random cases."""
    import torch
    assert lh.batch_path(k, m, nbytes, decode=True) == "jit-fused"
    stripes = 24
    data = lhutil.fill(k * m, stripes * k * nbytes).reshape(stripes, k, nbytes)
    rec = lh.encode_batch(torch.from_numpy(data).cuda(), m).cpu().numpy()
    rng = np.random.Generator(np.random.PCG64(k + m))
    cases = []
    for s in range(stripes):
        e = m if s < stripes // 2 else int(rng.integers(1, m + 1))
        erased = sorted({63} | set(rng.choice(63, size=e - 1, replace=False).tolist()))
        rrows = sorted(rng.choice(m, size=e, replace=False).tolist())
        slots = [("d", x) for x in range(k) if x not in erased]
        rng.shuffle(slots)
        rslots = [("r", j) for j in rrows]
        # one recovery block in slot 63, the others spread over the array
        slots = slots + rslots[:-1]
        for i, sl in enumerate(rslots[:-1]):
            pos = int(rng.integers(0, len(slots)))
            slots.remove(sl)
            slots.insert(pos, sl)
        slots.append(rslots[-1])
        assert len(slots) == k and slots[63][0] == "r"
        cases.append((slots, [x if kind == "d" else k + x for kind, x in slots]))
    blocks, rows = _received(data, rec, cases)
    exp_b, exp_r = _oracle_decode_all(oracle, k, m, nbytes, blocks, rows)
    d_blocks = torch.from_numpy(blocks).cuda()
    d_rows = torch.from_numpy(rows).cuda()
    status = lh.decode_batch(d_blocks, d_rows, m)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert np.array_equal(d_rows.cpu().numpy(), exp_r)
    assert np.array_equal(d_blocks.cpu().numpy(), exp_b)
    # duplicate row in slot 63 -> invalid, untouched
    bad = rows.copy()
    bad[:, 63] = bad[:, 0]
    d_blocks = torch.from_numpy(blocks).cuda()
    d_rows = torch.from_numpy(bad).cuda()
    status = lh.decode_batch(d_blocks, d_rows, m)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == -1).all()
    assert np.array_equal(d_rows.cpu().numpy(), bad)
    assert np.array_equal(d_blocks.cpu().numpy(), blocks)
