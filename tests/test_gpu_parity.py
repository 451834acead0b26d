"""GPU parity: the HIP codec (through the C ABI) against the reference's golden fixtures and
the C oracle.  Bit-exact everywhere (integer/byte work).  Run with `-m gpu` on an MI355X."""
import ctypes
import json
import os

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


@pytest.fixture(params=["jit", "generic"])
def path(request, monkeypatch):
    if request.param == "generic":
        monkeypatch.setenv("LONGHAIR_AMD_PATH", "generic")
    else:
        monkeypatch.delenv("LONGHAIR_AMD_PATH", raising=False)
    return request.param


def _load(name):
    return json.load(open(os.path.join(lhutil.GOLDEN, name)))


@pytest.fixture(params=["default", "gpu", "host-avx512bw", "host-avx2", "host-scalar"])
def policy(request, lh, monkeypatch):
    """Drop-in dispatch policy (include/cauchy_256_dispatch.h): every drop-in test runs under
    the library's default policy (AUTO, as an unchanged reference caller), on the GPU and on
    each instruction-set level of the host SIMD engine."""
    if request.param == "default":
        if "LONGHAIR_AMD_DISPATCH" not in os.environ:
            assert lh.dispatch_policy() == "auto"
        prev = lh.dispatch_policy()
    elif request.param == "gpu":
        prev = lh.set_dispatch("gpu")
    else:
        isa = request.param.split("-")[1]
        if isa == "avx512bw" and lh.host_isa() != "avx512bw":
            pytest.skip("host CPU without AVX-512BW")
        monkeypatch.setenv("LONGHAIR_AMD_HOST_ISA", isa)
        prev = lh.set_dispatch("host")
        assert lh.host_isa() == isa
    yield request.param
    lh.set_dispatch(prev)


class DropIn(lhutil._Codec):
    """The product's drop-in entry points driven exactly like the reference (host memory)."""

    def __init__(self, lh):
        lib = lh.lib()
        super().__init__(lib, lib.cauchy_256_encode, lib.cauchy_256_decode)


def _gpu_tensor(arr):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


# ----------------------------------------------------------------- drop-in ABI


def test_dropin_encode_golden_grid(lh, policy):
    codec = DropIn(lh)
    for k, m, bytes_, seed, rc, digest in _load("encode_grid.json")["cases"]:
        data = lhutil.fill(seed, k * bytes_)
        got_rc, rec = codec.encode(k, m, data, bytes_)
        assert got_rc == rc, (k, m, bytes_)
        if rc != 0:
            rec = rec[:bytes_]
        assert lhutil.h64(rec) == digest, (k, m, bytes_)


def test_dropin_encode_full_bytes(lh, policy):
    codec = DropIn(lh)
    for c in _load("encode_full.json"):
        data = np.frombuffer(bytes.fromhex(c["data"]), dtype=np.uint8)
        rc, rec = codec.encode(c["k"], c["m"], data, c["bytes"])
        assert rc == c["rc"]
        assert rec.tobytes().hex() == c["recovery"]


def test_dropin_decode_golden(lh, policy):
    codec = DropIn(lh)
    for c in _load("decode_cases.json"):
        k, m, bytes_ = c["k"], c["m"], c["bytes"]
        data = lhutil.fill(c["seed"], k * bytes_).reshape(k, bytes_)
        rc_e, rec = codec.encode(k, m, data, bytes_)
        assert rc_e == c["rc_encode"], c["tag"]
        rec = rec.reshape(m, bytes_)
        bufs = [(data[x] if kind == "d" else rec[x]).copy() for kind, x in c["slots"]]
        rc, rows = codec.decode(k, m, bufs, list(c["rows_in"]), bytes_)
        assert rc == c["rc"], c["tag"]
        assert rows == c["rows_out"], c["tag"]
        assert [lhutil.h64(b) for b in bufs] == c["digests"], c["tag"]


@pytest.mark.parametrize("k,m,nbytes,cases", [(29, 4, 1296, 40), (29, 1, 1296, 6), (128, 32, 8192, 3),
                                              (200, 56, 65536, 1), (17, 6, 520, 20), (250, 6, 16, 4), (2, 2, 8, 8)])
def test_dropin_random_vs_oracle(lh, oracle, policy, k, m, nbytes, cases):
    """Drop-in encode + decode of random stripes (random e, random recovery rows, shuffled
    slots) against the oracle, on the GPU and on the host engine."""
    codec = DropIn(lh)
    rng = np.random.Generator(np.random.PCG64(k * 1000 + m))
    for c in range(cases):
        data = lhutil.fill(int(rng.integers(0, 2**31)), k * nbytes).reshape(k, nbytes)
        rc, rec = codec.encode(k, m, data, nbytes)
        rc_o, rec_o = oracle.encode(k, m, data, nbytes)
        assert rc == rc_o == 0 and rec.tobytes() == rec_o.tobytes(), (k, m, c)
        rec = rec.reshape(m, nbytes)
        e = int(rng.integers(0, min(k, m) + 1))
        slots, rows = lhutil.erasure_case(int(rng.integers(0, 2**31)), k, m, e)
        bufs = [(data[x] if kind == "d" else rec[x]).copy() for kind, x in slots]
        exp = [b.copy() for b in bufs]
        rc, got_rows = codec.decode(k, m, bufs, rows, nbytes)
        rc_o, exp_rows = oracle.decode(k, m, exp, rows, nbytes)
        assert rc == rc_o and got_rows == exp_rows, (k, m, c, e)
        assert all(a.tobytes() == b.tobytes() for a, b in zip(bufs, exp)), (k, m, c, e)


@pytest.mark.parametrize("k,m,nbytes", [(29, 4, 1296), (128, 32, 8192)])
def test_dropin_concurrent_callers(lh, oracle, k, m, nbytes):
    """Drop-in calls from several threads at once on the GPU (policy GPU): each call takes one
    of the device's independent staging slots (own stream and buffers), so concurrent callers
    are not serialised; every result against the oracle (computed beforehand)."""
    import threading
    codec = DropIn(lh)
    cases = []
    rng = np.random.Generator(np.random.PCG64(k + 7 * m))
    for c in range(24):
        data = lhutil.fill(int(rng.integers(0, 2**31)), k * nbytes).reshape(k, nbytes)
        rc_o, rec_o = oracle.encode(k, m, data, nbytes)
        e = int(rng.integers(1, min(k, m) + 1))
        slots, rows = lhutil.erasure_case(int(rng.integers(0, 2**31)), k, m, e)
        rec = rec_o.reshape(m, nbytes)
        bufs = [(data[x] if kind == "d" else rec[x]).copy() for kind, x in slots]
        exp = [b.copy() for b in bufs]
        rc_d, exp_rows = oracle.decode(k, m, exp, rows, nbytes)
        assert rc_o == rc_d == 0
        cases.append((data, rec_o, bufs, rows, exp, exp_rows))
    errors = []

    def worker(t):
        try:
            for c in range(t, len(cases), 4):
                data, rec_o, bufs, rows, exp, exp_rows = cases[c]
                rc, rec = codec.encode(k, m, data, nbytes)
                assert rc == 0 and rec.tobytes() == rec_o.tobytes(), ("encode", c)
                rc, got_rows = codec.decode(k, m, bufs, rows, nbytes)
                assert rc == 0 and got_rows == exp_rows, ("rows", c)
                assert all(a.tobytes() == b.tobytes() for a, b in zip(bufs, exp)), ("decode", c)
        except Exception as ex:  # noqa: BLE001 -- reported below
            errors.append(ex)

    prev = lh.set_dispatch("gpu")
    try:
        threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=120)
    finally:
        lh.set_dispatch(prev)
    assert not errors, errors


def test_dropin_invalid_rows_untouched(lh, policy):
    """Duplicate or out-of-range rows: -1 and the blocks untouched (documented deviation:
    undefined behaviour in the reference, cauchy_256.cpp:612-614, :733)."""
    codec = DropIn(lh)
    k, m, nbytes = 6, 3, 16
    for rows in ([0, 1, 2, 3, 6, 6], [0, 1, 2, 3, 4, 9]):
        bufs = [lhutil.fill(i, nbytes) for i in range(k)]
        before = [b.copy() for b in bufs]
        rc, got = codec.decode(k, m, bufs, rows, nbytes)
        assert rc == -1 and got == rows
        assert all(a.tobytes() == b.tobytes() for a, b in zip(bufs, before))


def test_dropin_auto_policy_routes_by_size(lh, oracle):
    """AUTO: a small all-host call runs on the host engine (no kernel launched), a large one
    on the GPU (its kernels in the launch trace); both return the oracle's bytes."""
    codec = DropIn(lh)
    prev = lh.set_dispatch("auto", 1 << 20)
    try:
        for k, m, nbytes, on_gpu in ((29, 4, 1296, False), (128, 32, 8192, True)):
            data = lhutil.fill(k + m, k * nbytes)
            rc, rec = codec.encode(k, m, data, nbytes)
            assert rc == 0 and rec.tobytes() == oracle.encode(k, m, data, nbytes)[1].tobytes()
            assert bool(lh.last_launch()) == on_gpu, (k, m, lh.last_launch())
    finally:
        lh.set_dispatch(prev, 4 << 20)


def test_dropin_mixed_pointers(lh):
    """One call with host and device blocks (classified per pointer) gives the
    oracle's bytes under every policy."""
    import torch
    k, m, nbytes = 29, 4, 1296
    data = lhutil.fill(78, k * nbytes)
    ref_rc, ref_rec = lhutil.Oracle().encode(k, m, data, nbytes)
    d = _gpu_tensor(data)
    ptrs = (ctypes.POINTER(ctypes.c_ubyte) * k)()
    for x in range(k):
        addr = (d.data_ptr() if x % 2 else data.ctypes.data) + x * nbytes
        ptrs[x] = ctypes.cast(addr, ctypes.POINTER(ctypes.c_ubyte))
    for pol in ("gpu", "host"):
        prev = lh.set_dispatch(pol)
        try:
            rec = np.zeros(m * nbytes, dtype=np.uint8)
            assert lh.cauchy_256_encode(k, m, ptrs, rec, nbytes) == 0
            assert rec.tobytes() == ref_rec.tobytes()
        finally:
            lh.set_dispatch(prev)
    del torch


@pytest.mark.parametrize("k,m,nbytes,trace", [
    (29, 4, 1296, "lh_jit_encode(pointer table)"), (128, 32, 8192, "lh_jit_encode_win(pointer table)"),
    (200, 3, 64, "lh_apply_jump2_kernel(pointer table)"), (10, 1, 100, "lh_ptr_copy_kernel(gather)"),
    (1, 3, 40, "lh_ptr_copy_kernel(gather)")])
def test_dropin_device_pointers(lh, oracle, k, m, nbytes, trace):
    """Blocks that already live in device memory go through the same entry points: every
    pointer in device memory takes the pointer-table form (one copy of the k + m pointers,
    the blocks read and written where they lie), decode included; the results are the
    oracle's, the rows rewritten as by the reference."""
    import torch
    prev = lh.set_dispatch("gpu")
    try:
        data = lhutil.fill(77 + k, k * nbytes)
        ref_rc, ref_rec = oracle.encode(k, m, data, nbytes)
        pool = torch.zeros((k + m + 3) * (nbytes + 16), dtype=torch.uint8, device="cuda")
        base = pool.data_ptr()
        off = [((i * 7919) % (k + m + 3)) * (nbytes + 16) + (i % 5) for i in range(k + m)]  # scattered, odd offsets
        for x in range(k):
            pool[off[x]:off[x] + nbytes] = torch.from_numpy(data[x * nbytes:(x + 1) * nbytes].copy()).cuda()
        r = torch.zeros(m * nbytes, dtype=torch.uint8, device="cuda")
        ptrs = (ctypes.POINTER(ctypes.c_ubyte) * k)()
        for x in range(k):
            ptrs[x] = ctypes.cast(base + off[x], ctypes.POINTER(ctypes.c_ubyte))
        assert lh.cauchy_256_encode(k, m, ptrs, r.data_ptr(), nbytes) == ref_rc == 0
        assert trace in lh.last_launch(), lh.last_launch()
        assert r.cpu().numpy().tobytes() == ref_rec.tobytes()
        # decode: erase min(k, m) originals, recovery blocks into their own scattered places
        e = min(k, m)
        slots, rows = lhutil.erasure_case(k * 31 + m, k, m, e)
        rec = ref_rec.reshape(m, nbytes)
        blocks = (lh.Block * k)()
        bufs = []
        for i, (kind, x) in enumerate(slots):
            o = off[k + x] if kind == "r" else off[x]
            if kind == "r":
                pool[o:o + nbytes] = torch.from_numpy(rec[x].copy()).cuda()
            blocks[i].data = ctypes.cast(base + o, ctypes.POINTER(ctypes.c_ubyte))
            blocks[i].row = rows[i]
            bufs.append((data[x * nbytes:(x + 1) * nbytes] if kind == "d" else rec[x]).copy())
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows), nbytes)
        assert lh.cauchy_256_decode(k, m, blocks, nbytes) == rc == 0
        assert [blocks[i].row for i in range(k)] == exp_rows
        got = pool.cpu().numpy()
        for i, (kind, x) in enumerate(slots):
            o = off[k + x] if kind == "r" else off[x]
            assert got[o:o + nbytes].tobytes() == bufs[i].tobytes(), i
    finally:
        lh.set_dispatch(prev)


def test_dropin_device_pointers_invalid_size(lh):
    """All-device encode with m > 1 and block_bytes % 8 != 0: recovery block 0 is written and
    -1 returned, as the reference (the pointer-table form's gathered path)."""
    import torch
    k, m, nbytes = 5, 3, 12
    data = torch.randint(0, 256, (k, nbytes), dtype=torch.uint8, device="cuda")
    r = torch.full((m, nbytes), 9, dtype=torch.uint8, device="cuda")
    ptrs = (ctypes.POINTER(ctypes.c_ubyte) * k)()
    for x in range(k):
        ptrs[x] = ctypes.cast(data.data_ptr() + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
    assert lh.cauchy_256_encode(k, m, ptrs, r.data_ptr(), nbytes) == -1
    got = r.cpu().numpy()
    assert (got[0] == np.bitwise_xor.reduce(data.cpu().numpy(), axis=0)).all()
    assert (got[1:] == 9).all()


# ---------------------------------------------------------------- batched API


def _encode_batch_vs_oracle(lh, oracle, k, m, nbytes, stripes, seed):
    import torch
    host = lhutil.fill(seed, stripes * k * nbytes).reshape(stripes, k, nbytes)
    rec = lh.encode_batch(_gpu_tensor(host), m)
    torch.cuda.synchronize()
    got = rec.cpu().numpy()
    for s in range(stripes):
        rc, exp = oracle.encode(k, m, host[s], nbytes)
        assert rc == 0
        assert got[s].tobytes() == exp.tobytes(), (k, m, nbytes, s)
    return host, got


@pytest.mark.parametrize("k,m,nbytes,stripes", [
    (29, 4, 1296, 257), (29, 2, 1296, 64), (29, 3, 1296, 64), (29, 8, 1296, 32), (4, 2, 16, 100),
    (10, 6, 8, 200), (17, 6, 520, 40), (64, 5, 4096, 8), (3, 250, 24, 6), (250, 3, 24, 6),
    (128, 32, 8192, 3), (200, 56, 65536, 1), (2, 2, 8, 1000), (29, 4, 1304, 33), (9, 7, 72, 129),
    # windowed large-m path: one wave (16 rows) per workgroup, two waves (16 + 4), m = 6 (k = 250)
    (100, 16, 2048, 5), (40, 20, 4096, 4), (250, 6, 2048, 3),
])
def test_encode_batch_vs_oracle(lh, oracle, path, k, m, nbytes, stripes):
    _encode_batch_vs_oracle(lh, oracle, k, m, nbytes, stripes, seed=k * 7 + m + nbytes)


def _decode_scenarios(k, m, nbytes, stripes, seed, e=None):
    rng = np.random.Generator(np.random.PCG64(seed))
    slots, rows = [], []
    for s in range(stripes):
        ee = e if e is not None else int(rng.integers(0, min(k, m) + 1))
        sl, rw = lhutil.erasure_case(int(rng.integers(0, 2**31)), k, m, ee)
        slots.append(sl)
        rows.append(rw)
    return slots, rows


@pytest.mark.parametrize("k,m,nbytes,stripes,e", [
    (29, 4, 1296, 300, 4), (29, 4, 1296, 300, None), (29, 2, 16, 100, None), (10, 8, 24, 64, None),
    (17, 6, 520, 40, None), (128, 32, 8192, 3, 32), (128, 32, 1024, 8, None), (200, 56, 65536, 1, 56),
    (5, 3, 8, 200, None), (2, 2, 8, 50, 2), (29, 1, 1296, 50, None), (29, 1, 20, 50, None),
    (1, 3, 16, 10, None),
    # fused wide decode: 2 and 3 waves per workgroup, one wave (m = 6, k = 250), random e
    (100, 16, 2048, 12, None), (40, 20, 4096, 8, None), (250, 6, 2048, 8, None),
])
def test_decode_batch_vs_oracle(lh, oracle, path, k, m, nbytes, stripes, e):
    _decode_batch_vs_oracle(lh, oracle, k, m, nbytes, stripes, e)


def _decode_batch_vs_oracle(lh, oracle, k, m, nbytes, stripes, e):
    import torch
    data = lhutil.fill(k + m + nbytes, stripes * k * nbytes).reshape(stripes, k, nbytes)
    slots, rows = _decode_scenarios(k, m, nbytes, stripes, seed=nbytes + k, e=e)
    blocks = np.zeros((stripes, k, nbytes), dtype=np.uint8)
    recs = []
    for s in range(stripes):
        rc, rec = oracle.encode(k, m, data[s], nbytes)
        rec = rec.reshape(m, nbytes)
        recs.append(rec)
        for i, (kind, x) in enumerate(slots[s]):
            blocks[s, i] = data[s, x] if kind == "d" else rec[x]
    d_blocks = _gpu_tensor(blocks)
    d_rows = _gpu_tensor(np.array(rows, dtype=np.uint8))
    status = lh.decode_batch(d_blocks, d_rows, m)
    torch.cuda.synchronize()
    got_blocks, got_rows, got_status = d_blocks.cpu().numpy(), d_rows.cpu().numpy(), status.cpu().numpy()
    assert (got_status == 0).all()
    for s in range(stripes):
        bufs = [blocks[s, i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows[s]), nbytes)
        assert rc == 0
        assert list(got_rows[s]) == exp_rows, s
        for i in range(k):
            assert got_blocks[s, i].tobytes() == bufs[i].tobytes(), (s, i)


def test_decode_batch_invalid_rows(lh):
    import torch
    k, m, nbytes = 6, 3, 16
    blocks = torch.zeros((2, k, nbytes), dtype=torch.uint8, device="cuda")
    rows = torch.tensor([[0, 1, 2, 3, 4, 4], [0, 1, 2, 3, 4, 9]], dtype=torch.uint8, device="cuda")
    status = lh.decode_batch(blocks, rows, m)
    assert status.cpu().tolist() == [-1, -1]
    assert rows.cpu().tolist() == [[0, 1, 2, 3, 4, 4], [0, 1, 2, 3, 4, 9]]


def test_batch_invalid_params(lh):
    import torch
    x = torch.zeros((2, 200, 16), dtype=torch.uint8, device="cuda")
    with pytest.raises(lh.LonghairError):
        lh.encode_batch(x, 57)
    # Recovery block 0 was still produced, as the reference does before validating.
    y = torch.full((2, 200, 12), 3, dtype=torch.uint8, device="cuda")
    with pytest.raises(lh.LonghairError):
        lh.encode_batch(y, 4)


def test_baseline_scale_roundtrip(lh):
    """BASELINE.json configs[1] at full size: 65536 stripes of k=29, m=4, 1296 B: encode,
    erase 4 random originals per stripe, decode; every stripe must return its data, and a
    sample of stripes must match the oracle byte for byte."""
    import torch
    k, m, nbytes, stripes = 29, 4, 1296, 65536
    g = torch.Generator(device="cuda").manual_seed(1)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    rec = lh.encode_batch(data, m)
    # Per stripe: erase 4 originals (random), keep order of the rest, recovery at the end.
    perm = torch.argsort(torch.rand(stripes, k, device="cuda", generator=g), dim=1)
    keep = perm[:, : k - 4].sort(dim=1).values
    blocks = torch.empty_like(data)
    blocks[:, : k - 4] = torch.gather(data, 1, keep.unsqueeze(-1).expand(-1, -1, nbytes))
    blocks[:, k - 4:] = rec
    rows = torch.cat([keep, torch.arange(k, k + 4, device="cuda").expand(stripes, 4)], dim=1).to(torch.uint8)
    status = lh.decode_batch(blocks, rows, m)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    order = rows.long().argsort(dim=1)
    restored = torch.gather(blocks, 1, order.unsqueeze(-1).expand(-1, -1, nbytes))
    assert torch.equal(restored, data)
    oracle = lhutil.Oracle()
    for s in [0, 1, 2, 4095, 30000, stripes - 1]:
        rc, exp = oracle.encode(k, m, data[s].cpu().numpy(), nbytes)
        assert rec[s].cpu().numpy().tobytes() == exp.tobytes()


# ------------------------------------------------------------- host-batch pipeline


@pytest.mark.parametrize("writeback", ["kernel", "range"])
@pytest.mark.parametrize("k,m,nbytes,stripes,chunk", [(29, 4, 1296, 1000, 96), (17, 6, 520, 77, 0),
                                                      (29, 1, 1296, 50, 8), (128, 32, 8192, 5, 2)])
def test_host_batch_pipeline(lh, oracle, k, m, nbytes, stripes, chunk, writeback, monkeypatch):
    """Pinned-host pipeline against the oracle, with the recovered blocks written back by
    lh_writeback_kernel (default) or by the per-chunk slot-range copy."""
    import torch
    monkeypatch.setenv("LONGHAIR_AMD_PIPE_WRITEBACK", writeback)
    data = lhutil.fill(k * 3 + m, stripes * k * nbytes).reshape(stripes, k, nbytes)
    pinned = torch.from_numpy(data).pin_memory()
    rec = lh.encode_host_batch(pinned.numpy(), m, chunk_stripes=chunk)
    blocks = np.zeros_like(data)
    rows = np.zeros((stripes, k), dtype=np.uint8)
    slots, rws = _decode_scenarios(k, m, nbytes, stripes, seed=k + m)
    for s in range(stripes):
        rc, exp = oracle.encode(k, m, data[s], nbytes)
        assert rec[s].tobytes() == exp.tobytes(), s
        for i, (kind, x) in enumerate(slots[s]):
            blocks[s, i] = data[s, x] if kind == "d" else rec[s, x]
        rows[s] = rws[s]
    exp_blocks, exp_rows = blocks.copy(), rows.copy()
    for s in range(stripes):
        bufs = [exp_blocks[s, i].copy() for i in range(k)]
        rc, r = oracle.decode(k, m, bufs, list(exp_rows[s]), nbytes)
        exp_blocks[s] = np.stack(bufs)
        exp_rows[s] = r
    pb = torch.from_numpy(blocks).pin_memory().numpy()
    pr = torch.from_numpy(rows).pin_memory().numpy()
    status = lh.decode_host_batch(pb, pr, m, chunk_stripes=chunk)
    assert (status == 0).all()
    assert np.array_equal(pr, exp_rows)
    assert np.array_equal(pb, exp_blocks)
    if writeback == "kernel" and m > 1:
        # pageable buffers have no device mapping: the range copy takes over
        blocks2, rows2 = blocks.copy(), rows.copy()
        status = lh.decode_host_batch(blocks2, rows2, m, chunk_stripes=chunk)
        assert (status == 0).all()
        assert np.array_equal(rows2, exp_rows) and np.array_equal(blocks2, exp_blocks)


@pytest.mark.parametrize("offset", [8, 4])
def test_host_batch_unaligned(lh, oracle, offset):
    """Pinned blocks at an 8-byte (write-back kernel, 8-byte lanes) and a 4-byte offset
    (range copy) from a 16-byte boundary."""
    import torch
    k, m, nbytes, stripes = 29, 4, 1296, 40
    data = lhutil.fill(offset + 77, stripes * k * nbytes).reshape(stripes, k, nbytes)
    rec = np.stack([oracle.encode(k, m, data[s], nbytes)[1].reshape(m, nbytes) for s in range(stripes)])
    slots, rws = _decode_scenarios(k, m, nbytes, stripes, seed=offset)
    blocks = np.zeros_like(data)
    for s in range(stripes):
        for i, (kind, x) in enumerate(slots[s]):
            blocks[s, i] = data[s, x] if kind == "d" else rec[s, x]
    rows = np.array(rws, dtype=np.uint8)
    exp_blocks, exp_rows = blocks.copy(), rows.copy()
    for s in range(stripes):
        bufs = [exp_blocks[s, i].copy() for i in range(k)]
        rc, r = oracle.decode(k, m, bufs, list(exp_rows[s]), nbytes)
        exp_blocks[s] = np.stack(bufs)
        exp_rows[s] = r
    raw = torch.empty(blocks.nbytes + 64, dtype=torch.uint8).pin_memory().numpy()
    base = (-raw.ctypes.data) % 16 + offset
    pb = raw[base:base + blocks.nbytes].reshape(blocks.shape)
    assert pb.ctypes.data % 16 == offset
    pb[:] = blocks
    pr = torch.from_numpy(rows).pin_memory().numpy()
    status = lh.decode_host_batch(pb, pr, m, chunk_stripes=16)
    assert (status == 0).all()
    assert np.array_equal(pr, exp_rows)
    assert np.array_equal(pb, exp_blocks)


@pytest.mark.parametrize("writeback", ["kernel", "range"])
def test_host_batch_padded_stride(lh, oracle, monkeypatch, writeback):
    """Pinned stripes with a padded stripe stride through the C ABI: the write-back kernel
    and the range copy honour the stride, and the padding is never written."""
    import torch
    monkeypatch.setenv("LONGHAIR_AMD_PIPE_WRITEBACK", writeback)
    k, m, nbytes, stripes, pad = 17, 6, 520, 30, 72
    stride = k * nbytes + pad
    data = lhutil.fill(pad + 5, stripes * k * nbytes).reshape(stripes, k, nbytes)
    slots, rws = _decode_scenarios(k, m, nbytes, stripes, seed=pad)
    raw = torch.full((stripes * stride,), 0xA5, dtype=torch.uint8).pin_memory().numpy()
    view = raw.reshape(stripes, stride)
    exp = view.copy()
    rows = np.array(rws, dtype=np.uint8)
    exp_rows = rows.copy()
    for s in range(stripes):
        rc, rec = oracle.encode(k, m, data[s], nbytes)
        rec = rec.reshape(m, nbytes)
        blk = np.stack([data[s, x] if kind == "d" else rec[x] for kind, x in slots[s]])
        view[s, :k * nbytes] = blk.reshape(-1)
        bufs = [blk[i].copy() for i in range(k)]
        rc, r = oracle.decode(k, m, bufs, list(exp_rows[s]), nbytes)
        exp[s, :k * nbytes] = np.stack(bufs).reshape(-1)
        exp_rows[s] = r
    pr = torch.from_numpy(rows).pin_memory().numpy()
    status = np.zeros(stripes, dtype=np.int8)
    rc = lh.lib().cauchy_256_decode_host_batch(k, m, nbytes, stripes, raw.ctypes.data, stride, pr.ctypes.data,
                                               status.ctypes.data, 8)
    assert rc == 0 and (status == 0).all()
    assert np.array_equal(pr, exp_rows)
    assert np.array_equal(view, exp)


# ------------------------------------------------------------------- packet framing


@pytest.mark.parametrize("k,m,nbytes,stripes", [(29, 4, 1296, 64), (10, 6, 24, 33), (3, 2, 8, 5)])
def test_frame_unframe_decode(lh, k, m, nbytes, stripes):
    """Encode, frame into [row][block] packets, keep k random packets per stripe in a
    random order, unframe and decode: every stripe returns its data."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(k * m)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    rec = lh.encode_batch(data, m)
    packets = lh.frame_batch(data, rec)
    assert torch.equal(packets[:, :k, 1:], data) and torch.equal(packets[:, k:, 1:], rec)
    assert packets[:, :, 0].cpu().tolist() == [list(range(k + m))] * stripes
    pick = torch.argsort(torch.rand(stripes, k + m, device="cuda", generator=g), dim=1)[:, :k]
    received = torch.gather(packets, 1, pick.unsqueeze(-1).expand(-1, -1, nbytes + 1)).contiguous()
    blocks, rows = lh.unframe_batch(received)
    assert torch.equal(rows, pick.to(torch.uint8))
    status = lh.decode_batch(blocks, rows, m)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    order = rows.long().argsort(dim=1)
    assert torch.equal(torch.gather(blocks, 1, order.unsqueeze(-1).expand(-1, -1, nbytes)), data)


# ------------------------------------------------------------------- hipGraph capture


@pytest.mark.parametrize("k,m,nbytes,stripes", [(29, 4, 1296, 4096), (128, 32, 8192, 64)])
def test_batch_calls_capture_in_a_graph(lh, k, m, nbytes, stripes):
    """The batched calls only enqueue stream-ordered work (no device-wide synchronisation,
    no allocation once the shape is prepared), so an encode + decode step captures into a
    hipGraph (torch.cuda.graph) and replays with the same results."""
    import torch
    lh.prepare(k, m, nbytes, stripes)
    g = torch.Generator(device="cuda").manual_seed(k)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    perm = torch.argsort(torch.rand(stripes, k, device="cuda", generator=g), dim=1)
    keep = perm[:, : k - m]
    blocks = torch.empty_like(data)
    blocks[:, : k - m] = torch.gather(data, 1, keep.unsqueeze(-1).expand(-1, -1, nbytes))
    rows0 = torch.cat([keep, torch.arange(k, k + m, device="cuda").expand(stripes, m)], dim=1).to(torch.uint8)
    rows = rows0.clone()
    status = torch.empty((stripes,), dtype=torch.int8, device="cuda")
    rec_view = blocks[:, k - m:]

    def step():
        lh.encode_batch(data, m, recovery=rec_view)
        rows.copy_(rows0)
        lh.decode_batch(blocks, rows, m, status=status)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # warm-up on the capture stream (workspaces, zero page)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):  # the warmed-up stream: its workspace exists
        step()
    blocks[:, k - m:].zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    order = rows.long().argsort(dim=1)
    assert torch.equal(torch.gather(blocks, 1, order.unsqueeze(-1).expand(-1, -1, nbytes)), data)


def test_huge_stripe_stride_uses_a_safe_path(lh, oracle):
    """The specialised kernels address a wave's stripes through one 32-bit buffer range;
    strides beyond it (here 800 MB between stripes) must take a path without that limit
    and still give the oracle's bytes (encode and in-place decode)."""
    import torch
    k, m, nbytes, stripes, stride = 29, 4, 1296, 4, 800 << 20
    buf = torch.zeros(stride * (stripes - 1) + k * nbytes, dtype=torch.uint8, device="cuda")
    view = torch.as_strided(buf, (stripes, k, nbytes), (stride, nbytes, 1))
    host = lhutil.fill(31, stripes * k * nbytes).reshape(stripes, k, nbytes)
    view.copy_(torch.from_numpy(host))
    rec = lh.encode_batch(view, m)
    torch.cuda.synchronize()
    for s in range(stripes):
        rc, exp = oracle.encode(k, m, host[s], nbytes)
        assert rec[s].cpu().numpy().tobytes() == exp.tobytes(), s
    # decode in place: erase originals 0..3, recovery blocks in their slots
    for s in range(stripes):
        view[s, :m] = rec[s]
    rows = torch.tensor([[k + r for r in range(m)] + list(range(m, k))] * stripes, dtype=torch.uint8, device="cuda")
    status = lh.decode_batch(view, rows, m)
    torch.cuda.synchronize()
    assert (status.cpu() == 0).all()
    assert torch.equal(view.cpu(), torch.from_numpy(host))
    assert rows.cpu().tolist() == [list(range(k))] * stripes
    del buf


@pytest.mark.parametrize("k,m,nbytes,stripes", [
    (128, 32, 1024, 64), (200, 56, 256, 32), (128, 128, 64, 12), (60, 12, 512, 100), (9, 200, 64, 40),
    (128, 32, 8192, 16),  # wide decode (precompiled module)
])
def test_planner_closed_form_matches_elimination(lh, oracle, monkeypatch, k, m, nbytes, stripes):
    """The decode planner inverts e x e Cauchy submatrices in closed form (every m >= 7);
    LONGHAIR_AMD_PLAN_GJ forces the Gauss-Jordan elimination it replaced.  Both must give
    the oracle's bytes and rows, at random erasure counts up to e = min(k, m) (here up to
    128: two rows per lane), through the wide decode and the generic path (m > 64)."""
    import torch
    data = lhutil.fill(k * 7 + m, stripes * k * nbytes).reshape(stripes, k, nbytes)
    slots, rows = _decode_scenarios(k, m, nbytes, stripes, seed=k * m)
    blocks = np.zeros((stripes, k, nbytes), dtype=np.uint8)
    for s in range(stripes):
        rec = oracle.encode(k, m, data[s], nbytes)[1].reshape(m, nbytes)
        for i, (kind, x) in enumerate(slots[s]):
            blocks[s, i] = data[s, x] if kind == "d" else rec[x]
    outs = []
    for gj in (False, True):
        if gj:
            monkeypatch.setenv("LONGHAIR_AMD_PLAN_GJ", "1")
        d_blocks = _gpu_tensor(blocks)
        d_rows = _gpu_tensor(np.array(rows, dtype=np.uint8))
        status = lh.decode_batch(d_blocks, d_rows, m)
        torch.cuda.synchronize()
        assert (status.cpu() == 0).all()
        outs.append((d_blocks.cpu().numpy(), d_rows.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    for s in range(min(stripes, 8)):
        bufs = [blocks[s, i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows[s]), nbytes)
        assert rc == 0 and list(outs[0][1][s]) == exp_rows
        assert all(outs[0][0][s, i].tobytes() == bufs[i].tobytes() for i in range(k)), s


# Every knob of INTEGRATION.md section 6 that selects other kernel code has a parity test.
# These cover the separate planner of the e_max <= 4 decode and the JIT_DEFINES tuning hook
# (tools/precompile.py KNOB_JOBS compiles the variant modules at build time).
KNOB_VARIANTS = [
    ("nofused", {"LONGHAIR_AMD_NO_FUSED_PLAN": "1"}, ["lh_plan_small_kernel<4>", "lh_jit_decode"]),
    # the register-ring forms (LH_LDS=0: every shape the LDS staging does not take, jit.cpp)
    ("defines-lds0-pf2-nt0-noxcd", {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDS=0,LH_PF=2,LH_NT=0,LH_XCD=0"},
     ["lh_jit_decode_fused"]),
    ("defines-lds0-recfirst0-pfdec2", {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDS=0,LH_REC_FIRST=0,LH_PF_DEC=2"},
     ["lh_jit_decode_fused"]),
    # the LDS-staged forms' other ring depth, cache policy, column order and direct stores
    ("defines-ld2-nt0-ldsrecfirst-direct", {"LONGHAIR_AMD_JIT_DEFINES": "LH_LD=2,LH_NT=0,LH_LDS_NT_DEC=0,LH_LDS_REC_FIRST=1,LH_LDS_FLAT_ST=0"},
     ["lh_jit_decode_fused"]),
    # the decode ring refilled one and three slots at a time (default two, LH_LDG)
    ("defines-ldg1", {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDG=1"}, ["lh_jit_decode_fused"]),
    ("defines-ldg3", {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDG=3"}, ["lh_jit_decode_fused"]),
    # DMAs from asm (no compiler drain: the rings really run LH_LD - 1 columns deep, counted waits)
    ("defines-asm-dma", {"LONGHAIR_AMD_JIT_DEFINES": "LH_ASM_DMA=1"}, ["lh_jit_decode_fused"]),
    # the encode's one-column ring (LH_CPS=1; the pointer-table encode's form) and other
    # multi-column-step shapes: 3 columns (partial last step), 2-wave workgroups, two slots,
    # slot-image stores
    ("defines-cps1", {"LONGHAIR_AMD_JIT_DEFINES": "LH_CPS=1"}, ["lh_jit_decode_fused"]),
    ("defines-cps3-wpb2-ahead-flat", {"LONGHAIR_AMD_JIT_DEFINES": "LH_CPS=3,LH_WPB=2,LH_WGCU=2,LH_CPS_AHEAD=1,LH_CPS_FLAT=1"},
     ["lh_jit_decode_fused"]),
    # the decode's memory-order form (slots read in multi-slot steps, each slot's network picked
    # by its run-time row), with two step slots and with one (3 slots per step: partial last step)
    ("defines-dmo", {"LONGHAIR_AMD_JIT_DEFINES": "LH_DMO=1"}, ["lh_jit_decode_fused"]),
    ("defines-dmo-noahead-cps3", {"LONGHAIR_AMD_JIT_DEFINES": "LH_DMO=1,LH_DMO_AHEAD=0,LH_CPS=3"},
     ["lh_jit_decode_fused"]),
]


@pytest.mark.parametrize("name,env,dec_trace", KNOB_VARIANTS, ids=[v[0] for v in KNOB_VARIANTS])
def test_kernel_knob_variants(lh, oracle, monkeypatch, name, env, dec_trace):
    """k29/m4/1296 encode + decode through each knob's kernels, bytes and rewritten rows
    against the oracle (random e per stripe, the first at e = 4, shuffled slots)."""
    import test_gpu_boundaries as tb
    for key, v in env.items():
        monkeypatch.setenv(key, v)
    enc, dec = tb.roundtrip(lh, oracle, 29, 4, 1296, 96, seed=sum(map(ord, name)))
    assert enc == ["lh_jit_encode"], enc
    assert dec == dec_trace, dec
