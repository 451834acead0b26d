"""GPU parity of the pointer-table batch calls (include/cauchy_256_batch.h
cauchy_256_encode_batch_ptrs / cauchy_256_decode_batch_ptrs): the reference's per-block
pointers (cauchy_256.h:78 data_ptrs[], :103 Block.data) for a batch of stripes.

Every block is placed at a random position of a shared pool, at a random byte offset (odd
addresses included), so no two blocks of a stripe are adjacent or in order.  Results must be
bit-identical to the strided batch calls on the same inputs (those are checked against the
oracle in test_gpu_parity.py) and, on a sample of stripes, to the C oracle directly.  The
launch trace shows which form ran: the specialised kernels reading the blocks in place
("(pointer table)": the register networks, the windowed large-m kernels with the phase-B
kernel, and for shapes without a specialised module the generic jump apply) or the gather /
strided / scatter form (m = 1, k = 1, sub-blocks under 4 bytes, the lone-last-lane decode)."""
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


def _scatter(blocks, seed, max_off=15):
    """blocks: uint8 CUDA tensor [S, n, B].  Copies every block to a random place of a pool
    (random order, random byte offset 0..max_off); returns (pool, ptrs [S, n] int64, place)
    where place locates the blocks again (_gather)."""
    import torch
    S, n, B = blocks.shape
    rng = np.random.Generator(np.random.PCG64(seed))
    stride = B + max_off + 1
    order = rng.permutation(S * n)
    offs = rng.integers(0, max_off + 1, size=S * n)
    pool = torch.full((S * n * stride + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    p2 = pool[: S * n * stride].view(S * n, stride)
    flat = blocks.reshape(S * n, B)
    for o in np.unique(offs):
        sel = np.nonzero(offs == o)[0]
        p2[torch.from_numpy(order[sel]).cuda(), int(o):int(o) + B] = flat[torch.from_numpy(sel).cuda()]
    ptrs = torch.from_numpy((order * stride + offs).reshape(S, n).astype(np.int64) + pool.data_ptr()).cuda()
    return pool, ptrs, (S, n, B, stride, order, offs)


def _gather(pool, place):
    import torch
    S, n, B, stride, order, offs = place
    p2 = pool[: S * n * stride].view(S * n, stride)
    out = torch.empty((S * n, B), dtype=torch.uint8, device="cuda")
    for o in np.unique(offs):
        sel = np.nonzero(offs == o)[0]
        out[torch.from_numpy(sel).cuda()] = p2[torch.from_numpy(order[sel]).cuda(), int(o):int(o) + B]
    return out.reshape(S, n, B)


ENCODE = [
    # (k, m, bytes, stripes, form)
    (29, 4, 1296, 300, "lh_jit_encode(pointer table)"),
    (29, 8, 1296, 70, "lh_jit_encode(pointer table)"),
    (10, 6, 24, 130, "lh_jit_encode(pointer table)"),
    (64, 5, 4096, 9, "lh_jit_encode(pointer table)"),
    (128, 32, 8192, 3, "lh_jit_encode_win(pointer table)"),   # windowed large-m encode
    (40, 20, 4096, 6, "lh_jit_encode_win(pointer table)"),
    (200, 56, 65536, 2, "lh_jit_encode_win(pointer table)"),
    (40, 20, 1024, 5, "lh_apply_jump_kernel(pointer table)"),   # large m, sub % 256 != 0: generic, in place
    (200, 3, 64, 5, "lh_apply_jump2_kernel(pointer table)"),     # k > 128: generic, two-dword lanes (m <= 4)
    (40, 20, 24, 5, "lh_ptr_copy_kernel(gather)"),               # sub < 4: the bytewise generic kernel, gathered
    (10, 1, 100, 7, "lh_ptr_copy_kernel(gather)"),      # m = 1, any block size
    (1, 3, 40, 5, "lh_ptr_copy_kernel(gather)"),        # k = 1 copies
]


@pytest.mark.parametrize("k,m,nbytes,stripes,form", ENCODE)
def test_encode_batch_ptrs(lh, oracle, k, m, nbytes, stripes, form):
    import torch
    g = torch.Generator(device="cuda").manual_seed(k * 1000 + m)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    want = lh.encode_batch(data, m)
    dpool, dptr, _ = _scatter(data, seed=k + m)
    rpool, rptr, rplace = _scatter(torch.zeros((stripes, m, nbytes), dtype=torch.uint8, device="cuda"),
                                   seed=k * m + 1)
    lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr)
    torch.cuda.synchronize()
    assert form in lh.last_launch(), lh.last_launch()
    got = _gather(rpool, rplace)
    assert torch.equal(got, want)
    host = data.cpu().numpy()
    for s in (0, stripes - 1):
        rc, rec = oracle.encode(k, m, host[s], nbytes)
        assert rc == 0
        assert got[s].cpu().numpy().tobytes() == rec.tobytes(), s


def test_encode_batch_ptrs_invalid_writes_block0(lh):
    """m > 1 with bytes % 8 != 0: recovery block 0 is still written (the XOR of the data),
    the other recovery blocks are left alone, and the call fails, as the reference."""
    import torch
    k, m, nbytes, stripes = 5, 3, 12, 4
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda")
    dpool, dptr, _ = _scatter(data, seed=3)
    rpool, rptr, rplace = _scatter(torch.full((stripes, m, nbytes), 7, dtype=torch.uint8, device="cuda"), seed=4)
    with pytest.raises(lh.LonghairError):
        lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr)
    torch.cuda.synchronize()
    got = _gather(rpool, rplace).cpu().numpy()
    x = np.bitwise_xor.reduce(data.cpu().numpy(), axis=1)
    assert (got[:, 0] == x).all()
    assert (got[:, 1:] == 7).all()


DECODE = [
    (29, 4, 1296, 300, "lh_jit_decode_fused(pointer table)"),
    (29, 8, 1296, 70, "lh_jit_decode(pointer table)"),
    (10, 6, 24, 130, "lh_jit_decode(pointer table)"),
    (64, 3, 4096, 9, "lh_jit_decode_fused(pointer table)"),
    (128, 32, 8192, 3, "lh_jit_decode_wide(pointer table)"),  # planner, phase A and phase B through the table
    (40, 20, 4096, 6, "lh_jit_decode_wide(pointer table)"),
    (200, 56, 65536, 3, "lh_jit_decode_wide(pointer table)"),
    (40, 20, 1024, 5, "lh_apply_jump_kernel(pointer table)"),
    (200, 3, 64, 5, "lh_apply_jump_kernel(pointer table)"),
    (40, 20, 4104, 3, "lh_ptr_copy_kernel(gather)"),   # sub 513: the last dword lane alone in its workgroup
    (40, 20, 24, 5, "lh_ptr_copy_kernel(gather)"),
    (10, 1, 100, 7, "lh_ptr_copy_kernel(gather)"),
    (1, 3, 40, 5, "lh_ptr_copy_kernel(gather)"),
]


def _received(lh, k, m, nbytes, stripes, seed):
    """Encoded stripes, per stripe a random erasure pattern (e from 0 to min(k, m), the
    received blocks shuffled); stripe 1 (when there are 3+) gets a duplicate row (invalid)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    rec = lh.encode_batch(data, m)
    dh, rh = data.cpu().numpy(), rec.cpu().numpy()
    blocks = np.empty((stripes, k, nbytes), dtype=np.uint8)
    rows = np.empty((stripes, k), dtype=np.uint8)
    rng = np.random.Generator(np.random.PCG64(seed))
    for s in range(stripes):
        e = int(rng.integers(0, min(k, m) + 1))
        slots, r = lhutil.erasure_case(seed * 7919 + s, k, m, e)
        for i, (kind, x) in enumerate(slots):
            blocks[s, i] = dh[s, x] if kind == "d" else rh[s, x]
        rows[s] = r
    if stripes >= 3 and k >= 2:
        rows[1, 1] = rows[1, 0]
    return data, blocks, rows


@pytest.mark.parametrize("k,m,nbytes,stripes,form", DECODE)
def test_decode_batch_ptrs(lh, oracle, k, m, nbytes, stripes, form):
    import torch
    data, blocks, rows = _received(lh, k, m, nbytes, stripes, seed=k + 31 * m)
    # the strided call on the same inputs
    sb = torch.from_numpy(blocks).cuda()
    sr = torch.from_numpy(rows).cuda()
    sstat = lh.decode_batch(sb, sr, m)
    # the pointer-table call
    pool, ptrs, place = _scatter(torch.from_numpy(blocks).cuda(), seed=k * 3 + m)
    pr = torch.from_numpy(rows).cuda()
    pstat = lh.decode_batch_ptrs(k, m, nbytes, ptrs, pr)
    torch.cuda.synchronize()
    assert form in lh.last_launch(), lh.last_launch()
    got = _gather(pool, place)
    assert torch.equal(pstat, sstat)
    assert torch.equal(pr, sr)
    assert torch.equal(got, sb)
    # and the oracle on a sample of stripes (stripe 1 may be the invalid one)
    gh, gr = got.cpu().numpy(), pr.cpu().numpy()
    for s in sorted({0, stripes - 1}):
        bufs = [blocks[s, i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows[s]), nbytes)
        assert rc == 0
        assert list(gr[s]) == exp_rows, s
        for i in range(k):
            assert gh[s, i].tobytes() == bufs[i].tobytes(), (s, i)


def test_decode_batch_ptrs_roundtrip_baseline_shape(lh):
    """BASELINE configs[1] shape at 16 384 stripes through the pointer-table calls: encode
    from scattered data blocks, lose 4 random originals per stripe, decode from scattered
    received blocks; every stripe returns its data."""
    import torch
    k, m, nbytes, stripes = 29, 4, 1296, 16384
    g = torch.Generator(device="cuda").manual_seed(5)
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda", generator=g)
    dpool, dptr, dplace = _scatter(data, seed=11, max_off=7)
    rpool, rptr, rplace = _scatter(torch.zeros((stripes, m, nbytes), dtype=torch.uint8, device="cuda"), seed=12,
                                   max_off=7)
    lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr)
    # received: originals except 4 random ones, then recovery blocks 0..3 (pointers into the pools)
    perm = torch.argsort(torch.rand(stripes, k, device="cuda", generator=g), dim=1)
    keep = perm[:, : k - 4].sort(dim=1).values
    bptr = torch.cat([torch.gather(dptr, 1, keep), rptr], dim=1).contiguous()
    rows = torch.cat([keep, torch.arange(k, k + m, device="cuda").expand(stripes, m)], dim=1).to(torch.uint8)
    rows = rows.contiguous()
    lost = perm[:, k - 4:].sort(dim=1).values
    status = lh.decode_batch_ptrs(k, m, nbytes, bptr, rows)
    torch.cuda.synchronize()
    assert lh.last_launch() == ["lh_jit_decode_fused(pointer table)"]
    assert (status == 0).all()
    # the recovery slots now hold the lost originals, in ascending order, with their rows
    assert torch.equal(rows[:, k - 4:].long(), lost)
    got = _gather(rpool, rplace)
    assert torch.equal(got, torch.gather(data, 1, lost.unsqueeze(2).expand(stripes, 4, nbytes)))


@pytest.mark.parametrize("k,m,nbytes", [(40, 20, 24), (10, 1, 100), (1, 3, 40)])
def test_ptrs_gather_in_chunks(lh, oracle, monkeypatch, k, m, nbytes):
    """The gather / strided / scatter form over several workspace chunks (the chunk capped by
    LONGHAIR_AMD_PTR_CHUNK_BYTES at 3 stripes for the encode, 3-4 for the decode; 11
    stripes): encode and decode bit-identical to the strided calls."""
    import torch
    stripes = 11
    monkeypatch.setenv("LONGHAIR_AMD_PTR_CHUNK_BYTES", str(3 * (k + m) * nbytes + 3 * k))
    data, blocks, rows = _received(lh, k, m, nbytes, stripes, seed=k + m)
    want = lh.encode_batch(data, m)
    dpool, dptr, _ = _scatter(data, seed=5)
    rpool, rptr, rplace = _scatter(torch.zeros((stripes, m, nbytes), dtype=torch.uint8, device="cuda"), seed=6)
    lh.encode_batch_ptrs(k, m, nbytes, dptr, rptr)
    torch.cuda.synchronize()
    assert lh.last_launch()[0] == "lh_ptr_copy_kernel(gather)", lh.last_launch()
    assert torch.equal(_gather(rpool, rplace), want)
    sb, sr = torch.from_numpy(blocks).cuda(), torch.from_numpy(rows).cuda()
    sstat = lh.decode_batch(sb, sr, m)
    pool, ptrs, place = _scatter(torch.from_numpy(blocks).cuda(), seed=7)
    pr = torch.from_numpy(rows).cuda()
    pstat = lh.decode_batch_ptrs(k, m, nbytes, ptrs, pr)
    torch.cuda.synchronize()
    assert torch.equal(pstat, sstat) and torch.equal(pr, sr)
    assert torch.equal(_gather(pool, place), sb)


@pytest.mark.parametrize("k,m,nbytes", [(29, 4, 1296), (128, 32, 8192), (200, 3, 64)])
def test_prepare_ptrs(lh, k, m, nbytes):
    """cauchy_256_batch_prepare_ptrs: the pointer-table modules of a shape (cached at build
    time here), nothing for a shape without specialised kernels."""
    lh.prepare_ptrs(k, m, nbytes)
