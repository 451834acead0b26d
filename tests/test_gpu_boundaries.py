"""GPU parity at every kernel-selection boundary, each side asserted by the launch trace.

The product picks its kernels by shape (longhair_amd/csrc/jit.cpp jit_config_for /
jit_win_config_for, codec.cpp encode_batch / decode_batch, kernels.hip launch_plan /
launch_inverse).  For each boundary a pair of shapes straddles it; both are encoded and
decoded against the C oracle (bit-exact data and rewritten rows), with random erasure
counts (the first stripe always at e = e_max), random recovery rows and shuffled slots,
and `cauchy_256_last_launch` must name the kernels the boundary predicts -- so every
variant test runs the kernel it names.

The last test is a sweep shaped like the reference's own `main()` (every k in [1, 255],
tests/cauchy_256_tests.cpp:227-381) and `order_test` (random positions, :122-205).
`-m gpu`: needs an MI355X.  The specialised modules of every shape here are compiled at
build time (tools/precompile.py), so no test waits on hiprtc.
"""
import numpy as np
import pytest

import lhutil

pytestmark = pytest.mark.gpu

FUSED = ["lh_jit_decode_fused"]
SMALL4 = ["lh_plan_small_kernel<4>", "lh_jit_decode"]
SMALL8 = ["lh_plan_small_kernel<8>", "lh_jit_decode"]
# (e_max > 8: the in-place apply and phase B take their stripes by e, largest first)
GENERIC_CF = ["lh_plan_kernel(closed form)", "lh_order_kernel", "lh_apply_jump_kernel"]
GENERIC_S8 = ["lh_plan_small_kernel<8>", "lh_apply_jump_kernel"]
# the generic decode's fallback (sub < 4, or the overlapping last dword lane alone in its
# workgroup: sub = 256 t + 1..3): apply into a workspace, then scatter
OLD_CF = ["lh_plan_kernel(closed form)", "lh_apply_generic_kernel", "lh_scatter_kernel"]
JUMP = ["lh_apply_jump_kernel"]
JUMP2 = ["lh_apply_jump2_kernel"]  # two-dword lanes (codec.cpp jump_layout)
JUMP_FB = ["lh_apply_jump_kernel(fallback)"]  # the in-asm table (LONGHAIR_AMD_INV_FALLBACK)
GEN = {"LONGHAIR_AMD_PATH": "generic"}
PS4_JUMP = ["lh_plan_small_kernel<4>", "lh_apply_jump_kernel"]
PS4_JUMP2 = ["lh_plan_small_kernel<4>", "lh_apply_jump2_kernel"]
PS8_JUMP = ["lh_plan_small_kernel<8>", "lh_apply_jump_kernel"]
# (lh_order_kernel: phase B's stripes by e, largest first; kernels.hip launch_inverse)
WIDE16 = ["lh_plan_kernel(closed form)", "lh_jit_decode_wide", "lh_order_kernel", "lh_inverse_gt_kernel"]
WIDE64 = WIDE16  # (one phase-B kernel for every e_max since round 3)

# (id, k, m, bytes, stripes, env, encode kernels, decode kernels)
BOUNDARIES = [
    # fused in-kernel plan <-> separate planner: k <= 64
    ("k64-fused", 64, 4, 1296, 48, {}, ["lh_jit_encode"], FUSED),
    ("k65-planned", 65, 4, 1296, 48, {}, ["lh_jit_encode"], SMALL4),
    # ... and one stripe per <= 64 lanes (nch = 64 with 8-byte lanes; the decode of m = 3 at
    # 8128-byte blocks takes 8-byte lanes too, nch = 127: two waves per stripe)
    ("nch64-fused", 8, 4, 4096, 24, {}, ["lh_jit_encode"], FUSED),
    ("nch127-planned", 8, 3, 8128, 24, {}, ["lh_jit_encode"], SMALL4),
    # ... and e_max <= 4 (both sides of e_max = min(k, m) = 4 / 5, from k and from m)
    ("emax4-k", 4, 8, 64, 64, {}, ["lh_jit_encode"], FUSED),
    ("emax5-k", 5, 8, 64, 64, {}, ["lh_jit_encode"], SMALL8),
    ("emax4-m", 10, 4, 64, 64, {}, ["lh_jit_encode"], FUSED),
    ("emax5-m", 10, 5, 64, 64, {}, ["lh_jit_encode"], SMALL8),
    # specialised decode needs e_max * m <= 64 (e_max 8 / 9): small planner <-> Cauchy planner
    ("emax8", 9, 8, 64, 64, {}, ["lh_jit_encode"], SMALL8),
    ("emax9", 9, 9, 64, 64, {}, ["lh_jit_encode"], GENERIC_CF),
    ("emax8-k16", 16, 8, 64, 64, {}, ["lh_jit_encode"], SMALL8),
    ("emax9-k16", 16, 9, 64, 64, {}, ["lh_jit_encode"], GENERIC_CF),
    # generator from the CAUCHY_MATRIX_2..6 tables (m <= 6) <-> from the X/Y points (m >= 7)
    ("m6-jit", 20, 6, 64, 64, {}, ["lh_jit_encode"], SMALL8),
    ("m7-jit", 20, 7, 64, 64, {}, ["lh_jit_encode"], SMALL8),
    ("m6-generic", 20, 6, 64, 64, {"LONGHAIR_AMD_PATH": "generic"}, JUMP, GENERIC_S8),
    ("m7-generic", 20, 7, 64, 64, {"LONGHAIR_AMD_PATH": "generic"}, JUMP, GENERIC_S8),
    # register-resident encode network: m <= 12 (96 accumulator dwords) <-> windowed / generic
    ("enc-m12", 40, 12, 2048, 8, {}, ["lh_jit_encode"], WIDE16),
    ("enc-m13", 40, 13, 2048, 8, {}, ["lh_jit_encode_win"], WIDE16),
    ("enc-m12-small", 10, 12, 64, 32, {}, ["lh_jit_encode"], GENERIC_CF),
    ("enc-m13-small", 10, 13, 64, 32, {}, JUMP, GENERIC_CF),
    # windowed decode: m <= 64 (the used-row ballot) and sub % 256 == 0
    ("wide-m64", 20, 64, 2048, 8, {}, ["lh_jit_encode_win"], WIDE16),
    ("generic-m65", 20, 65, 2048, 8, {}, ["lh_jit_encode_win"], GENERIC_CF),
    ("wide-sub512", 40, 20, 4096, 8, {}, ["lh_jit_encode_win"], WIDE16),
    ("generic-sub513", 40, 20, 4104, 8, {}, JUMP, OLD_CF),
    # generic decode in place: every dword lane of a sub-block in one workgroup with its
    # overlapped neighbour (sub 516: jump apply) <-> not (sub 513 above: workspace + scatter)
    ("generic-sub516", 40, 20, 4128, 8, {}, JUMP, GENERIC_CF),
    # generic kernels below dword lanes (sub < 4) <-> the jump apply (sub = 4)
    ("generic-sub3", 30, 13, 24, 40, {}, ["lh_apply_generic_kernel"], OLD_CF),
    ("generic-sub4", 30, 13, 32, 40, {}, JUMP, GENERIC_CF),
    # two-dword lanes (codec.cpp jump_layout): at most 4 outputs, sub >= 8 (encode) and, in
    # place, sub >= 512 with the last two-dword lane in its neighbour's workgroup
    ("jump2-n4-sub7", 40, 4, 56, 64, GEN, JUMP, PS4_JUMP),
    ("jump2-n4-sub8", 40, 4, 64, 64, GEN, JUMP2, PS4_JUMP),
    ("jump2-n5-sub8", 40, 5, 64, 64, GEN, JUMP, PS8_JUMP),
    ("jump2-n4-sub504", 40, 4, 4032, 8, GEN, JUMP2, PS4_JUMP),
    ("jump2-n4-sub520", 40, 4, 4160, 8, GEN, JUMP2, PS4_JUMP2),
    ("jump2-n5-sub520", 40, 5, 4160, 8, GEN, JUMP, PS8_JUMP),
    ("jump2-n4-sub516", 40, 4, 4128, 8, GEN, JUMP2, PS4_JUMP),  # (sub % 8 = 4, nch 65: lone)
    # the in-asm one-dword table (and the address-probe fallback) for every jump apply
    ("jump2-n4-fallback", 40, 4, 4160, 8, dict(GEN, LONGHAIR_AMD_INV_FALLBACK="1"), JUMP_FB,
     ["lh_plan_small_kernel<4>", "lh_apply_jump_kernel(fallback)"]),
    # phase B: V rows staged 16 at a time for e_max <= 32, all at once above
    ("jump-emax32", 40, 32, 2048, 8, {}, ["lh_jit_encode_win"], WIDE16),
    ("jump-emax33", 40, 33, 2048, 8, {}, ["lh_jit_encode_win"], WIDE64),
]

# Phase-B kernel (kernels.hip launch_inverse): one kernel, lh_inverse_gt_kernel, with its
# outputs packed 8 per wave (e_max <= 32) or spread (above), and its in-asm-table fallback.
# (Round 3's other six forms were removed in round 4; the packing override in round 5.)
PHASE_B = [
    ({}, 32, "lh_inverse_gt_kernel"),
    ({}, 33, "lh_inverse_gt_kernel"),
    ({}, 64, "lh_inverse_gt_kernel"),
    ({"LONGHAIR_AMD_INV_FALLBACK": "1"}, 32, "lh_inverse_gt_kernel(fallback)"),
    ({"LONGHAIR_AMD_INV_FALLBACK": "1"}, 33, "lh_inverse_gt_kernel(fallback)"),
    ({"LONGHAIR_AMD_INV_FALLBACK": "1"}, 64, "lh_inverse_gt_kernel(fallback)"),
]


@pytest.fixture(scope="module")
def lh():
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import longhair_amd
    assert longhair_amd.cauchy_256_init() == 0
    return longhair_amd


def _gpu(arr):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


def _scenarios(k, m, stripes, seed, e_first=None):
    """Per stripe: random e in [0, e_max] (stripe 0: e_first, default e_max), random erased
    originals, random recovery rows, shuffled slot order (lhutil.erasure_case)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    e_max = min(k, m)
    out = []
    for s in range(stripes):
        e = (e_max if e_first is None else e_first) if s == 0 else int(rng.integers(0, e_max + 1))
        out.append(lhutil.erasure_case(int(rng.integers(0, 2**31)), k, m, e))
    return out


def roundtrip(lh, oracle, k, m, nbytes, stripes, seed, scen=None):
    """encode_batch + decode_batch of `stripes` stripes against the oracle.  Returns the
    launch traces (encode, decode)."""
    import torch
    data = lhutil.fill(seed, stripes * k * nbytes).reshape(stripes, k, nbytes)
    rec = lh.encode_batch(_gpu(data), m)
    torch.cuda.synchronize()
    enc_trace = lh.last_launch()
    got_rec = rec.cpu().numpy()
    scen = scen or _scenarios(k, m, stripes, seed)
    blocks = np.zeros((stripes, k, nbytes), dtype=np.uint8)
    rows = np.zeros((stripes, k), dtype=np.uint8)
    for s in range(stripes):
        rc, exp = oracle.encode(k, m, data[s], nbytes)
        assert rc == 0
        assert got_rec[s].tobytes() == exp.tobytes(), ("encode", k, m, nbytes, s)
        exp = exp.reshape(m, nbytes)
        slots, rws = scen[s]
        for i, (kind, x) in enumerate(slots):
            blocks[s, i] = data[s, x] if kind == "d" else exp[x]
        rows[s] = rws
    d_blocks, d_rows = _gpu(blocks), _gpu(rows)
    status = lh.decode_batch(d_blocks, d_rows, m)
    torch.cuda.synchronize()
    dec_trace = lh.last_launch()
    got, got_rows, st = d_blocks.cpu().numpy(), d_rows.cpu().numpy(), status.cpu().numpy()
    assert (st == 0).all()
    for s in range(stripes):
        bufs = [blocks[s, i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows[s]), nbytes)
        assert rc == 0
        assert list(got_rows[s]) == exp_rows, ("rows", k, m, nbytes, s)
        for i in range(k):
            assert got[s, i].tobytes() == bufs[i].tobytes(), ("decode", k, m, nbytes, s, i)
    return enc_trace, dec_trace


@pytest.mark.parametrize("case", BOUNDARIES, ids=[c[0] for c in BOUNDARIES])
def test_selection_boundary(lh, oracle, monkeypatch, case):
    name, k, m, nbytes, stripes, env, enc_k, dec_k = case
    for key, v in env.items():
        monkeypatch.setenv(key, v)
    enc, dec = roundtrip(lh, oracle, k, m, nbytes, stripes, seed=k * 1000 + m * 10 + nbytes)
    assert enc == enc_k, (name, enc)
    assert dec == dec_k, (name, dec)


@pytest.mark.parametrize("env,m,kernel", PHASE_B,
                         ids=[f"{'-'.join(k[17:] + v for k, v in e.items()) or 'default'}-m{m}" for e, m, _ in PHASE_B])
def test_phase_b_variant(lh, oracle, monkeypatch, env, m, kernel):
    """Every phase-B kernel of the split large-m decode against the oracle (k = 40, 2048-byte
    blocks, e_max = m), on both sides of e_max = 32."""
    for key, v in env.items():
        monkeypatch.setenv(key, v)
    k, nbytes = 40, 2048
    enc, dec = roundtrip(lh, oracle, k, m, nbytes, 8, seed=m * 31)
    assert dec == ["lh_plan_kernel(closed form)", "lh_jit_decode_wide", "lh_order_kernel", kernel], dec


def test_phase_b_chunks_per_workgroup(lh, oracle):
    """Phase-B workgroups over two consecutive 2 KiB chunks of a stripe (the tile pipeline
    carried across them): 6144-byte blocks = 3 chunks, so the second workgroup of a stripe has
    a one-chunk remainder; against the oracle."""
    enc, dec = roundtrip(lh, oracle, 40, 20, 6144, 7, seed=14)
    assert dec == ["lh_plan_kernel(closed form)", "lh_jit_decode_wide", "lh_order_kernel", "lh_inverse_gt_kernel"], dec


def _sweep_ms(k):
    return sorted({m for m in list(range(1, 9)) + [16, 32, 64, 256 - k] if 1 <= m and k + m <= 256})


def test_reference_main_sweep(lh, oracle, monkeypatch):
    """Every k in [1, 255] x m in {1..8, 16, 32, 64, 256 - k}: 3 stripes each, the first at
    e = min(k, m) erasures, the others at random e in [0, min(k, m)], random positions and
    recovery rows, shuffled slots, block sizes 8..64 bytes; encode_batch + decode_batch
    against the oracle.

    Shapes whose specialised module is in the build's code-object cache take it (every
    k <= 16 with m <= 8 is precompiled, tools/precompile.py SWEEP); the rest run the generic
    kernels -- LONGHAIR_AMD_JIT_COMPILE=0 keeps hiprtc out of the test (a k = 100 module
    takes minutes to compile).  The launch traces must show both families."""
    monkeypatch.setenv("LONGHAIR_AMD_JIT_COMPILE", "0")
    seen = set()
    n = 0
    for k in range(1, 256):
        for m in _sweep_ms(k):
            nbytes = 8 * (1 + (7 * k + m) % 8)
            scen = _scenarios(k, m, 3, seed=k * 257 + m)
            enc, dec = roundtrip(lh, oracle, k, m, nbytes, 3, seed=k * 997 + m, scen=scen)
            seen.update(enc + dec)
            n += 1
    assert n > 2500
    assert {"lh_jit_encode", "lh_jit_decode_fused", "lh_jit_decode", "lh_apply_generic_kernel", "lh_apply_jump_kernel",
            "lh_apply_jump2_kernel", "lh_xor_reduce_kernel"} <= seen, sorted(seen)


def _jit_sample(n=24, seed=2024):
    """A seeded sample of register-network shapes outside the boundary pairs and the sweep's
    precompiled set: k in [17, 128], m in [2, 12], blocks of 16..4096 bytes (k * m <= 700
    keeps the network within jit.cpp's kMaxNetworkOnes).  tools/precompile.py compiles every
    one at build time (the test itself never waits on hiprtc)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    while len(out) < n:
        k, m = int(rng.integers(17, 129)), int(rng.integers(2, 13))
        nbytes = 8 * int(rng.integers(2, 513))
        if k * m <= 700 and (k, m, nbytes) not in out:
            out.append((k, m, nbytes))
    return out


JIT_SAMPLE = _jit_sample()


@pytest.mark.parametrize("k,m,nbytes", JIT_SAMPLE, ids=[f"k{k}m{m}b{b}" for k, m, b in JIT_SAMPLE])
def test_specialised_sample(lh, oracle, k, m, nbytes):
    """The hiprtc-specialised kernels (one module per (k, m, bytes), the generator bits as
    constants) on a seeded sample of shapes: encode through lh_jit_encode, decode through the
    specialised kernel its e_max selects (fused plan, or the small planner + lh_jit_decode;
    the generic apply above e_max * m = 64), bytes and rewritten rows against the oracle,
    random e per stripe (the first at e_max), random recovery rows, shuffled slots."""
    assert lh.batch_path(k, m, nbytes) == "jit", (k, m, nbytes)
    enc_k, dec_k = lh.kernel_names(k, m, nbytes)
    enc, dec = roundtrip(lh, oracle, k, m, nbytes, 24, seed=k * 131 + m * 17 + nbytes)
    assert enc == ["lh_jit_encode"], enc
    assert [d.split("<")[0].split("(")[0] for d in dec] == dec_k, (dec, dec_k)


@pytest.mark.parametrize("k,nbytes", [(29, 1296), (5, 24), (2, 8)])
def test_m1_accepts_any_rows_like_the_reference(lh, oracle, k, nbytes):
    """m == 1 decode (cauchy_decode_m1, cauchy_256.cpp:487-535) accepts any rows: rows >= k
    are recovery blocks (the last in array order is the output), repeated originals are
    harmless, and with no recovery block blocks[0] is overwritten.  The batch path must
    give the oracle's bytes, rows and status 0 for all of them."""
    import torch
    rng = np.random.Generator(np.random.PCG64(k))
    cases = [
        [k + 5] + list(range(1, k)),                       # recovery row out of range for m = 1
        [0] * k,                                           # every slot claims original 0
        list(range(k - 1)) + [k],                          # one recovery block, last slot
        [k, k + 1] + list(range(2, k)) if k > 2 else [k, k + 1],  # two recovery blocks
        list(range(k)),                                    # no erasure: the quirk
        list(rng.integers(0, 256, k)),                     # anything
    ]
    for rows in cases:
        rows = [int(r) for r in rows][:k]
        blocks = lhutil.fill(k + len(rows), k * nbytes).reshape(1, k, nbytes)
        d_blocks, d_rows = _gpu(blocks), _gpu(np.array([rows], dtype=np.uint8))
        status = lh.decode_batch(d_blocks, d_rows, 1)
        torch.cuda.synchronize()
        bufs = [blocks[0, i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, 1, bufs, rows, nbytes)
        assert rc == 0
        assert int(status.cpu()[0]) == 0, rows
        assert list(d_rows.cpu().numpy()[0]) == exp_rows, rows
        got = d_blocks.cpu().numpy()[0]
        assert all(got[i].tobytes() == bufs[i].tobytes() for i in range(k)), rows


def test_capture_never_allocates(lh):
    """A decode captured into a graph on a stream whose workspace was never reserved must
    fail with -3 (nothing enqueued) instead of allocating graph-owned memory; after
    cauchy_256_batch_prepare_stream on that stream the same capture works and replays."""
    import torch
    k, m, nbytes, stripes = 200, 56, 65536 // 64, 16   # generic path (sub % 256 != 0): plan + work
    data = torch.randint(0, 256, (stripes, k, nbytes), dtype=torch.uint8, device="cuda")
    rec = lh.encode_batch(data, m)
    blocks = data.clone()
    blocks[:, :m] = rec
    rows0 = torch.tensor([[k + r for r in range(m)] + list(range(m, k))] * stripes, dtype=torch.uint8,
                         device="cuda")
    rows = rows0.clone()
    status = torch.empty((stripes,), dtype=torch.int8, device="cuda")
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    failed = None
    try:
        with torch.cuda.graph(graph, stream=s):
            try:
                lh.decode_batch(blocks, rows, m, status=status, stream=s)
            except lh.LonghairError as e:
                failed = e
    except RuntimeError:
        pass  # an empty capture may be rejected by torch; what matters is the codec's error
    assert failed is not None and failed.code == -3 and "capture" in str(failed)
    torch.cuda.synchronize()
    lh.prepare(k, m, nbytes, stripes, stream=s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        rows.copy_(rows0)
        lh.decode_batch(blocks, rows, m, status=status, stream=s)
    graph.replay()
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert torch.equal(blocks, data) and torch.equal(rows[0].cpu(), torch.arange(k, dtype=torch.uint8))


@pytest.mark.parametrize("off,pad", [(1, 0), (8, 0), (4, 12), (0, 2), (3, 5)])
def test_misaligned_batch_buffers(lh, oracle, off, pad):
    """The batch calls take any base address and stripe stride: the data, the recovery
    blocks and the decode buffer at odd offsets and strides (the LDS-staged k29/m4 kernels'
    DMAs then start off 16-byte boundaries); every stripe against the oracle, the bytes
    around the blocks untouched."""
    import torch
    k, m, nbytes, stripes = 29, 4, 1296, 50
    stride = k * nbytes + pad
    data = lhutil.fill(off * 7 + pad, stripes * k * nbytes).reshape(stripes, k, nbytes)
    xb = torch.full((off + stride * stripes + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    X = xb[off:].as_strided((stripes, k, nbytes), (stride, nbytes, 1))
    X.copy_(_gpu(data))
    rb = torch.full((off + (m * nbytes + pad) * stripes + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    R = rb[off:].as_strided((stripes, m, nbytes), (m * nbytes + pad, nbytes, 1))
    lh.encode_batch(X, m, recovery=R)
    torch.cuda.synchronize()
    rec = R.cpu().numpy()
    for s in range(stripes):
        rc, exp = oracle.encode(k, m, data[s], nbytes)
        assert rc == 0 and rec[s].tobytes() == exp.tobytes(), s
    # decode in place from a misaligned buffer
    scen = _scenarios(k, m, stripes, off * 31 + pad)
    db = torch.full((off + stride * stripes + 64,), 0x3C, dtype=torch.uint8, device="cuda")
    D = db[off:].as_strided((stripes, k, nbytes), (stride, nbytes, 1))
    blocks = np.empty_like(data)
    rows = np.empty((stripes, k), dtype=np.uint8)
    for s, (slots, rws) in enumerate(scen):
        for i, (kind, x) in enumerate(slots):
            blocks[s, i] = data[s, x] if kind == "d" else rec[s, x]
        rows[s] = rws
    D.copy_(_gpu(blocks))
    d_rows = _gpu(rows)
    lh.decode_batch(D, d_rows, m)
    torch.cuda.synchronize()
    got, got_rows = D.cpu().numpy(), d_rows.cpu().numpy()
    for s in range(stripes):
        bufs = [blocks[s, i].copy() for i in range(k)]
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows[s]), nbytes)
        assert list(got_rows[s]) == exp_rows, s
        assert all(got[s, i].tobytes() == bufs[i].tobytes() for i in range(k)), s
    raw = db.cpu().numpy()
    assert (raw[:off] == 0x3C).all() and (raw[off + stride * stripes:] == 0x3C).all()
    if pad:
        body = raw[off:off + stride * stripes].reshape(stripes, stride)
        assert (body[:, k * nbytes:] == 0x3C).all()


@pytest.mark.parametrize("align", [128, 64])
def test_aligned_decode_buffer(lh, oracle, align):
    """bench.py's aligned decode buffer (a padded stripe stride and an offset that put every
    stripe's recovery slots on an `align`-byte boundary) through the specialised k29/m4
    kernels: the encode writes straight into the recovery slots, the decode runs in place;
    every stripe against the oracle and the padding bytes untouched."""
    import torch
    import bench
    k, m, nbytes, stripes = 29, 4, 1296, 99
    off, stride = bench.aligned_layout(k, m, nbytes, align)
    buf = torch.full((off + stride * stripes,), 0x5A, dtype=torch.uint8, device="cuda")
    D = buf[off:].as_strided((stripes, k, nbytes), (stride, nbytes, 1))
    data = lhutil.fill(align + 1, stripes * k * nbytes).reshape(stripes, k, nbytes)
    scen = [lhutil.erasure_case(align * 1000 + s, k, m, m, shuffle=False) for s in range(stripes)]
    rows = np.array([rw for _, rw in scen], dtype=np.uint8)
    for s, (slots, _) in enumerate(scen):      # survivors first, the m recovery slots last
        D[s, : k - m] = torch.from_numpy(np.stack([data[s, x] for kind, x in slots if kind == "d"])).cuda()
    lh.encode_batch(_gpu(data), m, recovery=D[:, k - m:])
    assert lh.last_launch() == ["lh_jit_encode"]
    d_rows = _gpu(rows)
    status = lh.decode_batch(D, d_rows, m)
    torch.cuda.synchronize()
    assert lh.last_launch() == FUSED and (status.cpu() == 0).all()
    got, got_rows = D.cpu().numpy(), d_rows.cpu().numpy()
    for s in range(stripes):
        rc, rec = oracle.encode(k, m, data[s], nbytes)
        rec = rec.reshape(m, nbytes)
        bufs = [data[s, x].copy() if kind == "d" else rec[x].copy() for kind, x in scen[s][0]]
        rc, exp_rows = oracle.decode(k, m, bufs, list(rows[s]), nbytes)
        assert list(got_rows[s]) == exp_rows, s
        assert all(got[s, i].tobytes() == bufs[i].tobytes() for i in range(k)), s
    raw = buf.cpu().numpy()
    pad = np.ones(raw.size, dtype=bool)
    for s in range(stripes):
        pad[off + s * stride: off + s * stride + k * nbytes] = False
    assert (raw[pad] == 0x5A).all()


def test_exit_during_background_compile(tmp_path):
    """A short-lived process that meets a new shape and exits at once, its background hiprtc
    compilation still running (jit.cpp CompileWorker): the exit-time drain joins the
    worker while hiprtc is intact, so the process ends cleanly (exit code 0, no abort)."""
    import os
    import subprocess
    import sys
    code = (
        "import sys, torch; sys.path.insert(0, %r); import longhair_amd as lh\n"
        "assert lh.cauchy_256_init() == 0\n"
        "x = torch.zeros((8, 11, 72), dtype=torch.uint8, device='cuda')\n"
        "lh.encode_batch(x, 3); torch.cuda.synchronize()\n"
        "print('trace', lh.last_launch(), flush=True)\n"
    ) % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LONGHAIR_AMD_JIT_SYNC="0", LONGHAIR_AMD_CACHE_DIR=str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "lh_apply_jump" in r.stdout, r.stdout  # it ran on the generic kernels, compile in flight


def test_jit_compiles_in_background(lh, oracle, monkeypatch, tmp_path):
    """A batch call on a shape with no specialised module returns at once on the generic
    kernels while hiprtc compiles the module on a background thread (no lock held: other
    shapes' lookups proceed); a later call of the same shape launches the specialised
    kernels.  Bytes against the oracle on both paths (jit.cpp JitCache::get, kAsync)."""
    import os
    import time

    import torch
    monkeypatch.setenv("LONGHAIR_AMD_JIT_SYNC", "0")
    monkeypatch.setenv("LONGHAIR_AMD_CACHE_DIR", str(tmp_path))  # nothing cached on disk
    k, m, nbytes, stripes = 13, 3, 88, 40                     # a shape no other test uses
    data = lhutil.fill(77, stripes * k * nbytes).reshape(stripes, k, nbytes)
    expect = np.stack([oracle.encode(k, m, data[s], nbytes)[1].reshape(m, nbytes) for s in range(stripes)])
    x = _gpu(data)
    t0 = time.perf_counter()
    rec = lh.encode_batch(x, m)
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    assert lh.last_launch() == ["lh_apply_jump2_kernel"], lh.last_launch()
    assert first < 1.0, f"first call took {first:.2f} s"
    assert np.array_equal(rec.cpu().numpy(), expect)
    # another shape meanwhile: its (cached) module is not held up by the compilation
    t1 = time.perf_counter()
    lh.encode_batch(_gpu(lhutil.fill(1, 9 * 29 * 1296).reshape(9, 29, 1296)), 4)
    torch.cuda.synchronize()
    assert time.perf_counter() - t1 < 1.0
    deadline = time.time() + 100
    while True:
        rec = lh.encode_batch(x, m)
        torch.cuda.synchronize()
        trace = lh.last_launch()
        if trace == ["lh_jit_encode"]:
            break
        assert trace == ["lh_apply_jump2_kernel"], trace
        assert time.time() < deadline, "the background compilation did not finish in 100 s"
        time.sleep(0.25)
    assert np.array_equal(rec.cpu().numpy(), expect)
    assert any(f.endswith(".co") for f in os.listdir(tmp_path)), "the module was not written to the cache"
    # the decode has a module of its own (one role per module, jit.cpp): generic kernels while
    # it compiles in the background, then the fused decode (e_max = 3); bytes checked each time
    scen = _scenarios(k, m, stripes, 5)
    deadline = time.time() + 100
    while True:
        _, dec = roundtrip(lh, oracle, k, m, nbytes, stripes, seed=9, scen=scen)
        if dec == FUSED:
            break
        assert dec == ["lh_plan_small_kernel<4>", "lh_apply_jump_kernel"], dec
        assert time.time() < deadline, "the decode module's background compilation did not finish in 100 s"
        time.sleep(0.25)
