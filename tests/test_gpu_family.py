"""GPU parity of the block-size families (jit_codec.hip LH_FAMILY, jit.cpp jit_family_ok), the
encode's and the fused decode's: one module per (k, m) and role serves every qualifying block
size, the size a kernel argument (the reference serves any (k, m, bytes) at full
speed on its first call, cauchy_256.cpp:423-481).  Bytes against the C oracle at block sizes of every sub-block
alignment (sub mod 8 = 0, 2, 4, 6), one and several stripes per wave, partial waves, and
the last lane's partial word (one module serving several sizes: tests/test_family_build.py).
`-m gpu`: needs an MI355X."""
import os

import numpy as np
import pytest

import lhutil

pytestmark = pytest.mark.gpu

# (k, m, bytes, stripes): sub = bytes / 8 -> nch = ceil(sub / 8) lanes, 64 // nch stripes per wave
FAMILY_SHAPES = [
    (29, 4, 1296, 97),   # sub 162 (mod 8 = 2), 21 lanes, 3 stripes per wave: the headline shape
    (29, 4, 1312, 50),   # sub 164 (4)
    (29, 4, 2592, 9),    # sub 324 (4), 41 lanes, 1 stripe per wave
    (29, 4, 1280, 31),   # sub 160 (0): full last word
    (29, 4, 1328, 20),   # sub 166 (6)
    (29, 4, 4096, 5),    # sub 512: 64 lanes
    (29, 4, 64, 70),     # sub 8: one lane, 64 stripes per wave
    (10, 3, 384, 33),    # k 10: two steps of 5 columns, 6 lanes, 10 stripes per wave
    (17, 6, 784, 21),    # m 6 (the register budget's limit), k 17: last step of 2 columns
    (64, 2, 2112, 7),    # k 64, sub 264: 33 lanes
    (4, 5, 96, 40),      # k 4 (two steps of 2), sub 12
]


# The fused decode's family: (k, m, bytes, stripes); at least ceil(k / 8) lanes per stripe
FAMILY_DEC_SHAPES = [
    (29, 4, 1296, 97),   # sub 162 (mod 8 = 2), 21 lanes, 3 stripes per wave: the headline shape
    (29, 4, 1312, 50),   # sub 164 (4)
    (29, 4, 2592, 9),    # sub 324 (4), 41 lanes, 1 stripe per wave
    (29, 4, 1280, 31),   # sub 160 (0): full last word
    (29, 4, 1328, 20),   # sub 166 (6)
    (29, 4, 4096, 5),    # 64 lanes
    (29, 4, 464, 40),    # sub 58, 8 lanes: 4 Block.row bytes per lane, 8 stripes per wave
    (10, 3, 384, 33),    # 6 lanes, 10 stripes per wave, e <= 3
    (17, 4, 784, 21),    # sub 98 (2), 13 lanes
    (64, 2, 2112, 7),    # k 64, 33 lanes, e <= 2
    (4, 5, 96, 40),      # k 4 < m: e <= 4, 2 lanes, 32 stripes per wave
]



def family_sample(pairs=((5, 3), (13, 4), (22, 2), (37, 4), (50, 3), (64, 4)), sizes=25, seed=611):
    """A seeded sample for the families' randomised parity: for each (k, m) (one module per
    role serves all its sizes), `sizes` random 16-byte-multiple block sizes that both families
    serve, with a random stripe count.  tools/precompile.py builds the modules."""
    import longhair_amd as lh
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for k, m in pairs:
        got = 0
        while got < sizes:
            b = 16 * int(rng.integers(1, 257))
            if (lh.lib().cauchy_256_batch_path(k, m, b, 8) == 1 and lh.lib().cauchy_256_batch_path(k, m, b, 9) == 1
                    and (k, m, b) not in [o[:3] for o in out]):
                out.append((k, m, b, int(rng.integers(1, 40))))
                got += 1
    return out


FAMILY_SAMPLE_PAIRS = ((5, 3), (13, 4), (22, 2), (37, 4), (50, 3), (64, 4))


@pytest.fixture(scope="module")
def lh():
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import longhair_amd
    assert longhair_amd.cauchy_256_init() == 0
    return longhair_amd


@pytest.mark.parametrize("k,m,nbytes,stripes", FAMILY_SHAPES, ids=[f"k{k}m{m}b{b}" for k, m, b, _ in FAMILY_SHAPES])
def test_family_encode_matches_oracle(lh, oracle, monkeypatch, k, m, nbytes, stripes):
    import torch
    monkeypatch.setenv("LONGHAIR_AMD_JIT_DEFINES", "LH_FAMILY=1")
    monkeypatch.setenv("LONGHAIR_AMD_JIT_SYNC", "1")
    data = lhutil.fill(k * 1000 + nbytes, stripes * k * nbytes).reshape(stripes, k, nbytes)
    x = torch.from_numpy(data).cuda()
    # a strided recovery buffer with a gap between stripes (the bench layout's form)
    rbuf = torch.full((stripes, m + 1, nbytes), 0x5A, dtype=torch.uint8, device="cuda")
    rec = rbuf[:, :m]
    assert lh.lib().cauchy_256_batch_path(k, m, nbytes, 8) == 1  # served by the family module
    lh.encode_batch(x, m, recovery=rec)
    torch.cuda.synchronize()
    assert lh.last_launch() == ["lh_jit_encode(family)"], lh.last_launch()
    got = rec.cpu().numpy()
    for s in range(stripes):
        rc, exp = oracle.encode(k, m, data[s], nbytes)
        assert rc == 0 and got[s].tobytes() == exp.tobytes(), f"stripe {s}"
    assert (rbuf[:, m].cpu().numpy() == 0x5A).all()  # nothing written past the recovery blocks


@pytest.mark.parametrize("k,m,nbytes,stripes", FAMILY_DEC_SHAPES, ids=[f"k{k}m{m}b{b}" for k, m, b, _ in FAMILY_DEC_SHAPES])
def test_family_decode_matches_oracle(lh, oracle, monkeypatch, k, m, nbytes, stripes):
    """Bytes and rewritten rows of the fused decode's family module against the oracle: random
    e per stripe (the first at e_max), random recovery rows, shuffled slots (as every
    specialised decode is tested, test_gpu_boundaries.roundtrip)."""
    import test_gpu_boundaries as tb
    monkeypatch.setenv("LONGHAIR_AMD_JIT_DEFINES", "LH_FAMILY=1")
    monkeypatch.setenv("LONGHAIR_AMD_JIT_SYNC", "1")
    assert lh.lib().cauchy_256_batch_path(k, m, nbytes, 9) == 1  # served by the family module
    _, dec = tb.roundtrip(lh, oracle, k, m, nbytes, stripes, seed=k * 7 + nbytes)
    assert dec == ["lh_jit_decode_fused(family)"], dec


def test_family_serves_sizes_without_a_module(lh, oracle, monkeypatch, tmp_path):
    """Default policy: a k29/m4 block size with no size-specialised module cached, and no
    compiling allowed (as for every drop-in call), encodes and decodes on the (k, m) family
    modules that the precompile of another size left in the cache -- not on the generic
    kernels."""
    import test_gpu_boundaries as tb
    monkeypatch.delenv("LONGHAIR_AMD_JIT_DEFINES", raising=False)
    monkeypatch.setenv("LONGHAIR_AMD_CACHE_DIR", str(tmp_path))
    monkeypatch.setenv("LONGHAIR_AMD_PRECOMPILE_FAMILY", "1")
    assert lh.lib().cauchy_256_jit_precompile(29, 4, 1296) == 0  # the 1 296-byte modules + the families
    monkeypatch.setenv("LONGHAIR_AMD_JIT_COMPILE", "0")
    for nbytes, stripes in ((1456, 13), (2592, 5), (784, 40)):
        enc, dec = tb.roundtrip(lh, oracle, 29, 4, nbytes, stripes, seed=nbytes + 7)
        assert enc == ["lh_jit_encode(family)"], (nbytes, enc)
        assert dec == ["lh_jit_decode_fused(family)"], (nbytes, dec)


def test_family_random_sizes(lh, oracle, monkeypatch):
    """Randomised parity of both families: 150 seeded (k, m, bytes, stripes) cases over six
    (k, m) modules, encode and decode (random e, recovery rows and slot order per stripe)
    against the oracle, each through the family kernels."""
    import test_gpu_boundaries as tb
    monkeypatch.setenv("LONGHAIR_AMD_JIT_DEFINES", "LH_FAMILY=1")
    monkeypatch.setenv("LONGHAIR_AMD_JIT_SYNC", "1")
    cases = family_sample(FAMILY_SAMPLE_PAIRS)
    assert len(cases) == 150
    for k, m, nbytes, stripes in cases:
        enc, dec = tb.roundtrip(lh, oracle, k, m, nbytes, stripes, seed=k * 100003 + nbytes)
        assert enc == ["lh_jit_encode(family)"], (k, m, nbytes, enc)
        assert dec == ["lh_jit_decode_fused(family)"], (k, m, nbytes, dec)
