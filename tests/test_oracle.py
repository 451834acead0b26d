"""The C restatement (oracle/) against golden fixtures produced by the reference itself."""
import json
import os

import numpy as np
import pytest

import lhutil


def _load(name):
    return json.load(open(os.path.join(lhutil.GOLDEN, name)))


def test_tables_blob_digest():
    import hashlib
    blob = open(lhutil.TABLES, "rb").read()
    assert len(blob) == 34902
    assert hashlib.sha256(blob).hexdigest() == \
        "98a1ea9be26a57c0f378cc6324a108ec5dd5b08bb959c6be30f1a50e2ed36de8"


def test_fill_spec():
    # splitmix64(0) = 0xe220a8397b1dcdaf (the published splitmix64 test value), little-endian.
    assert lhutil.fill(0, 8).tobytes().hex() == "afcd1d7b39a820e2"
    a, b = lhutil.fill(7, 100), lhutil.fill(7, 100)
    assert (a == b).all() and not (lhutil.fill(8, 100) == a).all()


def test_encode_grid(oracle):
    for k, m, bytes_, seed, rc, digest in _load("encode_grid.json")["cases"]:
        data = lhutil.fill(seed, k * bytes_)
        got_rc, rec = oracle.encode(k, m, data, bytes_)
        assert got_rc == rc, (k, m, bytes_)
        if rc != 0:
            rec = rec[:bytes_]
        assert lhutil.h64(rec) == digest, (k, m, bytes_)


def test_encode_full_bytes(oracle):
    for c in _load("encode_full.json"):
        data = np.frombuffer(bytes.fromhex(c["data"]), dtype=np.uint8)
        rc, rec = oracle.encode(c["k"], c["m"], data, c["bytes"])
        assert rc == c["rc"]
        assert rec.tobytes().hex() == c["recovery"]


def _decode_case(codec, c):
    k, m, bytes_ = c["k"], c["m"], c["bytes"]
    data = lhutil.fill(c["seed"], k * bytes_).reshape(k, bytes_)
    rc_e, rec = codec.encode(k, m, data, bytes_)
    assert rc_e == c["rc_encode"]
    rec = rec.reshape(m, bytes_)
    bufs = [(data[x] if kind == "d" else rec[x]).copy() for kind, x in c["slots"]]
    rc, rows = codec.decode(k, m, bufs, list(c["rows_in"]), bytes_)
    return rc, rows, [lhutil.h64(b) for b in bufs], data


def test_decode_cases(oracle):
    for c in _load("decode_cases.json"):
        rc, rows, digests, data = _decode_case(oracle, c)
        assert rc == c["rc"], c["tag"]
        assert rows == c["rows_out"], c["tag"]
        assert digests == c["digests"], c["tag"]


def test_decode_roundtrip_recovers_originals(oracle):
    # Independent of fixtures: whatever the reference returns, it must equal the data.
    for c in _load("decode_cases.json"):
        if c["rc"] != 0 or c["tag"] in ("m1_no_erasure_quirk",):
            continue
        rc, rows, digests, data = _decode_case(oracle, c)
        for r, d in zip(rows, digests):
            assert d == lhutil.h64(data[r]), c["tag"]


@pytest.mark.skipif(not os.path.exists(lhutil.REF_SO), reason="reference build absent")
def test_oracle_vs_reference_random():
    ref, orc = lhutil.RefLib(), lhutil.Oracle()
    rng = np.random.Generator(np.random.PCG64(5))
    for _ in range(200):
        k = int(rng.integers(1, 255))
        m = int(rng.integers(1, 256 - k + 1))
        bytes_ = 8 * int(rng.integers(1, 5))
        data = lhutil.fill(int(rng.integers(0, 2**32)), k * bytes_)
        assert ref.encode(k, m, data, bytes_)[1].tobytes() == orc.encode(k, m, data, bytes_)[1].tobytes()
