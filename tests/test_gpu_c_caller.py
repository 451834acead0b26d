"""A native C program calls the drop-in boundary exactly as a user of the reference would:
compiled against include/cauchy_256.h and linked with -llonghair_amd (tests/native/c_caller.c,
order_test-style round trips, tests/cauchy_256_tests.cpp:122-205).  Its encode bytes and
codes must equal the reference's golden fixtures.  Runs under the library's default dispatch
policy (AUTO) and under the GPU and host policies.  `-m gpu`: the library needs an MI355X."""
import json
import os
import subprocess

import numpy as np
import pytest

import lhutil

pytestmark = pytest.mark.gpu

NATIVE = os.path.join(lhutil.REPO, "tests", "native")
EXE = os.path.join(NATIVE, "c_caller")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "-s", "-C", NATIVE])
    return EXE


@pytest.mark.parametrize("policy", ["default", "gpu", "host"])
def test_c_caller_matches_goldens(exe, policy, tmp_path):
    grid = json.load(open(os.path.join(lhutil.GOLDEN, "encode_grid.json")))["cases"]
    # every k in [1, 255] at some m, the invalid-parameter cases and the BASELINE shapes
    pick = [c for i, c in enumerate(grid) if i % 7 == 0 or c[4] != 0 or c[2] >= 1296]
    lines = "".join(f"{k} {m} {b} {seed}\n" for k, m, b, seed, rc, dig in pick)
    out = tmp_path / "rec.bin"
    r = subprocess.run([exe, policy, str(out)], input=lines, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    blob = out.read_bytes()
    off = 0
    for k, m, b, seed, rc, digest in pick:
        got_rc = int(np.frombuffer(blob[off:off + 4], dtype="<i4")[0])
        rec = np.frombuffer(blob[off + 4:off + 4 + m * b], dtype=np.uint8)
        off += 4 + m * b
        assert got_rc == rc, (k, m, b)
        assert lhutil.h64(rec if rc == 0 else rec[:b]) == digest, (k, m, b)
    assert off == len(blob)
