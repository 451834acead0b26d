"""CPU tests of the host SIMD engine behind the drop-in dispatch policy
(longhair_amd/csrc/host_codec.cpp, include/cauchy_256_dispatch.h): a standalone harness
(tests/native/host_engine_check.cpp) links the engine's host code and checks it against the
C oracle on random stripes, at every instruction-set level, also under ASan + UBSan.
The product library itself still refuses every codec call without a GPU
(tests/test_abi.py::test_no_silent_cpu_path); the engine is reached there only through the
GPU-gated drop-in entry points (tests/test_gpu_parity.py, policy fixture)."""
import os
import subprocess

import pytest

import lhutil

CSRC = os.path.join(lhutil.REPO, "longhair_amd", "csrc")
SRCS = [os.path.join(CSRC, f) for f in ("host_codec.cpp", "field.cpp", "blobs.cpp")]


def _build(tmp_path, extra):
    exe = str(tmp_path / "host_engine_check")
    cmd = ["g++", "-std=c++17", "-g", f"-I{CSRC}", f"-DLH_SRC_DIR={os.path.join(lhutil.REPO, 'longhair_amd')}",
           os.path.join(lhutil.REPO, "tests", "native", "host_engine_check.cpp"), *SRCS, "-ldl", "-o", exe, *extra]
    subprocess.check_call(cmd)
    return exe


@pytest.fixture(scope="module")
def oracle_so(oracle):
    return lhutil.ORACLE_SO


@pytest.mark.parametrize("sanitize", [False, True])
def test_host_engine_matches_oracle(tmp_path, oracle_so, sanitize):
    flags = ["-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"] \
        if sanitize else ["-O2"]
    exe = _build(tmp_path, flags)
    for isa in ("avx512bw", "avx2", "scalar"):
        env = dict(os.environ, LONGHAIR_AMD_HOST_ISA=isa, ASAN_OPTIONS="detect_leaks=1")
        r = subprocess.run([exe, oracle_so, lhutil.TABLES], capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert " 0 mismatches" in r.stdout
