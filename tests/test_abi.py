"""CPU-only checks of the C-ABI boundary (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

import lhutil

REPO = lhutil.REPO


def _declared_functions():
    names = set()
    for h in ("cauchy_256.h", "cauchy_256_batch.h", "cauchy_256_dispatch.h"):
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


def test_no_silent_cpu_path():
    """Without a GPU every codec call must fail loudly (-2), never compute on the CPU."""
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
    assert longhair_amd.cauchy_256_encode(k, m, ptrs, rec, nbytes) == -2
    assert not rec.any()
    # the host SIMD engine of the drop-in dispatch policy is no fallback either
    for policy in ("host", "auto"):
        prev = longhair_amd.set_dispatch(policy)
        try:
            assert longhair_amd.cauchy_256_encode(k, m, ptrs, rec, nbytes) == -2
            assert not rec.any()
        finally:
            longhair_amd.set_dispatch(prev)


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
    # two tables (in-asm indexed for 8 outputs; once per code object) of 256 bodies of
    # 8 v_bitop3_b32 + a return: the fixed 68-byte stride the jump assumes
    assert committed.count("v_bitop3_b32") == 2 * 256 * 8
    assert committed.count("s_setpc_b64 s[94:95]") == 2 * 256
    # every call statement (1..8 outputs) turns GPR indexing on once and off once, and
    # restores M0 (no path leaves the statement with indexing on)
    assert committed.count("lh_inv_gtab:") == 1 and committed.count("s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)") == 8
    assert committed.count("s_set_gpr_idx_off") == 8 + 1 and committed.count("s_mov_b32 m0, s97") == 8 + 1
