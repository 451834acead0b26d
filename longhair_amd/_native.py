"""Loader for the in-tree C-ABI library (no CPU fallback: a missing library raises)."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LONGHAIR_AMD_LIBRARY: another in-tree build of the same sources (the phase-B checked build,
# `make -C longhair_amd/csrc LH_DEBUG=1 OUT=$PWD/longhair_amd/liblonghair_amd_check.so
# BUILD=$PWD/longhair_amd/build_check`); the default is the product library.
library_path = os.path.join(_HERE, os.environ.get("LONGHAIR_AMD_LIBRARY", "liblonghair_amd.so"))
_lib = None


class Block(ctypes.Structure):
    """Same layout as the reference Block (cauchy_256.h:52-55)."""
    _fields_ = [("data", ctypes.POINTER(ctypes.c_ubyte)), ("row", ctypes.c_ubyte)]


# Every symbol include/cauchy_256.h, cauchy_256_batch.h, cauchy_256_dispatch.h and (test-only)
# cauchy_256_test.h declare.
EXPORTS = {
    "_cauchy_256_init": (ctypes.c_int, [ctypes.c_int]),
    "cauchy_256_encode": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "cauchy_256_decode": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "cauchy_256_encode_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                               ctypes.c_longlong, ctypes.c_void_p]),
    "cauchy_256_decode_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p]),
    "cauchy_256_encode_batch_ptrs": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "cauchy_256_decode_batch_ptrs": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p]),
    "cauchy_256_encode_host_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                                    ctypes.c_longlong, ctypes.c_int]),
    "cauchy_256_decode_host_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_int]),
    "cauchy_256_batch_prepare": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "cauchy_256_batch_prepare_ptrs": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "cauchy_256_batch_prepare_stream": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                       ctypes.c_void_p]),
    "cauchy_256_last_launch": (ctypes.c_char_p, []),
    "cauchy_256_batch_path": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "cauchy_256_jit_precompile": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "cauchy_256_frame_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong,
                                              ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]),
    "cauchy_256_unframe_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong,
                                                ctypes.c_void_p, ctypes.c_void_p]),
    "cauchy_256_last_error": (ctypes.c_char_p, []),
    "cauchy_256_set_dispatch": (ctypes.c_int, [ctypes.c_int, ctypes.c_longlong]),
    "cauchy_256_get_dispatch": (ctypes.c_int, []),
    "cauchy_256_host_isa": (ctypes.c_char_p, []),
}
# Bound only where the library exports them: the test-only hook lives in the checked build
# (liblonghair_amd_check.so, LH_TEST_HOOKS), not in the product library.
OPTIONAL_EXPORTS = {
    "cauchy_256_debug_throw_next": (None, []),
}


def bind(l):
    """Set the ctypes signatures of a loaded copy of the library (every EXPORTS symbol must
    exist; OPTIONAL_EXPORTS where present)."""
    for name, (res, args) in EXPORTS.items():
        f = getattr(l, name)
        f.restype = res
        f.argtypes = args
    for name, (res, args) in OPTIONAL_EXPORTS.items():
        if hasattr(l, name):
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
    return l


def lib():
    """The loaded library (loads on first use; raises OSError if it was never built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(library_path):
            raise OSError(f"{library_path} is missing: run `make -C longhair_amd/csrc` "
                          "(longhair_amd has no CPU fallback)")
        l = ctypes.CDLL(library_path)
        bind(l)
        _lib = l
    return _lib
