"""Shared helpers for tests, golden generation and bench (test infrastructure).

- `fill(seed, n)`: the fixed input-data spec.  Bytes are the little-endian words of
  splitmix64(seed * 2**32 + i), i = 0, 1, ...  Reproducible in numpy, C and HIP.
- `Oracle`: ctypes handle to oracle/liblh_oracle.so (the C restatement).
- `RefLib`: ctypes handle to oracle/_ref/liblonghair_ref.so (the reference itself,
  compiled from /root/reference by `make -C oracle ref`).  Only used to generate golden
  fixtures and as the CPU baseline; never by the product.
"""
import ctypes
import hashlib
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLES = os.path.join(REPO, "longhair_amd", "data", "cauchy_tables_256.bin")
ORACLE_SO = os.path.join(REPO, "oracle", "liblh_oracle.so")
REF_SO = os.path.join(REPO, "oracle", "_ref", "liblonghair_ref.so")
GOLDEN = os.path.join(REPO, "tests", "golden")

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    """Vectorised splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def fill(seed, n):
    """n pseudo-random bytes for `seed` (see module docstring)."""
    words = (n + 7) // 8
    ctr = np.arange(words, dtype=np.uint64) + np.uint64((seed & 0xFFFFFFFF) << 32)
    return splitmix64(ctr).view(np.uint8)[:n].copy()


def h64(buf):
    """16-hex-digit SHA-256 prefix of a byte buffer (fixture digest)."""
    return hashlib.sha256(np.ascontiguousarray(buf).tobytes()).hexdigest()[:16]


class Block(ctypes.Structure):
    """Reference Block layout (cauchy_256.h:52-55)."""
    _fields_ = [("data", ctypes.POINTER(ctypes.c_ubyte)), ("row", ctypes.c_ubyte)]


def _ptr(arr):
    return arr.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte))


class _Codec:
    """encode/decode over numpy buffers for a C library with the reference ABI."""

    def __init__(self, lib, enc, dec):
        self.lib = lib
        self._enc = enc
        self._dec = dec
        enc.restype = ctypes.c_int
        dec.restype = ctypes.c_int

    def encode(self, k, m, data, bytes_):
        """data: uint8 [k, bytes] (or [k*bytes]).  Returns (rc, recovery uint8 [m*bytes])."""
        data = np.ascontiguousarray(data).reshape(-1)
        rec = np.zeros(max(m, 1) * bytes_ + 64, dtype=np.uint8)
        ptrs = (ctypes.POINTER(ctypes.c_ubyte) * max(k, 1))()
        for x in range(k):
            ptrs[x] = ctypes.cast(data.ctypes.data + x * bytes_, ctypes.POINTER(ctypes.c_ubyte))
        rc = self._enc(ctypes.c_int(k), ctypes.c_int(m), ptrs, _ptr(rec), ctypes.c_int(bytes_))
        return rc, rec[: m * bytes_]

    def decode(self, k, m, bufs, rows, bytes_):
        """bufs: list of k uint8 arrays (modified in place), rows: list of k ints.
        Returns (rc, new_rows)."""
        blocks = (Block * k)()
        for i in range(k):
            blocks[i].data = _ptr(bufs[i])
            blocks[i].row = rows[i]
        rc = self._dec(ctypes.c_int(k), ctypes.c_int(m), blocks, ctypes.c_int(bytes_))
        return rc, [blocks[i].row for i in range(k)]


class Oracle(_Codec):
    def __init__(self, path=ORACLE_SO):
        lib = ctypes.CDLL(path)
        blob = open(TABLES, "rb").read()
        lib.lho_init.restype = ctypes.c_int
        assert lib.lho_init(ctypes.c_char_p(blob), ctypes.c_size_t(len(blob))) == 0
        super().__init__(lib, lib.lho_encode, lib.lho_decode)

    def cauchy_rows(self, k, m):
        out = np.zeros((m - 1) * k, dtype=np.uint8)
        self.lib.lho_cauchy_rows(ctypes.c_int(k), ctypes.c_int(m), _ptr(out))
        return out.reshape(m - 1, k)


class RefLib(_Codec):
    def __init__(self, path=REF_SO):
        lib = ctypes.CDLL(path)
        lib._cauchy_256_init.restype = ctypes.c_int
        assert lib._cauchy_256_init(ctypes.c_int(2)) == 0
        super().__init__(lib, lib.cauchy_256_encode, lib.cauchy_256_decode)


def erasure_case(seed, k, m, e, shuffle=True):
    """A decode scenario: erase `e` random originals, supply `e` random recovery rows,
    optionally shuffle the block order.  Returns (slots, rows) where slots[i] is
    ('d', x) for original x or ('r', j) for recovery block j, and rows[i] its row."""
    rng = np.random.Generator(np.random.PCG64(seed))
    erased = sorted(rng.choice(k, size=e, replace=False).tolist()) if e else []
    rec = sorted(rng.choice(m, size=e, replace=False).tolist()) if e else []
    slots = [("d", x) for x in range(k) if x not in erased] + [("r", j) for j in rec]
    if shuffle:
        order = rng.permutation(len(slots)).tolist()
        slots = [slots[i] for i in order]
    rows = [x if kind == "d" else k + x for kind, x in slots]
    return slots, rows
