"""longhair_amd -- MI355X-native Cauchy Reed-Solomon codec with the cauchy_256.h ABI.

Python view of the C-ABI library `liblonghair_amd.so` (built from longhair_amd/csrc by
`make -C longhair_amd/csrc` or `__graft_entry__.build()`):

* the reference interface, one stripe per call (catid/longhair cauchy_256.h:47-103):
  `cauchy_256_init()`, `cauchy_256_encode(k, m, data_ptrs, recovery_blocks, block_bytes)`,
  `cauchy_256_decode(k, m, blocks, block_bytes)` and the `Block` structure, taking the same
  arguments as the C functions (ctypes pointers / arrays) and returning the same codes;
* batched device-resident helpers on torch uint8 tensors: `encode_batch`, `decode_batch`.

There is no CPU implementation: importing works without a GPU, but every codec call
goes through the HIP library and fails loudly (LonghairError / non-zero codes) when no
device or no library is available.
"""
import ctypes

from ._native import Block, lib, library_path  # noqa: F401

CAUCHY_256_VERSION = 2

OK, EINVAL, ENODEV, EHIP = 0, -1, -2, -3


class LonghairError(RuntimeError):
    def __init__(self, code, what):
        msg = lib().cauchy_256_last_error().decode(errors="replace")
        super().__init__(f"{what} failed with code {code}: {msg}")
        self.code = code


def _cauchy_256_init(expected_version):
    return lib()._cauchy_256_init(ctypes.c_int(expected_version))


def cauchy_256_init():
    """Reference `cauchy_256_init()` macro: 0 on success (-1 version mismatch, -2 no GPU)."""
    return _cauchy_256_init(CAUCHY_256_VERSION)


def cauchy_256_encode(k, m, data_ptrs, recovery_blocks, block_bytes):
    """Reference cauchy_256_encode (cauchy_256.h:78): `data_ptrs` is a ctypes array of k
    `POINTER(c_ubyte)` (host or device memory), `recovery_blocks` a pointer/address with
    room for m * block_bytes bytes.  Returns 0 / -1 like the reference."""
    return lib().cauchy_256_encode(ctypes.c_int(k), ctypes.c_int(m), data_ptrs,
                                   ctypes.c_void_p(_addr(recovery_blocks)), ctypes.c_int(block_bytes))


def cauchy_256_decode(k, m, blocks, block_bytes):
    """Reference cauchy_256_decode (cauchy_256.h:103): `blocks` is a ctypes array of k
    `Block`; recovered originals are written in place and their `row` rewritten."""
    return lib().cauchy_256_decode(ctypes.c_int(k), ctypes.c_int(m), blocks, ctypes.c_int(block_bytes))


def _addr(x):
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, ctypes.Array) or isinstance(x, ctypes._Pointer):
        return ctypes.cast(x, ctypes.c_void_p).value
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    raise TypeError(f"cannot take the address of {type(x)}")


def _require(cond, msg, exc=ValueError):
    """API argument check that survives `python -O` (unlike assert): a bad tensor must raise,
    never reach a kernel as a wrong pointer."""
    if not cond:
        raise exc(msg)


def _cuda_tensor(t, dtype, name, shape=None, contiguous=False, device=None):
    """`t` must be a CUDA tensor of `dtype` (and `shape`, contiguity, `device` when given)."""
    import torch
    _require(isinstance(t, torch.Tensor), f"{name} must be a torch tensor", TypeError)
    _require(t.dtype == dtype, f"{name} must be {dtype}, got {t.dtype}", TypeError)
    _require(t.is_cuda, f"{name} must be a CUDA (device) tensor")
    if shape is not None:
        _require(tuple(t.shape) == tuple(shape), f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if contiguous:
        _require(t.is_contiguous(), f"{name} must be contiguous")
    if device is not None:
        _require(t.device == device, f"{name} must be on {device}, got {t.device}")


def _block_tensor(t, name):
    """uint8 CUDA tensor [stripes, blocks, bytes] with contiguous blocks (any stripe stride)."""
    import torch
    _cuda_tensor(t, torch.uint8, name)
    _require(t.dim() == 3, f"{name} must be [stripes, blocks, block_bytes]")
    _require(t.stride(2) == 1 and t.stride(1) == t.shape[2], f"{name}: blocks must be contiguous within a stripe")


def _stream_handle(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def encode_batch(data, m, recovery=None, stream=None):
    """Encode a batch of stripes resident on the GPU.

    data: uint8 CUDA tensor [stripes, k, block_bytes] (stripe-contiguous blocks).
    Returns the recovery tensor [stripes, m, block_bytes] (allocated if not given).
    Runs asynchronously on `stream` (default: torch's current stream)."""
    import torch
    _block_tensor(data, "data")
    stripes, k, nbytes = data.shape
    if recovery is None:
        recovery = torch.empty((stripes, m, nbytes), dtype=torch.uint8, device=data.device)
    _block_tensor(recovery, "recovery")
    _require(tuple(recovery.shape) == (stripes, m, nbytes), f"recovery must be [{stripes}, {m}, {nbytes}]")
    _require(recovery.device == data.device, "recovery must be on data's device")
    rc = lib().cauchy_256_encode_batch(k, m, nbytes, stripes, ctypes.c_void_p(data.data_ptr()),
                                       ctypes.c_longlong(data.stride(0)),
                                       ctypes.c_void_p(recovery.data_ptr()),
                                       ctypes.c_longlong(recovery.stride(0)),
                                       ctypes.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_encode_batch")
    return recovery


def decode_batch(blocks, rows, m, status=None, stream=None):
    """Decode a batch of stripes in place on the GPU.

    blocks: uint8 CUDA tensor [stripes, k, block_bytes] -- the k received blocks of each
            stripe in array order (the reference's Block[] order).
    rows:   uint8 CUDA tensor [stripes, k] -- each slot's Block.row; rewritten in place.
    Returns `status` (int8 [stripes], 0 ok / -1 invalid rows)."""
    import torch
    _block_tensor(blocks, "blocks")
    stripes, k, nbytes = blocks.shape
    _cuda_tensor(rows, torch.uint8, "rows", (stripes, k), True, blocks.device)
    if status is None:
        status = torch.empty((stripes,), dtype=torch.int8, device=blocks.device)
    _cuda_tensor(status, torch.int8, "status", (stripes,), True, blocks.device)
    rc = lib().cauchy_256_decode_batch(k, m, nbytes, stripes, ctypes.c_void_p(blocks.data_ptr()),
                                       ctypes.c_longlong(blocks.stride(0)),
                                       ctypes.c_void_p(rows.data_ptr()),
                                       ctypes.c_void_p(status.data_ptr()),
                                       ctypes.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_decode_batch")
    return status


def _ptr_table(t, stripes, n, name="pointer table"):
    import torch
    _cuda_tensor(t, torch.int64, name, (stripes, n), True)
    return ctypes.c_void_p(t.data_ptr())


def encode_batch_ptrs(k, m, block_bytes, data_ptrs, recovery_ptrs, stream=None):
    """Encode stripes whose blocks sit anywhere in device memory (cauchy_256_encode_batch_ptrs).

    data_ptrs:     int64 CUDA tensor [stripes, k] of device addresses (the reference's data_ptrs[]
                   per stripe, cauchy_256.h:78);
    recovery_ptrs: int64 CUDA tensor [stripes, m], where recovery block r of each stripe goes."""
    stripes = data_ptrs.shape[0]
    rc = lib().cauchy_256_encode_batch_ptrs(k, m, block_bytes, stripes, _ptr_table(data_ptrs, stripes, k, "data_ptrs"),
                                            _ptr_table(recovery_ptrs, stripes, m, "recovery_ptrs"),
                                            ctypes.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_encode_batch_ptrs")


def decode_batch_ptrs(k, m, block_bytes, block_ptrs, rows, status=None, stream=None):
    """Decode stripes whose k received blocks sit anywhere in device memory, in place
    (cauchy_256_decode_batch_ptrs; the reference's Block[] per stripe, cauchy_256.h:103).

    block_ptrs: int64 CUDA tensor [stripes, k] (Block.data of each slot);
    rows:       uint8 CUDA tensor [stripes, k] (Block.row), rewritten in place.
    Returns `status` (int8 [stripes], 0 ok / -1 invalid rows)."""
    import torch
    stripes = block_ptrs.shape[0]
    table = _ptr_table(block_ptrs, stripes, k, "block_ptrs")
    _cuda_tensor(rows, torch.uint8, "rows", (stripes, k), True, block_ptrs.device)
    if status is None:
        status = torch.empty((stripes,), dtype=torch.int8, device=rows.device)
    _cuda_tensor(status, torch.int8, "status", (stripes,), True, block_ptrs.device)
    rc = lib().cauchy_256_decode_batch_ptrs(k, m, block_bytes, stripes, table,
                                            ctypes.c_void_p(rows.data_ptr()), ctypes.c_void_p(status.data_ptr()),
                                            ctypes.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_decode_batch_ptrs")
    return status


def prepare_ptrs(k, m, block_bytes):
    """Compile the pointer-table forms of the shape's specialised kernels now
    (cauchy_256_batch_prepare_ptrs)."""
    rc = lib().cauchy_256_batch_prepare_ptrs(k, m, block_bytes)
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_batch_prepare_ptrs")


def encode_host_batch(data, m, recovery=None, chunk_stripes=0):
    """Encode stripes held in host memory (numpy uint8 [stripes, k, bytes], ideally pinned
    via a pinned torch CPU tensor's .numpy()); pipelined H2D / kernel / D2H."""
    import numpy as np
    _require(data.dtype == np.uint8 and data.ndim == 3 and data.flags.c_contiguous,
             "data must be a C-contiguous uint8 array [stripes, k, block_bytes]")
    stripes, k, nbytes = data.shape
    if recovery is None:
        recovery = np.empty((stripes, m, nbytes), dtype=np.uint8)
    rc = lib().cauchy_256_encode_host_batch(k, m, nbytes, stripes, data.ctypes.data, data.strides[0],
                                            recovery.ctypes.data, recovery.strides[0], chunk_stripes)
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_encode_host_batch")
    return recovery


def decode_host_batch(blocks, rows, m, chunk_stripes=0):
    """Decode stripes held in host memory in place (numpy uint8 [stripes, k, bytes] and
    rows [stripes, k]); returns the int8 status per stripe."""
    import numpy as np
    _require(blocks.dtype == np.uint8 and blocks.ndim == 3 and blocks.flags.c_contiguous,
             "blocks must be a C-contiguous uint8 array [stripes, k, block_bytes]")
    stripes, k, nbytes = blocks.shape
    _require(rows.dtype == np.uint8 and rows.shape == (stripes, k) and rows.flags.c_contiguous,
             f"rows must be a C-contiguous uint8 array [{stripes}, {k}]")
    status = np.zeros(stripes, dtype=np.int8)
    rc = lib().cauchy_256_decode_host_batch(k, m, nbytes, stripes, blocks.ctypes.data, blocks.strides[0],
                                            rows.ctypes.data, status.ctypes.data, chunk_stripes)
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_decode_host_batch")
    return status


def frame_batch(data, recovery, packets=None, stream=None):
    """Packets of a batch (the reference sends each block with its one-byte row,
    README.md:66-72): uint8 CUDA tensors data [S, k, B] and recovery [S, m, B] ->
    packets [S, k + m, B + 1], packet i = [row i][block i]."""
    import torch
    stripes, k, nbytes = data.shape
    m = recovery.shape[1]
    _block_tensor(data, "data")
    _block_tensor(recovery, "recovery")
    if packets is None:
        packets = torch.empty((stripes, k + m, nbytes + 1), dtype=torch.uint8, device=data.device)
    _cuda_tensor(packets, torch.uint8, "packets", (stripes, k + m, nbytes + 1), True, data.device)
    rc = lib().cauchy_256_frame_batch(k, m, nbytes, stripes, ctypes.c_void_p(data.data_ptr()), data.stride(0),
                                      ctypes.c_void_p(recovery.data_ptr()), recovery.stride(0),
                                      ctypes.c_void_p(packets.data_ptr()), packets.stride(0),
                                      ctypes.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_frame_batch")
    return packets


def unframe_batch(packets, blocks=None, rows=None, stream=None):
    """The k packets received per stripe (uint8 CUDA tensor [S, k, B + 1], any order)
    -> (blocks [S, k, B], rows [S, k]), the layout decode_batch takes."""
    import torch
    _cuda_tensor(packets, torch.uint8, "packets", None, True)
    _require(packets.dim() == 3, "packets must be [stripes, k, block_bytes + 1]")
    stripes, k, b1 = packets.shape
    if blocks is None:
        blocks = torch.empty((stripes, k, b1 - 1), dtype=torch.uint8, device=packets.device)
    if rows is None:
        rows = torch.empty((stripes, k), dtype=torch.uint8, device=packets.device)
    _block_tensor(blocks, "blocks")
    _require(tuple(blocks.shape) == (stripes, k, b1 - 1), "blocks must be [stripes, k, block_bytes]")
    _cuda_tensor(rows, torch.uint8, "rows", (stripes, k), True, packets.device)
    rc = lib().cauchy_256_unframe_batch(k, b1 - 1, stripes, ctypes.c_void_p(packets.data_ptr()), packets.stride(0),
                                        ctypes.c_void_p(blocks.data_ptr()), blocks.stride(0),
                                        ctypes.c_void_p(rows.data_ptr()), ctypes.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_unframe_batch")
    return blocks, rows


_POLICIES = {"gpu": 0, "auto": 1, "host": 2}


def set_dispatch(policy, host_max_work=-1):
    """Drop-in dispatch policy (include/cauchy_256_dispatch.h): 'auto' (default: small
    all-host-memory calls on the host SIMD engine), 'gpu' or 'host'.  Returns the
    previous policy name.  The library needs a GPU under every policy."""
    prev = lib().cauchy_256_set_dispatch(_POLICIES[policy], host_max_work)
    if prev < 0:
        raise LonghairError(prev, "cauchy_256_set_dispatch")
    return {v: k for k, v in _POLICIES.items()}[prev]


def dispatch_policy():
    return {v: k for k, v in _POLICIES.items()}[lib().cauchy_256_get_dispatch()]


def host_isa():
    """Instruction set of the host engine on this CPU ('avx512bw', 'avx2', 'scalar')."""
    return lib().cauchy_256_host_isa().decode()


def prepare(k, m, block_bytes, max_stripes=0, stream=None):
    """Compile the specialised kernels / reserve workspace for a shape (synchronous).
    Workspaces are per stream: prepare the stream a graph will be captured on."""
    rc = lib().cauchy_256_batch_prepare_stream(k, m, block_bytes, max_stripes,
                                               ctypes.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise LonghairError(rc, "cauchy_256_batch_prepare_stream")


def last_launch():
    """Kernels this thread's last entry-point call enqueued (cauchy_256_last_launch), in
    launch order; [] when it ran on the host engine or launched nothing."""
    s = lib().cauchy_256_last_launch().decode()
    return s.split(";") if s else []


def batch_path(k, m, block_bytes, decode=False):
    """'jit' when a run-time specialised network serves the shape ('jit-fused' for a
    decode whose plan is computed in the same kernel), else 'generic'."""
    code = lib().cauchy_256_batch_path(k, m, block_bytes, 1 if decode else 0)
    return {0: "generic", 1: "jit", 2: "jit-fused", 3: "jit-win", 4: "jit-wide"}[code]


def lds_staged(k, m, block_bytes, decode=False):
    """True when the shape's encode (decode) register network stages its columns by LDS-DMA
    (jit.cpp jit_config_for, jit_codec.hip LH_LDS)."""
    return lib().cauchy_256_batch_path(k, m, block_bytes, 5 if decode else 2) == 1


def jump_lanes(k, m, block_bytes, decode=False):
    """Dword lanes per sub-block of the generic jump kernel the library launches for this
    shape on the current device (codec.cpp jump_layout): 1 = lh_apply_jump_kernel, 2 =
    lh_apply_jump2_kernel, 0 = the generic kernels below dword lanes."""
    rc = lib().cauchy_256_batch_path(k, m, block_bytes, 7 if decode else 6)
    if rc < 0:
        raise LonghairError(rc, "cauchy_256_batch_path")
    return rc


def kernel_names(k, m, block_bytes):
    """Names of the kernels one encode_batch / decode_batch launches for this shape."""
    sub = block_bytes // 8
    small = sub < 4  # the generic kernels below dword lanes

    def lone_tail(w):  # decode in place: the overlapping last lane must share its neighbour's workgroup
        nch = (sub + w - 1) // w
        return sub % w != 0 and nch > 1 and (nch - 1) % 64 == 0

    old_dec = small or lone_tail(4)
    two_dec = not old_dec and jump_lanes(k, m, block_bytes, True) == 2  # (the library's own choice)
    two_enc = not small and jump_lanes(k, m, block_bytes) == 2
    jump_enc = "lh_apply_generic_kernel" if small else ("lh_apply_jump2_kernel" if two_enc else "lh_apply_jump_kernel")
    enc = {"generic": [jump_enc], "jit": ["lh_jit_encode"],
           "jit-win": ["lh_jit_encode_win"]}[batch_path(k, m, block_bytes)]
    order = ["lh_order_kernel"] if min(k, m) > 8 else []  # kernels.hip order_stripes
    dec = {"generic": ["lh_plan_kernel"] + (["lh_apply_generic_kernel", "lh_scatter_kernel"] if old_dec
                                            else order + ["lh_apply_jump2_kernel" if two_dec else "lh_apply_jump_kernel"]),
           "jit": ["lh_plan_small_kernel" if min(k, m) <= 8 else "lh_plan_kernel", "lh_jit_decode"],
           "jit-fused": ["lh_jit_decode_fused"],
           "jit-wide": ["lh_plan_kernel", "lh_jit_decode_wide"] + order + ["lh_inverse_gt_kernel"],
           }[batch_path(k, m, block_bytes, True)]
    if m == 1 or k == 1:
        enc, dec = ["lh_xor_reduce_kernel"], ["lh_plan_kernel", "lh_xor_reduce_kernel"]
    return enc, dec
