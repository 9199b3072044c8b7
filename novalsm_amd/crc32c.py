"""Python mirror of NovaLSM's crc32c interface, backed by libnova_crc32c.so.

Names and argument meaning follow util/crc32c.h:11-43 (``Extend``, ``Value``,
``Mask``, ``Unmask``, ``kMaskDelta``) so parity tests read like the reference's
util/crc32c_test.cc; the batch functions wrap the C-ABI in include/nova_crc32c.h.

Device batch functions take torch CUDA(HIP) tensors for data, descriptors and
outputs and run on the current torch stream.  They call the HIP kernels only:
if the native library is missing or no GPU is usable they raise -- there is
no CPU fallback on this path.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

from . import build as _build

kMaskDelta = 0xA282EAD8

APPEND_TYPE = 0x1
MASK_OUTPUT = 0x2
TB_QUIRK = 0x4
RAW = 0x8
HINT_LARGE_BLOCKS = 0x10  # scheduling hint: most blocks >= 16 KiB (include/nova_crc32c.h)


def TYPE(t: int) -> int:
    return (t & 0xFF) << 8


class NovaError(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None


def lib_path() -> str:
    return _build.LIB


def load(build_if_missing: bool = False) -> ctypes.CDLL:
    """Load the in-tree native library (never a site-packages copy)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        if not build_if_missing:
            raise ImportError(f"native library missing: {path} (run __graft_entry__.build())")
        _build.build()
    L = ctypes.CDLL(path)
    u32, u64, sz, vp, i32 = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p,
                             ctypes.c_int)
    sig = {
        "nova_crc32c_extend": (u32, [u32, ctypes.c_char_p, sz]),
        "nova_crc32c_value": (u32, [ctypes.c_char_p, sz]),
        "nova_crc32c_mask": (u32, [u32]),
        "nova_crc32c_unmask": (u32, [u32]),
        "nova_crc32c_combine": (u32, [u32, u32, u64]),
        "nova_port_accelerated_crc32c": (u32, [u32, ctypes.c_char_p, sz]),
        "nova_crc32c_batch": (i32, [vp, vp, vp, vp, vp, sz, u32, vp]),
        "nova_crc32c_batch_strided": (i32, [vp, u64, u32, sz, vp, vp, u32, vp]),
        "nova_sstable_write_trailers": (i32, [vp, vp, vp, sz, u32, vp]),
        "nova_sstable_verify_blocks": (i32, [vp, vp, vp, sz, vp, vp, vp]),
        "nova_crc32c_stream_host": (i32, [vp, u64, u32, sz, vp, u32, sz, i32]),
        "nova_log_write_crcs": (i32, [vp, vp, sz, vp]),
        "nova_log_verify_records": (i32, [vp, vp, sz, vp, vp, vp]),
        "nova_xor_parity": (i32, [vp, vp, sz, sz, vp, vp]),
        "nova_fill_splitmix64": (i32, [vp, sz, u64, u64, vp]),
        "nova_device_init": (i32, []),
        "nova_crc32c_plan": (i32, [sz, u64, ctypes.POINTER(i32), ctypes.POINTER(u32)]),
        "nova_crc32c_kernel_name": (ctypes.c_char_p, [i32]),
        "nova_crc32c_describe": (i32, [sz, u64, u64, i32, ctypes.c_char_p, sz]),
        "nova_crc32c_set_tuning": (None, [i32, u32]),
        "nova_error_string": (ctypes.c_char_p, [i32]),
        "nova_crc32c_abi_version": (i32, []),
        "nova_diag_set_variant": (None, [i32]),
        "nova_diag_set_static_pct": (None, [i32]),
        "nova_diag_set_blocks_per_group": (None, [i32]),
        "nova_diag_set_chunk_blocks": (None, [i32]),
        "nova_diag_set_stream_waves": (None, [i32]),
        "nova_diag_set_variable_kernel": (None, [i32]),
        "nova_diag_set_parity_variant": (None, [i32]),
        "nova_diag_set_rounds_sort": (None, [i32]),
        "nova_diag_set_trailer_single_pass": (None, [i32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().nova_error_string(rc).decode()
        raise NovaError(f"{what} failed: {msg} ({rc})")


def _bytes(data) -> bytes:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return bytes(data)
    if isinstance(data, str):
        return data.encode()
    return bytes(data)


# ---- scalar API: util/crc32c.h ------------------------------------------

def Extend(init_crc: int, data, n: Optional[int] = None) -> int:
    b = _bytes(data)
    n = len(b) if n is None else n
    return load().nova_crc32c_extend(init_crc & 0xFFFFFFFF, b, n)


def Value(data, n: Optional[int] = None) -> int:
    return Extend(0, data, n)


def Mask(crc: int) -> int:
    return load().nova_crc32c_mask(crc & 0xFFFFFFFF)


def Unmask(masked_crc: int) -> int:
    return load().nova_crc32c_unmask(masked_crc & 0xFFFFFFFF)


def Combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return load().nova_crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)


def AcceleratedCRC32C(crc: int, data) -> int:
    """port::AcceleratedCRC32C (port/port_stdcxx.h:179-189) backed by the GPU."""
    b = _bytes(data)
    return load().nova_port_accelerated_crc32c(crc & 0xFFFFFFFF, b, len(b))


# ---- device batches -------------------------------------------------------

def _stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    if not t.is_cuda:
        raise NovaError("device batch expects GPU tensors (no CPU fallback on this path)")
    return int(t.data_ptr())


def _require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise NovaError("no GPU available: the batched CRC32C path runs only on the HIP device")


def batch(data, offsets, lengths, init=None, flags: int = 0, out=None, stream=None):
    """Variable-length batch (nova_crc32c_batch). data: uint8 GPU tensor;
    offsets: int64/uint64 GPU tensor; lengths: int32/uint32 GPU tensor."""
    import torch
    _require_gpu()
    n = int(offsets.numel())
    if lengths.numel() != n:
        raise NovaError("offsets/lengths size mismatch")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=data.device)
    rc = load().nova_crc32c_batch(_ptr(data), _ptr(offsets), _ptr(lengths), _ptr(init),
                                  _ptr(out), n, flags, _stream_ptr(stream))
    _check(rc, "nova_crc32c_batch")
    return out


def batch_strided(data, stride: int, length: int, n_blocks: int, init=None, flags: int = 0,
                  out=None, stream=None, base_offset: int = 0):
    import torch
    _require_gpu()
    if n_blocks and base_offset + (n_blocks - 1) * stride + length > data.numel():
        raise NovaError("blocks exceed the data tensor")
    if out is None:
        out = torch.empty(n_blocks, dtype=torch.int32, device=data.device)
    rc = load().nova_crc32c_batch_strided(_ptr(data) + base_offset, stride, length, n_blocks,
                                          _ptr(init), _ptr(out), flags, _stream_ptr(stream))
    _check(rc, "nova_crc32c_batch_strided")
    return out


def write_trailers(buf, offsets, sizes, type_byte: int = 0, tb_quirk: bool = False, stream=None,
                   hint_large: bool = False):
    _require_gpu()
    flags = TYPE(type_byte) | (TB_QUIRK if tb_quirk else 0) | (HINT_LARGE_BLOCKS if hint_large else 0)
    rc = load().nova_sstable_write_trailers(_ptr(buf), _ptr(offsets), _ptr(sizes),
                                            int(offsets.numel()), flags, _stream_ptr(stream))
    _check(rc, "nova_sstable_write_trailers")
    return buf


def verify_blocks(buf, offsets, sizes, stream=None, ok=None, bad=None):
    """Returns (ok uint8 tensor, n_bad int32 tensor[1]).  A caller-supplied
    `bad` accumulates (zero it first)."""
    import torch
    _require_gpu()
    n = int(offsets.numel())
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=buf.device)
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=buf.device)
    rc = load().nova_sstable_verify_blocks(_ptr(buf), _ptr(offsets), _ptr(sizes), n, _ptr(ok),
                                           _ptr(bad), _stream_ptr(stream))
    _check(rc, "nova_sstable_verify_blocks")
    return ok, bad


def log_write_crcs(buf, record_offsets, stream=None):
    """db/log_writer.cc:99-114 for every record header at record_offsets (in place)."""
    _require_gpu()
    rc = load().nova_log_write_crcs(_ptr(buf), _ptr(record_offsets), int(record_offsets.numel()),
                                    _stream_ptr(stream))
    _check(rc, "nova_log_write_crcs")
    return buf


def log_verify_records(buf, record_offsets, stream=None, ok=None, bad=None):
    """db/log_reader.cc:251-262 per record -> (ok uint8 tensor, n_bad int32 tensor[1])."""
    import torch
    _require_gpu()
    n = int(record_offsets.numel())
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=buf.device)
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=buf.device)
    rc = load().nova_log_verify_records(_ptr(buf), _ptr(record_offsets), n, _ptr(ok), _ptr(bad),
                                        _stream_ptr(stream))
    _check(rc, "nova_log_verify_records")
    return ok, bad


def xor_parity(buf, frag_offsets, parity_len: int, out=None, stream=None):
    """ltc/stoc_file_client_impl.cpp:334-349 XOR parity block over fragments."""
    import torch
    _require_gpu()
    if out is None:
        out = torch.empty(parity_len, dtype=torch.uint8, device=buf.device)
    rc = load().nova_xor_parity(_ptr(buf), _ptr(frag_offsets), int(frag_offsets.numel()),
                                parity_len, _ptr(out), _stream_ptr(stream))
    _check(rc, "nova_xor_parity")
    return out


def stream_host(host_u8, stride: int, length: int, n_blocks: int, flags: int = 0,
                chunk_blocks: int = 4096, n_streams: int = 3):
    """Host-resident blocks (pinned torch CPU tensor or numpy array) -> CRCs (numpy u32)."""
    import numpy as np
    _require_gpu()
    out = np.empty(n_blocks, dtype=np.uint32)
    if hasattr(host_u8, "data_ptr"):
        ptr = int(host_u8.data_ptr())
    else:
        ptr = int(host_u8.ctypes.data)
    rc = load().nova_crc32c_stream_host(ptr, stride, length, n_blocks, int(out.ctypes.data),
                                        flags, chunk_blocks, n_streams)
    _check(rc, "nova_crc32c_stream_host")
    return out


def fill_splitmix64(t, seed: int, first_word: int = 0, stream=None):
    _require_gpu()
    rc = load().nova_fill_splitmix64(_ptr(t), t.numel() * t.element_size(), seed, first_word,
                                     _stream_ptr(stream))
    _check(rc, "nova_fill_splitmix64")
    return t


def set_tuning(lanes_per_unit: int = 0, seg_bytes: int = 0) -> None:
    load().nova_crc32c_set_tuning(lanes_per_unit, seg_bytes)


def plan(n_blocks: int, bytes_per_block: int):
    g = ctypes.c_int(0)
    s = ctypes.c_uint32(0)
    load().nova_crc32c_plan(n_blocks, bytes_per_block, ctypes.byref(g), ctypes.byref(s))
    return g.value, s.value


def describe(n_blocks: int, length: int, stride: int, variable: bool = False,
             large: bool = False) -> dict:
    import json
    buf = ctypes.create_string_buffer(512)
    v = (2 if large else 1) if variable else 0
    load().nova_crc32c_describe(n_blocks, length, stride, v, buf, 512)
    return json.loads(buf.value.decode())


def kernel_name(lanes_per_unit: int) -> str:
    return load().nova_crc32c_kernel_name(lanes_per_unit).decode()
