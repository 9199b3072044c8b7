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

import contextlib
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
_diag: Optional[ctypes.CDLL] = None
_active_diag = False  # wrappers route to the diagnostics library (diagnostics())

# C signatures (include/nova_crc32c.h).  The product library exports _SIG; the
# diagnostics build (libnova_crc32c_diag.so) exports _SIG and _DIAG_SIG.
_u32, _u64, _sz, _vp, _i32 = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p,
                              ctypes.c_int)
_pu64 = ctypes.POINTER(ctypes.c_uint64)
_SIG = {
    "nova_crc32c_extend": (_u32, [_u32, ctypes.c_char_p, _sz]),
    "nova_crc32c_value": (_u32, [ctypes.c_char_p, _sz]),
    "nova_crc32c_mask": (_u32, [_u32]),
    "nova_crc32c_unmask": (_u32, [_u32]),
    "nova_crc32c_combine": (_u32, [_u32, _u32, _u64]),
    "nova_port_accelerated_crc32c": (_u32, [_u32, ctypes.c_char_p, _sz]),
    "nova_port_stats": (None, [_pu64, _pu64, _pu64]),
    "nova_host_staging_release": (None, []),
    "nova_crc32c_batch": (_i32, [_vp, _vp, _vp, _vp, _vp, _sz, _u32, _vp]),
    "nova_crc32c_batch_strided": (_i32, [_vp, _u64, _u32, _sz, _vp, _vp, _u32, _vp]),
    "nova_sstable_write_trailers": (_i32, [_vp, _vp, _vp, _sz, _u32, _vp]),
    "nova_sstable_verify_blocks": (_i32, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "nova_sstable_verify_blocks_ex": (_i32, [_vp, _vp, _vp, _sz, _vp, _vp, _u32, _vp]),
    "nova_sst_queue_write_trailers": (_i32, [_vp, _vp, _vp, _sz, _u32, _vp]),
    "nova_sst_queue_verify_blocks": (_i32, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "nova_sst_queue_stats": (_i32, [_vp, _vp, _vp]),
    "nova_sst_queue_set_slots": (_i32, [ctypes.c_int]),
    "nova_sst_queue_hold": (_i32, [ctypes.c_int, _vp]),
    "nova_sst_engine_start": (_i32, []),
    "nova_sst_engine_stop": (_i32, []),
    "nova_sst_engine_stats": (_i32, [_vp, _vp, _vp, _vp]),
    "nova_sst_engine_set_idle_us": (_i32, [_u32]),
    "nova_sst_engine_set_enabled": (_i32, [ctypes.c_int]),
    "nova_sst_engine_set_trace": (_i32, [ctypes.c_int]),
    "nova_sst_engine_trace_stats": (_i32, [_vp, _vp]),
    "nova_sst_engine_trace_detail": (_i32, [_vp, _vp]),
    "nova_sst_engine_counters": (_i32, [_vp, _sz]),
    "nova_sst_engine_set_timeout_ms": (_i32, [_u32]),
    "nova_sst_engine_set_slice_us": (_i32, [_u32]),
    "nova_sst_engine_yield": (_i32, [_vp]),
    "nova_sst_engine_reset": (_i32, []),
    "nova_sst_engine_set_wait_delay_us": (None, [_u32]),
    "nova_sst_engine_set_give_up_us": (_i32, [_u32]),
    "nova_sst_engine_set_drop_chunks": (_i32, [_u32]),
    "nova_crc32c_stream_host": (_i32, [_vp, _u64, _u32, _sz, _vp, _u32, _sz, _i32]),
    "nova_crc32c_batch_host": (_i32, [_vp, _vp, _vp, _vp, _vp, _sz, _u32, _sz, _i32]),
    "nova_sstable_write_trailers_host": (_i32, [_vp, _vp, _vp, _sz, _u32, _sz, _i32]),
    "nova_sstable_verify_blocks_host": (_i32, [_vp, _vp, _vp, _sz, _vp, _vp, _sz, _i32]),
    "nova_log_write_crcs": (_i32, [_vp, _sz, _vp, _sz, _vp]),
    "nova_log_verify_records": (_i32, [_vp, _sz, _vp, _sz, _vp, _vp, _vp]),
    "nova_xor_parity": (_i32, [_vp, _vp, _sz, _sz, _vp, _vp]),
    "nova_fill_splitmix64": (_i32, [_vp, _sz, _u64, _u64, _vp]),
    "nova_device_init": (_i32, []),
    "nova_stream_release": (_i32, [_vp]),
    "nova_stream_slots": (_sz, []),
    "nova_crc32c_plan": (_i32, [_sz, _u64, ctypes.POINTER(_i32), ctypes.POINTER(_u32)]),
    "nova_crc32c_kernel_name": (ctypes.c_char_p, [_i32]),
    "nova_crc32c_describe": (_i32, [_sz, _u64, _u64, _i32, ctypes.c_char_p, _sz]),
    "nova_crc32c_set_tuning": (None, [_i32, _u32]),
    "nova_error_string": (ctypes.c_char_p, [_i32]),
    "nova_crc32c_abi_version": (_i32, []),
}
_DIAG_SIG = {
    "nova_diag_set_variant": (None, [_i32]),
    "nova_diag_set_stamps": (None, [_vp]),
    "nova_diag_set_static_pct": (None, [_i32]),
    "nova_diag_set_blocks_per_group": (None, [_i32]),
    "nova_diag_set_chunk_blocks": (None, [_i32]),
    "nova_diag_set_stream_waves": (None, [_i32]),
    "nova_diag_set_variable_kernel": (None, [_i32]),
    "nova_diag_set_parity_variant": (None, [_i32]),
    "nova_diag_set_rounds_sort": (None, [_i32]),
    "nova_diag_set_log_window": (None, [_i32]),
    "nova_diag_set_log_key": (None, [_i32]),
    "nova_diag_host_extend_loop": (_u32, [_vp, _sz, ctypes.c_uint64]),
    "nova_diag_lane_xor_probe": (_i32, [_vp, _vp, _vp, _vp]),
    "nova_diag_copy_ceiling": (_i32, [_vp, _vp, _sz, _vp, _vp, _i32, _i32, _vp]),
    "nova_diag_set_trailer_single_pass": (None, [_i32]),
    "nova_diag_set_burst_lanes": (None, [_i32]),
    "nova_diag_set_split": (None, [_i32]),
    "nova_diag_read_stream": (_i32, [_vp, _sz, _vp, _i32, _vp]),
    "nova_diag_log_field_scatter": (_i32, [_vp, _vp, _u64, _vp]),
    "nova_diag_read_ceiling": (_i32, [_vp, _sz, _vp, _i32, _i32, _vp]),
    "nova_diag_hold_cus": (_i32, [_u32, _vp]),
    "nova_diag_engine_groups": (_i32, [_u32, _u64, _u64, _vp]),
}
ABI_VERSION = 4

# log verify status codes (include/nova_crc32c.h, db/log_reader.cc:228-262)
LOG_CHECKSUM_MISMATCH = 0
LOG_OK = 1
LOG_BAD_LENGTH = 2
LOG_ZERO_RECORD = 3
LOG_TRUNCATED = 4
LOG_BLOCK_TRAILER = 5  # < 7 bytes left in a full block: skipped, not reported


def lib_path() -> str:
    return _build.LIB


def _open(path: str, sig: dict, optional: tuple = ()) -> ctypes.CDLL:
    """Bind `sig`; a name in `optional` (diagnostics entry points) may be
    absent -- an older diagnostics build in an A/B -- and then fails when used."""
    L = ctypes.CDLL(path)
    for name, (res, args) in sig.items():
        if name in optional and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.nova_crc32c_abi_version() != ABI_VERSION:
        raise ImportError(f"{path}: ABI {L.nova_crc32c_abi_version()} != {ABI_VERSION} (rebuild)")
    return L


def load(build_if_missing: bool = False) -> ctypes.CDLL:
    """The in-tree product library (never a site-packages copy)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        if not build_if_missing:
            raise ImportError(f"native library missing: {path} (run __graft_entry__.build())")
        _build.build()
    _lib = _open(path, _SIG)
    return _lib


def load_diag() -> ctypes.CDLL:
    """The diagnostics build (tools/ and tuning tests only: it can compute wrong
    CRCs on purpose, see include/nova_crc32c.h)."""
    global _diag
    if _diag is None:
        if not os.path.exists(_build.DIAG_LIB):
            raise ImportError(f"diagnostics library missing: {_build.DIAG_LIB}")
        _diag = _open(_build.DIAG_LIB, {**_SIG, **_DIAG_SIG}, tuple(_DIAG_SIG))
    return _diag


def _L() -> ctypes.CDLL:
    return load_diag() if _active_diag else load()


def enable_diagnostics() -> ctypes.CDLL:
    """For tools/: route every wrapper to the diagnostics library from now on."""
    global _active_diag
    D = load_diag()
    _active_diag = True
    return D


@contextlib.contextmanager
def diagnostics():
    """Route this module's wrappers to the diagnostics library inside the block
    (its nova_diag_* knobs are per calling thread); yields that library.  The
    knobs and the tuning are reset on exit."""
    global _active_diag
    D = load_diag()
    prev = _active_diag
    _active_diag = True
    try:
        yield D
    finally:
        _active_diag = prev
        D.nova_crc32c_set_tuning(0, 0)
        D.nova_diag_set_variant(0)
        D.nova_diag_set_static_pct(-1)
        D.nova_diag_set_blocks_per_group(0)
        D.nova_diag_set_chunk_blocks(0)
        D.nova_diag_set_stream_waves(0)
        D.nova_diag_set_variable_kernel(0)
        D.nova_diag_set_rounds_sort(2)
        D.nova_diag_set_log_window(0)
        D.nova_diag_set_log_key(0)
        D.nova_diag_set_trailer_single_pass(0)
        D.nova_diag_set_parity_variant(0)
        D.nova_diag_set_burst_lanes(0)
        D.nova_diag_set_split(0)


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _L().nova_error_string(rc).decode()
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
    return _L().nova_crc32c_extend(init_crc & 0xFFFFFFFF, b, n)


def Value(data, n: Optional[int] = None) -> int:
    return Extend(0, data, n)


def Mask(crc: int) -> int:
    return _L().nova_crc32c_mask(crc & 0xFFFFFFFF)


def Unmask(masked_crc: int) -> int:
    return _L().nova_crc32c_unmask(masked_crc & 0xFFFFFFFF)


def Combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return _L().nova_crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)


def AcceleratedCRC32C(crc: int, data) -> int:
    """port::AcceleratedCRC32C (port/port_stdcxx.h:179-189): the GPU for large
    buffers, the host Extend below NOVA_HOOK_MIN_BYTES and on any GPU failure."""
    b = _bytes(data)
    return _L().nova_port_accelerated_crc32c(crc & 0xFFFFFFFF, b, len(b))


def port_stats() -> dict:
    h, d, f = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    _L().nova_port_stats(ctypes.byref(h), ctypes.byref(d), ctypes.byref(f))
    return {"host": h.value, "device": d.value, "fallback": f.value}


# ---- device batches -------------------------------------------------------
# Every tensor argument is checked before its pointer reaches the C-ABI: the
# kernels read descriptors as raw u64/u32 arrays and data as bytes, so a wrong
# dtype, a non-contiguous view or a tensor on another device would be read
# silently as garbage.

def _stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _u64_dtypes():
    import torch
    return tuple(d for d in (torch.int64, getattr(torch, "uint64", None)) if d is not None)


def _u32_dtypes():
    import torch
    return tuple(d for d in (torch.int32, getattr(torch, "uint32", None)) if d is not None)


def _arg(t, name: str, dtypes, device=None, min_numel: int = 0) -> Optional[int]:
    """Pointer of a checked tensor argument (None passes through as NULL)."""
    if t is None:
        return None
    if not getattr(t, "is_cuda", False):
        raise NovaError(f"{name}: device batch expects GPU tensors (no CPU fallback on this path)")
    if t.dtype not in dtypes:
        raise NovaError(f"{name}: dtype {t.dtype} not in {[str(d) for d in dtypes]}")
    if not t.is_contiguous():
        raise NovaError(f"{name}: must be contiguous")
    if device is not None and t.device != device:
        raise NovaError(f"{name}: on {t.device}, data is on {device}")
    if t.numel() < min_numel:
        raise NovaError(f"{name}: {t.numel()} elements, need {min_numel}")
    return int(t.data_ptr())


def _data(t, name: str = "data") -> int:
    import torch
    return _arg(t, name, (torch.uint8,))


def _require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise NovaError("no GPU available: the batched CRC32C path runs only on the HIP device")


def batch(data, offsets, lengths, init=None, flags: int = 0, out=None, stream=None):
    """Variable-length batch (nova_crc32c_batch). data: uint8 GPU tensor;
    offsets: int64/uint64; lengths, init, out: int32/uint32 (same device)."""
    import torch
    _require_gpu()
    n = int(offsets.numel())
    if lengths.numel() != n:
        raise NovaError("offsets/lengths size mismatch")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=data.device)
    dv, u32, u64 = data.device, _u32_dtypes(), _u64_dtypes()
    rc = _L().nova_crc32c_batch(_data(data), _arg(offsets, "offsets", u64, dv),
                                _arg(lengths, "lengths", u32, dv),
                                _arg(init, "init", u32, dv, n), _arg(out, "out", u32, dv, n), n,
                                flags, _stream_ptr(stream))
    _check(rc, "nova_crc32c_batch")
    return out


def batch_strided(data, stride: int, length: int, n_blocks: int, init=None, flags: int = 0,
                  out=None, stream=None, base_offset: int = 0):
    import torch
    _require_gpu()
    ptr = _data(data)
    if n_blocks and base_offset + (n_blocks - 1) * stride + length > data.numel():
        raise NovaError("blocks exceed the data tensor")
    if out is None:
        out = torch.empty(n_blocks, dtype=torch.int32, device=data.device)
    dv, u32 = data.device, _u32_dtypes()
    rc = _L().nova_crc32c_batch_strided(ptr + base_offset, stride, length, n_blocks,
                                        _arg(init, "init", u32, dv, n_blocks),
                                        _arg(out, "out", u32, dv, n_blocks), flags,
                                        _stream_ptr(stream))
    _check(rc, "nova_crc32c_batch_strided")
    return out


def write_trailers(buf, offsets, sizes, type_byte: int = 0, tb_quirk: bool = False, stream=None,
                   hint_large: bool = False):
    _require_gpu()
    if sizes.numel() != offsets.numel():
        raise NovaError("offsets/sizes size mismatch")
    flags = TYPE(type_byte) | (TB_QUIRK if tb_quirk else 0) | (HINT_LARGE_BLOCKS if hint_large else 0)
    dv = buf.device
    rc = _L().nova_sstable_write_trailers(_data(buf, "buf"), _arg(offsets, "offsets", _u64_dtypes(), dv),
                                          _arg(sizes, "sizes", _u32_dtypes(), dv),
                                          int(offsets.numel()), flags, _stream_ptr(stream))
    _check(rc, "nova_sstable_write_trailers")
    return buf


def verify_blocks(buf, offsets, sizes, stream=None, ok=None, bad=None, hint_large: bool = False):
    """Returns (ok uint8 tensor, n_bad int32 tensor[1]).  A caller-supplied
    `bad` accumulates (zero it first).  hint_large: NOVA_CRC32C_HINT_LARGE_BLOCKS
    (nova_sstable_verify_blocks_ex)."""
    import torch
    _require_gpu()
    n = int(offsets.numel())
    if sizes.numel() != n:
        raise NovaError("offsets/sizes size mismatch")
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=buf.device)
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=buf.device)
    dv = buf.device
    args = (_data(buf, "buf"), _arg(offsets, "offsets", _u64_dtypes(), dv),
            _arg(sizes, "sizes", _u32_dtypes(), dv), n, _arg(ok, "ok", (torch.uint8,), dv, n),
            _arg(bad, "bad", _u32_dtypes(), dv, 1))
    if hint_large:
        rc = _L().nova_sstable_verify_blocks_ex(*args, HINT_LARGE_BLOCKS, _stream_ptr(stream))
    else:
        rc = _L().nova_sstable_verify_blocks(*args, _stream_ptr(stream))
    _check(rc, "nova_sstable_verify_blocks")
    return ok, bad


def queue_write_trailers(buf, offsets, sizes, type_byte: int = 0, tb_quirk: bool = False, stream=None):
    """nova_sst_queue_write_trailers: write_trailers through the coalescing
    queue (host-synchronous; concurrent callers share launches)."""
    _require_gpu()
    if sizes.numel() != offsets.numel():
        raise NovaError("offsets/sizes size mismatch")
    flags = TYPE(type_byte) | (TB_QUIRK if tb_quirk else 0)
    dv = buf.device
    rc = _L().nova_sst_queue_write_trailers(_data(buf, "buf"), _arg(offsets, "offsets", _u64_dtypes(), dv),
                                            _arg(sizes, "sizes", _u32_dtypes(), dv),
                                            int(offsets.numel()), flags, _stream_ptr(stream))
    _check(rc, "nova_sst_queue_write_trailers")
    return buf


def queue_verify_blocks(buf, offsets, sizes, ok, bad=None, stream=None):
    """nova_sst_queue_verify_blocks: verify_blocks through the coalescing
    queue (host-synchronous).  `bad` accumulates (zero it first)."""
    import torch
    _require_gpu()
    n = int(offsets.numel())
    if sizes.numel() != n:
        raise NovaError("offsets/sizes size mismatch")
    dv = buf.device
    rc = _L().nova_sst_queue_verify_blocks(_data(buf, "buf"), _arg(offsets, "offsets", _u64_dtypes(), dv),
                                           _arg(sizes, "sizes", _u32_dtypes(), dv), n,
                                           _arg(ok, "ok", (torch.uint8,), dv, n),
                                           _arg(bad, "bad", _u32_dtypes(), dv, 1), _stream_ptr(stream))
    _check(rc, "nova_sst_queue_verify_blocks")
    return ok, bad


def queue_set_slots(slots: int) -> None:
    """Batches the coalescing queue keeps in flight on this device (1..4; 0:
    NOVA_SST_QUEUE_SLOTS or the default 4)."""
    _check(_L().nova_sst_queue_set_slots(int(slots)), "nova_sst_queue_set_slots")


def queue_hold(hold: int) -> int:
    """Test hook: 1 holds the coalescing queue (no queued request leads a
    batch), 0 releases it, -1 only reads; returns the requests waiting."""
    v = ctypes.c_uint64(0)
    _check(_L().nova_sst_queue_hold(int(hold), ctypes.byref(v)), "nova_sst_queue_hold")
    return int(v.value)


def queue_stats() -> dict:
    v = [ctypes.c_uint64(0) for _ in range(3)]
    _check(_L().nova_sst_queue_stats(*[ctypes.byref(x) for x in v]), "nova_sst_queue_stats")
    return {"batches": v[0].value, "requests": v[1].value, "max_tables": v[2].value}


def engine_start() -> None:
    """Start the persistent per-SSTable engine now (queue_* calls start it too)."""
    _check(_L().nova_sst_engine_start(), "nova_sst_engine_start")


def engine_stop() -> None:
    """Stop the engine (requests in flight finish first; the next queue_* call
    starts it again)."""
    _check(_L().nova_sst_engine_stop(), "nova_sst_engine_stop")


def engine_stats() -> dict:
    v = [ctypes.c_uint64(0) for _ in range(3)]
    run = ctypes.c_int(0)
    _check(_L().nova_sst_engine_stats(*[ctypes.byref(x) for x in v], ctypes.byref(run)),
           "nova_sst_engine_stats")
    return {"requests": v[0].value, "launches": v[1].value, "fallbacks": v[2].value,
            "running": bool(run.value)}


ENGINE_COUNTERS = ("requests", "launches", "fallbacks", "running", "exits_idle", "exits_yield",
                   "exits_stop", "exits_lost", "timeouts", "errors", "taken_back", "unsafe",
                   "yield_waits", "yield_bumps", "broken", "backing_off", "exits_slice", "launch_us_max",
                   "launch_slow", "poll_gap_us_max", "sleep_waits", "max_spinners",
                   "ring_device", "host_marked_done", "waves", "storm_declined")


def engine_counters() -> dict:
    """nova_sst_engine_counters: the engine's lifetime counters (include/nova_crc32c.h)."""
    v = (ctypes.c_uint64 * len(ENGINE_COUNTERS))()
    _check(_L().nova_sst_engine_counters(v, len(ENGINE_COUNTERS)), "nova_sst_engine_counters")
    return dict(zip(ENGINE_COUNTERS, [int(x) for x in v]))


def engine_set_slice_us(us: int) -> None:
    """Engine instance time slice in us from the next instance (0: the
    NOVA_SST_ENGINE_SLICE_US default; None: no slice)."""
    v = 0xFFFFFFFF if us is None else int(us)
    _check(_L().nova_sst_engine_set_slice_us(v), "nova_sst_engine_set_slice_us")


def engine_set_timeout_ms(ms: int) -> None:
    """Host timeout of one engine request (0: NOVA_SST_ENGINE_TIMEOUT_MS)."""
    _check(_L().nova_sst_engine_set_timeout_ms(int(ms)), "nova_sst_engine_set_timeout_ms")


def engine_yield(stream=None) -> None:
    """Make the resident engine yield to work enqueued on `stream` (kernels of
    other libraries)."""
    _check(_L().nova_sst_engine_yield(_stream_ptr(stream)), "nova_sst_engine_yield")


def engine_reset() -> None:
    """End an engine backoff now."""
    _check(_L().nova_sst_engine_reset(), "nova_sst_engine_reset")


def engine_set_wait_delay_us(us: int) -> None:
    """Test hook (calling thread): start waiting for a submitted request `us` late."""
    _L().nova_sst_engine_set_wait_delay_us(int(us))


def engine_set_give_up_us(us: int) -> None:
    """Test hook: the engine's give-up time in us from the next instance (0:
    the default 20 s); a dispatcher with a request unfinished that long after
    the last arrival exits "lost"."""
    _check(_L().nova_sst_engine_set_give_up_us(int(us)), "nova_sst_engine_set_give_up_us")


def engine_set_drop_chunks(on: bool) -> None:
    """Test hook: from the next instance the engine's workers run no chunk, so
    with a short give-up time an instance ends "lost" with the requests it took
    unfinished."""
    _check(_L().nova_sst_engine_set_drop_chunks(1 if on else 0), "nova_sst_engine_set_drop_chunks")


def engine_set_enabled(on: int) -> None:
    """Route queue_* calls: 1 the persistent engine, 0 the coalescing queue,
    -1 the NOVA_SST_ENGINE default."""
    _check(_L().nova_sst_engine_set_enabled(int(on)), "nova_sst_engine_set_enabled")


def engine_set_idle_us(us: int) -> None:
    """Idle time before an engine instance exits (from the next instance)."""
    _check(_L().nova_sst_engine_set_idle_us(int(us)), "nova_sst_engine_set_idle_us")


def log_write_crcs(buf, record_offsets, stream=None, buf_len: Optional[int] = None):
    """db/log_writer.cc:99-114 for every record header at record_offsets (in
    place).  buf is a log image from a 32 KiB block boundary; buf_len defaults
    to its size."""
    _require_gpu()
    bl = int(buf.numel()) if buf_len is None else int(buf_len)
    if bl > buf.numel():
        raise NovaError("buf_len exceeds the buffer")
    rc = _L().nova_log_write_crcs(_data(buf, "buf"), bl,
                                  _arg(record_offsets, "record_offsets", _u64_dtypes(), buf.device),
                                  int(record_offsets.numel()), _stream_ptr(stream))
    _check(rc, "nova_log_write_crcs")
    return buf


def log_verify_records(buf, record_offsets, stream=None, ok=None, bad=None,
                       buf_len: Optional[int] = None):
    """db/log_reader.cc:196-262 per record -> (status uint8 tensor of LOG_*,
    n_bad int32 tensor[1] counting CHECKSUM_MISMATCH and BAD_LENGTH; a header
    in a full block's last 1-6 bytes is LOG_BLOCK_TRAILER, one at/past the end
    of the file or cut by its last partial block LOG_TRUNCATED, neither counted)."""
    import torch
    _require_gpu()
    n = int(record_offsets.numel())
    bl = int(buf.numel()) if buf_len is None else int(buf_len)
    if bl > buf.numel():
        raise NovaError("buf_len exceeds the buffer")
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=buf.device)
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=buf.device)
    dv = buf.device
    rc = _L().nova_log_verify_records(_data(buf, "buf"), bl,
                                      _arg(record_offsets, "record_offsets", _u64_dtypes(), dv), n,
                                      _arg(ok, "ok", (torch.uint8,), dv, n),
                                      _arg(bad, "bad", _u32_dtypes(), dv, 1), _stream_ptr(stream))
    _check(rc, "nova_log_verify_records")
    return ok, bad


def xor_parity(buf, frag_offsets, parity_len: int, out=None, stream=None):
    """ltc/stoc_file_client_impl.cpp:334-349 XOR parity block over fragments."""
    import torch
    _require_gpu()
    if out is None:
        out = torch.empty(parity_len, dtype=torch.uint8, device=buf.device)
    dv = buf.device
    rc = _L().nova_xor_parity(_data(buf, "buf"), _arg(frag_offsets, "frag_offsets", _u64_dtypes(), dv),
                              int(frag_offsets.numel()), parity_len,
                              _arg(out, "out", (torch.uint8,), dv, parity_len), _stream_ptr(stream))
    _check(rc, "nova_xor_parity")
    return out


# ---- host-resident paths ----------------------------------------------------

def _host_ptr(x, name: str) -> int:
    """Pointer of a host buffer: a CPU torch tensor (pinned or not) or a
    numpy array; must be contiguous."""
    if hasattr(x, "data_ptr"):
        if getattr(x, "is_cuda", False):
            raise NovaError(f"{name}: host path expects host memory")
        if not x.is_contiguous():
            raise NovaError(f"{name}: must be contiguous")
        return int(x.data_ptr())
    if not x.flags["C_CONTIGUOUS"]:
        raise NovaError(f"{name}: must be contiguous")
    return int(x.ctypes.data)


def _np_desc(offsets, lengths):
    import numpy as np
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    if o.shape != ln.shape:
        raise NovaError("offsets/lengths size mismatch")
    return o, ln


def stream_host(host_u8, stride: int, length: int, n_blocks: int, flags: int = 0,
                chunk_blocks: int = 4096, n_streams: int = 3):
    """Host-resident fixed-stride blocks (pinned torch CPU tensor or numpy array) -> CRCs (numpy u32)."""
    import numpy as np
    _require_gpu()
    out = np.empty(n_blocks, dtype=np.uint32)
    rc = _L().nova_crc32c_stream_host(_host_ptr(host_u8, "host"), stride, length, n_blocks,
                                      int(out.ctypes.data), flags, chunk_blocks, n_streams)
    _check(rc, "nova_crc32c_stream_host")
    return out


def batch_host(host_u8, offsets, lengths, init=None, flags: int = 0, chunk_bytes: int = 0,
               n_streams: int = 3):
    """Variable-length blocks in host memory (nova_crc32c_batch_host) -> numpy u32."""
    import numpy as np
    _require_gpu()
    o, ln = _np_desc(offsets, lengths)
    ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    out = np.empty(len(o), dtype=np.uint32)
    rc = _L().nova_crc32c_batch_host(_host_ptr(host_u8, "host"), int(o.ctypes.data),
                                     int(ln.ctypes.data),
                                     None if ini is None else int(ini.ctypes.data),
                                     int(out.ctypes.data), len(o), flags, chunk_bytes, n_streams)
    _check(rc, "nova_crc32c_batch_host")
    return out


def write_trailers_host(host_u8, offsets, sizes, type_byte: int = 0, tb_quirk: bool = False,
                        chunk_bytes: int = 0, n_streams: int = 3):
    _require_gpu()
    o, ln = _np_desc(offsets, sizes)
    flags = TYPE(type_byte) | (TB_QUIRK if tb_quirk else 0)
    rc = _L().nova_sstable_write_trailers_host(_host_ptr(host_u8, "host"), int(o.ctypes.data),
                                               int(ln.ctypes.data), len(o), flags, chunk_bytes,
                                               n_streams)
    _check(rc, "nova_sstable_write_trailers_host")
    return host_u8


def verify_blocks_host(host_u8, offsets, sizes, chunk_bytes: int = 0, n_streams: int = 3):
    """-> (ok numpy u8, n_bad int)."""
    import numpy as np
    _require_gpu()
    o, ln = _np_desc(offsets, sizes)
    ok = np.empty(len(o), dtype=np.uint8)
    bad = ctypes.c_uint32(0)
    rc = _L().nova_sstable_verify_blocks_host(_host_ptr(host_u8, "host"), int(o.ctypes.data),
                                              int(ln.ctypes.data), len(o), int(ok.ctypes.data),
                                              ctypes.addressof(bad), chunk_bytes, n_streams)
    _check(rc, "nova_sstable_verify_blocks_host")
    return ok, bad.value


def fill_splitmix64(t, seed: int, first_word: int = 0, stream=None):
    _require_gpu()
    if not t.is_contiguous():
        raise NovaError("fill_splitmix64: tensor must be contiguous")
    ptr = _arg(t, "t", (t.dtype,))
    rc = _L().nova_fill_splitmix64(ptr, t.numel() * t.element_size(), seed, first_word,
                                   _stream_ptr(stream))
    _check(rc, "nova_fill_splitmix64")
    return t


def stream_release(stream) -> None:
    """nova_stream_release: drop the claim-counter slot of a torch stream that
    ran batches (before the stream goes away)."""
    _check(_L().nova_stream_release(int(stream.cuda_stream)), "nova_stream_release")


def stream_slots() -> int:
    return int(_L().nova_stream_slots())


def set_tuning(lanes_per_unit: int = 0, seg_bytes: int = 0) -> None:
    """Per calling thread (include/nova_crc32c.h)."""
    _L().nova_crc32c_set_tuning(lanes_per_unit, seg_bytes)


def plan(n_blocks: int, bytes_per_block: int):
    g = ctypes.c_int(0)
    s = ctypes.c_uint32(0)
    _L().nova_crc32c_plan(n_blocks, bytes_per_block, ctypes.byref(g), ctypes.byref(s))
    return g.value, s.value


def describe(n_blocks: int, length: int, stride: int, variable: bool = False,
             large: bool = False, log: bool = False, log_verify: bool = False) -> dict:
    """The product's plan for a batch (nova_crc32c_describe); log / log_verify:
    n_blocks log records of mean span `length` written / verified."""
    import json
    buf = ctypes.create_string_buffer(512)
    v = 4 if log_verify else 3 if log else ((2 if large else 1) if variable else 0)
    _L().nova_crc32c_describe(n_blocks, length, stride, v, buf, 512)
    return json.loads(buf.value.decode())


def kernel_name(lanes_per_unit: int) -> str:
    return _L().nova_crc32c_kernel_name(lanes_per_unit).decode()
