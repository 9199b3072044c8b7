"""Synthetic SSTable-block data: the splitmix64 counter stream.

Word ``k`` of the stream seeded with ``seed`` is ``mix(seed + (k + 1) * GAMMA)``,
i.e. exactly the bytes a sequential splitmix64 generator started at ``seed``
emits (little-endian 8-byte words).  The same stream is produced on the device
by ``nova_fill_splitmix64`` (novalsm_amd/csrc/nova_crc32c_kernels.hip) so large
batches never need host initialisation, and by oracle/crc32c_oracle.c for the
checker.  BASELINE.md fixes the seeds: config 1 seed 1, config 2 seed 2, ...
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def splitmix64_words(seed: int, first_word: int, n_words: int) -> np.ndarray:
    k = np.arange(first_word + 1, first_word + 1 + n_words, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + k * GAMMA)


def splitmix64_bytes(seed: int, nbytes: int, first_byte: int = 0) -> np.ndarray:
    """``nbytes`` bytes of the stream starting at byte offset ``first_byte``."""
    w0 = first_byte // 8
    w1 = (first_byte + nbytes + 7) // 8
    words = splitmix64_words(seed, w0, max(0, w1 - w0))
    raw = words.view(np.uint8)
    s = first_byte - 8 * w0
    return raw[s:s + nbytes].copy()


# ---- log images -------------------------------------------------------------
LOG_BLOCK = 32768   # db/log_format.h:27 kBlockSize
LOG_HEADER = 7      # db/log_format.h:30 kHeaderSize
FULL, FIRST, MIDDLE, LAST = 1, 2, 3, 4  # db/log_format.h:14-24


def log_layout(payload_lens, block_offset: int = 0):
    """Physical layout of a log file written by log::Writer::AddRecord
    (db/log_writer.cc:53-97): logical records of the given payload sizes are
    cut into physical records [crc 4][len 2][type 1][payload] that never cross
    a 32 KiB block; a block remainder shorter than a header becomes a zero
    trailer.  Returns (offsets u64, lengths u32, types u8, trailer ranges
    [(start, end)], total bytes); offsets are from the file start, which sits
    block_offset bytes into its first block (Writer(dest, dest_length))."""
    offs, lens, types, pads = [], [], [], []
    pos = 0
    bo = block_offset % LOG_BLOCK
    for left in (int(x) for x in payload_lens):
        begin = True
        while True:
            leftover = LOG_BLOCK - bo
            if leftover < LOG_HEADER:  # :64-73 switch to a new block
                if leftover > 0:
                    pads.append((pos, pos + leftover))
                    pos += leftover
                bo = 0
            avail = LOG_BLOCK - bo - LOG_HEADER
            frag = min(left, avail)
            end = frag == left
            t = FULL if (begin and end) else FIRST if begin else LAST if end else MIDDLE
            offs.append(pos)
            lens.append(frag)
            types.append(t)
            pos += LOG_HEADER + frag
            bo += LOG_HEADER + frag
            left -= frag
            begin = False
            if left <= 0:  # an empty record still emits one zero-length fragment
                break
    return (np.array(offs, np.uint64), np.array(lens, np.uint32), np.array(types, np.uint8),
            pads, pos)


def log_image(seed: int, payload_lens, block_offset: int = 0):
    """A host log image over the layout above: splitmix64(seed) payload bytes,
    header length/type fields set, trailers zero, CRC fields NOT yet written.
    Returns (image u8, offsets, lengths, types)."""
    offs, lens, types, pads, total = log_layout(payload_lens, block_offset)
    img = splitmix64_bytes(seed, total)
    o = offs.astype(np.int64)
    img[o + 4] = (lens & 0xFF).astype(np.uint8)
    img[o + 5] = (lens >> 8).astype(np.uint8)
    img[o + 6] = types
    for a, b in pads:
        img[a:b] = 0
    return img, offs, lens, types


def big_string(partial: bytes, n: int) -> bytes:
    """BigString (db/log_test.cc:19-26): `partial` repeated, cut to n bytes."""
    reps = n // len(partial) + 1
    return (partial * reps)[:n]


def log_case_image(writes, mutations, crc_of):
    """The file a log::Writer leaves after AddRecord of each payload in
    `writes` (db/log_writer.cc:53-114: log_layout above, header CRC
    Mask(Value(type || payload)) from `crc_of(bytes) -> masked u32`), then the
    edits a reader test makes to it (db/log_test.cc:76-97):
      ("inc", offset, delta)   IncrementByte: byte += delta (mod 256)
      ("set", offset, value)   SetByte
      ("shrink", nbytes)       ShrinkSize: drop the file's last nbytes
      ("fixcrc", offset, len)  FixChecksum: the CRC of the header at offset
                               over its type byte and len payload bytes
    Returns (image u8, physical record offsets u64)."""
    offs, lens, types, pads, total = log_layout([len(w) for w in writes])
    img = np.zeros(total, np.uint8)
    k = 0
    for w in writes:  # the fragments of each logical record, in order
        done = 0
        while True:
            o, ln = int(offs[k]), int(lens[k])
            img[o + 4] = ln & 0xFF
            img[o + 5] = ln >> 8
            img[o + 6] = types[k]
            img[o + 7:o + 7 + ln] = np.frombuffer(w[done:done + ln], np.uint8)
            c = crc_of(bytes([int(types[k])]) + w[done:done + ln])
            img[o:o + 4] = np.frombuffer(int(c).to_bytes(4, "little"), np.uint8)
            done += ln
            k += 1
            if done >= len(w):
                break
    for m in mutations:
        if m[0] == "inc":
            img[m[1]] = (int(img[m[1]]) + m[2]) & 0xFF
        elif m[0] == "set":
            img[m[1]] = m[2] & 0xFF
        elif m[0] == "shrink":
            img = img[:img.size - m[1]].copy()
        elif m[0] == "fixcrc":
            o, ln = m[1], m[2]
            c = crc_of(img[o + 6:o + 7 + ln].tobytes())
            img[o:o + 4] = np.frombuffer(int(c).to_bytes(4, "little"), np.uint8)
        else:
            raise ValueError(m)
    return img, offs


def log_layout_fast(payload_lens):
    """log_layout(payload_lens) for a file starting at a block boundary, with the
    records that fit a block whole placed by one numpy step per 32 KiB block
    (log_layout walks them one by one: ~25 s for a 4 GiB image of 263-B
    records).  Same result (tests/test_host_api.py checks them equal)."""
    pl = np.asarray(payload_lens, dtype=np.int64)
    n = pl.size
    O, L, T, pads = [], [], [], []
    i, bo, pos = 0, 0, 0  # next logical record, offset in the block, block start
    rem, begin = 0, True
    win = 256
    while i < n:
        leftover = LOG_BLOCK - bo
        if leftover < LOG_HEADER:  # db/log_writer.cc:64-73
            if leftover > 0:
                pads.append((pos + bo, pos + LOG_BLOCK))
            pos += LOG_BLOCK
            bo = 0
            continue
        if not begin:  # the rest of record i: MIDDLE or LAST fragments
            frag = min(rem, LOG_BLOCK - bo - LOG_HEADER)
            end = frag == rem
            O.append(np.array([pos + bo], np.int64))
            L.append(np.array([frag], np.int64))
            T.append(np.array([LAST if end else MIDDLE], np.uint8))
            bo += LOG_HEADER + frag
            rem -= frag
            if end:
                i += 1
                begin = True
            continue
        # records i.. that fit this block whole: FULL
        while True:
            k = min(n - i, win)
            cs = np.cumsum(LOG_HEADER + pl[i:i + k])
            m = int(np.searchsorted(cs, leftover, side="right"))
            if m < k or i + k == n:
                break
            win *= 2
        if m:
            starts = cs[:m] - (LOG_HEADER + pl[i:i + m])
            O.append(pos + bo + starts)
            L.append(pl[i:i + m].copy())
            T.append(np.full(m, FULL, np.uint8))
            bo += int(cs[m - 1])
            i += m
            if m > 64:
                win = max(256, 2 * m)
            continue
        # record i begins here as a FIRST fragment (possibly empty)
        frag = leftover - LOG_HEADER
        O.append(np.array([pos + bo], np.int64))
        L.append(np.array([frag], np.int64))
        T.append(np.array([FIRST], np.uint8))
        bo += LOG_HEADER + frag
        rem = int(pl[i]) - frag
        begin = False
    total = pos + bo
    offs = np.concatenate(O).astype(np.uint64) if O else np.zeros(0, np.uint64)
    lens = np.concatenate(L).astype(np.uint32) if L else np.zeros(0, np.uint32)
    types = np.concatenate(T) if T else np.zeros(0, np.uint8)
    return offs, lens, types, pads, total
