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
