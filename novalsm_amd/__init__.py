"""novalsm_amd -- MI355X-native batched CRC32C block-checksum engine.

Drop-in for NovaLSM's per-SSTable-block checksum path (util/crc32c.cc
crc32c::Extend/Value/Mask/Unmask and its callers table/table_builder.cc,
ltc/stoc_file_client_impl.cpp, table/table.cc).  The product is the C-ABI
library novalsm_amd/lib/libnova_crc32c.so (include/nova_crc32c.h); this package
is its Python mirror for tests and benchmarks.
"""
from . import crc32c  # noqa: F401
from .crc32c import (  # noqa: F401
    Extend, Value, Mask, Unmask, Combine, kMaskDelta, NovaError,
)

__all__ = ["crc32c", "Extend", "Value", "Mask", "Unmask", "Combine", "kMaskDelta",
           "NovaError"]
