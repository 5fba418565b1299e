"""lsmdb_amd -- MI355X-native (gfx950) SST block codec for lsmdb.

Drop-in for the reference's SST block path (table/builder.go encode, table/iterator.go +
table/table.go decode).  Layout:
  csrc/        HIP kernels (decode.hip, encode.hip) + the C ABI (api.hip, include/lsmgpu.h)
  _lib.py      ctypes binding of the C ABI (fails loudly if liblsmgpu.so is missing)
  codec.py     Codec: host-buffer and device-resident batch calls
  table.py     host mirror of the Go `table` package (Builder, OpenTable, Iterator, ...)
  y.py         ValueStruct codec, key helpers, MergeIterator (the Go `y` helpers)
  bloom.py     bbloom-shaped bloom tail (hash parity unpinned)
"""
__version__ = "0.1.0"

__all__ = ["codec", "table", "y", "bloom"]
