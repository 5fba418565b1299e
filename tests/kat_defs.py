"""Known-answer tests hand-derived from the reference source (NOT produced by the oracle).

Each expected byte string is written from the Go code by hand (struct.pack restatements of
table/builder.go:23-45,84-160 and y/iterator.go:48-62), so these pin the oracle and the GPU
path independently of either.
"""
from __future__ import annotations

import struct

FF8 = b"\xff" * 8  # KeyWithTs(k, 0): BE64(MaxUint64 - 0) (y/y.go:68-73)


def hdr(plen: int, klen: int, vlen: int, prev: int) -> bytes:
    """header.Encode (builder.go:30-35)"""
    return struct.pack(">HHHI", plen, klen, vlen, prev)


TERM_VS = b"\x00\x00\x00"  # ValueStruct{}.EncodeTo: meta 0, usermeta 0, uvarint(0)
NOPREV = 0xFFFFFFFF

# ---------------------------------------------------------------- builder KATs
# TestConcatIteratorOneTable's table: {"k1":"a1","k2":"a2"}, Meta 'A' (table_test.go:326-346)
K1, K2 = b"k1" + FF8, b"k2" + FF8
V1, V2 = b"A\x00\x00a1", b"A\x00\x00a2"
TWO_ENTRY_DATA = (hdr(0, 10, 5, NOPREV) + K1 + V1 +
                  hdr(0, 10, 5, 0) + K2 + V2 +
                  hdr(0, 0, 3, 25) + TERM_VS)
TWO_ENTRY_INDEX = struct.pack(">II", 63, 1)
assert len(TWO_ENTRY_DATA) == 63
assert TWO_ENTRY_DATA.hex() == (
    "0000000a0005ffffffff" "6b31ffffffffffffffff" "4100006131"
    "0000000a000500000000" "6b32ffffffffffffffff" "4100006132"
    "00000000000300000019" "000000")

# buildTable(t, [][]string{}) (table_test.go:514): one terminator-only block
EMPTY_DATA = hdr(0, 0, 3, NOPREV) + TERM_VS
EMPTY_INDEX = struct.pack(">II", 13, 1)

# resultInterval = 2, three entries "key0000".."key0002" -> "0".."2": cut before entry 2
_K = [b"key%04d" % i + FF8 for i in range(3)]
_V = [b"A\x00\x00" + (b"%d" % i) for i in range(3)]
CUT_DATA = (hdr(0, 15, 4, NOPREV) + _K[0] + _V[0] +
            hdr(0, 15, 4, 0) + _K[1] + _V[1] +
            hdr(0, 0, 3, 29) + TERM_VS +              # block 0 ends at 71
            hdr(0, 15, 4, NOPREV) + _K[2] + _V[2] +
            hdr(0, 0, 3, 0) + TERM_VS)               # block 1 ends at 113
CUT_INDEX = struct.pack(">III", 71, 113, 2)
CUT_KEYS, CUT_VS = _K, _V
assert len(CUT_DATA) == 113

BUILDER_KATS = [
    # (name, keys, vs, entries_per_block, expected data, expected index)
    ("two_entry", [K1, K2], [V1, V2], 100, TWO_ENTRY_DATA, TWO_ENTRY_INDEX),
    ("empty", [], [], 100, EMPTY_DATA, EMPTY_INDEX),
    ("cut_every_2", CUT_KEYS, CUT_VS, 2, CUT_DATA, CUT_INDEX),
    ("cut_exact_multiple", CUT_KEYS[:2], CUT_VS[:2], 2,
     CUT_DATA[:71], struct.pack(">II", 71, 1)),  # Finish does not open a new block
]

# ---------------------------------------------------------------- ValueStruct KATs
# (meta, user_meta, expires_at, value, expected encoding, EncodedSize)
VS_KATS = [
    (0x41, 0, 0, b"a1", b"A\x00\x00a1", 5),
    (0x41, 7, 1, b"", b"A\x07\x01", 3),
    (0, 0, 127, b"x", b"\x00\x00\x7fx", 4),
    (0, 0, 128, b"x", b"\x00\x00\x80\x01x", 5),
    (0, 0, 300, b"", b"\x00\x00\xac\x02", 4),
    (1, 2, 1 << 63, b"v", b"\x01\x02" + b"\x80" * 9 + b"\x01" + b"v", 13),
    (1, 2, (1 << 64) - 1, b"", b"\x01\x02" + b"\xff" * 9 + b"\x01", 12),
    (0x41, 0, 0, b"z" * 70000, None, (70000 + 3) & 0xFFFF),  # uint16 truncation (F7)
]

# ---------------------------------------------------------------- decode KATs
# hand-built blocks -> (expected [(key, value)], expected status); statuses as include/lsmgpu.h
OK, VALUE_OVERFLOW, FIRST_PLEN, TRUNC_HEADER, PREFIX_OOB = 0, 1, 2, 3, 4

_base = b"abcdefghij"
PLEN_BLOCK = (hdr(0, 10, 2, NOPREV) + _base + b"V0" +         # key abcdefghij
              hdr(4, 3, 2, 0) + b"xyz" + b"V1" +               # baseKey[:4] ++ xyz
              hdr(12, 0, 1, 22) + b"Z" +                       # baseKey[:12]: cap semantics
              hdr(0, 0, 3, 37) + TERM_VS)
DECODE_KATS = [
    ("prefix_compressed", PLEN_BLOCK,
     [(b"abcdefghij", b"V0"), (b"abcdxyz", b"V1"), (b"abcdefghijV0", b"Z")], OK),
    ("two_entry", TWO_ENTRY_DATA, [(K1, V1), (K2, V2)], OK),
    ("empty_table_block", EMPTY_DATA, [], OK),
    ("zero_length_block", b"", [], OK),
    ("no_terminator", hdr(0, 10, 5, NOPREV) + K1 + V1, [(K1, V1)], OK),
    ("value_overflow", hdr(0, 10, 5, NOPREV) + K1 + V1 + hdr(0, 10, 50, 0) + K2 + V2,
     [(K1, V1)], VALUE_OVERFLOW),
    ("key_overrun", hdr(0, 10, 5, NOPREV) + K1 + V1 + hdr(0, 200, 0, 0) + K2,
     [(K1, V1)], VALUE_OVERFLOW),
    ("first_plen_nonzero", hdr(3, 10, 5, NOPREV) + K1 + V1, [], FIRST_PLEN),
    ("truncated_header", hdr(0, 10, 5, NOPREV) + K1 + V1 + b"\x00\x00\x00\x0a\x00", [(K1, V1)],
     TRUNC_HEADER),
    ("prefix_oob", hdr(0, 10, 5, NOPREV) + K1 + V1 + hdr(200, 1, 1, 0) + b"q" + b"r",
     [(K1, V1)], PREFIX_OOB),
    ("zero_vlen", hdr(0, 10, 0, NOPREV) + K1 + hdr(0, 10, 0, 0) + K2 + hdr(0, 0, 3, 20) + TERM_VS,
     [(K1, b""), (K2, b"")], OK),
]
