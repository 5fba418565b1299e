"""Host mirror of the reference's `y` helpers used on the SST path.

ValueStruct wire codec (y/iterator.go:11-62), key/timestamp conventions (y/y.go:67-107),
the y.Iterator protocol (y/iterator.go:64-72) and MergeIterator (y/iterator.go:74-227).
Names follow the Go API (snake_case aliases are provided for Python callers).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List, Optional, Protocol

MAX_U64 = (1 << 64) - 1


class AssertionFailed(AssertionError):
    """y.AssertTrue / AssertTruef (y/error.go:24-37) -- log.Fatal in Go, an exception here."""


def assert_true(cond: bool, msg: str = "assert failed") -> None:
    if not cond:
        raise AssertionFailed(msg)


def size_varint(x: int) -> int:
    """y/iterator.go:20-29"""
    n = 0
    while True:
        n += 1
        x >>= 7
        if x == 0:
            return n


def put_uvarint(x: int) -> bytes:
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def uvarint(b: bytes) -> tuple[int, int]:
    """encoding/binary.Uvarint: (value, n) with n == 0 (short) or n < 0 (overflow)."""
    x = 0
    s = 0
    for i, c in enumerate(b):
        if i == 10:
            return 0, -(i + 1)
        if c < 0x80:
            if i == 9 and c > 1:
                return 0, -(i + 1)
            return x | (c << s), i + 1
        x |= (c & 0x7F) << s
        s += 7
    return 0, 0


@dataclass
class ValueStruct:
    """y/iterator.go:11-18.  `version` is not serialised (internal only)."""
    meta: int = 0
    user_meta: int = 0
    expires_at: int = 0
    value: bytes = b""
    version: int = 0

    # Go-style accessors
    @property
    def Meta(self) -> int:  # noqa: N802
        return self.meta

    @property
    def Value(self) -> bytes:  # noqa: N802
        return self.value

    def encoded_size(self) -> int:
        """y/iterator.go:31-38 (uint16 result: silently truncated)."""
        sz = len(self.value) + 2
        if self.expires_at == 0:
            return (sz + 1) & 0xFFFF
        return (sz + size_varint(self.expires_at)) & 0xFFFF

    def full_encoded_size(self) -> int:
        """The number of bytes encode() writes (never truncated)."""
        return 2 + len(put_uvarint(self.expires_at)) + len(self.value)

    def encode(self) -> bytes:
        """y/iterator.go:48-62 Encode/EncodeTo"""
        return bytes((self.meta & 0xFF, self.user_meta & 0xFF)) + put_uvarint(self.expires_at) + bytes(self.value)

    @classmethod
    def decode(cls, b: bytes) -> "ValueStruct":
        """y/iterator.go:40-46 (a short buffer raises like Go's index panic)."""
        if len(b) < 2:
            raise IndexError("ValueStruct.Decode: buffer shorter than 2 bytes")
        x, n = uvarint(b[2:])
        # Go: ExpiresAt, sz = binary.Uvarint(b[2:]); Value = b[2+sz:] (sz<=0 keeps Go's slicing)
        if n <= 0:
            return cls(b[0], b[1], 0, bytes(b[2 + n:]) if 2 + n >= 0 else b"")
        return cls(b[0], b[1], x, bytes(b[2 + n:]))


# ------------------------------------------------------------------ y/y.go:67-107
def key_with_ts(key: bytes, ts: int) -> bytes:
    """y/y.go:67-73 KeyWithTs"""
    return bytes(key) + struct.pack(">Q", MAX_U64 - ts)


def parse_ts(key: bytes) -> int:
    """y/y.go:75-81"""
    if len(key) <= 8:
        return 0
    return MAX_U64 - struct.unpack(">Q", key[-8:])[0]


def _bytes_compare(a: bytes, b: bytes) -> int:
    return (a > b) - (a < b)


def compare_keys(key1: bytes, key2: bytes) -> int:
    """y/y.go:83-90 CompareKeys (asserts both keys carry an 8-byte ts suffix)."""
    assert_true(len(key1) > 8 and len(key2) > 8, "CompareKeys: key length <= 8")
    c = _bytes_compare(key1[:-8], key2[:-8])
    if c:
        return c
    return _bytes_compare(key1[-8:], key2[-8:])


def parse_key(key: Optional[bytes]) -> Optional[bytes]:
    """y/y.go:92-100 ParseKey"""
    if key is None:
        return None
    assert_true(len(key) > 8, f"key={key!r}")
    return key[:-8]


def same_key(src: bytes, dst: bytes) -> bool:
    """y/y.go:102-107"""
    if len(src) != len(dst):
        return False
    return parse_key(src) == parse_key(dst)


# Go-named aliases
KeyWithTs = key_with_ts
ParseTs = parse_ts
CompareKeys = compare_keys
ParseKey = parse_key
SameKey = same_key


class Iterator(Protocol):
    """y.Iterator (y/iterator.go:64-72)."""

    def Next(self) -> None: ...  # noqa: E704,N802
    def Rewind(self) -> None: ...  # noqa: E704,N802
    def Seek(self, key: bytes) -> None: ...  # noqa: E704,N802
    def Key(self) -> Optional[bytes]: ...  # noqa: E704,N802
    def Value(self) -> ValueStruct: ...  # noqa: E704,N802
    def Valid(self) -> bool: ...  # noqa: E704,N802
    def Close(self) -> None: ...  # noqa: E704,N802


class MergeIterator:
    """y/iterator.go:74-227: k-way merge; equal keys de-duplicated, lower index ("nice") wins.

    The Go version keeps a container/heap; since Less is a strict order on (key, nice) the
    observable sequence is the same as taking the minimum under Less each step.
    """

    def __init__(self, iters: List[Iterator], reversed: bool = False):
        self.all = list(iters)
        self.reversed = reversed
        self.h: List[int] = []  # indices of live iterators
        self.cur_key: Optional[bytes] = None
        self._init_heap()

    def _less(self, i: int, j: int) -> bool:
        cmp = compare_keys(self.all[i].Key(), self.all[j].Key())
        if cmp < 0:
            return not self.reversed
        if cmp > 0:
            return self.reversed
        return i < j

    def _top(self) -> Optional[int]:
        best = None
        for i in self.h:
            if best is None or self._less(i, best):
                best = i
        return best

    def _init_heap(self) -> None:
        self.h = [i for i, it in enumerate(self.all) if it.Valid()]
        t = self._top()
        self.cur_key = self.all[t].Key() if t is not None else None

    def Valid(self) -> bool:  # noqa: N802
        t = self._top()
        return t is not None and self.all[t].Valid()

    def Key(self) -> Optional[bytes]:  # noqa: N802
        t = self._top()
        return self.all[t].Key() if t is not None else None

    def Value(self) -> ValueStruct:  # noqa: N802
        t = self._top()
        return self.all[t].Value() if t is not None else ValueStruct()

    def Next(self) -> None:  # noqa: N802
        t = self._top()
        if t is None:
            return
        self.all[t].Next()
        while self.h:
            self.h = [i for i in self.h if self.all[i].Valid()]
            t = self._top()
            if t is None:
                break
            if self.all[t].Key() != self.cur_key:
                break
            self.all[t].Next()
        t = self._top()
        if t is None or not self.all[t].Valid():
            return
        self.cur_key = self.all[t].Key()

    def Rewind(self) -> None:  # noqa: N802
        for it in self.all:
            it.Rewind()
        self._init_heap()

    def Seek(self, key: bytes) -> None:  # noqa: N802
        for it in self.all:
            it.Seek(key)
        self._init_heap()

    def Close(self) -> None:  # noqa: N802
        for it in self.all:
            it.Close()


def NewMergeIterator(iters: List[Iterator], reversed: bool) -> MergeIterator:  # noqa: N802
    return MergeIterator(iters, reversed)
