"""Host mirror of the reference `table` package (table/builder.go, table.go, iterator.go).

The byte work runs on the GPU through the C ABI:
  * Builder.Finish      -> lsmgpu_encode_values + lsmgpu_encode_blocks (gfx950 encode kernel)
  * OpenTable           -> lsmgpu_parse_index + lsmgpu_decode_blocks   (gfx950 decode kernel)
What stays here is the reference's control logic, transliterated so the reference's own
tests (table/table_test.go) read the same: the Iterator / blockIterator state machines
become cursors over the decoded SoA batch, reproducing Go's observable behaviour (including
its seek, prev-chain and end-of-block rules).  There is no CPU decode fallback.
"""
from __future__ import annotations

import mmap
import os
import struct
from typing import List, Optional

import numpy as np

from . import bloom as _bloom
from .codec import Codec, HostDecoded, default_codec, parse_index
from .y import MAX_U64, ValueStruct, assert_true, compare_keys, parse_key

RESULT_INTERVAL = 100  # table/builder.go:13-15 resultInterval
# Finish's bloom tail: "all_ones" (default) = every bit set, so a Go reader's DoesNotHave never
# skips the table -- always correct, whatever bbloom's exact bytes are; "bbloom" = the restated
# bbloom filter built on the device (Builder(bloom="bbloom") or LSMDB_AMD_BLOOM=bbloom).  The
# restated bbloom bytes are parity unpinned (DESIGN.md "Bloom tail"), so the
# default stays all-ones until they are checked against Go.
BLOOM_BBLOOM = "bbloom"
BLOOM_ALL_ONES = "all_ones"
DEFAULT_BLOOM = os.environ.get("LSMDB_AMD_BLOOM", BLOOM_ALL_ONES)
MAX_U32 = 0xFFFFFFFF
FILE_SUFFIX = ".sst"

# options/options.go FileLoadingMode
FILE_IO = 0
LOAD_TO_RAM = 1
MEMORY_MAP = 2


class EOFError_(Exception):
    """io.EOF marker used by the iterator state machines."""


EOF = EOFError_("EOF")


class TableError(Exception):
    pass


# ================================================================== Builder (builder.go)
class Builder:
    """table.Builder (builder.go:47-198).  Entries are staged on the host; Finish() encodes
    every block on the GPU.  `Add` keeps Go's running sizes so ReachedCapacity/Empty answer
    exactly as the reference does at every point."""

    def __init__(self, entries_per_block: int = RESULT_INTERVAL, block_bytes: int = 0,
                 codec: Optional[Codec] = None, bloom: Optional[str] = None):
        self.bloom = bloom or DEFAULT_BLOOM
        if self.bloom not in (BLOOM_BBLOOM, BLOOM_ALL_ONES):
            raise ValueError(f"bloom must be {BLOOM_BBLOOM!r} or {BLOOM_ALL_ONES!r}")
        self.entries_per_block = entries_per_block
        self.block_bytes = block_bytes
        self._codec = codec
        self._keys: List[bytes] = []
        self._vals: List[ValueStruct] = []
        # Go-side running state (builder.go:47-59)
        self._counter = 0
        self._buf_len = 0
        self._base_offset = 0
        self._nrestarts = 0
        self._finished = False

    # builder.go:69,71
    def Close(self) -> None:  # noqa: N802
        pass

    def Empty(self) -> bool:  # noqa: N802
        return self._buf_len == 0

    def Add(self, key: bytes, value: ValueStruct) -> None:  # noqa: N802
        """builder.go:125-137.  Rejects (instead of corrupting) what Go cannot represent:
        len(key) <= 8 panics in y.ParseKey (y.go:98); an empty key would be written as a
        terminator; an encoded value > 65535 B is silently truncated by EncodedSize."""
        if self._finished:
            raise TableError("Add after Finish")
        key = bytes(key)
        assert_true(len(key) > 8, f"key={key!r}")  # y.ParseKey via addHelper (builder.go:88)
        if len(key) > 0xFFFF:
            raise ValueError("key longer than 65535 bytes (uint16 klen)")
        vlen = value.full_encoded_size()
        if vlen > 0xFFFF:
            raise ValueError("encoded value longer than 65535 bytes (uint16 vlen)")
        esz = 10 + len(key) + vlen
        cut = self.entries_per_block > 0 and self._counter >= self.entries_per_block
        if not cut and self.block_bytes > 0 and self._counter > 0:
            cut = (self._buf_len - self._base_offset) + esz + 13 > self.block_bytes
        if cut:  # finishBlock + restart (builder.go:126-134)
            self._buf_len += 13
            self._nrestarts += 1
            self._counter = 0
            self._base_offset = self._buf_len
        self._buf_len += esz
        self._counter += 1
        self._keys.append(key)
        self._vals.append(value)

    def ReachedCapacity(self, cap: int) -> bool:  # noqa: N802
        """builder.go:140-143"""
        estimate = self._buf_len + 8 + 4 * self._nrestarts + 8
        return estimate > cap

    def Finish(self) -> bytes:  # noqa: N802
        """builder.go:163-198: blocks + index on the GPU, then the bloom tail."""
        self._finished = True
        codec = self._codec or default_codec()
        n = len(self._keys)
        keys = b"".join(self._keys)
        key_end = np.cumsum([len(k) for k in self._keys], dtype=np.uint64).astype(np.uint32) \
            if n else np.zeros(0, np.uint32)
        if n:
            meta = np.fromiter((v.meta & 0xFF for v in self._vals), np.uint8, n)
            umeta = np.fromiter((v.user_meta & 0xFF for v in self._vals), np.uint8, n)
            exp = np.fromiter((v.expires_at for v in self._vals), np.uint64, n)
            vals = b"".join(bytes(v.value) for v in self._vals)
            val_end = np.cumsum([len(v.value) for v in self._vals], dtype=np.uint64).astype(np.uint32)
            vs, vs_end = codec.encode_values_host(meta, umeta, exp, vals, val_end)
        else:
            vs, vs_end = b"", np.zeros(0, np.uint32)
        body, _data_len, _restarts = codec.encode_host(keys, key_end, vs, vs_end,
                                                       self.entries_per_block, self.block_bytes)
        if self.bloom == BLOOM_ALL_ONES:
            bdata = _bloom.all_ones_json(n)
        else:
            bdata = codec.bloom_tail_host(keys, key_end)  # builder.go:164-181,189-195 (device)
        return body + bdata + struct.pack(">I", len(bdata))


def NewTableBuilder(entries_per_block: int = RESULT_INTERVAL) -> Builder:  # noqa: N802
    return Builder(entries_per_block)


# ================================================================== Table (table.go)
class _KeyOffset:
    __slots__ = ("key", "offset", "len", "fblk")

    def __init__(self, key: bytes, offset: int, ln: int, fblk: int):
        self.key, self.offset, self.len, self.fblk = key, offset, ln, fblk


class Table:
    """table.Table (table.go:31-47): the whole file is decoded on the GPU at open time."""

    def __init__(self):
        self.fd_name: Optional[str] = None
        self.table_size = 0
        self.block_index: List[_KeyOffset] = []
        self.ref = 1
        self.loading_mode = MEMORY_MAP
        self.raw: bytes = b""
        self.smallest: Optional[bytes] = None
        self.biggest: Optional[bytes] = None
        self.id = 0
        self.bloom_json = b""
        self._bloom = None  # (bitset, setLocs), parsed at open (table.go:186); None: Has = true
        self._bloom_dev = None  # the bitset on the device, uploaded at the first batch probe
        self._codec: Optional[Codec] = None
        self.dec: Optional[HostDecoded] = None
        self._owns_file = False

    # -- refcount (table.go:49-71): the file is deleted when the count drops to 0
    def IncrRef(self) -> None:  # noqa: N802
        self.ref += 1

    def DecrRef(self) -> None:  # noqa: N802
        self.ref -= 1
        if self.ref == 0 and self.fd_name and self._owns_file:
            try:
                os.remove(self.fd_name)
            except FileNotFoundError:
                pass

    def Close(self) -> None:  # noqa: N802
        pass

    def Size(self) -> int:  # noqa: N802
        return self.table_size

    def Smallest(self) -> Optional[bytes]:  # noqa: N802
        return self.smallest

    def Biggest(self) -> Optional[bytes]:  # noqa: N802
        return self.biggest

    def Filename(self) -> Optional[str]:  # noqa: N802
        return self.fd_name

    def ID(self) -> int:  # noqa: N802
        return self.id

    def DoesNotHave(self, key: bytes) -> bool:  # noqa: N802
        """table.go:301: !bf.Has(key) (key as the caller passes it: level_handler.go:221-224
        strips the ts first).  One key: hashed on the host, no device round trip -- it is
        Get's cheap skip, probed once per table per lookup."""
        if self._bloom is None:
            return False
        bitset, locs = self._bloom
        return not _bloom.has(bitset, locs, bytes(key))

    def DoesNotHaveBatch(self, keys) -> np.ndarray:  # noqa: N802
        """DoesNotHave for many keys in one device probe: bool array (True = not present).
        The filter is uploaded once per Table and probed in place."""
        keys = list(keys)
        if self._bloom is None:
            return np.zeros(len(keys), bool)
        bitset, locs = self._bloom
        codec = self._codec or default_codec()
        if self._bloom_dev is None:
            import torch
            self._bloom_dev = torch.from_numpy(bitset.view(np.int64).copy()).to(codec.device)
        return ~codec.bloom_has_cached(self._bloom_dev, locs, keys)

    def NewIterator(self, reversed: bool) -> "Iterator":  # noqa: N802
        return Iterator(self, reversed)

    # block(idx) (table.go:271-282) -> cursor over block idx of the sorted block index
    def block(self, idx: int) -> "BlockIterator":
        assert_true(idx >= 0, f"idx={idx}")
        if idx >= len(self.block_index):
            raise TableError("block out of index")
        return BlockIterator(self, self.block_index[idx])


def ParseFileID(name: str):  # noqa: N802
    """table.go:303-316"""
    name = os.path.basename(name)
    if not name.endswith(FILE_SUFFIX):
        return 0, False
    stem = name[: -len(FILE_SUFFIX)]
    try:
        fid = int(stem, 10)
    except ValueError:
        return 0, False
    assert_true(fid >= 0)
    return fid, True


def IDToFilename(fid: int) -> str:  # noqa: N802
    return "%06d" % fid + FILE_SUFFIX


def NewFilename(fid: int, dir: str) -> str:  # noqa: N802
    return os.path.join(dir, IDToFilename(fid))


def _be16(b, o):
    return (b[o] << 8) | b[o + 1]


def _be32(b, o):
    return (b[o] << 24) | (b[o + 1] << 16) | (b[o + 2] << 8) | b[o + 3]


def OpenTable(path_or_bytes, loading_mode: int = MEMORY_MAP, codec: Optional[Codec] = None,  # noqa: N802
              file_id: Optional[int] = None, decoder=None) -> Table:
    """table.go:88-144.  Accepts a path (the file is deleted by DecrRef at ref 0, like Go) or
    the table bytes themselves.  `decoder(data, blk_off, blk_len)` defaults to the HIP batch
    decode (Codec.decode_host); tests may inject another decoder to exercise this host logic
    without a GPU."""
    t = Table()
    t.loading_mode = loading_mode
    t._codec = codec
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
        raw = bytes(path_or_bytes)
        t.id = file_id or 0
    else:
        path = os.fspath(path_or_bytes)
        fid, ok = ParseFileID(path)
        if not ok and file_id is None:
            raise TableError(f"Invalid filename: {os.path.basename(path)}")
        t.id = fid if ok else file_id
        t.fd_name = path
        t._owns_file = True
        with open(path, "rb") as f:
            if loading_mode == MEMORY_MAP and os.path.getsize(path) > 0:
                with mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
                    raw = bytes(m)
            else:
                raw = f.read()
    t.raw = raw
    t.table_size = len(raw)
    if decoder is None:
        decoder = (codec or default_codec()).decode_host
    _read_index(t, decoder)
    it = t.NewIterator(False)
    it.Rewind()
    if it.Valid():
        t.smallest = it.Key()
    it.Close()
    it2 = t.NewIterator(True)
    it2.Rewind()
    if it2.Valid():
        t.biggest = it2.Key()
    it2.Close()
    return t


def _read_index(t: Table, decoder) -> None:
    """table.go:177-269 readIndex: tail parse, every block decoded on the GPU, first keys
    (with the plen==0 assertion, table.go:239), then the sort by key (table.go:267)."""
    raw = t.raw
    off, ln, bo, bl = parse_index(raw)
    t.bloom_json = raw[bo: bo + bl]
    try:  # table.go:186 bbloom.JSONUnmarshal at open time
        t._bloom = _bloom.parse(t.bloom_json)
    except ValueError:
        # Deliberate divergence: Go's bbloom.JSONUnmarshal ignores JSON errors and builds a
        # filter from whatever it parsed (so a Go reader may skip such a table); the exact
        # lenient result is parity unpinned (no bbloom source here).  A tail the restated parser
        # cannot load is treated as Has() = true: never skip, never a wrong miss.
        t._bloom = None
    data_end = int(off[-1] + ln[-1]) if off.size else 0
    t.dec = decoder(np.frombuffer(raw, np.uint8)[:data_end] if data_end
                    else np.zeros(16, np.uint8), off, ln)
    kos = []
    for b in range(off.size):
        o, n = int(off[b]), int(ln[b])
        if o + 10 > len(raw):
            raise TableError("While reading first header in block")
        plen, klen = _be16(raw, o), _be16(raw, o + 2)
        assert_true(plen == 0, f"Key offset: {o}, h.plen = {plen}")
        if o + 10 + klen > len(raw):
            raise TableError("While reading first key in block")
        kos.append(_KeyOffset(raw[o + 10: o + 10 + klen], o, n, b))
    if len(kos) > 1:
        import functools
        kos.sort(key=functools.cmp_to_key(lambda a, b: compare_keys(a.key, b.key)))
    t.block_index = kos


# ================================================================== blockIterator (iterator.go:13-169)
class BlockIterator:
    """blockIterator over one decoded block.  Go's byte cursor `pos` and `last` header are
    modelled by block-relative header positions; entry boundaries come from the GPU decode,
    the raw `prev` back-pointers from the block bytes (iterator.go:137-155)."""

    def __init__(self, t: Table, ko: _KeyOffset):
        self.t = t
        d = t.dec
        fb = ko.fblk
        self.base = ko.offset
        self.len = ko.len
        self.e0 = int(d.blk_first[fb])
        self.n = int(d.blk_first[fb + 1]) - self.e0
        # block-relative header start of every entry, and the end of the last one
        if self.n:
            kp = (d.view[self.e0: self.e0 + self.n] & 0xFFFFFFFF).astype(np.int64) - self.base
            kl = ((d.view[self.e0: self.e0 + self.n] >> 32) & 0xFFFF).astype(np.int64)
            vl = ((d.view[self.e0: self.e0 + self.n] >> 48) & 0xFFFF).astype(np.int64)
            self.hpos = kp - 10
            self.stop = int(kp[-1] + kl[-1] + vl[-1])
        else:
            self.hpos = np.zeros(0, np.int64)
            self.stop = 0
        self.idx_of = {int(p): i for i, p in enumerate(self.hpos)}
        # the decode stopped at a header Go cannot parse: reaching it panics there (a header
        # slice past the block, or baseKey[:plen] past the base key -- iterator.go:96,121)
        self.panics = int(d.blk_status[fb]) in (3, 4)  # BLK_TRUNC_HEADER, BLK_PREFIX_OOB
        self.Reset()

    # raw header field `prev` at block-relative position p (builder.go:23-43)
    def _prev_at(self, p: int) -> int:
        if p < 0 or p + 10 > self.len:
            raise TableError(f"header at {p} is outside the block (Go reads past the slice)")
        return _be32(self.t.raw, self.base + p + 6)

    def Reset(self) -> None:  # noqa: N802
        self.pos = 0
        self.err: Optional[Exception] = None
        self.init = False
        self.cur = -1            # current entry index (valid when err is None and init)
        self.last_pos = None     # block-relative position of the last header seen
        self.last_prev = 0       # header{}.prev after Reset

    def Init(self) -> None:  # noqa: N802
        if not self.init:
            self.Next()

    def Valid(self) -> bool:  # noqa: N802
        return self.err is None

    def Error(self):  # noqa: N802
        return self.err

    def Close(self) -> None:  # noqa: N802
        pass

    def Seek(self, key: bytes, whence: int = 0) -> None:  # noqa: N802
        """iterator.go:58-79"""
        self.err = None
        if whence == 0:
            self.Reset()
        done = False
        self.Init()
        while self.Valid():
            if compare_keys(self.Key(), key) >= 0:
                done = True
                break
            self.Next()
        if not done:
            self.err = EOF

    def SeekToFirst(self) -> None:  # noqa: N802
        self.err = None
        self.Init()

    def SeekToLast(self) -> None:  # noqa: N802
        self.err = None
        self.Init()
        while self.Valid():
            self.Next()
        self.Prev()

    def _enter(self, i: int) -> None:
        self.cur = i
        self.last_pos = int(self.hpos[i])
        self.last_prev = self._prev_at(self.last_pos)

    def Next(self) -> None:  # noqa: N802
        """iterator.go:112-135"""
        self.init = True
        self.err = None
        if self.pos >= self.len:
            self.err = EOF
            return
        i = self.idx_of.get(self.pos)
        if i is None:
            # the terminator (or the header the decode stopped at): itr.last = h, io.EOF
            if self.pos != self.stop:
                raise TableError("cursor left the decoded entry chain")
            if self.panics:
                raise TableError("Go panics on this header (truncated, or plen past the base key)")
            self.last_pos = self.pos
            self.last_prev = self._prev_at(self.pos)
            self.pos += 10
            self.err = EOF
            return
        self._enter(i)
        self.pos = int(self.hpos[i + 1]) if i + 1 < self.n else self.stop

    def Prev(self) -> None:  # noqa: N802
        """iterator.go:137-155"""
        if not self.init:
            return
        self.err = None
        if self.last_prev == MAX_U32:
            self.err = EOF
            self.pos = 0
            return
        i = self.idx_of.get(self.last_prev)
        if i is None:
            raise TableError(f"prev pointer {self.last_prev} is not an entry boundary")
        self._enter(i)
        self.pos = int(self.hpos[i + 1]) if i + 1 < self.n else self.stop

    def Key(self) -> Optional[bytes]:  # noqa: N802
        if self.err is not None:
            return None
        return self.t.dec.key(self.e0 + self.cur)

    def Value(self) -> Optional[bytes]:  # noqa: N802
        if self.err is not None:
            return None
        return self.t.dec.value(self.e0 + self.cur)


# ================================================================== Iterator (iterator.go:171-386)
class Iterator:
    """table.Iterator; the same state machine as iterator.go:171-386."""

    def __init__(self, t: Table, reversed: bool = False):
        t.IncrRef()
        self.t = t
        self.bpos = 0
        self.bi: Optional[BlockIterator] = None
        self.err: Optional[Exception] = None
        self.reversed = reversed
        self.next()

    def Close(self) -> None:  # noqa: N802
        self.t.DecrRef()

    def reset(self) -> None:
        self.bpos = 0
        self.err = None

    def Valid(self) -> bool:  # noqa: N802
        return self.err is None

    def seekToFirst(self) -> None:  # noqa: N802
        if len(self.t.block_index) == 0:
            self.err = EOF
            return
        self.bpos = 0
        self.bi = self.t.block(self.bpos)
        self.bi.SeekToFirst()
        self.err = self.bi.Error()

    def seekToLast(self) -> None:  # noqa: N802
        n = len(self.t.block_index)
        if n == 0:
            self.err = EOF
            return
        self.bpos = n - 1
        self.bi = self.t.block(self.bpos)
        self.bi.SeekToLast()
        self.err = self.bi.Error()

    def seekHelper(self, block_idx: int, key: bytes) -> None:  # noqa: N802
        self.bpos = block_idx
        self.bi = self.t.block(block_idx)
        self.bi.Seek(key, 0)
        self.err = self.bi.Error()

    def seekFrom(self, key: bytes, whence: int) -> None:  # noqa: N802
        self.err = None
        if whence == 0:
            self.reset()
        bi = self.t.block_index
        lo, hi = 0, len(bi)  # sort.Search(len, CompareKeys(ko.key, key) > 0)
        while lo < hi:
            mid = (lo + hi) // 2
            if compare_keys(bi[mid].key, key) > 0:
                hi = mid
            else:
                lo = mid + 1
        idx = lo
        if idx == 0:
            self.seekHelper(0, key)
            return
        self.seekHelper(idx - 1, key)
        if self.err is EOF:
            if idx == len(bi):
                return
            self.seekHelper(idx, key)

    def seek(self, key: bytes) -> None:
        self.seekFrom(key, 0)

    def seekForPrev(self, key: bytes) -> None:  # noqa: N802
        self.seekFrom(key, 0)
        if self.Key() != key:
            self.prev()

    def next(self) -> None:
        self.err = None
        while True:
            if self.bpos >= len(self.t.block_index):
                self.err = EOF
                return
            if self.bi is None:
                self.bi = self.t.block(self.bpos)
                self.bi.SeekToFirst()
                return
            self.bi.Next()
            if not self.bi.Valid():
                self.bpos += 1
                self.bi = None
                continue
            return

    def prev(self) -> None:
        self.err = None
        while True:
            if self.bpos < 0:
                self.err = EOF
                return
            if self.bi is None:
                self.bi = self.t.block(self.bpos)
                self.bi.SeekToLast()
                return
            self.bi.Prev()
            if not self.bi.Valid():
                self.bpos -= 1
                self.bi = None
                continue
            return

    def Key(self) -> Optional[bytes]:  # noqa: N802
        return self.bi.Key() if self.bi is not None else None

    def Value(self) -> ValueStruct:  # noqa: N802
        v = self.bi.Value() if self.bi is not None else None
        if v is None:
            raise IndexError("Value() on an invalid block iterator (Go panics in Decode)")
        return ValueStruct.decode(v)

    def Next(self) -> None:  # noqa: N802
        self.prev() if self.reversed else self.next()

    def Rewind(self) -> None:  # noqa: N802
        self.seekToLast() if self.reversed else self.seekToFirst()

    def Seek(self, key: bytes) -> None:  # noqa: N802
        self.seekForPrev(key) if self.reversed else self.seek(key)


# ================================================================== ConcatIterator (iterator.go:388-496)
class ConcatIterator:
    def __init__(self, tbls: List[Table], reversed: bool = False):
        self.reversed = reversed
        self.iters = [t.NewIterator(reversed) for t in tbls]
        self.tables = list(tbls)
        self.idx = -1
        self.cur: Optional[Iterator] = None

    def setIdx(self, idx: int) -> None:  # noqa: N802
        self.idx = idx
        self.cur = None if idx < 0 or idx >= len(self.iters) else self.iters[idx]

    def Rewind(self) -> None:  # noqa: N802
        if not self.iters:
            return
        self.setIdx(len(self.iters) - 1 if self.reversed else 0)
        self.cur.Rewind()

    def Valid(self) -> bool:  # noqa: N802
        return self.cur is not None and self.cur.Valid()

    def Key(self) -> Optional[bytes]:  # noqa: N802
        return self.cur.Key()

    def Value(self) -> ValueStruct:  # noqa: N802
        return self.cur.Value()

    def Seek(self, key: bytes) -> None:  # noqa: N802
        n = len(self.tables)
        if not self.reversed:
            lo, hi = 0, n
            while lo < hi:
                mid = (lo + hi) // 2
                if compare_keys(self.tables[mid].Biggest(), key) >= 0:
                    hi = mid
                else:
                    lo = mid + 1
            idx = lo
        else:
            lo, hi = 0, n
            while lo < hi:
                mid = (lo + hi) // 2
                if compare_keys(self.tables[n - 1 - mid].Smallest(), key) <= 0:
                    hi = mid
                else:
                    lo = mid + 1
            idx = n - 1 - lo
        if idx >= n or idx < 0:
            self.setIdx(-1)
            return
        self.setIdx(idx)
        self.cur.Seek(key)

    def Next(self) -> None:  # noqa: N802
        self.cur.Next()
        if self.cur.Valid():
            return
        while True:
            self.setIdx(self.idx - 1 if self.reversed else self.idx + 1)
            if self.cur is None:
                return
            self.cur.Rewind()
            if self.cur.Valid():
                break

    def Close(self) -> None:  # noqa: N802
        for it in self.iters:
            it.Close()


def NewConcatIterator(tbls: List[Table], reversed: bool) -> ConcatIterator:  # noqa: N802
    return ConcatIterator(tbls, reversed)


__all__ = ["Builder", "NewTableBuilder", "Table", "OpenTable", "Iterator", "BlockIterator",
           "ConcatIterator", "NewConcatIterator", "ParseFileID", "IDToFilename", "NewFilename",
           "RESULT_INTERVAL", "FILE_IO", "LOAD_TO_RAM", "MEMORY_MAP", "EOF", "parse_key",
           "MAX_U64"]
