"""SST images for the batched table-open tests (table/table.go:88-144,177-269): well-formed
tables of every config shape, tables whose block index is out of key order (readIndex sorts
it), empty / terminator-less / prefix-compressed last blocks (SeekToLast + Prev quirks), and
malformed tables for every LSMGPU_TBL_* status.  Built with the oracle Builder (test only)."""
import struct

import numpy as np

TAIL = b"{}" + (2).to_bytes(4, "big")  # a bbloom-shaped 2-byte JSON + its length


def ts_key(user: bytes, ts: int) -> bytes:
    """y.KeyWithTs (y/y.go:67-72): user key ++ BE64(MaxUint64 - ts)."""
    return user + (0xFFFFFFFFFFFFFFFF - ts).to_bytes(8, "big")


def with_tail(data: bytes, ends) -> bytes:
    """[data blocks][restarts BE32 x N][N BE32] + bloom tail (builder.go:146-198)."""
    idx = b"".join(int(e).to_bytes(4, "big") for e in ends) + len(ends).to_bytes(4, "big")
    return data + idx + TAIL


def blocks_of(oracle, sst: bytes):
    off, ln, _, _ = oracle.parse_index(sst + TAIL)
    return [sst[int(o): int(o) + int(n)] for o, n in zip(off, ln)]


def reorder(oracle, sst: bytes, perm) -> bytes:
    """The same blocks in another physical order (restarts rewritten)."""
    bl = blocks_of(oracle, sst)
    data, ends = b"", []
    for i in perm:
        data += bl[i]
        ends.append(len(data))
    return with_tail(data, ends)


def entry(plen, key, val, prev):
    return struct.pack(">HHHI", plen, len(key), len(val), prev) + key + val


def cases(oracle):
    """[(label, sst bytes)]"""
    out = []
    rng = np.random.default_rng(5)
    keys = [ts_key(b"key%06d" % i, int(rng.integers(1, 1 << 40))) for i in range(950)]
    vss = [b"A\x00\x00" + bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
           for _ in keys]
    sst, _, _ = oracle.build(keys, vss, entries_per_block=100)
    out.append(("ts keys, 100/blk", sst + TAIL))
    hexk = [b"%016x" % i for i in range(3000)]
    sst4, _, _ = oracle.build(hexk, [b"A\x00\x00" + b"v" * 100] * 3000, entries_per_block=100,
                              block_bytes=4096)
    out.append(("C2-like 4 KiB", sst4 + TAIL))
    out.append(("single entry", oracle.build([ts_key(b"only", 7)], [b"A\x00\x00x"])[0] + TAIL))
    out.append(("empty table", oracle.build([], [])[0] + TAIL))
    nb = len(blocks_of(oracle, sst))
    perm = list(range(nb))[::-1]
    out.append(("reversed block order", reorder(oracle, sst, perm)))
    perm2 = list(rng.permutation(nb))
    out.append(("shuffled block order", reorder(oracle, sst, perm2)))
    # last block without a terminator: SeekToLast ends at pos >= len, Prev() goes to the
    # last decoded header's prev = the second-to-last entry
    b = entry(0, ts_key(b"za", 1), b"A\x00\x00a", 0xFFFFFFFF)
    p1 = len(b)
    b += entry(0, ts_key(b"zb", 1), b"A\x00\x00b", 0)
    b += entry(0, ts_key(b"zc", 1), b"A\x00\x00c", p1)
    first = blocks_of(oracle, sst)[0]
    out.append(("last block unterminated", with_tail(first + b, [len(first), len(first) + len(b)])))
    # single unterminated entry: last.prev = MaxUint32 -> Prev() is io.EOF, biggest nil
    one = entry(0, ts_key(b"zz", 1), b"A\x00\x00z", 0xFFFFFFFF)
    out.append(("last block one unterminated entry", with_tail(first + one, [len(first), len(first) + len(one)])))
    # prefix-compressed last block: biggest = baseKey[:plen] ++ diff
    base = ts_key(b"zzprefix-compressed", 3)
    pc = entry(0, base, b"A\x00\x00q", 0xFFFFFFFF)
    q1 = len(pc)
    pc += entry(12, b"-tail" + b"\x00" * 8, b"A\x00\x00r", 0)
    pc += struct.pack(">HHHI", 0, 0, 3, q1) + b"\x00\x00\x00"
    out.append(("prefix-compressed last block", with_tail(first + pc, [len(first), len(first) + len(pc)])))
    # first block empty (terminator only): smallest nil (seekToFirst does not advance)
    term = struct.pack(">HHHI", 0, 0, 3, 0xFFFFFFFF) + b"\x00\x00\x00"
    out.append(("empty first block, one block", with_tail(term, [len(term)])))
    # value overflow in the last block's final entry: Prev() from the overflowing header
    vo = entry(0, ts_key(b"zv1", 1), b"A\x00\x00a", 0xFFFFFFFF)
    v1 = len(vo)
    vo += struct.pack(">HHHI", 0, len(ts_key(b"zv2", 1)), 500, 0) + ts_key(b"zv2", 1) + b"A\x00"
    out.append(("value overflow in last block", with_tail(first + vo, [len(first), len(first) + len(vo)])))
    # ---- malformed
    out.append(("bad tail: bloom length", sst[:-4] + (1 << 30).to_bytes(4, "big") + TAIL))
    bad_restart = bytearray(sst + TAIL)
    ridx = len(sst) - 4 - 4 * nb  # restart array position
    bad_restart[ridx + 4: ridx + 8] = (1).to_bytes(4, "big")  # non-monotone
    out.append(("bad tail: restarts", bytes(bad_restart)))
    fp = bytearray(sst + TAIL)
    o2 = int(oracle.parse_index(sst + TAIL)[0][1])
    fp[o2: o2 + 2] = (3).to_bytes(2, "big")  # plen of block 1's first header
    out.append(("first plen", bytes(fp)))
    short = [b"k%03d" % i for i in range(300)]  # 4-B keys: CompareKeys asserts len > 8
    out.append(("short keys, 3 blocks", oracle.build(short, [b"A\x00\x00"] * 300)[0] + TAIL))
    out.append(("short keys, 1 block", oracle.build(short[:50], [b"A\x00\x00"] * 50)[0] + TAIL))
    rd = bytearray(first)
    rd[2:4] = (0xFFFF).to_bytes(2, "big")  # first key runs past the file
    out.append(("first key past the file", with_tail(bytes(rd), [len(rd)])))
    return out
