"""ctypes access to the CPU ORACLE (oracle/build/libsstref.so) -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, byref, c_int, c_int64, c_size_t, c_uint8, c_uint16, c_uint32, c_uint64, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libsstref.so")


class Totals(ctypes.Structure):
    _fields_ = [("n_entries", c_uint64), ("key_bytes", c_uint64), ("val_bytes", c_uint64),
                ("first_bad_block", c_int64), ("n_bad_blocks", c_uint64), ("overflow", c_int)]


class TableInfo(ctypes.Structure):
    _fields_ = [("nblk", c_uint32), ("bloom_off", c_uint32), ("bloom_len", c_uint32),
                ("status", ctypes.c_int32), ("has_smallest", ctypes.c_int32),
                ("smallest_off", c_uint32), ("smallest_len", c_uint32),
                ("has_biggest", ctypes.c_int32), ("big_base_off", c_uint32), ("big_plen", c_uint32),
                ("big_diff_off", c_uint32), ("big_klen", c_uint32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s"], check=True)
        L = ctypes.CDLL(ORACLE_SO)
        L.sstref_uvarint_size.argtypes = [c_uint64]
        L.sstref_uvarint_size.restype = c_int
        L.sstref_vs_encoded_size.argtypes = [c_uint64, c_size_t]
        L.sstref_vs_encoded_size.restype = c_uint16
        L.sstref_vs_encode.argtypes = [c_uint8, c_uint8, c_uint64, c_void_p, c_size_t, c_void_p]
        L.sstref_vs_encode.restype = c_size_t
        L.sstref_vs_decode.argtypes = [c_void_p, c_size_t, POINTER(c_uint8), POINTER(c_uint8),
                                       POINTER(c_uint64)]
        L.sstref_vs_decode.restype = c_int
        L.sstref_builder_new.argtypes = [c_uint32, c_uint32]
        L.sstref_builder_new.restype = c_void_p
        L.sstref_builder_free.argtypes = [c_void_p]
        L.sstref_builder_add.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_size_t]
        L.sstref_builder_reached_capacity.argtypes = [c_void_p, c_int64]
        L.sstref_builder_reached_capacity.restype = c_int
        L.sstref_builder_empty.argtypes = [c_void_p]
        L.sstref_builder_empty.restype = c_int
        L.sstref_builder_finish.argtypes = [c_void_p, POINTER(c_size_t), POINTER(c_size_t),
                                            POINTER(POINTER(c_uint32)), POINTER(c_size_t)]
        L.sstref_builder_finish.restype = POINTER(c_uint8)
        L.sstref_build.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_uint32,
                                   c_uint32, c_void_p, c_size_t, POINTER(c_size_t), c_void_p,
                                   c_size_t, POINTER(c_size_t)]
        L.sstref_build.restype = c_size_t
        L.sstref_parse_index.argtypes = [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t,
                                         POINTER(c_size_t), POINTER(c_size_t), POINTER(c_size_t)]
        L.sstref_parse_index.restype = c_int
        L.sstref_decode_blocks.argtypes = [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t,
                                           c_void_p, c_size_t, c_void_p, c_void_p, c_size_t,
                                           c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                           POINTER(Totals)]
        L.sstref_decode_blocks.restype = c_int
        L.sstref_decode_bench.argtypes = [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, c_int,
                                          c_int, POINTER(c_uint64)]
        L.sstref_decode_bench.restype = ctypes.c_double
        L.sstref_compare_keys.argtypes = [c_void_p, c_size_t, c_void_p, c_size_t]
        L.sstref_compare_keys.restype = c_int
        L.sstref_siphash24.argtypes = [c_uint64, c_uint64, c_void_p, c_size_t]
        L.sstref_siphash24.restype = c_uint64
        L.sstref_bloom_params.argtypes = [ctypes.c_double, ctypes.c_double, POINTER(c_uint64),
                                          POINTER(c_uint64), POINTER(c_uint32)]
        L.sstref_bloom_has.argtypes = [c_void_p, c_uint64, c_uint32, c_uint64, c_void_p, c_size_t]
        L.sstref_bloom_has.restype = c_int
        L.sstref_bloom_json.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p, c_size_t]
        L.sstref_bloom_json.restype = c_size_t
        L.sstref_bloom_build.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_uint64, c_uint32,
                                         c_uint64]
        L.sstref_bloom_build.restype = c_int
        L.sstref_open_table.argtypes = [c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_size_t, POINTER(TableInfo)]
        L.sstref_open_table.restype = c_int
        L.sstref_merge.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t]
        L.sstref_merge.restype = c_size_t
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data if a.size else None


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b.view(np.uint8).reshape(-1))
    a = np.frombuffer(bytes(b), dtype=np.uint8)
    return a if a.size else np.zeros(1, np.uint8)[:0]


def vs_encode(meta: int, user_meta: int, expires_at: int, value: bytes) -> bytes:
    out = np.zeros(len(value) + 12, np.uint8)
    v = _u8(value)
    n = lib().sstref_vs_encode(meta, user_meta, expires_at, _p(v), len(value), _p(out))
    return out[:n].tobytes()


def vs_encoded_size(expires_at: int, value_len: int) -> int:
    return lib().sstref_vs_encoded_size(expires_at, value_len)


def columns(keys, vss):
    """(keys bytes, key_end u32, vs bytes, vs_end u32) from lists."""
    kb = b"".join(keys)
    vb = b"".join(vss)
    ke = np.cumsum([len(k) for k in keys], dtype=np.uint64).astype(np.uint32) if keys else np.zeros(0, np.uint32)
    ve = np.cumsum([len(v) for v in vss], dtype=np.uint64).astype(np.uint32) if vss else np.zeros(0, np.uint32)
    return kb, ke, vb, ve


def build_cols(kb: bytes, ke: np.ndarray, vb: bytes, ve: np.ndarray, entries_per_block: int = 100,
               block_bytes: int = 0):
    """Builder.Add x n + Finish minus bloom -> (bytes [data][index], data_len, restarts)."""
    kba, vba = _u8(kb), _u8(vb)
    ke = np.ascontiguousarray(ke, np.uint32)
    ve = np.ascontiguousarray(ve, np.uint32)
    n = ke.size
    cap = 10 * n + len(kb) + len(vb) + 13 * (n + 1) + 4 * (n + 2) + 64
    out = np.zeros(cap, np.uint8)
    rs = np.zeros(n + 2, np.uint32)
    dl, nr = c_size_t(0), c_size_t(0)
    ln = lib().sstref_build(_p(kba), _p(ke), _p(vba), _p(ve), n, entries_per_block, block_bytes,
                            _p(out), cap, byref(dl), _p(rs), rs.size, byref(nr))
    assert ln > 0
    return out[:ln].tobytes(), dl.value, rs[: nr.value].copy()


def build(keys, vss, entries_per_block: int = 100, block_bytes: int = 0):
    return build_cols(*columns(keys, vss), entries_per_block, block_bytes)


def parse_index(sst: bytes):
    a = _u8(sst)
    n, bo, bl = c_size_t(0), c_size_t(0), c_size_t(0)
    rc = lib().sstref_parse_index(_p(a), a.size, None, None, 0, byref(n), byref(bo), byref(bl))
    if rc == -1:
        raise ValueError("malformed tail")
    off = np.zeros(max(n.value, 1), np.uint32)
    ln = np.zeros(max(n.value, 1), np.uint32)
    rc = lib().sstref_parse_index(_p(a), a.size, _p(off), _p(ln), off.size, byref(n), byref(bo), byref(bl))
    if rc != 0:
        raise ValueError("malformed tail")
    return off[: n.value], ln[: n.value], bo.value, bl.value


class Decoded:
    def __init__(self, **kw):
        self.__dict__.update(kw)

    def key(self, i):
        a = int(self.key_end[i - 1]) if i else 0
        return self.key_data[a: int(self.key_end[i])].tobytes()

    def value(self, i):
        a = int(self.val_end[i - 1]) if i else 0
        return self.val_data[a: int(self.val_end[i])].tobytes()


def decode(data, blk_off, blk_len) -> Decoded:
    """The oracle decode of every block (blockIterator forward walk)."""
    d = _u8(data)
    off = np.ascontiguousarray(blk_off, np.uint32)
    ln = np.ascontiguousarray(blk_len, np.uint32)
    nblk = off.size
    cap = max(int(ln.astype(np.uint64).sum()), 16)
    ent_cap = cap // 10 + 1
    for _ in range(2):
        kd = np.zeros(cap, np.uint8)
        vd = np.zeros(cap, np.uint8)
        ke = np.zeros(ent_cap, np.uint32)
        ve = np.zeros(ent_cap, np.uint32)
        vw = np.zeros(ent_cap, np.uint64)
        bf = np.zeros(nblk + 1, np.uint32)
        bs = np.zeros(max(nblk, 1), np.int32)
        t = Totals()
        rc = lib().sstref_decode_blocks(_p(d) if d.size else None, d.size, _p(off), _p(ln), nblk,
                                        _p(kd), kd.size, _p(ke), _p(vd), vd.size, _p(ve), _p(vw),
                                        ent_cap, _p(bf), _p(bs), byref(t))
        if rc == 0:
            n = t.n_entries
            return Decoded(n_entries=n, key_data=kd[: t.key_bytes], key_end=ke[:n],
                           val_data=vd[: t.val_bytes], val_end=ve[:n], view=vw[:n], blk_first=bf,
                           blk_status=bs[:nblk], first_bad_block=t.first_bad_block,
                           n_bad_blocks=t.n_bad_blocks)
        cap = max(t.key_bytes, t.val_bytes, 16)
        ent_cap = max(t.n_entries, 1)
    raise RuntimeError("oracle decode overflow")


def decode_sst(sst: bytes) -> Decoded:
    off, ln, _, _ = parse_index(sst)
    return decode(sst, off, ln)


def decode_bench(data: np.ndarray, blk_off, blk_len, nthreads: int, reps: int):
    d = _u8(data)
    off = np.ascontiguousarray(blk_off, np.uint32)
    ln = np.ascontiguousarray(blk_len, np.uint32)
    cs = c_uint64(0)
    secs = lib().sstref_decode_bench(_p(d), d.size, _p(off), _p(ln), off.size, nthreads, reps, byref(cs))
    return secs, cs.value


_ = (c_int64,)


def open_table(sst: bytes, cap: int = 1 << 20) -> dict:
    """OpenTable's index work (sstref_open_table; table.go:88-144,177-269): per-block
    [off,len), first keys, sorted order, smallest / biggest (as bytes, or None)."""
    a = _u8(sst)
    off = np.zeros(cap, np.uint32)
    ln = np.zeros(cap, np.uint32)
    ko = np.zeros(cap, np.uint32)
    kl = np.zeros(cap, np.uint32)
    order = np.zeros(cap, np.uint32)
    info = TableInfo()
    lib().sstref_open_table(_p(a), a.size, _p(off), _p(ln), _p(ko), _p(kl), _p(order), cap,
                            byref(info))
    n = info.nblk if info.status != 5 else 0
    raw = bytes(a)
    smallest = raw[info.smallest_off: info.smallest_off + info.smallest_len] if info.has_smallest else None
    biggest = None
    if info.has_biggest:
        biggest = (raw[info.big_base_off: info.big_base_off + info.big_plen] +
                   raw[info.big_diff_off: info.big_diff_off + info.big_klen])
    return dict(status=info.status, nblk=info.nblk, bloom_off=info.bloom_off,
                bloom_len=info.bloom_len, blk_off=off[:n].copy(), blk_len=ln[:n].copy(),
                key_off=ko[:n].copy(), key_len=kl[:n].copy(), order=order[:n].copy(),
                smallest=smallest, biggest=biggest,
                smallest_view=(info.has_smallest, info.smallest_off, info.smallest_len),
                biggest_view=(info.has_biggest, info.big_base_off, info.big_plen,
                              info.big_diff_off, info.big_klen))


def merge(key_data, key_end, run_first) -> np.ndarray:
    """MergeIterator order (sstref_merge): source entry index of each output entry."""
    kd = _u8(key_data) if len(key_data) else np.zeros(1, np.uint8)
    ke = np.ascontiguousarray(key_end, dtype=np.uint32)
    rf = np.ascontiguousarray(run_first, dtype=np.uint32)
    out = np.zeros(max(ke.size, 1), np.uint32)
    n = lib().sstref_merge(_p(kd), _p(ke), _p(rf), rf.size - 1, _p(out), out.size)
    assert n != ctypes.c_size_t(-1).value
    return out[:n].copy()


# ---- bloom tail (oracle/bbloom.c: bbloom restated; table/builder.go:164-195)
def siphash24(k0: int, k1: int, msg: bytes) -> int:
    b = _u8(msg)
    return int(lib().sstref_siphash24(k0, k1, _p(b), len(msg)))


def bloom_params(n: int, wrongs: float = 0.01) -> tuple[int, int, int]:
    """(size in bits, setLocs, exponent) of bbloom.New(float64(n), wrongs)."""
    sz, locs, ex = c_uint64(), c_uint64(), c_uint32()
    lib().sstref_bloom_params(float(n), wrongs, byref(sz), byref(locs), byref(ex))
    return sz.value, locs.value, ex.value


def bloom_build(keys: bytes, key_end: np.ndarray) -> tuple[np.ndarray, int, int, int]:
    """Finish's filter over keys WITH ts (ParseKey strips 8 B): (bitset u64, bits, locs, exp)."""
    ke = np.ascontiguousarray(key_end, np.uint32)
    bits, locs, ex = bloom_params(ke.size)
    bs = np.zeros(bits // 64, np.uint64)
    kb = _u8(keys)
    rc = lib().sstref_bloom_build(_p(kb), _p(ke), ke.size, _p(bs), bits, ex, locs)
    if rc != 0:
        raise ValueError("key of <= 8 B (y.go:98)")
    return bs, bits, locs, ex


def bloom_has(bitset: np.ndarray, bits: int, locs: int, ex: int, key: bytes) -> bool:
    kb = _u8(key)
    return bool(lib().sstref_bloom_has(_p(bitset), bits, ex, locs, _p(kb), len(key)))


def bloom_json(bitset: np.ndarray, bits: int, locs: int) -> bytes:
    n = int(lib().sstref_bloom_json(_p(bitset), bits, locs, None, 0))
    out = np.zeros(n, np.uint8)
    lib().sstref_bloom_json(_p(bitset), bits, locs, _p(out), n)
    return out.tobytes()
