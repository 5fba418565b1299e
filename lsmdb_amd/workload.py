"""Synthetic SST workloads of BASELINE.json's configs.

All generation is vectorised numpy with seed 0x5EED0000 + config#.  Columns are returned in
the C-ABI layout: (keys bytes, key_end u32, vs bytes, vs_end u32) where vs are encoded
ValueStructs ([Meta][UserMeta][uvarint ExpiresAt][Value], y/iterator.go:48-62).

  C1  table_test path: 10k entries, 16 B keys / 100 B values, 100 entries/block
  C2  4 KiB blocks (byte target 4096), 16 B hex keys / 100 B values  <- the headline
  C3  64 B keys / 1 KiB values, 4 KiB byte target (3 entries/block)
  C4  64 MiB SSTs (ReachedCapacity), 16 B / 100 B, 100 entries/block
  C5  user keys Zipf(1.2) over [8,256] B + 8 B ts, 100 B values, 32 KiB byte target
Keys are strictly increasing; 10 % of entries carry a non-zero ExpiresAt spread over every
uvarint width 1-10 and 5 % are 15-B value-pointer entries (12-B value, Meta |= bitValuePointer,
db.go:486-505).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SEED_BASE = 0x5EED0000
# one-line workload labels per config (bench.py's config.workload)
DESCRIPTIONS = {
    1: "100 entries/block (reference resultInterval), 16 B keys / 100 B values",
    2: "byte target 4 KiB, 16 B keys / 100 B values",
    3: "byte target 4 KiB, 64 B keys / 1 KiB values",
    4: "100 entries/block in 64 MiB SSTs, 16 B keys / 100 B values",
    5: "byte target 32 KiB, Zipf(1.2) 8-256 B user keys + 8 B ts / 100 B values",
}
HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
META_A = 0x41          # 'A' as in table_test.go
BIT_VALUE_POINTER = 2  # structs.go:33-40


@dataclass
class Columns:
    keys: np.ndarray     # u8
    key_end: np.ndarray  # u32
    vs: np.ndarray       # u8 (encoded ValueStructs)
    vs_end: np.ndarray   # u32
    entries_per_block: int
    block_bytes: int

    @property
    def n(self) -> int:
        return int(self.key_end.size)


def _ends(lengths: np.ndarray) -> np.ndarray:
    return np.cumsum(lengths, dtype=np.uint64).astype(np.uint32)


def hex_keys(n: int, start: int = 0) -> np.ndarray:
    """fmt.Sprintf("%016x", i) for i in [start, start+n) (BenchmarkRead, table_test.go:595)."""
    i = np.arange(start, start + n, dtype=np.uint64)
    shifts = np.arange(60, -4, -4, dtype=np.uint64)
    digits = ((i[:, None] >> shifts[None, :]) & np.uint64(15)).astype(np.intp)
    return HEX[digits]  # (n, 16) u8


def _varints(x: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """uvarint encodings of u64 x: (bytes (n,10) u8, lengths (n,))."""
    n = x.size
    out = np.zeros((n, 10), dtype=np.uint8)
    lens = np.ones(n, dtype=np.int64)
    v = x.astype(np.uint64).copy()
    for j in range(10):
        more = v >= np.uint64(0x80)
        out[:, j] = (v & np.uint64(0x7F)).astype(np.uint8) | (more.astype(np.uint8) << 7)
        lens += more
        v = v >> np.uint64(7)
    return out, lens


def encode_values(rng: np.random.Generator, n: int, value_len: int, exp_frac: float = 0.10,
                  vptr_frac: float = 0.05) -> tuple[np.ndarray, np.ndarray]:
    """Encoded ValueStruct column: (vs bytes u8, vs_end u32)."""
    exp = np.zeros(n, dtype=np.uint64)
    has_exp = rng.random(n) < exp_frac
    k = int(has_exp.sum())  # spread over every uvarint width 1..10
    r = rng.integers(0, np.iinfo(np.uint64).max, size=k, dtype=np.uint64, endpoint=True)
    exp[has_exp] = (r >> rng.integers(0, 64, size=k).astype(np.uint64)) | np.uint64(1)
    vptr = rng.random(n) < vptr_frac
    vlen = np.where(vptr, 12, value_len).astype(np.int64)
    meta = np.where(vptr, META_A | BIT_VALUE_POINTER, META_A).astype(np.uint8)
    var, vl = _varints(exp)
    sizes = 2 + vl + vlen
    ends = np.cumsum(sizes)
    starts = ends - sizes
    total = int(ends[-1]) if n else 0
    out = rng.integers(0, 256, size=total, dtype=np.uint8)  # value bytes (PRNG)
    out[starts] = meta
    out[starts + 1] = 0  # UserMeta
    for j in range(10):
        m = vl > j
        out[starts[m] + 2 + j] = var[m, j]
    return out, ends.astype(np.uint32)


def config_columns(cfg: int, n: int, seed_offset: int = 0) -> Columns:
    rng = np.random.default_rng(SEED_BASE + cfg + 1000 * seed_offset)
    start = seed_offset * (1 << 40)
    if cfg in (1, 2, 4):
        keys = hex_keys(n, start).reshape(-1)
        key_end = _ends(np.full(n, 16, np.int64))
        vs, vs_end = encode_values(rng, n, 100)
        epb, bb = (100, 0) if cfg in (1, 4) else (0, 4096)
        return Columns(keys, key_end, vs, vs_end, epb, bb)
    if cfg == 3:
        # 64 B keys: 56 B user key (hex counter + filler) + 8 B ts (KeyWithTs)
        klen = 64
        user = np.full((n, klen - 8), ord("k"), dtype=np.uint8)
        user[:, :16] = hex_keys(n, start)
        ts = rng.integers(1, 1 << 40, size=n, dtype=np.uint64)
        tsb = (np.uint64((1 << 64) - 1) - ts).astype(">u8").view(np.uint8).reshape(n, 8)
        keys = np.concatenate([user, tsb], axis=1).reshape(-1)
        key_end = _ends(np.full(n, klen, np.int64))
        vs, vs_end = encode_values(rng, n, 1024)
        return Columns(keys, key_end, vs, vs_end, 0, 4096)
    if cfg == 5:
        # user key length ~ Zipf(1.2) clipped to [8,256]; 8-B BE counter prefix keeps order
        ul = np.clip(rng.zipf(1.2, size=n) + 7, 8, 256).astype(np.int64)
        klen = ul + 8
        key_end64 = np.cumsum(klen)
        ks = key_end64 - klen
        keys = rng.integers(ord("a"), ord("z") + 1, size=int(key_end64[-1]), dtype=np.uint8)
        ctr = (np.arange(n, dtype=np.uint64) + np.uint64(start)).astype(">u8").view(np.uint8).reshape(n, 8)
        for j in range(8):
            keys[ks + j] = ctr[:, j]
        ts = rng.integers(1, 1 << 40, size=n, dtype=np.uint64)
        tsb = (np.uint64((1 << 64) - 1) - ts).astype(">u8").view(np.uint8).reshape(n, 8)
        te = key_end64 - 8
        for j in range(8):
            keys[te + j] = tsb[:, j]
        vs, vs_end = encode_values(rng, n, 100)
        return Columns(keys, key_end64.astype(np.uint32), vs, vs_end, 0, 32768)
    raise ValueError(f"unknown config {cfg}")


def entries_for_bytes(cfg: int, target_bytes: int) -> int:
    """An entry count giving at least target_bytes of block data for a config (an over-estimate:
    the per-entry sizes below are under the generators' means -- C2 ~125.8 B with its
    terminators, C3 ~1,105 B, C5 ~216 B; trim_to_bytes trims to the exact byte target)."""
    per = {1: 118, 2: 118, 3: 1050, 4: 118, 5: 190}[cfg]
    return max(1, target_bytes // per + 64)


def data_len_prefix(key_end: np.ndarray, vs_end: np.ndarray, plan: np.ndarray) -> np.ndarray:
    """Block-data bytes of the first e entries, e = 1..n (Builder: 10-B header + key + vs per
    entry, a 13-B terminator per block; plan = first entry of each block + end sentinel)."""
    e = np.arange(1, key_end.size + 1, dtype=np.int64)
    nblk = np.searchsorted(plan[:-1].astype(np.int64), e - 1, side="right")
    return 10 * e + key_end.astype(np.int64) + vs_end.astype(np.int64) + 13 * nblk


def trim_to_bytes(cols: Columns, plan: np.ndarray, target_bytes: int) -> Columns:
    """The shortest prefix of cols whose block data reaches target_bytes (Builder's cut rule is
    greedy, so the prefix's plan is the prefix of the plan)."""
    dl = data_len_prefix(cols.key_end, cols.vs_end, plan)
    idx = np.nonzero(dl >= target_bytes)[0]
    if idx.size == 0:
        raise ValueError(f"columns hold {int(dl[-1])} B < target {target_bytes} B")
    n = int(idx[0]) + 1
    kt, vt = int(cols.key_end[n - 1]), int(cols.vs_end[n - 1])
    return Columns(cols.keys[:kt], cols.key_end[:n], cols.vs[:vt], cols.vs_end[:n],
                   cols.entries_per_block, cols.block_bytes)


__all__ = ["Columns", "config_columns", "hex_keys", "encode_values", "entries_for_bytes",
           "data_len_prefix", "trim_to_bytes"]
