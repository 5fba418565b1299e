"""GPU bloom tail (csrc/bloom.hip) vs the oracle restatement (oracle/bbloom.c): bit-exact
filters and JSON, probes, and the table round trip (Builder.Finish -> OpenTable ->
DoesNotHave).  bbloom-specific bytes are parity unpinned against Go (see test_bloom_oracle)."""
import numpy as np
import pytest
import torch

from lsmdb_amd import bloom, workload
from lsmdb_amd.codec import bloom_params
from lsmdb_amd.y import key_with_ts

pytestmark = pytest.mark.gpu


def _rand_keys(n, seed, lo=9, hi=300):
    rng = np.random.default_rng(seed)
    ln = rng.integers(lo, hi + 1, n)
    kb = rng.integers(0, 256, int(ln.sum()), dtype=np.uint8).tobytes()
    return kb, np.cumsum(ln).astype(np.uint32)


def _device(codec, kb, ke):
    dev = torch.device("cuda", 0)
    kd = torch.from_numpy(np.frombuffer(kb + b"\0" * 16, np.uint8).copy()).to(dev)
    return kd, torch.from_numpy(ke.view(np.int32).copy()).to(dev)


@pytest.mark.parametrize("case", ["random", "short", "word", "c2_hex", "c5_zipf", "one"])
def test_bloom_build_vs_oracle(codec, oracle, case):
    if case == "random":
        kb, ke = _rand_keys(30000, 1)
    elif case == "short":    # 9-15 B keys: 1-7 B bloom keys (tail word only)
        kb, ke = _rand_keys(20000, 2, 9, 15)
    elif case == "word":     # 16 / 24 B: whole words, empty tail
        kb, ke = _rand_keys(20000, 3, 16, 16)
    elif case == "c2_hex":   # BenchmarkRead keys: ParseKey keeps the first 8 hex digits
        c = workload.config_columns(2, 50000, 0)
        kb, ke = c.keys.tobytes(), c.key_end
    elif case == "c5_zipf":  # Zipf user keys + 8-B ts
        c = workload.config_columns(5, 20000, 0)
        kb, ke = c.keys.tobytes(), c.key_end
    else:
        kb, ke = b"k" * 9, np.array([9], np.uint32)
    n = int(ke.size)
    bs, bits, locs, _ = oracle.bloom_build(kb, ke)
    assert bloom_params(n)[:2] == (bits, locs)
    kd, ked = _device(codec, kb, ke)
    o = codec.bloom_build_device(kd, ked, n)
    codec.synchronize()
    assert int(o["flags"].cpu()[0]) == 0
    got = o["bitset"].cpu().numpy().view(np.uint64)
    assert np.array_equal(got, bs), f"{case}: filter bits differ"
    assert o["json"].cpu().numpy().tobytes() == oracle.bloom_json(bs, bits, locs)


@pytest.mark.parametrize("n", [0, 1, 519540])
def test_bloom_tail_sizes(codec, oracle, n):
    """Empty table (setLocs = 1 << 63, 512 zero bits), one key, and one C4 64 MiB table's
    519,540 keys (a 2^23-bit filter)."""
    c = workload.config_columns(4, max(n, 1), 4)
    kb, ke = (c.keys.tobytes(), c.key_end) if n else (b"", np.zeros(0, np.uint32))
    raw = codec.bloom_tail_host(kb, ke)
    bs, bits, locs, _ = oracle.bloom_build(kb, ke)
    assert raw == oracle.bloom_json(bs, bits, locs)
    got, glocs = bloom.parse(raw)
    assert np.array_equal(got, bs) and glocs == locs


def test_bloom_short_key_flag(codec):
    with pytest.raises(ValueError):
        codec.bloom_tail_host(b"x" * 9 + b"12345678", np.array([9, 17], np.uint32))


def test_bloom_has_vs_oracle(codec, oracle):
    kb, ke = _rand_keys(40000, 5, 9, 64)
    bs, bits, locs, ex = oracle.bloom_build(kb, ke)
    starts = np.concatenate([[0], ke[:-1]])
    present = [kb[starts[i]: ke[i] - 8] for i in range(0, 40000, 3)]
    qb, qe = _rand_keys(30000, 6, 0, 40)  # absent keys, lengths 0-40 (empty key included)
    qs = np.concatenate([[0], qe[:-1]])
    absent = [qb[qs[i]: qe[i]] for i in range(30000)]
    got = codec.bloom_has_host(bs, locs, present + absent)
    assert got[: len(present)].all()  # no false negatives
    want = np.array([oracle.bloom_has(bs, bits, locs, ex, k) for k in present + absent])
    assert np.array_equal(got, want)
    assert got[len(present):].mean() < 0.03


def test_table_doesnothave_roundtrip(codec, tmp_path):
    """Builder.Finish writes the device filter; OpenTable + DoesNotHave (level_handler.go:221-224
    probes ParseKey(key)) never rejects a present key."""
    from lsmdb_amd import table as T
    from lsmdb_amd.y import ValueStruct
    b = T.Builder(bloom=T.BLOOM_BBLOOM, codec=codec)
    keys = [key_with_ts(b"user%06d" % i, 1) for i in range(0, 3000, 2)]
    for k in keys:
        b.Add(k, ValueStruct(meta=0x41, value=b"v" * 20))
    path = tmp_path / "000007.sst"
    path.write_bytes(b.Finish())
    t = T.OpenTable(str(path), T.MEMORY_MAP, codec=codec)
    assert not t.DoesNotHaveBatch([k[:-8] for k in keys]).any()
    assert not t.DoesNotHave(keys[17][:-8])
    missing = [b"user%06d" % i for i in range(1, 3000, 2)]
    assert t.DoesNotHaveBatch(missing).mean() > 0.95
    t.DecrRef()
    # one-key host probes (DoesNotHave) agree with the device batch probe key by key
    probe = [k[:-8] for k in keys[:200]] + missing[:200]
    batch = t.DoesNotHaveBatch(probe)
    assert [t.DoesNotHave(k) for k in probe] == batch.tolist()


def test_table_all_ones_tail(codec, tmp_path):
    """Builder(bloom="all_ones"): the conservative tail for Go readers -- never a skip."""
    from lsmdb_amd import table as T
    from lsmdb_amd.y import ValueStruct
    b = T.Builder(bloom=T.BLOOM_ALL_ONES, codec=codec)
    for i in range(500):
        b.Add(key_with_ts(b"user%06d" % i, 1), ValueStruct(meta=0x41, value=b"v"))
    path = tmp_path / "000008.sst"
    path.write_bytes(b.Finish())
    t = T.OpenTable(str(path), T.MEMORY_MAP, codec=codec)
    missing = [b"nope%06d" % i for i in range(300)]
    assert not t.DoesNotHaveBatch(missing).any() and not t.DoesNotHave(missing[0])
    assert sum(1 for _ in _iter(t)) == 500
    t.DecrRef()


def _iter(t):
    it = t.NewIterator(False)
    it.Rewind()
    while it.Valid():
        yield it.Key()
        it.Next()
