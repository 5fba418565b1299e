"""The bloom-tail oracle (oracle/bbloom.c, bbloom v0.0.0-20190825152654 restated) on CPU.

Pinned: SipHash-2-4 against the published test vectors (Aumasson & Bernstein; key 00..0f,
message 00 01 .. n-1), bbloom's initial state decoding to one (k0, k1) pair both ways, and
bbloom.New's sizing at the reference's call (table/builder.go:164, wrongs = 0.01).  The
bbloom-specific hash split / bit order / JSON bytes are PARITY UNPINNED (no Go toolchain, the
library is not vendored, no reference test checks bloom bytes): the properties below are
what bbloom guarantees (no false negatives, ~1 % false positives at the sized load).
"""
import base64
import json

import numpy as np
import pytest

KEY = bytes(range(16))
K0 = int.from_bytes(KEY[:8], "little")
K1 = int.from_bytes(KEY[8:], "little")


@pytest.mark.parametrize("n,expect", [
    (0, 0x726fdb47dd0e0e31),
    (1, 0x74f839c593dc67fd),
    (2, 0x0d6c8009d9a94f5a),
    (15, 0xa129ca6149be45e5),  # the paper's worked example
])
def test_siphash24_vectors(oracle, n, expect):
    assert oracle.siphash24(K0, K1, bytes(range(n))) == expect


def test_bbloom_initial_state():
    """bbloom's sipHash starts from v0..v3 = these literals; each pair of the SipHash
    constants must decode to the same k0 / k1 (0xdeadbeaf, 0xfaebdaed) that bbloom.c uses."""
    v0, v1, v2, v3 = (8317987320269560794, 7237128889637516672, 7816392314733513934,
                      8387220255325274014)
    assert v0 ^ 0x736f6d6570736575 == v2 ^ 0x6c7967656e657261 == 0xdeadbeaf
    assert v1 ^ 0x646f72616e646f6d == v3 ^ 0x7465646279746573 == 0xfaebdaed


@pytest.mark.parametrize("n,bits,locs", [
    (1, 512, 7),            # getSize's 512-bit floor
    (53, 512, 7),           # 53 * 9.585 = 508 bits
    (54, 1024, 7),
    (10000, 1 << 17, 7),    # C1: 95,850 bits -> 2^17
    (519540, 1 << 23, 7),   # C4: one 64 MiB table, 4.98 M bits -> 2^23 (1 MiB filter)
])
def test_bloom_params(oracle, n, bits, locs):
    b, l, e = oracle.bloom_params(n)
    assert (b, l) == (bits, locs) and b == 1 << e
    from lsmdb_amd import bloom as host  # the JSON sizing the Python mirror uses agrees
    assert host.bbloom_params(float(n)) == (bits, locs)


def test_bloom_empty_table(oracle):
    """keyCount = 0: size 0 -> 512 bits, locs = ceil(0 / 0) = NaN -> uint64 1 << 63 (amd64)."""
    bs, bits, locs, _ = oracle.bloom_build(b"", np.zeros(0, np.uint32))
    assert bits == 512 and locs == 1 << 63 and not bs.any()
    doc = json.loads(oracle.bloom_json(bs, bits, locs))
    assert doc == {"FilterSet": base64.b64encode(bytes(64)).decode(), "SetLocs": 1 << 63}


def _keys(n, seed, lo=9, hi=40):
    rng = np.random.default_rng(seed)
    ln = rng.integers(lo, hi + 1, n)
    kb = rng.integers(0, 256, int(ln.sum()), dtype=np.uint8).tobytes()
    return kb, np.cumsum(ln).astype(np.uint32)


def test_bloom_properties(oracle):
    kb, ke = _keys(20000, 1)
    bs, bits, locs, ex = oracle.bloom_build(kb, ke)
    starts = np.concatenate([[0], ke[:-1]])
    for i in range(0, 20000, 97):  # every added key (minus its 8-B ts) is present
        assert oracle.bloom_has(bs, bits, locs, ex, kb[starts[i]: ke[i] - 8])
    qb, qe = _keys(20000, 2, 20, 30)  # fresh keys: ~1 % false positives (bbloom's target)
    qs = np.concatenate([[0], qe[:-1]])
    fp = sum(oracle.bloom_has(bs, bits, locs, ex, qb[qs[i]: qe[i]]) for i in range(20000))
    assert fp < 20000 * 0.02
    # popcount: 7 locs per key into 2^18 bits -> 1 - exp(-7n/m) of the bits set
    ones = int(np.unpackbits(bs.view(np.uint8)).sum())
    expect = bits * (1 - np.exp(-locs * 20000 / bits))
    assert abs(ones - expect) < 0.02 * bits
    doc = json.loads(oracle.bloom_json(bs, bits, locs))
    assert doc["SetLocs"] == locs
    assert base64.b64decode(doc["FilterSet"]) == bs.tobytes()


def test_bloom_rejects_short_keys(oracle):
    with pytest.raises(ValueError):
        oracle.bloom_build(b"12345678", np.array([8], np.uint32))


def test_host_probe_matches_oracle(oracle):
    """bloom.has (DoesNotHave's one-key host probe) against the oracle's sstref_bloom_has on
    filters the oracle built (random keys, keys of every length 1..40)."""
    import os
    import numpy as np
    from lsmdb_amd import bloom
    rng = np.random.default_rng(5)
    keys = [bytes(rng.integers(0, 256, int(rng.integers(9, 48)), dtype=np.uint8)) for _ in range(3000)]
    kb = b"".join(keys)
    ke = np.cumsum([len(k) for k in keys]).astype(np.uint32)
    bs, bits, locs, ex = oracle.bloom_build(kb, ke)
    present = [k[:-8] for k in keys[:500]]
    absent = [os.urandom(n) for n in range(1, 41)] * 10
    for k in present + absent:
        assert bloom.has(bs, locs, k) == oracle.bloom_has(bs, bits, locs, ex, k), k
    assert all(bloom.has(bs, locs, k) for k in present)


def test_all_ones_tail_parses():
    from lsmdb_amd import bloom
    for n in (0, 1, 100, 519540):
        bs, locs = bloom.parse(bloom.all_ones_json(n))
        assert (bs == np.uint64(0xFFFFFFFFFFFFFFFF)).all() and bs.size * 64 == bloom.bbloom_params(n)[0]
        assert bloom.has(bs, min(locs, 64), b"anything")
