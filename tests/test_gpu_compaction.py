"""Device-resident compaction ("decode + encode into full compaction"):
the input tables of compactBuildTables (levels.go:239-298) decoded in one GPU batch, merged
(lsmgpu_merge_runs_async), cut where Builder.ReachedCapacity starts a new table
(lsmgpu_cut_tables_async) and encoded (lsmgpu_encode_tables_async), or -- gather mode -- merged
without its bytes and encoded straight from the decoded tables through the merge's source
index (lsmgpu_encode_tables_gather_async / lsmgpu_bloom_tables_gather_async).  Checked byte for byte
against the oracle: sstref_merge order, then the oracle Builder driven exactly like the Go loop
(`if builder.ReachedCapacity(cap) { break }; builder.Add(key, value)`, levels.go:265-271)."""
import ctypes

import numpy as np
import pytest

import open_cases as C

pytestmark = pytest.mark.gpu


def _oracle_tables(oracle, keys, vss, cap, bloom=False):
    """The Go loop's tables: Finish minus bloom, or (bloom=True) the complete .sst bytes --
    Finish's bbloom JSON over the table's keys (oracle/bbloom.c) + its BE32 length."""
    L = oracle.lib()
    out, i, n = [], 0, len(keys)
    while i < n:
        i0 = i
        b = L.sstref_builder_new(100, 0)
        while i < n:
            if L.sstref_builder_reached_capacity(b, cap):
                break
            k, v = keys[i], vss[i]
            L.sstref_builder_add(b, k, len(k), v, len(v))
            i += 1
        ol, dl, nr = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        rs = ctypes.POINTER(ctypes.c_uint32)()
        ptr = L.sstref_builder_finish(b, ctypes.byref(ol), ctypes.byref(dl), ctypes.byref(rs),
                                      ctypes.byref(nr))
        img = ctypes.string_at(ptr, ol.value)
        L.sstref_builder_free(b)
        if bloom:
            kb, ke = oracle.columns(keys[i0:i], vss[i0:i])[:2]
            bs, bits, locs, _ = oracle.bloom_build(kb, ke)
            js = oracle.bloom_json(bs, bits, locs)
            img += js + len(js).to_bytes(4, "big")
        out.append(img)
    return out


@pytest.mark.parametrize("gather", [False, True])
@pytest.mark.parametrize("bloom", [False, True])
@pytest.mark.parametrize("cap", [1 << 17, 1 << 20, 3 << 20])  # 1 << 17: > 32 tables
def test_device_compaction(codec, oracle, cap, bloom, gather):
    import torch
    from lsmdb_amd import workload
    parts = []
    for s in range(3):
        c = workload.config_columns(4, 50000, seed_offset=0)  # one key space: overlapping tables
        idx = np.nonzero(np.random.default_rng(40 + s).random(50000) < 0.6)[0]
        keys = [bytes(c.keys[(c.key_end[i - 1] if i else 0): c.key_end[i]]) for i in idx]
        vss = [bytes(c.vs[(c.vs_end[i - 1] if i else 0): c.vs_end[i]]) for i in idx]
        parts.append(oracle.build(keys, vss, entries_per_block=100)[0])
    data = b"".join(parts)
    offs, lens, firsts, base = [], [], [], 0
    for p in parts:
        o, l, _, _ = oracle.parse_index(p + C.TAIL)
        firsts.append(sum(len(x) for x in offs))
        offs.append(o + base)
        lens.append(l)
        base += len(p)
    off = np.concatenate(offs).astype(np.uint32)
    ln = np.concatenate(lens).astype(np.uint32)
    dec = codec.decode_host(data, off, ln)
    rf = np.array([int(dec.blk_first[b]) for b in firsts] + [int(dec.blk_first[-1])], np.uint32)
    kd, ke = dec.key_data.tobytes(), dec.key_end
    vd, ve = dec.val_data.tobytes(), dec.val_end
    # device: merge -> cut -> encode, all on the device buffers
    dev = torch.device("cuda", codec.device)
    t = lambda a, dt: torch.from_numpy(np.array(a, copy=True).view(dt)).to(dev)
    d_kd, d_ke = t(np.frombuffer(kd + b"\0" * 16, np.uint8), np.uint8), t(ke, np.int32)
    d_vd, d_ve = t(np.frombuffer(vd + b"\0" * 16, np.uint8), np.uint8), t(ve, np.int32)
    m = codec.merge_device(d_kd, d_ke, d_vd, d_ve, t(rf, np.int32), int(rf[-1]), gather=not gather)
    codec.synchronize()
    r = m["result"].cpu().numpy()
    n_out, kb, vb = int(r[0]), int(r[1]), int(r[2])
    if not gather:
        o = codec.compact_tables_device(m["key_data"], m["key_end"], m["val_data"], m["val_end"],
                                        n_out, kb, vb, cap, bloom=bloom)
    else:  # the merged order only; bytes read from the decoded tables through src
        o = codec.cut_tables_device(m["key_end"], m["val_end"], n_out, cap, bloom=bloom)
        codec.synchronize()
        cr = o["result"].cpu().numpy()
        o["ntables"], o["bytes"] = int(cr[0]), int(cr[2])
        o["out"] = torch.empty(o["bytes"] + 16, dtype=torch.uint8, device=dev)
        o["flags"] = torch.zeros(4, dtype=torch.int32, device=dev)
        codec.encode_tables_gather_device(o, d_kd, d_ke, d_vd, d_ve, m["src"], m["key_end"],
                                          m["val_end"], kb, vb, o["out"], o["flags"])
        if bloom:
            o["bloom_flags"] = torch.zeros(1, dtype=torch.int32, device=dev)
            codec.bloom_tables_device(o, d_kd, d_ke, o["out"], o["bloom_flags"], src=m["src"])
    codec.synchronize()
    assert int(o["flags"][0].item()) == 0
    if bloom:
        assert int(o["bloom_flags"][0].item()) == 0
    # oracle: merge order, then the Go Builder loop
    src = oracle.merge(kd, ke, rf)
    ks = [kd[(ke[i - 1] if i else 0): ke[i]] for i in src]
    vs = [vd[(ve[i - 1] if i else 0): ve[i]] for i in src]
    ref = _oracle_tables(oracle, ks, vs, cap, bloom)
    assert o["ntables"] == len(ref) and len(ref) >= 2
    img = o["out"].cpu().numpy().tobytes()
    tout = o["tbl_out"].cpu().numpy()
    for k, want in enumerate(ref):
        assert img[int(tout[k]): int(tout[k + 1])] == want, f"table {k}"
