"""Compaction replay on one MI355X (levels.go:239-298 compactBuildTables with L >= 1: one top
table merged with the concatenated bottom tables), device-resident end to end:
  decode  all blocks of the 1 + 8 input tables (64 MiB each, C4 shape) in one batch
  merge   2 runs (top = nice 0, bottom = nice 1): y.MergeIterator, top wins on equal keys
  cut     the merged stream into output tables where Builder.ReachedCapacity(64 MiB) starts a
          new one (levels.go:265-271)
  encode  every output table (100-entry blocks, Builder.Add / finishBlock / blockIndex) in one
          launch, reading each entry's bytes from the decoded tables through the merge's source
          index (GATHER=0: the merge writes merged key / value streams and the encoder reads them)
Top keys are updates of every 8th bottom key (same key, new value): the merge drops 1/9 of its
input.  HIP-event times (median of 5) per stage; the oracle merge (sstref_merge, 1 thread)
timed on the host for the same runs; the merged keys/values checked against it.
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

PER_TABLE = 519540  # ReachedCapacity(64 MiB) at 100 entries/block, 16 B / 100 B


def timed(torch, stream, fn, reps=5):
    ts, out = [], None
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        out = fn()
        b.record(stream)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), out


def main():
    import torch
    from lsmdb_amd import workload
    from lsmdb_amd import codec as C
    nbot = int(os.environ.get("BOTTOM_TABLES", "8"))
    dev = torch.device("cuda", 0)
    codec = C.Codec(0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    codec.set_stream(stream.cuda_stream)

    bot = workload.config_columns(4, PER_TABLE * nbot)
    ke_b, ve_b = bot.key_end.astype(np.int64), bot.vs_end.astype(np.int64)
    top_idx = np.arange(0, PER_TABLE * nbot, 8)[:PER_TABLE]
    rng = np.random.default_rng(11)
    top_keys = np.concatenate([bot.keys[(ke_b[i - 1] if i else 0): ke_b[i]] for i in top_idx])
    top_ke = np.cumsum(ke_b[top_idx] - np.where(top_idx > 0, ke_b[top_idx - 1], 0)).astype(np.uint32)
    vlen = 103
    top_vs = np.tile(np.frombuffer(b"A\x00\x00" + bytes(100), np.uint8), top_idx.size).copy()
    top_vs[3::vlen] = rng.integers(0, 256, top_idx.size, dtype=np.uint8)
    top_ve = (np.arange(1, top_idx.size + 1) * vlen).astype(np.uint32)

    def encode(keys, ke, vs, ve, epb=100):
        n = ke.size
        nb = (n + epb - 1) // epb
        kt, vt = int(ke[-1]), int(vs.size)
        out_len = 10 * n + kt + vt + 13 * nb + 4 * nb + 4
        d = torch.empty(out_len + 16, dtype=torch.uint8, device=dev)
        fl = torch.zeros(4, dtype=torch.int32, device=dev)
        codec.encode_device_async(torch.from_numpy(keys).to(dev), torch.from_numpy(ke.view(np.int32)).to(dev),
                                  torch.from_numpy(vs).to(dev), torch.from_numpy(ve.view(np.int32)).to(dev),
                                  n, kt, vt, d, fl, entries_per_block=epb)
        data_len = 10 * n + kt + vt + 13 * nb
        ends = d[data_len: data_len + 4 * nb].cpu().numpy().view(">u4").astype(np.int64)
        return d[:data_len], ends

    # input tables: top, then the bottom tables (consecutive key ranges)
    tables = [encode(top_keys, top_ke, top_vs, top_ve)]
    for t in range(nbot):
        lo, hi = t * PER_TABLE, (t + 1) * PER_TABLE
        k0, k1 = (ke_b[lo - 1] if lo else 0), ke_b[hi - 1]
        v0, v1 = (ve_b[lo - 1] if lo else 0), ve_b[hi - 1]
        tables.append(encode(bot.keys[k0:k1].copy(), (ke_b[lo:hi] - k0).astype(np.uint32),
                             bot.vs[v0:v1].copy(), (ve_b[lo:hi] - v0).astype(np.uint32)))
    data = torch.cat([d for d, _ in tables])
    offs, lens, first_blk, base = [], [], [], 0
    for d, ends in tables:
        first_blk.append(sum(len(o) for o in offs))
        o = np.concatenate([[0], ends[:-1]])
        offs.append(o + base)
        lens.append(ends - o)
        base += d.numel()
    off = np.concatenate(offs).astype(np.uint32)
    ln = np.concatenate(lens).astype(np.uint32)
    n_in = int(top_idx.size + PER_TABLE * nbot)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
    bufs = codec.alloc_decode(data.numel(), data.numel(), off.size, C.MODE_MATERIALIZE, ent_cap=n_in)
    torch.cuda.synchronize()

    t_dec, _ = timed(torch, stream, lambda: codec.decode_device_async(
        data, d_off, d_len, int(ln.max()), C.MODE_MATERIALIZE, bufs, data_len=data.numel()))
    blk_first = bufs.blk_first.cpu().numpy().view(np.uint32)
    run_first = torch.tensor([0, int(blk_first[first_blk[1]]), n_in], dtype=torch.int32, device=dev)
    # gather (default): the merge writes the merged order only and the encoder / bloom read
    # each entry's bytes from the decoded tables through src (one copy, as builder.Add makes);
    # GATHER=0: the merge also writes merged key / value streams and the encoder reads those
    gather = os.environ.get("GATHER", "1") != "0"
    t_merge, m = timed(torch, stream, lambda: codec.merge_device(
        bufs.key_data, bufs.key_end, bufs.val_data, bufs.val_end, run_first, n_in,
        gather=not gather))
    r = m["result"].cpu().numpy()
    n_out, kb, vb = int(r[0]), int(r[1]), int(r[2])

    # output tables: ReachedCapacity(64 MiB) cut, then every table encoded in one launch
    mk, mke, mv, mve = m["key_data"], m["key_end"], m["val_data"], m["val_end"]
    t_cut, cut = timed(torch, stream, lambda: codec.cut_tables_device(mke, mve, n_out, 64 << 20,
                                                                      bloom=True))
    cr = cut["result"].cpu().numpy()
    ntab_out, out_bytes = int(cr[0]), int(cr[2])
    cut["ntables"] = ntab_out
    d_out = torch.empty(out_bytes + 16, dtype=torch.uint8, device=dev)
    fl = torch.zeros(4, dtype=torch.int32, device=dev)
    if gather:
        t_enc, _ = timed(torch, stream, lambda: codec.encode_tables_gather_device(
            cut, bufs.key_data, bufs.key_end, bufs.val_data, bufs.val_end, m["src"], mke, mve,
            kb, vb, d_out, fl))
        bargs = (bufs.key_data, bufs.key_end, d_out)
        bsrc = m["src"]
    else:
        t_enc, _ = timed(torch, stream, lambda: codec.encode_tables_device(
            cut, mk, mke, mv, mve, kb, vb, d_out, fl))
        bargs, bsrc = (mk, mke, d_out), None
    # Finish's bloom tails (complete .sst files); the host reads the cut's small arrays first
    bfl = torch.zeros(1, dtype=torch.int32, device=dev)
    codec.bloom_tables_device(cut, *bargs, bfl, src=bsrc)  # warm-up (and sizes the scratch)
    t_bloom, _ = timed(torch, stream, lambda: codec.bloom_tables_device(cut, *bargs, bfl, src=bsrc))

    # oracle merge on the host, and the check
    import oracle_ffi
    oracle_ffi.lib()
    kd = bufs.key_data[: int(bufs.key_end[n_in - 1].item())].cpu().numpy()
    ke = bufs.key_end[:n_in].cpu().numpy().view(np.uint32)
    t0 = time.perf_counter()
    src = oracle_ffi.merge(kd, ke, np.array([0, int(blk_first[first_blk[1]]), n_in], np.uint32))
    cpu_merge_s = time.perf_counter() - t0
    ok = (r[3] == 0 and src.size == n_out and
          np.array_equal(m["src"][:n_out].cpu().numpy().view(np.uint32), src))
    in_bytes = int(data.numel())
    print(json.dumps({
        "what": "compaction replay: decode 1+%d C4 tables -> merge (2 runs) -> encode + bloom "
                "(complete .sst files)" % nbot,
        "input_table_bytes": in_bytes, "entries_in": n_in, "entries_out": n_out,
        "output_tables": ntab_out, "output_bytes": out_bytes,
        "decode_ms": round(t_dec, 4), "merge_ms": round(t_merge, 4), "cut_ms": round(t_cut, 4),
        "encode_ms": round(t_enc, 4), "bloom_ms": round(t_bloom, 4),
        "total_ms": round(t_dec + t_merge + t_cut + t_enc + t_bloom, 4),
        "input_gibs": round(in_bytes / ((t_dec + t_merge + t_cut + t_enc + t_bloom) / 1e3) /
                            (1 << 30), 2),
        "cpu_oracle_merge_ms": round(cpu_merge_s * 1e3, 1),
        "merge_matches_oracle": bool(ok), "gather": gather}))
    codec.close()


if __name__ == "__main__":
    main()
