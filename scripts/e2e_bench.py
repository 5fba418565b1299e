"""End-to-end decode from host memory (SURVEY §8(d) "End-to-end"): the C2 1 GiB shard in pinned
host memory (what hipHostRegister makes of the mmap'd .sst), decoded in chunks of whole blocks
with three streams and double-buffered device slots:
  copy-in   chunk c: H2D of its block bytes                       (stream A)
  decode    chunk c: walk-scan-copy, materialize mode             (stream B, after A's event)
  copy-out  chunk c: D2H of key / value streams + end offsets     (stream C, after B's event)
so chunk c+1's H2D and chunk c-1's D2H overlap chunk c's decode.  Reported beside the PCIe
bound measured on the same box (pinned H2D and D2H of the same byte counts, and both at once).
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from lsmdb_amd import codec as C
    import bench
    chunk_bytes = int(os.environ.get("CHUNK_MIB", "64")) << 20
    dev = torch.device("cuda", 0)
    codec = C.Codec(0)
    w = bench.build_device_sst(codec, torch, dev, 2, 1 << 30, 0)
    data_len, offs, lens = w["data_len"], w["offs"], w["lens"]
    host = torch.empty(data_len, dtype=torch.uint8).pin_memory()
    host.copy_(w["d_sst"][:data_len])
    del w
    torch.cuda.empty_cache()

    # chunks of whole blocks (~chunk_bytes each); block offsets rebased to the chunk
    bounds, b0 = [], 0
    ends = offs.astype(np.int64) + lens
    while b0 < offs.size:
        limit = int(offs[b0]) + chunk_bytes
        b1 = int(np.searchsorted(ends, limit, side="right"))
        b1 = max(b1, b0 + 1)
        bounds.append((b0, b1))
        b0 = b1
    chunks = []
    for b0, b1 in bounds:
        base = int(offs[b0])
        size = int(ends[b1 - 1]) - base
        o = torch.from_numpy((offs[b0:b1] - base).astype(np.uint32).view(np.int32)).to(dev)
        l = torch.from_numpy(lens[b0:b1].astype(np.uint32).view(np.int32)).to(dev)
        chunks.append(dict(base=base, size=size, off=o, len=l, max=int(lens[b0:b1].max()),
                           nblk=b1 - b0))
    cap = max(c["size"] for c in chunks)
    max_nblk = max(c["nblk"] for c in chunks)
    ent_cap = cap // 10 + 1
    nslots = int(os.environ.get("SLOTS", "3"))
    # view mode: the host already holds the SST bytes (the mmap), so only the 8-B entry index
    # {key position, klen, vlen} comes back and keys / values are sliced from the host copy
    view = os.environ.get("E2E_MODE", "materialize") == "view"
    mode = C.MODE_VIEW if view else C.MODE_MATERIALIZE
    slots = [dict(d=torch.empty(cap + 64, dtype=torch.uint8, device=dev),
                  bufs=codec.alloc_decode(cap, 0 if view else cap, max_nblk, mode, ent_cap=ent_cap))
             for _ in range(nslots)]
    # host outputs (pinned): key + value streams and end offsets of the whole shard
    out_k = torch.empty(data_len, dtype=torch.uint8).pin_memory()
    out_v = torch.empty(data_len, dtype=torch.uint8).pin_memory()
    out_ke = torch.empty(data_len // 10, dtype=torch.int32).pin_memory()
    out_ve = torch.empty(data_len // 10, dtype=torch.int32).pin_memory()
    out_view = torch.empty(data_len // 10, dtype=torch.int64).pin_memory()
    sa, sb, sc = (torch.cuda.Stream(device=dev) for _ in range(3))
    codec.set_stream(sb.cuda_stream)

    # per-chunk output sizes (from a first decode pass) so the D2H copies are sized statically
    sizes = []
    for c in chunks:
        s = slots[0]
        s["d"][: c["size"]].copy_(host[c["base"]: c["base"] + c["size"]])
        torch.cuda.synchronize()
        codec.decode_device_async(s["d"], c["off"], c["len"], c["max"], mode,
                                  s["bufs"], data_len=c["size"])
        codec.synchronize()
        r = s["bufs"].result.cpu().numpy()
        sizes.append((int(r[0]), int(r[1]), int(r[2])))
    torch.cuda.synchronize()

    def run():
        ev_in = [torch.cuda.Event() for _ in chunks]
        ev_dec = [torch.cuda.Event() for _ in chunks]
        ev_out = [torch.cuda.Event() for _ in chunks]
        pos_e = pos_k = pos_v = 0
        for i, c in enumerate(chunks):
            s = slots[i % nslots]
            with torch.cuda.stream(sa):
                if i >= nslots:
                    sa.wait_event(ev_dec[i - nslots])  # slot's input no longer read
                s["d"][: c["size"]].copy_(host[c["base"]: c["base"] + c["size"]], non_blocking=True)
                ev_in[i].record(sa)
            sb.wait_event(ev_in[i])
            if i >= nslots:
                sb.wait_event(ev_out[i - nslots])  # slot's outputs copied out
            codec.decode_device_async(s["d"], c["off"], c["len"], c["max"], mode,
                                      s["bufs"], data_len=c["size"])
            ev_dec[i].record(sb)
            n, kb, vb = sizes[i]
            with torch.cuda.stream(sc):
                sc.wait_event(ev_dec[i])
                b = s["bufs"]
                if view:
                    out_view[pos_e: pos_e + n].copy_(b.view[:n], non_blocking=True)
                else:
                    out_k[pos_k: pos_k + kb].copy_(b.key_data[:kb], non_blocking=True)
                    out_v[pos_v: pos_v + vb].copy_(b.val_data[:vb], non_blocking=True)
                    out_ke[pos_e: pos_e + n].copy_(b.key_end[:n], non_blocking=True)
                    out_ve[pos_e: pos_e + n].copy_(b.val_end[:n], non_blocking=True)
                ev_out[i].record(sc)
            pos_e, pos_k, pos_v = pos_e + n, pos_k + kb, pos_v + vb
        torch.cuda.synchronize()
        return pos_e, pos_k, pos_v

    run()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        n_tot, k_tot, v_tot = run()
        ts.append(time.perf_counter() - t0)
    e2e = float(np.median(ts))
    out_bytes = 8 * n_tot if view else k_tot + v_tot + 8 * n_tot

    # PCIe bound on this box: pinned H2D, D2H of the same byte counts, and both at once
    dbuf = torch.empty(data_len, dtype=torch.uint8, device=dev)
    obuf = torch.empty(out_bytes, dtype=torch.uint8, device=dev)
    hout = torch.empty(out_bytes, dtype=torch.uint8).pin_memory()

    def wall(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    wall(lambda: dbuf.copy_(host, non_blocking=True))
    h2d = wall(lambda: dbuf.copy_(host, non_blocking=True))
    d2h = wall(lambda: hout.copy_(obuf, non_blocking=True))

    def both():
        with torch.cuda.stream(sa):
            dbuf.copy_(host, non_blocking=True)
        with torch.cuda.stream(sc):
            hout.copy_(obuf, non_blocking=True)
    duplex = wall(both)
    print(json.dumps({
        "what": "end-to-end decode from pinned host memory (H2D + decode + D2H, 3 streams)",
        "mode": "view" if view else "materialize",
        "input_bytes": data_len, "output_bytes": out_bytes, "chunks": len(chunks), "slots": nslots,
        "chunk_bytes": chunk_bytes, "entries": n_tot,
        "e2e_ms": round(e2e * 1e3, 2), "e2e_input_gibs": round(data_len / e2e / (1 << 30), 2),
        "pcie_h2d_gbs": round(data_len / h2d / 1e9, 1),
        "pcie_d2h_gbs": round(out_bytes / d2h / 1e9, 1),
        "pcie_duplex_ms": round(duplex * 1e3, 2),
        "bound_ms": round(max(duplex, h2d, d2h) * 1e3, 2),
        "frac_of_pcie_bound": round(max(duplex, h2d, d2h) / e2e, 3),
        "entries_match": n_tot == sum(s[0] for s in sizes)}))
    codec.close()


if __name__ == "__main__":
    main()
