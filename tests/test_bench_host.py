"""Host-side accounting of the bench line (no GPU): the walk's fetched-line pricing
(bench.walk_fetch_bytes, VERDICT r3 "price the walk by the lines it fetches") against a walk of
the blocks in Python that records every 8-B header read the way iterator.go:112-135 makes them,
and the PMC traffic summary's kernel selection (scripts/traffic_summary.py)."""
import csv
import os
import subprocess
import sys

import numpy as np
import pytest

from lsmdb_amd import workload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _blocks(oracle, parts):
    data = b"".join(parts)
    offs, lens, base = [], [], 0
    for p in parts:
        o, ln, _, _ = oracle.parse_index(p + b"{}" + (2).to_bytes(4, "big"))
        offs.append(o + base)
        lens.append(ln)
        base += len(p)
    return data, np.concatenate(offs).astype(np.uint32), np.concatenate(lens).astype(np.uint32)


def _header_lines(data, off, ln):
    """128-B lines holding the 8 bytes of every header the iterator reads (iterator.go:112-135):
    each entry's, plus the header it stops at when 10 bytes remain."""
    lines = set()
    for o, n in zip(off.tolist(), ln.tolist()):
        pos = 0
        while pos + 10 <= n:
            h = o + pos
            lines.update((h >> 7, (h + 7) >> 7))
            plen = int.from_bytes(data[h:h + 2], "big")
            klen = int.from_bytes(data[h + 2:h + 4], "big")
            vlen = int.from_bytes(data[h + 4:h + 6], "big")
            if (klen | plen) == 0:  # the terminator (Builder data: plen is always 0)
                break
            end = pos + 10 + klen + vlen
            if end > n:
                break
            pos = end
    return len(lines) * 128


@pytest.mark.parametrize("cfg,n", [(2, 6000), (3, 1500), (5, 2500)])
def test_walk_fetch_bytes_matches_header_walk(oracle, cfg, n):
    torch = pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench
    c = workload.config_columns(cfg, n, 7)
    parts = [oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, c.entries_per_block,
                               c.block_bytes)[0]]
    data, off, ln = _blocks(oracle, parts)
    ref = oracle.decode(data, off, ln)
    w = {"d_off": torch.from_numpy(off.view(np.int32).copy()),
         "d_len": torch.from_numpy(ln.view(np.int32).copy())}
    view = torch.from_numpy(np.asarray(ref.view).view(np.int64).copy())
    bf = torch.from_numpy(np.asarray(ref.blk_first).view(np.int32).copy())
    got = bench.walk_fetch_bytes(torch, w, view, bf)
    assert got == _header_lines(data, off, ln)
    if cfg == 2:  # C2's ~129-B entries: the walk touches every line of the input
        assert got >= 0.95 * len(data)
    if cfg == 3:  # C3's ~1.1 KB entries: a small share of the lines
        assert got < 0.3 * len(data)


def test_traffic_summary_sums_only_the_materialize_pipeline(tmp_path):
    """The view-only walk bench.py runs once to price the walk is not part of the decode."""
    names = ["void lsmgpu::wsc_walk_kernel<0, 256u, 32u, 19456u>(lsmgpu::DecodeParams)",
             "lsmgpu::wsc_copy_kernel(lsmgpu::DecodeParams)",
             "void lsmgpu::wsc_walk_kernel<3, 256u, 32u, 19456u>(lsmgpu::DecodeParams)",
             "void at::native::elementwise_kernel(...)"]
    rd, wr, fe, wsz = (tmp_path / f"{k}.csv" for k in ("rd", "wr", "fe", "ws"))

    def write(path, counters):
        with open(path, "w", newline="") as f:
            wtr = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            wtr.writeheader()
            d = 0
            for rep in range(3):
                for i, nm in enumerate(names):
                    d += 1
                    for cn, val in counters.items():
                        wtr.writerow({"Dispatch_Id": d, "Kernel_Name": nm, "Counter_Name": cn,
                                      "Counter_Value": val * (i + 1)})
    write(rd, {"TCC_EA0_RDREQ_sum": 10, "TCC_EA0_RDREQ_32B_sum": 0, "TCC_EA0_RDREQ_64B_sum": 0,
               "TCC_EA0_RDREQ_128B_sum": 10})
    write(wr, {"TCC_EA0_WRREQ_sum": 4, "TCC_EA0_WRREQ_64B_sum": 4})
    write(fe, {"FETCH_SIZE": 1})
    write(wsz, {"WRITE_SIZE": 1})
    bj = tmp_path / "bench.json"
    bj.write_text('{"roofline": {"algorithmic_bytes_per_launch": 1000}, '
                  '"config": {"workload": "C2 (configs[1]): 1000 B of SST data blocks"}}\n')
    out = tmp_path / "out.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "traffic_summary.py"), str(rd),
                    str(wr), str(fe), str(wsz), str(bj), str(out)], check=True, cwd=ROOT,
                   capture_output=True)
    import json
    j = json.loads(out.read_text())
    assert j["kernels"] == [n.split("(")[0][:90] for n in names[:2]]
    # walk (x1) + copy (x2) only: 3 x 10 128-B reads, 3 x 4 64-B writes
    assert j["read_bytes"] == 3 * 10 * 128 and j["write_bytes"] == 3 * 4 * 64
