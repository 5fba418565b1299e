"""Generates the golden fixtures in tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

Each fixture is DATA: the SST bytes `[data blocks][restarts BE32 x N][N BE32]` (the bbloom tail is
excluded: its parity is unpinned) plus the expected decode -- per-entry end
offsets as .npy and SHA-256 digests of the key / value streams -- and the SHA-256 of the seeded
input columns, so the generator itself is pinned too.  The bytes come from the C oracle
(oracle/sstref.c, a restatement of table/builder.go:84-198 and table/iterator.go:93-135), which
tests/test_oracle_kat.py pins to hand-derived known answers; tests/test_golden.py re-derives every
fixture from the oracle (CPU) and tests/test_gpu_golden.py checks the gfx950 encoder and decoder
against the committed files (GPU).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from lsmdb_amd import workload  # noqa: E402
import oracle_ffi as ofi  # noqa: E402
import kat_defs as kd  # noqa: E402

# (name, config, entries, entries_per_block or None = the config's rule, block_bytes or None)
SST_CASES = [
    ("c1_table_test", 1, 10_000, None, None),   # table_test.go path: 10k entries, 100 / block
    ("c2_4k_blocks", 2, 3_000, None, None),     # headline shape: 4 KiB byte target
    ("c3_64k_1k", 3, 300, None, None),          # 64 B keys / 1 KiB values, 4 KiB target
    ("c5_zipf_32k", 5, 2_000, None, None),      # Zipf keys, 32 KiB target
    ("c1_cut_7", 1, 1_000, 7, 0),               # odd resultInterval
]


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def blocks_of(restarts):
    """Block i = [restarts[i-1] or 0, restarts[i]) (table/table.go:203-215)."""
    r = np.asarray(restarts, np.uint64)
    off = np.concatenate([[0], r[:-1]]).astype(np.uint32)
    return off, (r - off).astype(np.uint32)


def sst_case(name, cfg, n, epb, bb):
    c = workload.config_columns(cfg, n)
    epb = c.entries_per_block if epb is None else epb
    bb = c.block_bytes if bb is None else bb
    sst, data_len, restarts = ofi.build_cols(c.keys.tobytes(), c.key_end, c.vs.tobytes(), c.vs_end,
                                             epb, bb)
    off, ln = blocks_of(restarts)
    dec = ofi.decode(sst[:data_len], off, ln)
    assert dec.n_entries == n and dec.n_bad_blocks == 0
    assert dec.key_data.tobytes() == c.keys.tobytes() and dec.val_data.tobytes() == c.vs.tobytes()
    with open(os.path.join(HERE, name + ".sst"), "wb") as f:
        f.write(sst)
    np.save(os.path.join(HERE, name + ".key_end.npy"), dec.key_end.astype("<u4"))
    np.save(os.path.join(HERE, name + ".val_end.npy"), dec.val_end.astype("<u4"))
    np.save(os.path.join(HERE, name + ".blk_first.npy"), dec.blk_first.astype("<u4"))
    return {
        "file": name + ".sst", "config": cfg, "entries": n, "entries_per_block": epb,
        "block_bytes": bb, "data_len": int(data_len), "nblocks": int(restarts.size),
        "sst_sha256": sha(sst), "key_sha256": sha(dec.key_data), "val_sha256": sha(dec.val_data),
        "key_bytes": int(dec.key_data.size), "val_bytes": int(dec.val_data.size),
        "input_sha256": {"keys": sha(c.keys), "key_end": sha(c.key_end.astype("<u4")),
                         "vs": sha(c.vs), "vs_end": sha(c.vs_end.astype("<u4"))},
    }


def blocks_case():
    """Every decode KAT block concatenated (misaligned offsets), one batch: statuses + entries."""
    blocks = [blk for _, blk, _, _ in kd.DECODE_KATS]
    data = bytearray(b"\x5a" * 3)  # leading junk: block 0 starts at an odd offset
    off, ln = [], []
    for b in blocks:
        off.append(len(data))
        ln.append(len(b))
        data += b + b"\xa5"  # one junk byte between blocks
    dec = ofi.decode(bytes(data), np.array(off, np.uint32), np.array(ln, np.uint32))
    with open(os.path.join(HERE, "kat_blocks.bin"), "wb") as f:
        f.write(bytes(data))
    entries = [[dec.key(i).hex(), dec.value(i).hex()] for i in range(dec.n_entries)]
    return {
        "file": "kat_blocks.bin", "names": [nm for nm, _, _, _ in kd.DECODE_KATS],
        "blk_off": off, "blk_len": ln, "blk_status": [int(s) for s in dec.blk_status],
        "blk_first": [int(x) for x in dec.blk_first], "entries": entries,
        "first_bad_block": int(dec.first_bad_block), "n_bad_blocks": int(dec.n_bad_blocks),
    }


def main():
    manifest = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/sstref.c",
                "seed_base": hex(workload.SEED_BASE), "sst": {}, "blocks": None}
    for case in SST_CASES:
        manifest["sst"][case[0]] = sst_case(*case)
    manifest["blocks"] = blocks_case()
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
