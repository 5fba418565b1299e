"""Loader for the committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest() -> dict:
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def sst_names() -> list[str]:
    return list(manifest()["sst"].keys())


def load_sst(name: str):
    """(case dict, sst bytes, blk_off, blk_len, key_end, val_end, blk_first)."""
    c = manifest()["sst"][name]
    with open(os.path.join(GOLDEN, c["file"]), "rb") as f:
        sst = f.read()
    n = c["nblocks"]
    index = np.frombuffer(sst[c["data_len"]: c["data_len"] + 4 * n], dtype=">u4").astype(np.uint64)
    assert int.from_bytes(sst[-4:], "big") == n
    off = np.concatenate([[0], index[:-1]]).astype(np.uint32)
    ln = (index - off).astype(np.uint32)
    ld = lambda s: np.load(os.path.join(GOLDEN, f"{name}.{s}.npy"))  # noqa: E731
    return c, sst, off, ln, ld("key_end"), ld("val_end"), ld("blk_first")


def load_blocks():
    b = manifest()["blocks"]
    with open(os.path.join(GOLDEN, b["file"]), "rb") as f:
        data = f.read()
    return b, data, np.array(b["blk_off"], np.uint32), np.array(b["blk_len"], np.uint32)
