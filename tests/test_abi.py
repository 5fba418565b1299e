"""The C-ABI library: loads, exports every symbol include/lsmgpu.h declares, host-only entry
points (tail parse, block planner) match the oracle; kernel resource budgets hold.  No GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

from lsmdb_amd import _lib, codec, workload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lsmgpu.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lsmgpu_[a-z_0-9]+)\s*\(", txt)))


def test_header_symbols_exported():
    names = header_functions()
    assert len(names) >= 14
    lib = _lib.lib()
    for n in names:
        assert hasattr(lib, n), f"{n} not exported by liblsmgpu.so"
    assert set(names) == set(_lib.EXPORTED_SYMBOLS)


def test_exports_via_nm():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for n in header_functions():
        assert n in syms


def test_version_and_strerror():
    lib = _lib.lib()
    assert lib.lsmgpu_abi_version() == 4
    for code in range(0, 12):
        assert lib.lsmgpu_strerror(code)
    assert lib.lsmgpu_strerror(_lib.ERR_CAPACITY) == b"output buffer too small"


def test_open_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.LsmgpuError) as e:
        codec.Codec(0)
    assert e.value.code == _lib.ERR_NO_DEVICE


@pytest.mark.parametrize("cfg,n", [(1, 10000), (2, 5000), (3, 500), (5, 3000), (1, 0)])
def test_parse_index_matches_oracle(oracle, cfg, n):
    if n == 0:
        body, _, _ = oracle.build([], [], 100)
    else:
        c = workload.config_columns(cfg, n)
        body, _, _ = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, c.entries_per_block,
                                       c.block_bytes)
    sst = body + b'{"FilterSet":"","SetLocs":7}' + (28).to_bytes(4, "big")
    a = codec.parse_index(sst)
    b = oracle.parse_index(sst)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2:] == b[2:]


@pytest.mark.parametrize("bad", [b"", b"\x00" * 7, b"\x00\x00\x00\x00\xff\xff\xff\xff",
                                 b"\x00" * 8 + b"\x00\x00\x00\x05",
                                 b"\x00\x00\x00\x10" + b"\x00\x00\x00\x02" + b"\x00\x00\x00\x00"])
def test_parse_index_malformed(bad):
    with pytest.raises(_lib.LsmgpuError) as e:
        codec.parse_index(bad)
    assert e.value.code == _lib.ERR_BAD_TAIL


@pytest.mark.parametrize("cfg,n", [(1, 10000), (2, 20000), (3, 1000), (5, 20000)])
def test_plan_blocks_matches_oracle_restarts(oracle, cfg, n):
    c = workload.config_columns(cfg, n)
    plan = codec.plan_blocks(c.key_end, c.vs_end, c.entries_per_block, c.block_bytes)
    _, _, restarts = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, c.entries_per_block,
                                       c.block_bytes)
    assert plan.size - 1 == restarts.size
    # block end = 10*e + key bytes + vs bytes + 13 per block, at each plan boundary
    ke = np.concatenate([[0], c.key_end.astype(np.int64)])
    ve = np.concatenate([[0], c.vs_end.astype(np.int64)])
    e = plan[1:].astype(np.int64)
    ends = 10 * e + ke[e] + ve[e] + 13 * np.arange(1, plan.size)
    assert np.array_equal(ends, restarts.astype(np.int64))


def _resource_usage(src):
    out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                          "-Rpass-analysis=kernel-resource-usage", src, "-o", os.devnull],
                         capture_output=True, text=True, cwd=os.path.dirname(src))
    assert out.returncode == 0, out.stderr[-2000:]
    res, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
            continue
        m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|ScratchSize \[bytes/lane\]): (\d+)", line)
        if m and cur:
            res[cur][m.group(1)] = int(m.group(2))
    return res


def test_decode_resource_budget():
    """launch_cfg sizes the persistent grid from kDecodeSgprs: the compiled kernels must stay
    within it (or the grid could exceed residency); no scratch spills."""
    src = os.path.join(ROOT, "lsmdb_amd", "csrc", "decode.hip")
    budget = int(re.search(r"kDecodeSgprs = (\d+)", open(src).read()).group(1))
    res = _resource_usage(src)
    kernels = {k: v for k, v in res.items() if "decode_kernel" in k}
    assert kernels
    for k, v in kernels.items():
        assert v["TotalSGPRs"] <= budget, (k, v)
        assert v["ScratchSize [bytes/lane]"] == 0, (k, v)


@pytest.mark.parametrize("cfg,n", [(1, 10000), (2, 3000), (3, 200), (5, 2000), (1, 0)])
def test_encode_size_query_without_device(oracle, cfg, n):
    """INTEGRATION.md's finishBlocks step 1: lsmgpu_encode_blocks with out == NULL (and a NULL
    ctx: host arrays) reports the exact image size, data length and restart count."""
    import ctypes
    from ctypes import byref, c_uint64
    if n:
        c = workload.config_columns(cfg, n)
        ke, ve, epb, bb = c.key_end, c.vs_end, c.entries_per_block, c.block_bytes
        body, dl, rs = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, epb, bb)
    else:
        ke = ve = np.zeros(0, np.uint32)
        epb, bb = 100, 0
        body, dl, rs = oracle.build([], [], 100)
    ol, dlen, nr = c_uint64(0), c_uint64(0), c_uint64(0)
    rc = _lib.lib().lsmgpu_encode_blocks(None, None, codec._ptr(ke), None, codec._ptr(ve), ke.size,
                                         0, epb, bb, None, 0, byref(ol), byref(dlen), None, 0,
                                         byref(nr))
    assert rc == _lib.OK
    assert ol.value == len(body) and dlen.value == dl and nr.value == len(rs)
    _ = ctypes


def test_encode_size_query_rejects_short_key():
    from ctypes import byref, c_uint64
    ke = np.array([16, 24], np.uint32)  # second key is 8 B: y.ParseKey's len > 8 assertion
    ve = np.array([5, 10], np.uint32)
    ol, dl, nr = c_uint64(0), c_uint64(0), c_uint64(0)
    rc = _lib.lib().lsmgpu_encode_blocks(None, None, codec._ptr(ke), None, codec._ptr(ve), 2, 0,
                                         100, 0, None, 0, byref(ol), byref(dl), None, 0, byref(nr))
    assert rc == _lib.ERR_KEY_LEN
    # a real call (out != NULL) still needs a context
    rc = _lib.lib().lsmgpu_encode_blocks(None, None, codec._ptr(ke), None, codec._ptr(ve), 2, 0,
                                         100, 0, codec._ptr(np.zeros(64, np.uint8)), 64, byref(ol),
                                         byref(dl), None, 0, byref(nr))
    assert rc == _lib.ERR_ARG
