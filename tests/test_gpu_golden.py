"""gfx950 encode/decode (through the C ABI) vs the committed golden fixtures."""
import numpy as np
import pytest

import golden_io as G
from lsmdb_amd import workload

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", G.sst_names())
def test_gpu_decode_golden(codec, name):
    c, sst, off, ln, key_end, val_end, blk_first = G.load_sst(name)
    d = codec.decode_host(sst[: c["data_len"]], off, ln)
    assert d.n_entries == c["entries"] and d.n_bad_blocks == 0
    assert not d.blk_status.any()
    assert np.array_equal(d.key_end, key_end) and np.array_equal(d.val_end, val_end)
    assert np.array_equal(d.blk_first, blk_first)
    assert G.sha(d.key_data) == c["key_sha256"] and G.sha(d.val_data) == c["val_sha256"]


@pytest.mark.parametrize("name", G.sst_names())
def test_gpu_encode_golden(codec, name):
    c, sst, *_ = G.load_sst(name)
    cols = workload.config_columns(c["config"], c["entries"])
    out, data_len, restarts = codec.encode_host(cols.keys, cols.key_end, cols.vs, cols.vs_end,
                                                c["entries_per_block"], c["block_bytes"])
    assert data_len == c["data_len"] and restarts.size == c["nblocks"]
    assert G.sha(out) == c["sst_sha256"]


def test_gpu_decode_golden_blocks(codec):
    b, data, off, ln = G.load_blocks()
    d = codec.decode_host(data, off, ln)
    assert [int(s) for s in d.blk_status] == b["blk_status"]
    assert [int(x) for x in d.blk_first] == b["blk_first"]
    assert [[d.key(i).hex(), d.value(i).hex()] for i in range(d.n_entries)] == b["entries"]
    assert d.first_bad_block == b["first_bad_block"] and d.n_bad_blocks == b["n_bad_blocks"]
