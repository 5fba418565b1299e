"""One lsmgpu_ctx per OS thread, several threads at once (include/lsmgpu.h: "one lsmgpu_ctx per
OS thread"; the cgo shim's model, and compactBuildTables' per-table goroutines,
levels.go:281-298).  Two host threads, each with its own Codec on device 0, decode different
shards -- a large batch (the lane walk + copy), a small one (100 blocks: the group walk) -- and run a whole
compaction at the same time, several rounds; every output is checked against the oracle.
ctypes drops the GIL inside each library call, so the threads' HIP work really overlaps."""
import threading

import pytest

from lsmdb_amd.codec import Codec

from test_gpu_parity import _assert_same, _cols, _sst_blocks
from test_gpu_shim import _bottom_run, _oracle_compaction, _tables

pytestmark = pytest.mark.gpu


def _shard(oracle, cfg, n, seed):
    c = _cols(cfg, n, seed=seed)
    sst = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, c.entries_per_block, c.block_bytes)[0]
    return _sst_blocks(oracle, [sst])


@pytest.mark.parametrize("path", [None, "wsc"])
def test_two_contexts_concurrently(oracle, monkeypatch, path):
    if path:
        monkeypatch.setenv("LSMGPU_DECODE_PATH", path)
    jobs = [
        [_shard(oracle, 2, 60000, 51), _shard(oracle, 1, 10000, 52)],   # ~1,900 + 100 blocks
        [_shard(oracle, 5, 30000, 53), _shard(oracle, 4, 10000, 54)],   # 32 KiB / 100-entry
    ]
    refs = [[oracle.decode(*s) for s in shards] for shards in jobs]
    comp = [(_tables(oracle, 2, 3000, 60 + i) + _bottom_run(oracle, 2, 2500), [0, 1, 2, 4])
            for i in range(2)]
    want = [_oracle_compaction(oracle, ssts, rf, 1 << 20, False) for ssts, rf in comp]
    errors = []
    start = threading.Barrier(2)

    def worker(i):
        try:
            with Codec(0) as codec:
                start.wait(timeout=60)
                for rnd in range(3):
                    for s, ref in zip(jobs[i], refs[i]):
                        _assert_same(codec.decode_host(*s), ref, f"thread {i} round {rnd}")
                    ssts, rf = comp[i]
                    assert codec.compact_host(ssts, rf, 1 << 20) == want[i], f"thread {i} compaction"
        except Exception as e:  # reported by the main thread
            errors.append((i, repr(e)))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=110)
    assert not any(t.is_alive() for t in threads), "a worker thread did not finish"
    assert not errors, errors
