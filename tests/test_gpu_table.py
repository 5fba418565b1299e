"""table_test.go end to end: lsmdb_amd.table.Builder (gfx950 encoder) -> .sst file ->
OpenTable (gfx950 decoder) -> Iterator / ConcatIterator / MergeIterator."""
import pytest

import table_cases as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(codec):
    return C.GpuEnv(codec)


@pytest.mark.parametrize("n", C.NS)
def test_seek_to_first(env, n):
    C.seek_to_first(env, n)


@pytest.mark.parametrize("n", C.NS)
def test_seek_to_last(env, n):
    C.seek_to_last(env, n)


def test_seek(env):
    C.seek(env)


def test_seek_for_prev(env):
    C.seek_for_prev(env)


@pytest.mark.parametrize("n", C.NS)
def test_iterate_from_start(env, n):
    C.iterate_from_start(env, n)


@pytest.mark.parametrize("n", C.NS)
def test_iterate_from_end(env, n):
    C.iterate_from_end(env, n)


def test_table(env):
    C.table_seek_iterate(env)


def test_iterate_back_and_forth(env):
    C.iterate_back_and_forth(env)


def test_uni_iterator(env):
    C.uni_iterator(env)


def test_concat_iterator_one_table(env):
    C.concat_one_table(env)


def test_concat_iterator(env):
    C.concat_iterator(env)


@pytest.mark.parametrize("rev", [False, True])
def test_merging_iterator(env, rev):
    C.merging_iterator(env, rev)


@pytest.mark.parametrize("which", [1, 2])
def test_merging_iterator_take(env, which):
    C.merging_take(env, which)


def test_file_lifecycle(env):
    C.file_lifecycle(env)


def test_builder_bytes_match_oracle(env, oracle):
    """Builder.Finish (GPU) == oracle Builder bytes over [0, index_end), bloom tail parsed."""
    kvs = C.test_kvs("key", 1234)
    raw = env.build_bytes(kvs)
    cpu = C.CpuEnv(oracle).build_bytes(kvs)
    assert raw == cpu
