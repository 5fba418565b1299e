"""table_test.go scenarios on the host mirror with oracle-decoded blocks (no GPU needed).

This checks the transliterated Iterator / blockIterator / ConcatIterator / MergeIterator
control logic against the reference's own known answers; tests/test_gpu_table.py runs the
same scenarios end to end through the gfx950 encoder and decoder.
"""
import pytest

import table_cases as C


@pytest.fixture(scope="module")
def env(oracle):
    return C.CpuEnv(oracle)


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
