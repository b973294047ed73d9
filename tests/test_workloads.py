"""Synthetic-input generators (bench plumbing) against the oracle / reference fixtures."""
import numpy as np

from narwhal_amd import workloads as W
from oracle import oracle as O


def test_fixture_seeds_match_stdrng(golden):
    s = W.fixture_seeds(1000)
    o = O.stdrng_seeds(1000)
    assert all(bytes(s[i]) == o[i] for i in range(1000))
    ref = [k["seed"] for k in golden["keys"]["stdrng_zero_seed_keys"]]
    assert [bytes(s[i]).hex() for i in range(4)] == ref


def test_chacha20_counter_offset():
    a = W.chacha20_keystream(bytes(range(32)), 5)
    b = W.chacha20_keystream(bytes(range(32)), 3, counter=2)
    assert a[128:] == b
    assert a == O.chacha20(bytes(range(32)), bytes(8), 0, 320)
