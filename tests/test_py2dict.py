"""CPython 2.7 dict order of the reducer's connection table (SURVEY.md trap 8):
the product's replay (ruleset-analysis_amd/py2dict.py) against published
CPython 2.7 values and against the oracle's structure-level restatement of
dictobject.c (oracle/py2dict.py)."""
import random

import pytest

from oracle import py2dict as opy2
from ruleset_analysis_amd import py2dict


def test_published_hash_values():
    # 64-bit CPython 2.7: hash('a') == 12416037344; 32-bit: -468864544
    assert py2dict.string_hash('a') == 12416037344
    assert opy2.string_hash('a') == 12416037344
    M = (1 << 32) - 1
    x = (ord('a') << 7) & M
    x = ((1000003 * x) & M) ^ ord('a')
    x ^= 1
    assert x - (1 << 32) == -468864544          # the same recurrence at 32 bits
    assert py2dict.string_hash('') == 0


def test_published_dict_order():
    # Python 2.7: {'a': 1, 'b': 2, 'c': 3} prints {'a': 1, 'c': 3, 'b': 2}
    keys = ['a', 'b', 'c']
    assert [keys[i] for i in py2dict.iteration_order(keys)] == ['a', 'c', 'b']
    assert opy2.py2_keys(keys) == ['a', 'c', 'b']


def test_vectorised_hash_equals_scalar():
    rng = random.Random(7)
    keys = ['%s;%d.%d.%d.%d;10.0.%d.%d;%d' % (rng.choice(['TCP', 'UDP', 'tcp']), rng.randrange(256),
                                              rng.randrange(256), rng.randrange(256), rng.randrange(256),
                                              rng.randrange(256), rng.randrange(256), rng.randrange(65536))
            for _ in range(2000)] + ['x', 'ab', '\xff\xfe']
    hv = py2dict.string_hashes(keys)
    assert [int(h) for h in hv] == [py2dict.string_hash(k) for k in keys]
    assert [int(h) for h in hv] == [opy2.string_hash(k) & ((1 << 64) - 1) for k in keys]


@pytest.mark.parametrize('n', [1, 5, 6, 7, 8, 40, 1000, 60000])
def test_replay_agrees_with_oracle(n):
    rng = random.Random(n)
    keys = list(dict.fromkeys('TCP;%d.%d.%d.%d;192.0.2.%d;%d' % (rng.randrange(256), rng.randrange(256),
                                                                  rng.randrange(256), rng.randrange(256),
                                                                  rng.randrange(3), rng.choice([80, 443]))
                              for _ in range(n)))
    got = [keys[i] for i in py2dict.iteration_order(keys)]
    assert got == opy2.py2_keys(keys)
    assert sorted(got) == sorted(keys)


def test_table_order_ties_follow_dict_order():
    from ruleset_analysis_amd.report import table_order
    spell = ['TCP'] * 3
    frm = ['1.1.1.1', '2.2.2.2', '3.3.3.3']
    to = ['192.0.2.1'] * 3
    port = ['80'] * 3
    order = table_order(spell, frm, to, port, [10, 20, 30])
    keys = [';'.join((spell[k], frm[k], to[k], port[k])) for k in range(3)]
    assert [keys[k] for k in order] == opy2.py2_keys(keys)
