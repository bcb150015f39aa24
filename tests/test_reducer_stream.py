"""The reducer drop-in (connlist-reducer.py:62-211) on the GPU parse: the
device's per-line reducer fields (textparse_line.h reduce_line, compiled for
the CPU here) against the Python restatement of the reference's regex, and the
streaming job (reducer_stream) against the oracle reducer on golden mapper
streams with noise, non-canonical text, odd timestamps, chunk boundaries
everywhere and the reference's error deaths."""
import ctypes
import random

import numpy as np
import pytest

from golden_io import load_case, split_lines
from oracle.crosscheck_2to3 import oracle_db
from oracle.mapper import map_lines
from oracle.reducer import reduce_lines
from ruleset_analysis_amd import acldb, textparse
from ruleset_analysis_amd.compile import F_BUILT, F_HIT, TUPLE_DTYPE
from ruleset_analysis_amd.logparse import reducer_fields, reducer_timestamp
from ruleset_analysis_amd.py2text import PY2_WS
from ruleset_analysis_amd.report import dotted
from test_textparse import _harness, _mutate

RED_KEYED, RED_NOISE, RED_SAME = 0, 1, 0x100


def _mapper_stream(case):
    dbj, text, _report, _sha, params = load_case(case)
    acls, fws = oracle_db(dbj)
    out = []
    map_lines(split_lines(text), params['host'], acls, fws, out)
    return dbj, params, ''.join(out).splitlines(True)


def _mutate_stream(lines, seed, bad_month=False):
    """Sorted mapper stream with the reducer's corner cases mixed in."""
    rng = random.Random(seed)
    out = []
    for l in lines:
        r = rng.random()
        if '\t' in l and r < 0.25:
            key, val = l.split('\t', 1)
            val = _mutate(val.rstrip('\n'), rng)
            if not bad_month:
                val = val.replace('Foo', 'Jul')
            l = key + '\t' + val.replace('\n', ' ') + '\n'
        elif r < 0.27:
            l = rng.choice(['no tab here\n', 'a;b\tvalue\n', 'fw1;acl;x\tvalue\n', '\n', '   \t  \n',
                            ' fw1;outside_access_in;1\t \n'])
        out.append(l)
        if '\t' in l and rng.random() < 0.02:     # the same key with non-canonical address / port text
            key, val = l.split('\t', 1)
            out.append(key + '\t' + val.replace(' for outside:', ' for outside:0', 1).replace('/', '/0', 1))
    return sorted(out, key=lambda s: s.encode('latin-1'))


def _oracle(dbj, lines, cap):
    acls, _fws = oracle_db(dbj)
    out = []
    exc = None
    try:
        reduce_lines(lines, acls, cap, out=out)
    except (KeyError, IndexError, ValueError) as e:
        exc = e
    return ''.join(l + '\n' for l in out), exc


# ---- CPU: the device's reducer-line parse -------------------------------------------------------------

def _reduce_on_cpu(lib, lines, spells, word):
    data = ''.join(lines).encode('latin-1')
    off = np.cumsum([0] + [len(l.encode('latin-1')) for l in lines]).astype(np.uint64)
    sp = textparse.spell_table(spells)
    n = len(lines)
    tup = np.zeros(n, TUPLE_DTYPE)
    ts = np.zeros(n, np.uint32)
    disp = np.zeros(n, np.uint32)
    buf = np.zeros((len(data) + 8) // 4 * 4, np.uint8)
    buf[:len(data)] = np.frombuffer(data, np.uint8)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    lib.reduce_lines_host(p(buf), p(off), ctypes.c_uint64(n), p(sp), ctypes.c_uint32(len(sp)), p(tup), p(ts), p(disp),
                          ctypes.c_int(word))
    return tup, ts, disp


def _key_of(line):
    s = line.strip(PY2_WS)
    return s.split('\t', 1)[0] if '\t' in s else None


@pytest.mark.parametrize('case,seed,word', [('small_200r', 1, 1), ('cap5_zipf', 2, 0), ('multi_acl', 3, 2)])
def test_device_reducer_fields_on_cpu_equal_reference_regex(case, seed, word):
    """Every line the device decides (not RSA_LINE_HOST) has the reducer's own
    hit flag, BUILT match, key strings and timestamp; noise is exactly the
    lines without a tab after strip; the same-key flag is key-string equality."""
    lib = _harness()
    _dbj, _params, lines = _mapper_stream(case)
    lines = _mutate_stream(lines, seed, bad_month=True)
    spells = list(textparse.DEFAULT_SPELLS)
    tup, ts, disp = _reduce_on_cpu(lib, lines, spells, word)
    kind = disp & 0xFF
    n_host = 0
    prev_key = None
    for i, line in enumerate(lines):
        key = _key_of(line)
        assert (kind[i] == RED_NOISE) == (key is None), line
        assert bool(disp[i] & RED_SAME) == (key is not None and key == prev_key), line
        prev_key = key
        if kind[i] == textparse.LINE_HOST:
            n_host += 1
            continue
        if key is None:
            continue
        hit, res = reducer_fields(line.strip(PY2_WS).split('\t', 1)[1])
        assert bool(tup[i]['flags'] & F_HIT) == hit, line
        assert bool(tup[i]['flags'] & F_BUILT) == (res is not None), line
        if res is not None:
            assert (spells[tup[i]['pspell']], dotted(tup[i]['src']), dotted(tup[i]['dst']), str(tup[i]['dport'])) == \
                (res[5], res[6], res[8], res[9]), line
            if hit:
                assert textparse.ts_unpack(ts[i]) == reducer_timestamp(res), line
    assert 0 < n_host < len(lines) // 4


# ---- GPU: the streaming job ---------------------------------------------------------------------------

def _run_stream(engine, dbj, lines, cap, chunk):
    from ruleset_analysis_amd.reducer_stream import ReducerStream
    out = []
    job = ReducerStream(engine, acldb.load_json(dbj), cap, out.append, chunk=chunk)
    data = ''.join(lines).encode('latin-1')
    exc = None
    try:
        for a in range(0, len(data), 1000):
            job.feed(data[a:a + 1000])
        job.finish()
    except (KeyError, IndexError, ValueError) as e:
        exc = e
    return ''.join(out), exc


@pytest.mark.gpu
@pytest.mark.parametrize('case,cap', [('small_200r', 1000), ('cap5_zipf', 5), ('multi_acl', 3), ('cap1', 1)])
@pytest.mark.parametrize('chunk', [4096, 1 << 16, 64 << 20])
def test_gpu_reducer_stream_golden_equals_oracle(engine, case, cap, chunk):
    dbj, _params, lines = _mapper_stream(case)
    lines = sorted(lines, key=lambda s: s.encode('latin-1'))
    want, wexc = _oracle(dbj, lines, cap)
    got, gexc = _run_stream(engine, dbj, lines, cap, chunk)
    assert wexc is None and gexc is None
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize('seed', [1, 2, 3])
@pytest.mark.parametrize('chunk', [4096, 64 << 20])
def test_gpu_reducer_stream_mutated_equals_oracle(engine, seed, chunk):
    """Noise lines, bad keys, non-canonical address/port text (two spellings
    of one address stay two connections), odd protocol spellings and
    timestamps, lines the BUILT regex misses, with the cap engaged."""
    dbj, _params, lines = _mapper_stream(['cap5_zipf', 'small_200r', 'multi_acl'][seed - 1])
    lines = _mutate_stream(lines, seed)
    want, wexc = _oracle(dbj, lines, 5)
    got, gexc = _run_stream(engine, dbj, lines, 5, chunk)
    assert type(gexc) is type(wexc)
    assert got == want


@pytest.mark.gpu
def test_gpu_reducer_stream_dies_where_the_reference_dies(engine):
    """An unknown host (KeyError) or rule index (IndexError) kills the job at
    that line: the blocks printed before it are the reference's."""
    dbj, params, lines = _mapper_stream('small_200r')
    lines = sorted(lines, key=lambda s: s.encode('latin-1'))
    k = len(lines) // 2
    for bad in ('nohost;x;1\tv\n', '%s;outside_access_in;99999\tv\n' % params['host']):
        ls = lines[:k] + [bad] + lines[k:]
        want, wexc = _oracle(dbj, ls, 1000)
        got, gexc = _run_stream(engine, dbj, ls, 1000, 4096)
        assert wexc is not None and type(gexc) is type(wexc)
        assert got == want


@pytest.mark.gpu
def test_gpu_reducer_stream_bad_month_only_before_the_cap(engine):
    """A month months.index rejects kills the reference only on a line that
    still reaches the BUILT branch (hit, dict not full): after the cap froze
    the rule it is just a hit."""
    dbj, _params, lines = _mapper_stream('cap5_zipf')
    lines = sorted(lines, key=lambda s: s.encode('latin-1'))
    keys = [_key_of(l) for l in lines]
    hits = [i for i, l in enumerate(lines) if '-6-302013' in l and ' Jul ' in l]
    # a late line of a long run (its rule froze long before) and the first line of a run
    runs = {}
    for i in hits:
        runs.setdefault(keys[i], []).append(i)
    long_run = max(runs.values(), key=len)
    late, early = long_run[-1], long_run[0]
    for i, dies in ((late, False), (early, True)):
        ls = list(lines)
        ls[i] = ls[i].replace(' Jul ', ' Foo ', 1)
        want, wexc = _oracle(dbj, ls, 5)
        got, gexc = _run_stream(engine, dbj, ls, 5, 1 << 16)
        assert (wexc is not None) == dies and type(gexc) is type(wexc)
        assert got == want
