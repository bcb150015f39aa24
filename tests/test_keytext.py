"""Reducer keys whose text is not the canonical form of the connection tuple
(``connlist-reducer.py:152-172`` keys its dict by the BUILT regex's strings:
``010.1.2.3`` and ``10.1.2.3`` are two connections, ``/080`` and ``/80`` two
ports).  The host parse interns such keys (``report.KeyText``) and the fused
job aggregates them under their own ids; the reports equal the oracle's
``mapper | sort | reducer``."""
import random
import re

import numpy as np
import pytest

from oracle.crosscheck_2to3 import oracle_db
from oracle import pipeline as op
from ruleset_analysis_amd import acldb, logparse, synth
from ruleset_analysis_amd.compile import CompiledRules, F_SWAP, TUPLE_DTYPE
from ruleset_analysis_amd.keytext import INTERNED


def _lines(n, seed):
    dbj, info = synth.make_db(13, 300, interfaces=('outside', 'partner'))
    tr = synth.make_traffic((dbj, info), n, seed=seed, zipf=1.2)
    rng = random.Random(seed)
    out, base = [], []
    for l in synth.render_lines(tr):
        base.append(l.rstrip('\n') + '\n')
        r = rng.random()
        if r < 0.05:
            l = l.replace(' for outside:', ' for outside:0', 1)                  # from address '051.0.0.1'
        elif r < 0.10:
            l = re.sub(r'( to [a-z]+:[0-9.]+)/([0-9]+)', r'\1/0\2', l, count=1)    # port '0993'
        elif r < 0.12:
            l = re.sub(r'( to [a-z]+:)([0-9.]+)', r'\g<1>00\2', l, count=1)        # to address '0010.1.2.3'
        out.append(l.rstrip('\n') + '\n')
    return dbj, out, base


def test_host_parse_interns_noncanonical_keys():
    dbj, lines, canon = _lines(4000, 3)
    db = acldb.load_json(dbj)
    P = logparse.parse_logs([('fw1', lines)], db, CompiledRules(db))
    assert P.error is None
    assert len(P.keyx) > 150
    Q = logparse.parse_logs([('fw1', canon)], db, CompiledRules(db))
    assert not Q.keyx
    # the connection tuples (what the classifier sees) do not change
    for f in ('src', 'dst', 'sport', 'dport', 'list', 'flags'):
        assert np.array_equal(P.tuples[f], Q.tuples[f]), f
    for i, k in P.keyx.items():
        res = logparse.reducer_fields(lines[i].strip(logparse.PY2_WS))[1]
        assert P.keytext.values[k] == (res[5], res[6], res[8], res[9])


def test_key_tuples_rewrites_only_interned_rows():
    import torch
    tup = np.zeros(5, TUPLE_DTYPE)
    tup['src'], tup['dst'], tup['sport'], tup['dport'] = 11, 22, 33, 44
    tup['flags'] = 0x07 | F_SWAP
    tup['list'] = 9
    t = torch.from_numpy(tup.view(np.int32).reshape(-1, 4).copy())
    out = logparse.key_tuples(torch, t, {1: 5, 3: 0x89ABCDEF})
    assert out is not t
    o = out.numpy().reshape(-1).view(TUPLE_DTYPE)
    assert np.array_equal(o[[0, 2, 4]], tup[[0, 2, 4]])
    assert tuple(o[1][['src', 'dst', 'sport', 'dport', 'list', 'flags', 'pspell']].tolist()) == \
        (5, 0, 0, 0, 9, 0x07, INTERNED)
    assert int(o[3]['src']) == 0x89ABCDEF
    assert logparse.key_tuples(torch, t, {}) is t


@pytest.mark.gpu
@pytest.mark.parametrize('text_path', [False, True])
def test_gpu_fused_job_noncanonical_keys_equal_oracle(engine, text_path):
    from ruleset_analysis_amd.pipeline import analyze, analyze_text
    dbj, lines, _canon = _lines(20000, 5)
    db = acldb.load_json(dbj)
    acls, fws = oracle_db(dbj)
    for cap in (5, 1000):
        _m, _s, want, _b = op.run_pipeline(''.join(lines), 'fw1', acls, fws, cap=cap)
        if text_path:
            got, _ = analyze_text([('fw1', ''.join(lines).encode('latin-1'))], db, cap=cap, engine=engine)
        else:
            got, _ = analyze([('fw1', lines)], db, cap=cap, engine=engine)
        assert got == want
    assert sum(1 for l in want if re.search(r' 0[0-9]+\.', l)) > 20     # interned rows were printed
