"""The C oracle (classify + reducer replay over packed arrays) agrees with the
Python oracle pipeline on every golden case: per-rule line counts, hits and the
connection tables (rows in first-seen order)."""
import numpy as np
import pytest

from conftest import golden_cases
from golden_io import load_case, split_lines
from oracle import coracle
from oracle import pipeline as op
from oracle.crosscheck_2to3 import oracle_db


def _dotted(v):
    v = int(v)
    return '%d.%d.%d.%d' % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


@pytest.mark.parametrize('case', golden_cases())
def test_c_oracle_vs_python_oracle(case):
    dbj, text, _report, _sha, params = load_case(case)
    cap = params['cap']
    R = coracle.OracleRules(dbj)
    cols, ts, order, ts_table, spell = coracle.inputs_from_text(R, params['host'], split_lines(text))
    res = coracle.run(R, cols, ts, order, cap)
    acls, fws = oracle_db(dbj)
    _m, _s, _red, blocks = op.run_pipeline(text, params['host'], acls, fws, cap=cap)
    by_key = {b['key']: b for b in blocks}
    got_keys = [R.key(g) for g in np.nonzero(res['matches'])[0]]
    assert sorted(got_keys) == sorted(by_key)
    rows = res['rows']
    for g in np.nonzero(res['matches'])[0]:
        b = by_key[R.key(g)]
        assert int(res['matches'][g]) == b['matches']
        assert int(res['hits'][g]) == b['hits']
        sel = np.nonzero(rows['gid'] == g)[0]
        mine = [['%s;%s;%s;%d' % (spell[rows['pspell'][k]], _dotted(rows['for_ip'][k]), _dotted(rows['to_ip'][k]),
                                  rows['to_port'][k]), int(rows['count'][k]), ts_table[rows['first'][k]],
                 ts_table[rows['last'][k]]] for k in sel]
        theirs = sorted(b['conns'], key=lambda r: r[0])
        assert sorted(mine, key=lambda r: r[0]) == theirs
        assert (int(res['n_conns'][g]) >= cap) == b['capped']
