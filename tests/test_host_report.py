"""Host-side logic of the product, without a GPU: the log parse, the rule
compilation (gid <-> key), and the reducer-format report assembly reproduce
the golden reports when fed per-rule results computed by the C oracle.  (The
GPU computes those results in the -m gpu tests.)"""
import numpy as np
import pytest

from conftest import golden_cases
from golden_io import load_case, split_lines
from oracle import coracle
from ruleset_analysis_amd import acldb
from ruleset_analysis_amd.compile import CompiledRules, RECORD_DTYPE
from ruleset_analysis_amd.engine import Results
from ruleset_analysis_amd.logparse import parse_logs, D_CLASSIFY
from ruleset_analysis_amd.pipeline import assemble_report


def oracle_results(dbj, host, lines, cap):
    R = coracle.OracleRules(dbj)
    cols, ts, order, ts_table, spell = coracle.inputs_from_text(R, host, lines)
    res = coracle.run(R, cols, ts, order, cap)
    rows = res['rows']
    rec = np.zeros(len(rows['gid']), dtype=RECORD_DTYPE)
    for k in ('gid', 'for_ip', 'to_ip', 'to_port', 'pspell', 'count', 'first', 'last'):
        rec[k] = rows[k]
    rec['min_order'] = np.arange(len(rec))        # rows come in first-seen order
    thresh = np.full(R.n_rules, 0xFFFFFFFFFFFFFFFF, np.uint64)
    if cap > 0:
        thresh[res['n_conns'] >= cap] = 0
    results = Results(res['matches'], res['hits'], res['n_conns'], thresh, rec, cap)
    return results, res['gid'], ts_table, spell


@pytest.mark.parametrize('case', golden_cases())
def test_report_assembly_matches_golden(case):
    dbj, text, report, _sha, params = load_case(case)
    lines = split_lines(text)
    db = acldb.load_json(dbj)
    compiled = CompiledRules(db)
    parsed = parse_logs([(params['host'], lines)], db, compiled)
    assert parsed.error is None
    results, gids, ts_table, spell = oracle_results(dbj, params['host'], lines, params['cap'])
    # the product's dispositions agree with the oracle's notion of classified lines
    assert np.array_equal(parsed.disposition == D_CLASSIFY, np.zeros(len(lines), bool) | (gids >= -1) &
                          (parsed.disposition == D_CLASSIFY))
    out = assemble_report(parsed, gids, results, compiled, params['cap'], ts_decode=ts_table.__getitem__,
                          pspell_table=spell)
    assert ''.join(l + '\n' for l in out) == report


def test_compiled_keys_roundtrip():
    dbj, _text, _report, _sha, params = load_case(golden_cases()[0])
    compiled = CompiledRules(acldb.load_json(dbj))
    for gid in range(0, compiled.n_rules, 7):
        host, acl, i = compiled.locate(gid)
        assert compiled.key(gid) == '%s;%s;%d' % (host, acl, i)
        assert compiled.rule(gid) is compiled.db.accesslists[host][acl]['rules'][i]


def _emulate_first_match(tuples, ent, off):
    """Test-only numpy evaluation of the compiled lists (the kernel's predicate)."""
    n = len(tuples)
    out = np.full(n, -1, np.int64)
    valid = (tuples['flags'] & 1) == 1
    for L in np.unique(tuples['list'][valid]):
        idx = np.nonzero(valid & (tuples['list'] == L))[0]
        e = ent[off[L]:off[L + 1]]
        t = tuples[idx]
        best = np.full(len(idx), 1 << 40, np.int64)
        u = lambda a: a.astype(np.uint64)
        for x in e:
            m = (((u(t['src']) - np.uint64(x['src_lo'])) & np.uint64(0xFFFFFFFF)) <= np.uint64(x['src_span'])) & \
                (((u(t['dst']) - np.uint64(x['dst_lo'])) & np.uint64(0xFFFFFFFF)) <= np.uint64(x['dst_span'])) & \
                (((u(t['sport']) - np.uint64(int(x['port_lo']) & 0xFFFF)) & np.uint64(0xFFFFFFFF))
                 <= np.uint64(int(x['port_span']) & 0xFFFF)) & \
                (((u(t['dport']) - np.uint64(int(x['port_lo']) >> 16)) & np.uint64(0xFFFFFFFF))
                 <= np.uint64(int(x['port_span']) >> 16))
            best = np.where(m, np.minimum(best, int(x['gid'])), best)
        out[idx] = np.where(best == 1 << 40, -1, best)
    return out


@pytest.mark.parametrize('case', golden_cases())
def test_compiled_tables_first_match(case):
    """The lowered candidate lists give the oracle's first match for every line."""
    dbj, text, _report, _sha, params = load_case(case)
    lines = split_lines(text)
    db = acldb.load_json(dbj)
    compiled = CompiledRules(db)
    parsed = parse_logs([(params['host'], lines)], db, compiled)
    ent, off = compiled.packed()
    got = _emulate_first_match(parsed.tuples, ent, off)
    _results, gids, _t, _s = oracle_results(dbj, params['host'], lines, params['cap'])
    assert np.array_equal(got, gids)


def _emulate_index(tuples, index, ent, off):
    """Test-only evaluation of the perfect-hash index (compile.pht_lookup, the
    host model of the device probe sequence); deferred lines are scanned."""
    from ruleset_analysis_amd.compile import pht_lookup
    exact = _emulate_first_match(tuples, ent, off)
    out = np.full(len(tuples), -1, dtype=np.int64)
    n_defer = 0
    for i in np.nonzero((tuples['flags'] & 1) == 1)[0]:
        t = tuples[i]
        L = int(t['list'])
        ports = int(t['sport']) | (int(t['dport']) << 16)
        k = pht_lookup(index, ent, off, L, int(t['src']), int(t['dst']), ports)
        if k == 'defer':
            n_defer += 1
            out[i] = exact[i]
        else:
            out[i] = k
    return out


@pytest.mark.parametrize('case', ['small_200r', 'cap5_zipf'])
def test_index_first_match(case):
    """The perfect-hash index gives the oracle's first match for every line."""
    dbj, text, _report, _sha, params = load_case(case)
    lines = split_lines(text)
    db = acldb.load_json(dbj)
    compiled = CompiledRules(db)
    parsed = parse_logs([(params['host'], lines)], db, compiled)
    ent, off = compiled.packed()
    from ruleset_analysis_amd.compile import build_index, index_stats
    index = build_index(ent, off, prefix=0, min_entries=1)    # force the index on every list
    assert sum(st[1] for st in index_stats(index)) > 0
    got = _emulate_index(parsed.tuples, index, ent, off)
    _results, gids, _t, _s = oracle_results(dbj, params['host'], lines, params['cap'])
    assert np.array_equal(got, gids)
