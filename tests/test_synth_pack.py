"""synth.pack (used by the bench for 10^8-line workloads, no text) produces
exactly what the host log parser produces from the rendered text: same tuples
for every classified line, same timestamp strings, same relative order among
the lines that can enter a connection table."""
import numpy as np
import pytest

from ruleset_analysis_amd import acldb, synth
from ruleset_analysis_amd.compile import CompiledRules, F_HIT, F_BUILT
from ruleset_analysis_amd.logparse import parse_logs, D_CLASSIFY


@pytest.mark.parametrize('population', [None, 10 ** 8])
def test_pack_equals_parse_of_render(population):
    dbj, info = synth.make_db(7, 300, interfaces=('outside', 'partner'))
    if population:       # BASELINE config 5's connection population
        tr = synth.make_traffic_population((dbj, info), 6000, seed=8, s=1.1, population=population)
    else:
        tr = synth.make_traffic((dbj, info), 6000, seed=8, zipf=1.2)
    lines = [l + '\n' for l in synth.render_lines(tr)]
    db = acldb.load_json(dbj)
    comp_a = CompiledRules(db)
    parsed = parse_logs([('fw1', lines)], db, comp_a)
    if population:
        assert len(np.unique(tr['rank'])) < 0.8 * len(lines)     # connections repeat
    assert parsed.error is None
    comp_b = CompiledRules(db)
    tup, ts, order = synth.pack(tr, comp_b)
    cls = parsed.disposition == D_CLASSIFY
    assert np.array_equal(cls, (tup['flags'] & 1) == 1)
    a, b = parsed.tuples[cls], tup[cls]
    for f in ('src', 'dst', 'sport', 'dport', 'flags'):
        assert np.array_equal(a[f], b[f]), f
    # list ids are assigned lazily in first-use order: compare the (host, acl, proto) they denote
    assert [comp_a.list_keys[i] for i in a['list']] == [comp_b.list_keys[i] for i in b['list']]
    built = (a['flags'] & F_BUILT) != 0
    assert [parsed.pspell_table[i] for i in a['pspell'][built]] == [synth.PSPELL[i] for i in b['pspell'][built]]
    hb = cls & ((parsed.tuples['flags'] & (F_HIT | F_BUILT)) == (F_HIT | F_BUILT))
    assert [parsed.ts_table[c] for c in parsed.ts[hb]] == [synth.ts_decode(c) for c in ts[hb]]
    idx = np.nonzero(hb)[0]
    assert np.array_equal(np.argsort(parsed.order[idx], kind='stable'), np.argsort(order[idx], kind='stable'))
    assert len(np.unique(order)) == len(order)


def test_population_is_fixed_across_chunks():
    """Chunks of one log (different sampling seeds, same pop_seed) draw from
    one population: a rank maps to the same connection in both."""
    dbj, info = synth.make_db(9, 200, interfaces=('outside', 'partner'))
    a = synth.make_traffic_population((dbj, info), 20000, seed=1, pop_seed=5)
    b = synth.make_traffic_population((dbj, info), 20000, seed=2, pop_seed=5)
    common = np.intersect1d(a['rank'], b['rank'])
    assert len(common) > 100
    ia = {r: i for i, r in enumerate(a['rank'].tolist())}
    ib = {r: i for i, r in enumerate(b['rank'].tolist())}
    for r in common[:200].tolist():
        i, j = ia[r], ib[r]
        if a['form'][i] != synth.F_OUTBOUND and b['form'][j] != synth.F_OUTBOUND:
            assert (a['src'][i], a['dst'][i], a['dport'][i], a['ifc'][i], a['proto'][i]) == \
                (b['src'][j], b['dst'][j], b['dport'][j], b['ifc'][j], b['proto'][j])


def test_make_db_shapes():
    dbj, _info = synth.make_db(3, 500)
    acl = dbj['accesslists']['fw1']['outside_access_in']
    assert len(acl['rules']) == 500
    assert [r['ruleindex'] for r in acl['rules']] == list(range(500))
    assert acl['rules'][-1]['original'].endswith('deny ip any any')
    assert 'ip' in acl['protocols']
    for p, idx in acl['protocols'].items():
        assert all(acl['rules'][i]['protocol'] == p for i in idx)
