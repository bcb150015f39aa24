"""BASELINE config 4 (FortiGate long scan, >= 1M expanded rules) on the GPU:
the fused job over run-compressed candidate lists with the (chained)
perfect-hash index gives the C oracle's per-rule results, where the oracle
scans the fully expanded rules of the restated FortiGate preprocessor line by
line, exactly like mapper.py:168-189."""
import numpy as np
import pytest

from oracle import coracle
from ruleset_analysis_amd import fortigate, native, synth, synth_fg
from ruleset_analysis_amd.compile import CompiledRules
from ruleset_analysis_amd.engine import DeviceBatch
from ruleset_analysis_amd.pipeline import built_hit_count

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def cfg4():
    text, info = synth_fg.make_config(4)                  # 160 policies, 3 wide-range: ~3.4M rules
    db = fortigate.build_db(text)
    comp = CompiledRules(db)
    comp.ensure_lists()
    return text, info, db, comp, coracle.OracleRules.from_fortigate(text)


def _job_vs_oracle(engine, text, info, comp, R, n, seed, cap, chunk=None, index=True, kind=None):
    tr = synth_fg.make_traffic(info, n, seed=seed)
    tup, ts, order = synth.pack(tr, comp)
    engine.load_compiled(comp, index=index, chunk=chunk, kind=kind)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    res = engine.run([b], cap, capacity=max(built_hit_count(tup), 1))
    gids = engine.last_gids[0].cpu().numpy()
    cols, ots, oorder = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ots, oorder, cap)
    assert np.array_equal(gids, ref['gid'])
    assert np.array_equal(res.matches, ref['matches'])
    assert np.array_equal(res.hits, ref['hits'])
    got = sorted((int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']),
                  int(r['count']), int(r['first']), int(r['last'])) for r in res.records)
    rows = ref['rows']
    want = sorted(zip(*(rows[k].astype(int).tolist() for k in ('gid', 'pspell', 'for_ip', 'to_ip', 'to_port',
                                                                'count', 'first', 'last'))))
    assert got == want
    assert np.array_equal(res.thresh != 0xFFFFFFFFFFFFFFFF, (ref['n_conns'] >= cap) & (cap > 0))
    return ref


def test_cfg4_parity_indexed(engine, cfg4):
    text, info, db, comp, R = cfg4
    assert comp.n_rules >= 1_000_000
    ref = _job_vs_oracle(engine, text, info, comp, R, 12000, seed=41, cap=1000)
    assert ref['evals'] > 10 ** 5 * 12000 * 0.1            # the reference scans ~1e5+ rules per line
    assert (ref['gid'] >= 0).mean() > 0.4


@pytest.mark.parametrize('kind', ['pht', 'bucket', 'bucket-filtered'])
def test_cfg4_parity_chained_index_capped(engine, cfg4, kind):
    """Index records of at most 4096 entries (chained) and a small cap."""
    text, info, db, comp, R = cfg4
    _job_vs_oracle(engine, text, info, comp, R, 12000, seed=42, cap=20, chunk=4096, kind=kind)


@pytest.mark.parametrize('kind', ['bucket', 'bucket-filtered'])
def test_cfg4_parity_bucket_index(engine, cfg4, kind):
    text, info, db, comp, R = cfg4
    _job_vs_oracle(engine, text, info, comp, R, 12000, seed=44, cap=1000, kind=kind)


@pytest.mark.parametrize('pair,defer,n', [(1, 0, 12001), (0, 0, 12001), (1, 1, 777), (1, 0, 63)])
def test_cfg4_bucket_two_lines_per_lane(engine, cfg4, pair, defer, n):
    """The global bucket image's two-lines-per-lane classifier (k_classify_pair,
    RSA_OPT_CLASSIFY_PAIR) against the oracle: odd line counts (the second
    line of the last lanes past the end), chained records, forced deferral
    (every indexed line through k_tail), and the one-line classifier."""
    text, info, db, comp, R = cfg4
    engine.set_option(native.RSA_OPT_CLASSIFY_PAIR, pair)
    engine.set_option(native.RSA_OPT_FORCE_DEFER, defer)
    try:
        _job_vs_oracle(engine, text, info, comp, R, n, seed=45 + n, cap=30, chunk=4096, kind='bucket')
    finally:
        engine.set_option(native.RSA_OPT_CLASSIFY_PAIR, 1)
        engine.set_option(native.RSA_OPT_FORCE_DEFER, 0)


def test_cfg4_sampled_lines_at_4m(engine, cfg4):
    """4M lines of config 4 through the fused job (bucket index, cap 1000):
    the first match of 16K lines drawn uniformly from the whole batch equals
    the C oracle's scan of the expanded rules (a line's first match does not
    depend on the others), and the per-rule line and hit counters equal the
    histograms of the job's own gids (every line)."""
    text, info, db, comp, R = cfg4
    n = 4_000_000
    tr = synth_fg.make_traffic(info, n, seed=46)
    tup, ts, order = synth.pack(tr, comp)
    engine.load_compiled(comp)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    res = engine.run([b], 1000, capacity=max(built_hit_count(tup), 1))
    gids = engine.last_gids[0].cpu().numpy()
    pick = np.sort(np.random.default_rng(7).choice(n, 16384, replace=False))
    sub = {k: (np.asarray(v)[pick] if isinstance(v, np.ndarray) and len(v) == n else v) for k, v in tr.items()}
    cols, _ts, _order = coracle.inputs_from_traffic(R, sub)
    g_ref, _evals = coracle.classify(R, cols['list'], cols['proto'], cols['src'], cols['dst'], cols['sport'],
                                     cols['dport'])
    assert np.array_equal(gids[pick], g_ref)
    ok = gids >= 0
    hit = ok & ((tup['flags'] & 2) != 0)
    assert np.array_equal(res.matches[:comp.n_rules].astype(np.int64),
                          np.bincount(gids[ok], minlength=comp.n_rules)[:comp.n_rules])
    assert np.array_equal(res.hits[:comp.n_rules].astype(np.int64),
                          np.bincount(gids[hit], minlength=comp.n_rules)[:comp.n_rules])
    assert (g_ref >= 0).mean() > 0.3


def test_cfg4_parity_linear_scan(engine, cfg4):
    text, info, db, comp, R = cfg4
    _job_vs_oracle(engine, text, info, comp, R, 6000, seed=43, cap=1000, index=False)


def test_cfg4_compressed_equals_expanded_at_1m_lines(engine, cfg4):
    """1M lines: the compressed, indexed classifier equals a GPU linear scan of
    the UNcompressed lists (one entry per expanded rule, millions per list)."""
    text, info, db, comp, R = cfg4
    tr = synth_fg.make_traffic(info, 1_000_000, seed=44)
    tup, ts, order = synth.pack(tr, comp)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    engine.load_compiled(comp)
    g_idx = engine.classify_only(b).cpu().numpy()
    full = CompiledRules(db, run_min=0)
    for k in comp.list_keys:
        full.list_id(*k)
    ent, _off = full.packed()
    assert len(ent) > 2_000_000
    tup2, _ts2, _o2 = synth.pack(tr, full)
    assert np.array_equal(tup2, tup)                    # same list ids
    b2 = DeviceBatch.from_numpy(tup2, ts, order, engine.device)
    engine.load_compiled(full, index=False)
    g_full = engine.classify_only(b2).cpu().numpy()
    assert np.array_equal(g_idx, g_full)
    assert (g_idx >= 0).sum() > 400_000


def test_cfg4_natural_chain_over_65534_entries(engine):
    """300 policies: the compressed outside list exceeds one record's 0xFFFE
    entries, so the index is a chain without forcing."""
    text, info = synth_fg.make_config(9, n_policies=300, n_wide=2)
    db = fortigate.build_db(text)
    comp = CompiledRules(db)
    comp.ensure_lists()
    _ent, off = comp.packed()
    assert int(np.diff(off).max()) > 0xFFFE
    R = coracle.OracleRules.from_fortigate(text)
    _job_vs_oracle(engine, text, info, comp, R, 8000, seed=45, cap=1000)
