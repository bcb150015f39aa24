"""Parity of the HIP path (through the C ABI) with the oracle.

* golden cases: the fused GPU job prints the converted reference's report byte
  for byte, and the GPU-classified mapper stream hashes to the reference's;
* seeded synthetic workloads (no text): per-rule line counts, hit counts and
  connection tables (count, first seen, last seen; cap semantics included) are
  bit-exact against the C oracle, which replays the reducer loop line by line.
"""
import hashlib

import numpy as np
import pytest

from conftest import golden_cases
from golden_io import load_case, split_lines
from oracle import coracle
from ruleset_analysis_amd import acldb, native, synth
from ruleset_analysis_amd.compile import CompiledRules
from ruleset_analysis_amd.engine import DeviceBatch
from ruleset_analysis_amd.logparse import parse_logs
from ruleset_analysis_amd.pipeline import analyze, built_hit_count
from ruleset_analysis_amd.report import mapper_output

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('case', golden_cases())
def test_golden_report(engine, case):
    dbj, text, report, _sha, params = load_case(case)
    out, _res = analyze([(params['host'], split_lines(text))], acldb.load_json(dbj), cap=params['cap'],
                        engine=engine)
    assert ''.join(l + '\n' for l in out) == report


@pytest.mark.parametrize('case', golden_cases())
def test_golden_mapper_stream(engine, case):
    dbj, text, _report, sha, params = load_case(case)
    db = acldb.load_json(dbj)
    compiled = CompiledRules(db)
    parsed = parse_logs([(params['host'], split_lines(text))], db, compiled)
    engine.load_compiled(compiled)
    engine.reset(max(built_hit_count(parsed.tuples), 1), params['cap'])
    b = DeviceBatch.from_numpy(parsed.tuples, parsed.ts, parsed.order, engine.device)
    gids = engine.classify_only(b).cpu().numpy() if parsed.n else np.zeros(0, np.int32)
    text_out = mapper_output(parsed, gids, compiled)
    assert hashlib.sha256(text_out.encode('latin-1')).hexdigest() == sha


def _gpu_vs_oracle(engine, n_rules, n_lines, cap, seed, zipf=None, interfaces=('outside',), batches=1,
                   shuffle=False, index=True, broad=True, prefix=0, kind=None, population=None, sync_cap=True,
                   capacity=None):
    dbj, info = synth.make_db(seed, n_rules, interfaces=interfaces, broad=broad)
    if population:
        tr = synth.make_traffic_population((dbj, info), n_lines, seed=seed + 1, s=zipf, population=population)
    else:
        tr = synth.make_traffic((dbj, info), n_lines, seed=seed + 1, zipf=zipf)
    if shuffle:   # input order no longer follows the sort order
        perm = np.random.default_rng(seed).permutation(n_lines)
        for k in ('src', 'dst', 'sport', 'dport', 'proto', 'ifc', 'form', 't', 'cid'):
            tr[k] = tr[k][perm]
    db = acldb.load_json(dbj)
    compiled = CompiledRules(db)
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled, index=index, prefix=prefix, kind=kind)
    cuts = np.linspace(0, n_lines, batches + 1).astype(int)
    bs = [DeviceBatch.from_numpy(tup[a:b], ts[a:b], order[a:b], engine.device) for a, b in zip(cuts[:-1], cuts[1:])]
    res = engine.run(bs, cap, capacity=capacity or max(built_hit_count(tup), 1), sync_cap=sync_cap)
    gids = np.concatenate([g.cpu().numpy() for g in engine.last_gids])
    R = coracle.OracleRules(dbj)
    cols, ots, oorder = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ots, oorder, cap)
    assert np.array_equal(gids, ref['gid'])
    assert np.array_equal(res.matches, ref['matches'])
    assert np.array_equal(res.hits, ref['hits'])
    rows = ref['rows']
    rec = res.records
    key_r = lambda g, a: (int(a['pspell']), int(a['for_ip']), int(a['to_ip']), int(a['to_port']))
    ro = np.argsort(rows['gid'], kind='stable')
    go = np.argsort(rec['gid'], kind='stable')
    ref_by = {}
    for k in ro:
        ref_by.setdefault(int(rows['gid'][k]), {})[(int(rows['pspell'][k]), int(rows['for_ip'][k]),
                                                    int(rows['to_ip'][k]), int(rows['to_port'][k]))] = (
            int(rows['count'][k]), int(rows['first'][k]), int(rows['last'][k]))
    got_by = {}
    for k in go:
        r = rec[k]
        got_by.setdefault(int(r['gid']), {})[key_r(None, r)] = (int(r['count']), int(r['first']), int(r['last']))
    assert got_by.keys() == ref_by.keys()
    for g in ref_by:
        assert got_by[g] == ref_by[g], g
    capped_gpu = res.thresh != 0xFFFFFFFFFFFFFFFF
    capped_ref = (ref['n_conns'] >= cap) & (cap > 0)
    assert np.array_equal(capped_gpu, capped_ref)
    return res, ref


def test_synth_parity_uncapped(engine):
    _gpu_vs_oracle(engine, 600, 200000, 1000, seed=11)


def test_emit_buffer_regrows(engine):
    """The engine's kept emission buffer starts too small: the library reports
    the count it needed, the engine grows the buffer and emits again; the
    records still match the oracle exactly."""
    engine._emit_buf, engine._emit_cap = None, 0
    engine._emit_buffer(1)
    _gpu_vs_oracle(engine, 400, 60000, 30, seed=41)
    assert engine._emit_cap > 1


def test_synth_parity_linear_scan(engine):
    _gpu_vs_oracle(engine, 3000, 200000, 100, seed=18, index=False)


@pytest.mark.parametrize('kind', ['pht', 'bucket'])
def test_synth_parity_deferred_tail(engine, kind):
    """Every index lookup forced through the exact deferred-line kernel."""
    from ruleset_analysis_amd import native
    engine.set_option(native.RSA_OPT_FORCE_DEFER, 1)
    try:
        _gpu_vs_oracle(engine, 2000, 300000, 50, seed=23, zipf=1.2, broad=False, prefix=0, kind=kind)
    finally:
        engine.set_option(native.RSA_OPT_FORCE_DEFER, 0)


@pytest.mark.parametrize('kind', ['bucket', 'bucket-filtered'])
def test_synth_parity_bucket_index(engine, kind):
    """The partial-key bucket index (RSA5, both forms) against the oracle."""
    _gpu_vs_oracle(engine, 3000, 300000, 40, seed=61, zipf=1.2, broad=False, kind=kind)


@pytest.mark.parametrize('cap', [5, 1000000])
def test_synth_parity_cap_count_on_device(engine, cap):
    """rsa_resolve_cap without the host read (the count stays on the device)
    and the recount run unconditionally: its kernels skip their work on the
    device when no rule is capped.  Equal to the oracle with rules capped and
    with none (bench.py's job takes this form)."""
    _gpu_vs_oracle(engine, 2000, 300000, cap, seed=31, zipf=1.1, sync_cap=False)


def test_synth_parity_region_count_from_previous_job(engine):
    """rsa_reset sizes the region count from the previous job's pass-1 record
    count (RSA_OPT_REGION_RECORDS): with 64 records per region and a table of
    2^23 slots, jobs after the first run at 4096 regions of 2048 slots instead
    of 1024 (and merge through the 4096-entry k_reduce<1>); every job stays
    equal to the oracle, and so does the policy off."""
    engine.set_option(native.RSA_OPT_REGION_RECORDS, 64)
    try:
        for seed in (33, 35):
            _gpu_vs_oracle(engine, 2000, 300000, 5, seed=seed, zipf=1.1, capacity=1 << 22)
        engine.set_option(native.RSA_OPT_REGION_RECORDS, 0)
        _gpu_vs_oracle(engine, 2000, 300000, 5, seed=37, zipf=1.1, capacity=1 << 22)
    finally:
        engine.set_option(native.RSA_OPT_REGION_RECORDS, 49152)


def test_synth_parity_wave_cap_scatter(engine):
    """Cap resolution through the wave-grouped scatter (taken above 16384
    capped rules; forced here) agrees with the oracle like the LDS-ranked one."""
    from ruleset_analysis_amd import native
    engine.set_option(native.RSA_OPT_WAVE_CAP_SCATTER, 1)
    try:
        _gpu_vs_oracle(engine, 2000, 300000, 5, seed=29, zipf=1.1)
    finally:
        engine.set_option(native.RSA_OPT_WAVE_CAP_SCATTER, 0)


@pytest.mark.parametrize('kind', ['pht', 'bucket', 'bucket-filtered'])
@pytest.mark.parametrize('broad,prefix', [(True, 64), (False, 64), (False, 0), (False, 4096)])
def test_index_and_scan_agree_10k(engine, broad, prefix, kind):
    """Both indexes (the bucket index and the pruned perfect-hash index, after
    a linear prefix) and the plain linear scan classify identically, half of
    the lines unmatched (full-list scans)."""
    dbj, info = synth.make_db(19, 10000, broad=broad)
    tr = synth.make_traffic((dbj, info), 1_000_000, seed=20, p_unmatched=0.5)
    compiled = CompiledRules(acldb.load_json(dbj))
    tup, _ts, _order = synth.pack(tr, compiled)
    b = DeviceBatch.from_numpy(tup, _ts, _order, engine.device)
    engine.load_compiled(compiled, index=True, prefix=prefix, kind=kind)
    g_idx = engine.classify_only(b).cpu().numpy()
    engine.use_index(False)
    g_scan = engine.classify_only(b).cpu().numpy()
    assert np.array_equal(g_idx, g_scan)
    assert (g_idx >= 0).sum() > 0


def test_synth_parity_10k_rules_spread(engine):
    """Realistic ACL (no catch-all permit): first matches spread over 10k rules."""
    _gpu_vs_oracle(engine, 10000, 300000, 20, seed=25, broad=False)


def test_synth_parity_capped_zipf(engine):
    res, ref = _gpu_vs_oracle(engine, 400, 300000, 25, seed=12, zipf=1.1)
    assert (ref['n_conns'] >= 25).sum() > 10          # the cap is really engaged


def test_synth_parity_multi_acl_batches(engine):
    _gpu_vs_oracle(engine, 500, 240000, 60, seed=13, interfaces=('outside', 'partner', 'vpn', 'dmz2'), batches=3)


def test_synth_parity_cap1(engine):
    _gpu_vs_oracle(engine, 200, 50000, 1, seed=14, zipf=1.5)


def test_synth_parity_10k_rules(engine):
    _gpu_vs_oracle(engine, 10000, 150000, 1000, seed=15)


def test_synth_parity_tightened_filter(engine):
    # > 4M lines in one batch: the library aggregates the first 1M lines (the
    # default slice is 1/256 of the batch, at least 1M), derives the per-rule
    # filter, refines it after 4M lines (and 16M in a longer batch) and skips
    # the table for lines beyond it
    res, ref = _gpu_vs_oracle(engine, 800, 5_000_000, 40, seed=16, zipf=1.2)
    assert (ref['n_conns'] >= 40).sum() > 0           # the cap is engaged


def test_synth_parity_tightened_filter_shuffled(engine):
    _gpu_vs_oracle(engine, 800, 5_000_000, 40, seed=17, zipf=1.2, shuffle=True)


@pytest.mark.parametrize('steps,slice_,growth', [(1, 256, 4), (2, 256, 16), (4, 256, 4), (3, 16, 4), (2, 256, 2)])
def test_synth_parity_filter_schedule(engine, steps, slice_, growth):
    """Other filter schedules: 1, 2 or 4 refinements, a 1/16 first slice,
    growth 2 and 16 (the default: 3 refinements growing 4x)."""
    from ruleset_analysis_amd import native
    engine.set_option(native.RSA_OPT_FILTER_STEPS, steps)
    engine.set_option(native.RSA_OPT_FILTER_SLICE, slice_)
    engine.set_option(native.RSA_OPT_FILTER_GROWTH, growth)
    try:
        _gpu_vs_oracle(engine, 1500, 5_000_000, 40, seed=24, zipf=1.1, broad=False,
                       interfaces=('outside', 'partner'))
    finally:
        engine.set_option(native.RSA_OPT_FILTER_STEPS, 3)
        engine.set_option(native.RSA_OPT_FILTER_SLICE, 256)
        engine.set_option(native.RSA_OPT_FILTER_GROWTH, 4)


def test_recount_after_moved_bounds_repeated_jobs(engine):
    """Shuffled 5M-line jobs (the last slice finds new connections below some
    rules' bounds, so thresholds move) run three times on one context: the
    tentative pass-2 fields of the last slice and the full replay with its
    backoff must give the oracle's result every time."""
    dbj, info = synth.make_db(29, 900)
    tr = synth.make_traffic((dbj, info), 5_000_000, seed=30, zipf=1.15)
    perm = np.random.default_rng(29).permutation(5_000_000)
    for k in ('src', 'dst', 'sport', 'dport', 'proto', 'ifc', 'form', 't', 'cid'):
        tr[k] = tr[k][perm]
    compiled = CompiledRules(acldb.load_json(dbj))
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    R = coracle.OracleRules(dbj)
    cols, ots, oorder = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ots, oorder, 40)
    rows = ref['rows']
    want = sorted(zip(*(rows[k].astype(int).tolist() for k in ('gid', 'pspell', 'for_ip', 'to_ip', 'to_port', 'count',
                                                                  'first', 'last'))))
    for _ in range(3):
        res = engine.run([b], 40, capacity=built_hit_count(tup))
        assert np.array_equal(res.matches, ref['matches']) and np.array_equal(res.hits, ref['hits'])
        got = sorted((int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']),
                      int(r['count']), int(r['first']), int(r['last'])) for r in res.records)
        assert got == want
    assert (ref['n_conns'] >= 40).sum() > 10


def test_capacity_above_table_limit_is_clamped(engine):
    """rsa_reset clamps a capacity above the largest table (callers pass the
    hit-line count, an upper bound) instead of refusing the job."""
    dbj, info = synth.make_db(33, 200)
    tr = synth.make_traffic((dbj, info), 20000, seed=34)
    compiled = CompiledRules(acldb.load_json(dbj))
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    res = engine.run([b], 1000, capacity=10 ** 12)
    R = coracle.OracleRules(dbj)
    cols, ots, oorder = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ots, oorder, 1000)
    assert np.array_equal(res.matches, ref['matches']) and len(res.records) == len(ref['rows']['gid'])
    engine.reset(1024, 1000)   # back to a small table for the other tests


def test_synth_parity_no_precheck(engine):
    """Slot updates without the plain-load pre-check (every field by atomics)."""
    from ruleset_analysis_amd import native
    engine.set_option(native.RSA_OPT_PRECHECK, 0)
    try:
        _gpu_vs_oracle(engine, 1500, 5_000_000, 40, seed=26, zipf=1.1, broad=False, shuffle=True)
    finally:
        engine.set_option(native.RSA_OPT_PRECHECK, 1)


def test_deterministic(engine):
    dbj, info = synth.make_db(21, 800)
    tr = synth.make_traffic((dbj, info), 100000, seed=22, zipf=1.2)
    compiled = CompiledRules(acldb.load_json(dbj))
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    outs = []
    for _ in range(2):
        res = engine.run([b], 30, capacity=built_hit_count(tup))
        rec = np.sort(res.records, order=['gid', 'for_ip', 'to_ip', 'to_port', 'pspell'])
        outs.append((res.matches.copy(), res.hits.copy(), res.thresh.copy(), rec))
    for a, c in zip(outs[0], outs[1]):
        assert np.array_equal(a, c)


def test_export_import_roundtrip(engine):
    """Pass-1 records exported from one table and imported into a fresh one
    (the multi-GPU merge path) give the same final tables."""
    dbj, info = synth.make_db(31, 300)
    tr = synth.make_traffic((dbj, info), 80000, seed=32, zipf=1.3)
    compiled = CompiledRules(acldb.load_json(dbj))
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    cap = 1000000
    ref = engine.run([b], cap, capacity=built_hit_count(tup))
    exported = engine.emit_device('pass1').clone()
    engine.reset(built_hit_count(tup), cap)
    engine.import_records(exported, 0)
    assert engine.resolve_cap() == 0
    got = engine.results(cap)
    f = ['gid', 'for_ip', 'to_ip', 'to_port', 'pspell', 'count', 'first', 'last', 'min_order']
    assert np.array_equal(np.sort(got.records[f], order=f), np.sort(ref.records[f], order=f))


def test_cfg2_shape_20m_lines(engine):
    """BASELINE config 2's shape (one ACL of 1k expanded rules, no catch-all
    permit) at 20M lines, cap 1000, against the C oracle."""
    res, ref = _gpu_vs_oracle(engine, 1000, 20_000_000, 1000, seed=2, broad=False)
    assert int(res.matches.sum()) > 10_000_000


def test_cfg5_shape_zipf_multi_acl_10m_lines(engine):
    """BASELINE config 5's shape: 4 interface ACLs x 2.5k rules, Zipf 1.1
    over rules, cap 1000 engaged, 10M lines, shuffled input order."""
    res, ref = _gpu_vs_oracle(engine, 2500, 10_000_000, 1000, seed=5, zipf=1.1,
                              interfaces=('outside', 'partner', 'vpn', 'extranet'), broad=False, shuffle=True)
    assert (ref['n_conns'] >= 1000).sum() > 20          # the cap is engaged on many rules


@pytest.mark.parametrize('shuffle', [False, True])
def test_cfg5_population_zipf_10m_lines(engine, shuffle):
    """BASELINE config 5 as SURVEY.md 8d defines it: 4 interface ACLs x 2.5k
    rules, every line's (src, dst, dport) drawn Zipf s=1.1 from a population
    of 1e8 connections (hot connections repeat: the reducer's count/first/last
    updates of one key, connlist-reducer.py:167-172), cap 1000 engaged,
    10M lines, in time order and shuffled, against the C oracle."""
    res, ref = _gpu_vs_oracle(engine, 2500, 10_000_000, 1000, seed=5, zipf=1.1, population=10 ** 8,
                              interfaces=('outside', 'partner', 'vpn', 'extranet'), broad=False, shuffle=shuffle)
    assert (ref['n_conns'] >= 1000).sum() > 20
    assert int(ref['rows']['count'].max()) > 10000      # one connection seen many times


@pytest.mark.parametrize('n_lines,cap,shuffle', [(600_000, 1000, False), (600_000, 20, True), (5_000_000, 40, False)])
def test_hot_split_every_region(engine, n_lines, cap, shuffle):
    """Every region holding a record takes the hot-region path
    (RSA_OPT_HOT_MIN=1): its segment is cut into slices pre-combined on all
    CUs (k_hot_combine), pass 1 and the pass-2 recount, then merged by its
    k_reduce workgroup -- per-rule results equal the C oracle's; the 5M-line
    case runs the filter slices (four segments per region in pass 2)."""
    engine.set_option(native.RSA_OPT_HOT_MIN, 1)
    try:
        _gpu_vs_oracle(engine, 800, n_lines, cap, seed=21, zipf=1.1, population=10 ** 6, shuffle=shuffle)
    finally:
        engine.set_option(native.RSA_OPT_HOT_MIN, 65536)


def test_hot_split_off_equals_on(engine):
    """The skewed 10M-line shape with the hot split off (one workgroup reads a
    hot region alone) gives the same records as with it on."""
    engine.set_option(native.RSA_OPT_HOT_SPLIT, 0)
    try:
        _gpu_vs_oracle(engine, 2500, 3_000_000, 1000, seed=5, zipf=1.1, population=10 ** 8,
                       interfaces=('outside', 'partner'), broad=False)
    finally:
        engine.set_option(native.RSA_OPT_HOT_SPLIT, 1)


@pytest.mark.parametrize('zipf,n_lines', [(None, 2_000_000), (1.2, 3_000_000)])
def test_count_by_rule_block_past_lds(engine, zipf, n_lines):
    """20000 rules (past the 13312 LDS counters): the per-rule line and hit
    counters by rule-block counting sort (k_cnt_*; >2^18 lines in a block, so
    blocks split into several tasks) equal one device atomic per
    line (RSA_OPT_COUNT_SORT=0) and the host's bincount of the pass-1 gids."""
    from ruleset_analysis_amd.compile import F_HIT
    dbj, info = synth.make_db(71, 20000, broad=False)
    tr = synth.make_traffic((dbj, info), n_lines, seed=72, zipf=zipf)
    compiled = CompiledRules(acldb.load_json(dbj))
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    out = []
    for on in (1, 0):
        engine.set_option(native.RSA_OPT_COUNT_SORT, on)
        try:
            b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
            res = engine.run([b], 1000, capacity=max(built_hit_count(tup), 1))
            out.append((res.matches.copy(), res.hits.copy(), engine.last_gids[0].cpu().numpy()))
        finally:
            engine.set_option(native.RSA_OPT_COUNT_SORT, 1)
    (m1, h1, g1), (m0, h0, g0) = out
    assert np.array_equal(g1, g0)
    assert np.array_equal(m1, m0) and np.array_equal(h1, h0)
    nr = len(m1)
    ok = g1 >= 0
    assert np.array_equal(m1, np.bincount(g1[ok], minlength=nr))
    hit = ok & ((tup['flags'] & F_HIT) != 0)
    assert np.array_equal(h1, np.bincount(g1[hit], minlength=nr))
    assert np.bincount(g1[ok] >> 13).max() > 1 << 18          # a block of several tasks
