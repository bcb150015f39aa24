"""BASELINE config 3's rule set at 16M lines (the job runs the filter slices
1M, 4M and the rest of the batch, each bounded by the thresholds resolved
after the previous one) and at the bench's full 125M-line shard (slices 1M,
4M, 16M, the rest), checked against the C oracle where the
oracle can follow it: the first match of 16K lines drawn uniformly from the
batch, and for 48 rules -- capped ones, the heaviest uncapped ones, random
ones -- every connection record, reduced by the oracle from all of those
rules' lines (a rule's records depend only on its own lines).  The lines of
the chosen rules are re-classified by the oracle too, so a line the GPU put
in one of them must belong there."""
import numpy as np
import pytest

from oracle import coracle
from ruleset_analysis_amd import acldb, synth
from ruleset_analysis_amd.compile import CompiledRules
from ruleset_analysis_amd.engine import DeviceBatch
from ruleset_analysis_amd.pipeline import built_hit_count

pytestmark = pytest.mark.gpu
NO = 0xFFFFFFFFFFFFFFFF
FIELDS = ('gid', 'pspell', 'for_ip', 'to_ip', 'to_port', 'count', 'first', 'last')


def _sub(tr, idx, n):
    return {k: (np.asarray(v)[idx] if isinstance(v, np.ndarray) and len(v) == n else v) for k, v in tr.items()}


def _classify(R, cols):
    return coracle.classify(R, cols['list'], cols['proto'], cols['src'], cols['dst'], cols['sport'],
                            cols['dport'])[0]


@pytest.mark.parametrize('n', [16_000_000, 125_000_000])
def test_cfg3_rules_sampled_against_oracle(engine, n):
    cap = 1000
    dbj, info = synth.make_db(3, 10000, interfaces=('outside',), broad=False)
    compiled = CompiledRules(acldb.load_json(dbj))
    compiled.ensure_lists()
    tr = synth.make_traffic((dbj, info), n, seed=3 * 1_000_003, t0=15 * 86400, span=3 * 3600, cid0=1_000_000)
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    res = engine.run([b], cap, capacity=max(built_hit_count(tup), 1))
    gids = engine.last_gids[0].cpu().numpy()
    R = coracle.OracleRules(dbj)
    nr = compiled.n_rules
    # (1) first match of a uniform sample of lines
    pick = np.sort(np.random.default_rng(11).choice(n, 16384, replace=False))
    cols, _ts, _o = coracle.inputs_from_traffic(R, _sub(tr, pick, n))
    assert np.array_equal(gids[pick], _classify(R, cols))
    # (2) whole rules: capped, heaviest uncapped, random
    capped = np.nonzero(res.thresh[:nr] != NO)[0]
    lines_of = np.bincount(gids[gids >= 0], minlength=nr)[:nr]
    unc = np.nonzero((res.thresh[:nr] == NO) & (lines_of > 0))[0]
    rng = np.random.default_rng(12)
    assert len(capped) >= 16 and len(unc) >= 32
    heavy = unc[np.argsort(lines_of[unc])[::-1][:16]]
    rules = np.unique(np.concatenate([rng.choice(capped, 16, replace=False), heavy,
                                      rng.choice(unc, 16, replace=False)]))
    sel = np.nonzero(np.isin(gids, rules))[0]
    cols, ts_s, o_s = coracle.inputs_from_traffic(R, _sub(tr, sel, n))
    g_ref = _classify(R, cols)
    assert np.array_equal(gids[sel], g_ref)
    ref = coracle.reduce(R, g_ref, cols['flags'], cols['pspell'], cols['src'], cols['dst'], cols['sport'],
                         cols['dport'], ts_s, o_s, cap)
    assert np.array_equal(res.matches[rules], ref['matches'][rules])
    assert np.array_equal(res.hits[rules], ref['hits'][rules])
    assert np.array_equal(res.thresh[rules] != NO, ref['n_conns'][rules] >= cap)
    recs = res.records[np.isin(res.records['gid'], rules)]
    got = sorted(zip(*(recs[k].astype(np.int64).tolist() for k in FIELDS)))
    want = sorted(zip(*(ref['rows'][k].astype(np.int64).tolist() for k in FIELDS)))
    assert got == want
    assert len(want) > 16 * cap
