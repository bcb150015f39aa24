"""BASELINE config 4 on the host: the FortiGate preprocessor restatement
(ruleset-analysis_amd/fortigate.py) expands a synthetic config exactly as the
oracle's loop-by-loop restatement of preprosess_fortigate_acl.py does, and the
run-compressed candidate lists (plus the chained perfect-hash index) classify
like the C oracle's scan of the fully expanded rules."""
import numpy as np
import pytest

from cpu_model import classify_entries
from oracle import coracle
from oracle import fortigate as ofg
from ruleset_analysis_amd import fortigate, synth, synth_fg
from ruleset_analysis_amd.compile import CompiledRules, STEP_SPORT, compress_runs, pht_lookup, RULE_DTYPE


@pytest.fixture(scope='module')
def small_fg():
    text, info = synth_fg.make_config(7, n_policies=30, n_wide=1, n_mid=1, n_syslog=2, wide_members=(2, 3))
    return text, info, fortigate.build_db(text)


def test_expansion_identical_to_oracle(small_fg):
    text, info, db = small_fg
    host, fws, acls = ofg.expand(text)
    assert fws == db.firewalls
    assert set(acls) == set(db.accesslists[host])
    for a, A in acls.items():
        c = ofg.as_columns(A)
        r = db.accesslists[host][a]['rules']
        assert len(r) == len(A)
        assert np.array_equal(c['action'], r.action.astype(np.uint8))
        assert [r.proto_names[k] for k in r.proto] == c['proto']
        assert np.array_equal(c['src'], r.src) and np.array_equal(c['dst'], r.dst)
        assert np.array_equal(c['src_len'], np.uint64(1) << (32 - r.src_len.astype(np.uint64)))
        assert np.array_equal(c['dst_len'], np.uint64(1) << (32 - r.dst_len.astype(np.uint64)))
        assert np.array_equal(c['sport'], r.sport) and np.array_equal(c['dport'], r.dport)
        po = db.accesslists[host][a]['protocols']
        assert set(po) == set(A.protocols)
        for k in po:
            assert np.array_equal(po[k], A.protocols[k])
    assert sum(len(A) for A in acls.values()) > 100000


def test_policy_order_is_python2_dict_order(small_fg):
    """preprosess_fortigate_acl.py:362 iterates obj['policy'].keys(): Python 2
    dict order of the policy-id strings, not config order (SURVEY.md trap 10)."""
    text, info, db = small_fg
    host = info['host']
    rules = db.accesslists[host]['outside-in']['rules']
    seen = []
    for i in range(len(rules)):
        pid = rules.rulenums[rules.rulenum[i]]
        if not seen or seen[-1] != pid:
            seen.append(pid)
    from oracle.py2dict import py2_keys
    outside = [p[0] for p in info['policies'] if p[1] == 'Outside']
    want = [k for k in py2_keys([p[0] for p in info['policies']]) if k in outside]
    assert seen == want and seen != sorted(seen, key=int)


def test_materialised_rule_matches_reference_fields(small_fg):
    text, info, db = small_fg
    rules = db.accesslists[info['host']]['outside-in']['rules']
    r = rules[5]
    assert r.ruleindex == 5 and r.original.startswith('access-list outside-in ')
    assert isinstance(r.sport, list) and len(r.sport) == 1 and len(r.comments) == 1
    assert 'remark section-' in r.comments[0]


def test_reference_quirks():
    base = '\n'.join(['config router setting', 'set hostname "FG-X1"', 'end',
                      'config firewall address', 'edit "a"', 'set subnet 10.0.0.0 255.255.255.0', 'next',
                      'edit "f"', 'set type fqdn', 'set fqdn "host.example"', 'next', 'end',
                      'config firewall addrgrp', 'edit "g"', 'set member "a" "f"', 'next', 'end',
                      'config firewall service custom', 'edit "ANY-TCP"', 'set protocol TCP/UDP/SCTP',
                      'set tcp-portrange 1-65535', 'next', 'edit "ALL"', 'set protocol IP', 'next', 'end',
                      'config firewall service group', 'end',
                      'config firewall policy',
                      'edit 1', 'set srcintf "Outside"', 'set srcaddr "g"', 'set dstaddr "a"', 'set action accept',
                      'set status enable', 'set service "ANY-TCP" "ALL"', "set comments ''", 'set global-label "x"',
                      'next',
                      'edit 2', 'set srcintf "Wan2"', 'set srcaddr "a"', 'set dstaddr "a"', 'set action accept',
                      'set status enable', 'set service "ALL"', "set comments ''", 'set global-label "x"', 'next',
                      'end', ''])
    db = fortigate.build_db(base)
    acl = db.accesslists['FG-X1']['outside-in']
    # the fqdn member cannot be resolved offline: skipped (the reference's failed lookup)
    assert len(acl['rules']) == 2
    assert acl['rules'][0].sport == [-1] and acl['rules'][0].dport == [-1]     # 1-65535 -> NO_PORT
    assert db.firewalls['FG-X1'] == {'X1-outside': {'in': 'outside-in'}, 'X1-': {'in': ''}}
    host, fws, acls = ofg.expand(base)
    assert fws == db.firewalls and len(acls['outside-in']) == 2
    # an ACL whose policies expand to no rule has no proto2rule entry: KeyError (:427)
    with pytest.raises(KeyError):
        fortigate.build_db(base.replace('set dstaddr "a"', 'set dstaddr "f"'))


def test_run_compression_exact():
    """Stepped run entries reproduce the expanded indices exactly (ASA nesting:
    dport outermost, stride = |dst| x |src|; source-port runs too)."""
    rows = []
    gid = 0
    for dp in range(1000, 1100):                  # dport -> dst -> src
        for d in range(3):
            for s in range(2):
                rows.append((0x0B000000 + s, 0, 0x0A000000 + d, 0, 0 | (dp << 16), 0xFFFF, gid, 0))
                gid += 1
    for sp in range(512, 600):                    # a source-port run, stride 1
        rows.append((0, 0xFFFFFFFF, 0x0A0000FF, 0, sp | (514 << 16), 0, gid, 0))
        gid += 1
    arr = np.array(rows, dtype=np.uint64)
    ent = np.zeros(len(rows), RULE_DTYPE)
    for j, name in enumerate(RULE_DTYPE.names):
        ent[name] = arr[:, j]
    comp = compress_runs(ent)
    assert len(comp) == 7 and (comp['step'] != 0).all()
    assert set(int(x) for x in comp['step'] & ~np.uint32(STEP_SPORT)) == {6, 1}
    assert np.all(np.diff(comp['gid'].astype(np.int64)) >= 0)
    rng = np.random.default_rng(1)
    n = 4000
    tup = np.zeros(n, synth.np.dtype([('src', '<u4'), ('dst', '<u4'), ('sport', '<u2'), ('dport', '<u2'),
                                      ('list', '<u2'), ('flags', 'u1'), ('pspell', 'u1')]))
    tup['src'] = rng.choice([0x0B000000, 0x0B000001, 0x0C000000], n)
    tup['dst'] = rng.choice([0x0A000000, 0x0A000001, 0x0A000002, 0x0A0000FF], n)
    tup['sport'] = rng.integers(500, 700, n)
    tup['dport'] = rng.choice([514, 999, 1000, 1050, 1099, 1100], n)
    tup['flags'] = 1
    off = np.array([0, len(ent)], np.uint32)
    assert np.array_equal(classify_entries(ent, off, tup), classify_entries(comp, np.array([0, len(comp)], np.uint32),
                                                                             tup))


@pytest.mark.parametrize('chunk', [None, 700])
def test_compressed_index_classifies_like_oracle(small_fg, chunk):
    text, info, db = small_fg
    comp = CompiledRules(db)
    comp.ensure_lists()
    ent, off = comp.packed()
    assert (ent['step'] != 0).sum() > 5
    tr = synth_fg.make_traffic(info, 3000, seed=8)
    tup, _ts, _order = synth.pack(tr, comp)
    R = coracle.OracleRules.from_fortigate(text)
    cols, _ots, _oorder = coracle.inputs_from_traffic(R, tr)
    ref, evals = coracle.classify(R, cols['list'], cols['proto'], cols['src'], cols['dst'], cols['sport'],
                                  cols['dport'])
    assert evals > 50 * len(tup)                     # long scans in the reference
    assert np.array_equal(classify_entries(ent, off, tup), ref)
    index = comp.index(chunk=chunk, kind='pht')
    if chunk:
        assert int(index[0][4]) > int(index[0][2])     # chained records exist
    for i in range(0, len(tup), 3):
        t = tup[i]
        if not t['flags'] & 1:
            continue
        k = pht_lookup(index, ent, off, int(t['list']), int(t['src']), int(t['dst']),
                       int(t['sport']) | (int(t['dport']) << 16))
        assert k == 'defer' or k == ref[i], i
