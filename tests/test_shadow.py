"""Shadowed-rule analysis (preprosess_access_lists.py:508-521): the GPU pairwise
containment scan (rsa_shadowed) against the C oracle's double loop, which is
itself pinned to the Python oracle's literal `rule in accesslists[acl][i]`
(oracle.firewallrule's FirewallRule.__contains__, firewallrule.py:128-174)."""
import numpy as np
import pytest

from oracle import coracle
from oracle.crosscheck_2to3 import oracle_db
from ruleset_analysis_amd import acldb, fortigate, synth, synth_fg
from ruleset_analysis_amd.shadow import shadow_messages, shadow_table, shadowed


def _python_shadow(rules):
    out = []
    for index, rule in enumerate(rules):
        cov = -1
        for i in range(index):
            if rule in rules[i]:
                cov = i
                break
        out.append(cov)
    return np.array(out, np.int32)


def test_c_oracle_shadow_equals_python_oracle():
    dbj, info = synth.make_db(91, 300)
    acls, _fws = oracle_db(dbj)
    R = coracle.OracleRules(dbj)
    n_shadowed = 0
    for acl in acls['fw1']:
        want = _python_shadow(acls['fw1'][acl]['rules'])
        got = coracle.shadow(R, 'fw1', acl)
        assert np.array_equal(got, want), acl
        n_shadowed += int((want >= 0).sum())
    assert n_shadowed > 0


def test_shadow_table_columns_equal_objects():
    text, info = synth_fg.make_config(7, n_policies=12, n_wide=0, n_mid=0, n_syslog=1)
    db = fortigate.build_db(text)
    rules = db.accesslists[info['host']]['outside-in']['rules']
    cols = shadow_table(rules)
    objs = shadow_table([rules[i] for i in range(len(rules))])
    for f in ('src_lo', 'src_span', 'dst_lo', 'dst_span', 'sport', 'dport', 'action', 'v4'):
        assert np.array_equal(cols[f], objs[f]), f
    # protocol ids may be numbered differently, but 'ip' is 0 and equality is preserved
    assert np.array_equal(cols['proto'] == 0, objs['proto'] == 0)


def test_laminar_codes_keep_containment():
    """IPv6 prefix networks -> 32-bit intervals: a contains b exactly when
    a's interval holds b's (random nested and disjoint prefixes)."""
    from ruleset_analysis_amd.shadow import laminar_codes
    rng = np.random.default_rng(11)
    nets = []
    for _ in range(400):
        plen = int(rng.integers(0, 129))
        base = int(rng.integers(0, 4)) << 126 | int(rng.integers(0, 1 << 62)) << 64 | int(rng.integers(0, 1 << 63))
        nets.append((base >> (128 - plen) << (128 - plen) if plen else 0, plen))
    nets += [(0, 0), nets[3], (nets[5][0], 128)]
    codes = laminar_codes(nets)
    last = lambda t: t[0] + (1 << (128 - t[1])) - 1
    for a in set(nets):
        for b in set(nets):
            inside = b[0] >= a[0] and last(b) <= last(a)
            (la, sa), (lb, sb) = codes[a], codes[b]
            assert inside == (lb >= la and lb + sb <= la + sa), (a, b)


def test_shadow_table_ipv6_columns_equal_objects():
    """asa_ipv6: the columnar rows (family codes, interval codes of the IPv6
    sides) equal the rows of the materialised FirewallRule objects."""
    import os
    from conftest import ROOT
    from ruleset_analysis_amd import asa
    with open(os.path.join(ROOT, 'tests', 'golden_asa', 'asa_ipv6', 'config.txt')) as f:
        db = asa.build_db(f.read())
    for acl, e in db.accesslists['v6-fw'].items():
        rules = e['rules']
        cols = shadow_table(rules)
        objs = shadow_table([rules[i] for i in range(len(rules))])
        for f in ('src_lo', 'src_span', 'dst_lo', 'dst_span', 'sport', 'dport', 'action', 'v4'):
            assert np.array_equal(cols[f], objs[f]), (acl, f)
    assert set(shadow_table(db.accesslists['v6-fw']['outside_in']['rules'])['v4'].tolist()) == {1, 3, 4, 5}


@pytest.mark.gpu
def test_gpu_shadow_equals_oracle_asa(engine):
    dbj, info = synth.make_db(92, 10000, interfaces=('outside', 'partner'))
    db = acldb.load_json(dbj)
    R = coracle.OracleRules(dbj)
    for acl, e in db.accesslists['fw1'].items():
        got = shadowed(engine, shadow_table(e['rules']))
        want = coracle.shadow(R, 'fw1', acl)
        assert np.array_equal(got, want), acl
    msgs = shadow_messages(engine, {a: e['rules'] for a, e in db.accesslists['fw1'].items()})
    assert msgs and msgs[0].startswith('Found rule which never gets hits since it is covered by a more generic rule')
    assert msgs[1].startswith('Specific rule ') and msgs[2].startswith('Generic rule ')


@pytest.mark.gpu
def test_gpu_shadow_equals_oracle_fortigate(engine):
    text, info = synth_fg.make_config(93, n_policies=40, n_wide=1, wide_members=(2, 2))
    db = fortigate.build_db(text)
    R = coracle.OracleRules.from_fortigate(text)
    for acl in ('outside-in', 'inside-in'):
        rules = db.accesslists[info['host']][acl]['rules']
        got = shadowed(engine, shadow_table(rules))
        want = coracle.shadow(R, info['host'], acl)
        assert np.array_equal(got, want), acl
        if acl == 'outside-in':
            assert len(rules) > 200000 and (got >= 0).sum() > 0


def _multiport_rules(seed, n):
    """Random rules with [NO_PORT], single ports and port lists (duplicates and
    -1 inside lists included), few addresses and ports so containments occur;
    the product's FirewallRule and the oracle's, built from the same fields."""
    import random
    from oracle.firewallrule import FirewallRule as OracleRule
    from ruleset_analysis_amd.firewallrule import FirewallRule
    rng = random.Random(seed)
    nets = ['any', '10.0.0.0/8', '10.1.0.0/16', '10.1.2.0/24', '10.1.2.3', '192.168.0.0/16', '192.168.1.1']
    pool = [22, 53, 80, 443, 8080]

    def ports():
        r = rng.random()
        if r < 0.35:
            return [-1]
        if r < 0.65:
            return [rng.choice(pool)]
        return [rng.choice(pool + [-1] * (r > 0.95)) for _ in range(rng.randrange(2, 5))]

    prod, orac = [], []
    for k in range(n):
        args = (rng.random() < 0.8, rng.choice(['ip', 'tcp', 'udp']), 'line %d' % k, rng.choice(nets), rng.choice(nets))
        sp, dp = ports(), ports()
        prod.append(FirewallRule(*args, sport=list(sp), dport=list(dp), ruleindex=k))
        orac.append(OracleRule(*args, sport=list(sp), dport=list(dp), ruleindex=k))
    return prod, orac


def test_shadow_table_port_lists():
    prod, _orac = _multiport_rules(5, 300)
    t = shadow_table(prod)
    for r, row in zip(prod, t):
        for side, v in ((r.sport, int(row['sport'])), (r.dport, int(row['dport']))):
            if len(side) == 1:
                assert v == side[0]
            else:
                at = -v - 2
                assert list(t.ports[at + 1:at + 1 + t.ports[at]]) == side


@pytest.mark.gpu
@pytest.mark.parametrize('seed', [1, 2])
def test_gpu_shadow_port_lists_equal_python_oracle(engine, seed):
    """Rules with multi-port sides (list containment, firewallrule.py:162-171):
    the GPU cover equals the oracle's literal double loop of `in` tests."""
    prod, orac = _multiport_rules(seed, 3000)
    got = shadowed(engine, shadow_table(prod))
    want = _python_shadow(orac)
    assert np.array_equal(got, want)
    assert (want >= 0).sum() > 100
