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
