"""ASA preprocessor restatement (asa.py, preprosess_access_lists.py:28-550):
pinned to the lib2to3-converted reference on the committed configs
(tests/golden_asa, written by oracle/crosscheck_asa.py: digest of the whole
DB, first rules, the -v shadowed-rule messages), the reference's error exits,
and the fused GPU job over a DB it builds against the Python oracle."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle.crosscheck_asa import dump_db, digest
from ruleset_analysis_amd import asa, synth_asa

GOLDEN_ASA = os.path.join(ROOT, 'tests', 'golden_asa')
CASES = sorted(os.listdir(GOLDEN_ASA))


def _case(name):
    d = os.path.join(GOLDEN_ASA, name)
    with open(os.path.join(d, 'config.txt'), encoding='latin-1', newline='') as f:
        text = f.read()
    with open(os.path.join(d, 'db.sha256')) as f:
        sha = f.read().strip()
    with open(os.path.join(d, 'summary.json')) as f:
        summary = json.load(f)
    with open(os.path.join(d, 'shadow.json')) as f:
        shadow = json.load(f)
    return text, sha, summary, shadow


@pytest.mark.parametrize('case', CASES)
def test_asa_db_equals_converted_reference(case):
    text, sha, summary, _shadow = _case(case)
    db = asa.build_db(text)
    dump = json.loads(json.dumps(dump_db(db), sort_keys=True))
    assert dump['firewalls'] == summary['firewalls']
    for acl, s in summary['acls'].items():
        e = [a for hs in dump['accesslists'].values() for n, a in hs.items() if n == acl][0]
        assert len(e['rules']) == s['n_rules']
        assert {p: len(v) for p, v in e['protocols'].items()} == s['protocols']
        assert e['rules'][:20] == s['first_rules']
    assert digest(dump) == sha


def test_asa_neq_and_names():
    text = ('hostname h\naccess-list a extended permit tcp any host 10.0.0.1 neq www\n'
            'access-list a extended permit udp any eq domain any range 1 3\naccess-group a in interface outside\n')
    db = asa.build_db(text)
    rules = db.accesslists['h']['a']['rules']
    assert len(rules) == 65535 + 3
    dp = rules.dport[:65535]
    assert 80 not in set(dp.tolist()) and dp[0] == 0 and dp[-1] == 65535 and dp[80] == 81
    assert [int(x) for x in rules.sport[65535:]] == [53, 53, 53]
    assert [int(x) for x in rules.dport[65535:]] == [1, 2, 3]
    assert rules[65535].ruleindex == 65535 and rules[65535].rulenum == 2
    assert db.firewalls == {'h': {'outside': {'in': 'a'}}}


def test_asa_reference_errors():
    with pytest.raises(SystemExit):
        asa.build_db('access-list a extended permit ip any any\n')                        # no hostname
    with pytest.raises(SystemExit):
        asa.build_db('hostname h\naccess-list a standard permit 10.0.0.0 255.0.0.0\n')   # regex fails
    with pytest.raises(SystemExit):
        asa.build_db('hostname h\naccess-list a extended permit tcp any any eq notaport\n')
    with pytest.raises(SystemExit):
        asa.build_db('hostname h\naccess-list a extended permit tcp 10.0.0.1 255.255.255.0 any\n')  # host bits
    with pytest.raises(KeyError):
        asa.build_db('hostname h\naccess-list a extended permit tcp object-group NOPE any\n')
    with pytest.raises(KeyError):
        asa.build_db('hostname h\naccess-list a remark only a remark\n')
    msgs = []
    with pytest.raises(SystemExit):
        asa.build_db('hostname h\naccess-list a extended permit tcp any any eq 99999999\n'
                     'access-list a extended permit tcp any any neq 70000\n', log=msgs.append)
    assert msgs[0].startswith('ERROR - Unable to parse one of the lines in the config, aborting.')


def test_asa_comments_shared_across_acls():
    text = ('hostname h\naccess-list a remark r1\naccess-list a remark r2\n'
            'access-list a extended permit ip any any\naccess-list b extended permit ip any any\n'
            'access-list b remark r3\naccess-list a extended permit tcp any any eq 1\n')
    db = asa.build_db(text)
    a, b = db.accesslists['h']['a']['rules'], db.accesslists['h']['b']['rules']
    assert a[0].comments == ['access-list a remark r1', 'access-list a remark r2']
    assert b[0].comments == a[0].comments          # one comment list until the next remark
    assert a[1].comments == ['access-list b remark r3'] and a[1].rulenum == 4


def test_synth_asa_configs_parse():
    for seed in range(4):
        text, info = synth_asa.make_config(seed + 10, 150, wide=seed % 2 == 1)
        db = asa.build_db(text)
        assert set(db.accesslists[info['hostname']]) == set(info['acls'])
        for acl in info['acls']:
            rules = db.accesslists[info['hostname']][acl]['rules']
            assert len(rules) > 0 and rules[len(rules) - 1].original.endswith('deny ip any any')


def _shadow_lines(acl, rules, cover):
    out = []
    for index in np.nonzero(cover >= 0)[0]:
        index, i = int(index), int(cover[index])
        out.append('Found rule which never gets hits since it is covered by a more generic rule above it in '
                   'access-list {0}.'.format(acl))
        out.append('Specific rule ' + str(index) + ': ' + str(rules[index]))
        out.append('Generic rule ' + str(i) + ': ' + str(rules[i]))
    return out


@pytest.mark.parametrize('case', CASES)
def test_c_oracle_shadow_equals_reference_messages(case):
    """The C oracle's double loop (the checker of the GPU scan) on the DB asa.py
    builds reproduces the converted reference's -v messages."""
    from oracle import coracle
    from ruleset_analysis_amd import acldb
    text, _sha, _summary, shadow = _case(case)
    db = asa.build_db(text)
    dbj = acldb.to_json_obj(db)
    for hs in dbj['accesslists'].values():
        for e in hs.values():
            e['protocols'] = {p: [int(x) for x in v] for p, v in e['protocols'].items()}
    R = coracle.OracleRules(json.loads(json.dumps(dbj)))
    n = 0
    for host, acls in db.accesslists.items():
        for acl, e in acls.items():
            got = _shadow_lines(acl, e['rules'], coracle.shadow(R, host, acl))
            assert got == shadow.get(acl, []), acl
            n += len(got)
    assert n == sum(len(v) for v in shadow.values())


# ---- GPU ----------------------------------------------------------------------------------------------

def _traffic_lines(db, host, n, seed):
    """Log lines for connections drawn inside the permit tcp/udp rules of the DB."""
    rng = np.random.default_rng(seed)
    out = []
    ifc_of = {e['in']: ifc for ifc, e in db.firewalls[host].items() if 'in' in e}
    for k in range(n):
        acl = sorted(ifc_of)[k % len(ifc_of)]
        rules = db.accesslists[host][acl]['rules']
        i = int(rng.integers(0, len(rules)))
        while rules.fam[i]:               # IPv6 rules match no IPv4 connection: draw from the others
            i = int(rng.integers(0, len(rules)))
        proto = rules.proto_names[rules.proto[i]]
        proto = proto if proto in ('tcp', 'udp') else 'tcp'
        sl, dl = int(rules.src_len[i]), int(rules.dst_len[i])
        src = int(rules.src[i]) | int(rng.integers(0, 1 << (32 - sl))) if sl < 32 else int(rules.src[i])
        dst = int(rules.dst[i]) | int(rng.integers(0, 1 << (32 - dl))) if dl < 32 else int(rules.dst[i])
        sp = int(rules.sport[i]) if rules.sport[i] >= 0 else int(rng.integers(1024, 65536))
        dp = int(rules.dport[i]) if rules.dport[i] >= 0 else int(rng.integers(1, 1024))
        dot = lambda v: '%d.%d.%d.%d' % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)
        s, d = dot(src & 0xFFFFFFFF), dot(dst & 0xFFFFFFFF)
        t = 'Jul 15 %02d:%02d:%02d' % (k // 3600 % 24, k // 60 % 60, k % 60)
        mid = '302013' if proto == 'tcp' else '302015'
        out.append('%s Jul 15 2013 %s: %%ASA-6-%s: Built inbound %s connection %d for %s:%s/%d (%s/%d) to inside:%s/%d '
                   '(%s/%d)\n' % (t, t[7:], mid, proto.upper(), 100000 + k, ifc_of[acl], s, sp, s, sp, d, dp, d, dp))
    return out


@pytest.mark.gpu
def test_gpu_fused_job_on_asa_db_equals_oracle(engine):
    from oracle.crosscheck_2to3 import oracle_db
    from oracle import pipeline as op
    from ruleset_analysis_amd import acldb
    from ruleset_analysis_amd.pipeline import analyze_text
    text, info = synth_asa.make_config(31, 250, n_net_groups=10)
    db = asa.build_db(text)
    lines = _traffic_lines(db, info['hostname'], 20000, 5)
    dbj = acldb.to_json_obj(db)
    for hs in dbj['accesslists'].values():
        for e in hs.values():
            e['protocols'] = {p: [int(x) for x in v] for p, v in e['protocols'].items()}
    acls, fws = oracle_db(json.loads(json.dumps(dbj)))
    _m, _s, want, _b = op.run_pipeline(''.join(lines), info['hostname'], acls, fws, cap=20)
    got, _ = analyze_text([(info['hostname'], ''.join(lines).encode('latin-1'))], db, cap=20, engine=engine)
    assert got == want
    assert sum(1 for l in got if l.startswith('Total number of hits:')) > 20


def test_ipv6_rules_keep_positions_and_never_match():
    """asa_ipv6: IPv6 rules sit between IPv4 rules with their ruleindex and
    are absent from every compiled candidate list (IPy never contains an IPv4
    address in an IPv6 network)."""
    from ruleset_analysis_amd.compile import CompiledRules
    text, _sha, _summary, _shadow = _case('asa_ipv6')
    db = asa.build_db(text)
    rules = db.accesslists['v6-fw']['outside_in']['rules']
    six = np.flatnonzero(rules.fam)
    assert len(six) and six[0] == 1 and len(six) < len(rules)
    assert str(rules[1].src) == '2001:db8::1' and rules[1].ruleindex == 1
    comp = CompiledRules(db)
    comp.ensure_lists()
    gids = set()
    for lst in comp._lists:
        gids.update(int(g) for g in lst['gid'])
    base = comp.base[('v6-fw', 'outside_in')]
    assert not gids & {base + int(i) for i in six}
    assert base + 0 in gids


@pytest.mark.gpu
def test_gpu_fused_job_on_ipv6_db_equals_oracle(engine):
    """The fused job over the asa_ipv6 DB (IPv6 rules between IPv4 ones) gives
    the oracle's report: gids past an IPv6 rule keep their ruleindex."""
    from oracle.crosscheck_2to3 import oracle_db
    from oracle import pipeline as op
    from ruleset_analysis_amd import acldb
    from ruleset_analysis_amd.pipeline import analyze_text
    text, _sha, _summary, _shadow = _case('asa_ipv6')
    db = asa.build_db(text)
    lines = _traffic_lines(db, 'v6-fw', 5000, 9)
    dbj = acldb.to_json_obj(db)
    for hs in dbj['accesslists'].values():
        for e in hs.values():
            e['protocols'] = {p: [int(x) for x in v] for p, v in e['protocols'].items()}
    acls, fws = oracle_db(json.loads(json.dumps(dbj)))
    _m, _s, want, _b = op.run_pipeline(''.join(lines), 'v6-fw', acls, fws, cap=50)
    got, _ = analyze_text([('v6-fw', ''.join(lines).encode('latin-1'))], db, cap=50, engine=engine)
    assert got == want
    assert sum(1 for l in got if l.startswith('Total number of hits:')) >= 4


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_gpu_shadowed_messages_equal_reference(engine, case):
    from ruleset_analysis_amd.shadow import shadow_messages
    text, _sha, _summary, shadow = _case(case)
    db = asa.build_db(text)
    for host, acls in db.accesslists.items():
        for acl, e in acls.items():
            try:
                got = shadow_messages(engine, {acl: e['rules']})
            except NotImplementedError:          # icmp rules with a type per side are outside the kernel
                continue
            assert got == shadow.get(acl, []), acl
