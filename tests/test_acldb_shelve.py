"""accesslists.db as the reference writes it: a dbm file of protocol-0 pickles
holding old-style ``firewallrule.FirewallRule`` instances (INST opcode) and
``IPy.IP`` objects (copy_reg._reconstructor).  The restricted unpickler maps
them onto the drop-in classes and refuses anything else."""
import dbm.ndbm
import pickle

import pytest

from ruleset_analysis_amd import acldb
from ruleset_analysis_amd.firewallrule import FirewallRule


def _s(x):
    return "S'%s'\n" % x


def _ip_pickle(ip, plen):
    # new-style IPy.IP as Python 2 pickles it at protocol 0
    return ("ccopy_reg\n_reconstructor\n(cIPy\nIP\nc__builtin__\nobject\nNtR(d" + _s('ip') + "L%dL\n" % ip +
            's' + _s('_prefixlen') + 'I%d\n' % plen + 's' + _s('_ipversion') + 'I4\nsb')


def _rule_pickle(action, proto, original, src, dst, sport, dport, rulenum, ruleindex):
    def lst(v):
        return '(l' + ''.join('I%d\na' % p for p in v)
    body = ('(ifirewallrule\nFirewallRule\n(d' + _s('action') + ('I01\n' if action else 'I00\n') + 's' +
            _s('protocol') + _s(proto) + 's' + _s('original') + _s(original) + 's' + _s('src') + _ip_pickle(*src) +
            's' + _s('dst') + _ip_pickle(*dst) + 's' + _s('sport') + lst(sport) + 's' + _s('dport') + lst(dport) +
            's' + _s('comments') + '(ls' + _s('rulenum') + 'I%d\ns' % rulenum + _s('ruleindex') +
            'I%d\nsb' % ruleindex)
    return body


def test_load_python2_shelve(tmp_path):
    r0 = _rule_pickle(True, 'tcp', 'access-list a extended permit tcp any host 10.0.0.5 eq 443', (0, 0),
                      (0x0A000005, 32), [-1], [443], 1, 0)
    r1 = _rule_pickle(False, 'ip', 'access-list a extended deny ip any any', (0, 0), (0, 0), [-1], [-1], 2, 1)
    acl = ("(d" + _s('fw1') + "(d" + _s('a') + "(d" + _s('rules') + "(l" + r0 + "a" + r1 + "a" + "s" +
           _s('protocols') + "(d" + _s('tcp') + "(lI0\nas" + _s('ip') + "(lI1\nass" + _s('timestamp') +
           "F1373846400.0\nsss.")
    fws = "(d" + _s('fw1') + "(d" + _s('outside') + "(d" + _s('in') + _s('a') + "sss."
    path = str(tmp_path / 'accesslists')
    db = dbm.ndbm.open(path, 'c')
    db[b'accesslists'] = acl.encode('latin-1')
    db[b'firewalls'] = fws.encode('latin-1')
    db.close()
    loaded = acldb.load(path + '.db')
    assert loaded.firewalls == {'fw1': {'outside': {'in': 'a'}}}
    rules = loaded.accesslists['fw1']['a']['rules']
    assert [type(r) for r in rules] == [FirewallRule, FirewallRule]
    assert str(rules[0]) == 'permit tcp 0.0.0.0/0 -> 10.0.0.5:[443]'
    assert str(rules[1]) == 'deny ip 0.0.0.0/0 -> 0.0.0.0/0'
    assert rules[0].ruleindex == 0 and rules[1].rulenum == 2
    assert loaded.accesslists['fw1']['a']['protocols'] == {'tcp': [0], 'ip': [1]}
    conn = FirewallRule(True, 'tcp', 'x', '1.2.3.4', '10.0.0.5', sport=1234, dport=443)
    assert conn in rules[0]


def test_unpickler_refuses_other_globals(tmp_path):
    path = str(tmp_path / 'evil')
    db = dbm.ndbm.open(path, 'c')
    db[b'accesslists'] = b"cos\nsystem\n(S'true'\ntR."
    db[b'firewalls'] = b'(d.'
    db.close()
    with pytest.raises(pickle.UnpicklingError):
        acldb.load(path + '.db')


def test_json_roundtrip(tmp_path):
    from ruleset_analysis_amd import synth
    dbj, _ = synth.make_db(4, 50)
    db = acldb.load_json(dbj)
    acldb.save_json(db, str(tmp_path / 'x.json'))
    db2 = acldb.load(str(tmp_path / 'x.json'))
    a = db.accesslists['fw1']['outside_access_in']['rules']
    b = db2.accesslists['fw1']['outside_access_in']['rules']
    assert [str(r) for r in a] == [str(r) for r in b]
    assert [r.__dict__ == s.__dict__ for r, s in zip(a, b)] == [True] * len(a)
