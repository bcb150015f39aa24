"""Python 2 byte-string text semantics (ruleset-analysis_amd/py2text.py) in
the preprocessor and postprocessor restatements: the reference strips and
splits config lines on the six ASCII whitespace bytes only, so NBSP (\\xa0),
NEL (\\x85) and \\x1c-\\x1f stay inside tokens; lower() and int() are ASCII."""
import pytest

from oracle.crosscheck_fortigate import EDGES, recorded_resolver
from ruleset_analysis_amd import asa, fortigate
from ruleset_analysis_amd.firewallrule import FirewallRule
from ruleset_analysis_amd.py2text import py2_int, py2_isdigit, py2_lower, py2_split, py2_strip


def test_helpers():
    assert py2_strip(' \t\xa0x\x85\r\n') == '\xa0x\x85'
    assert py2_split(' a\xa0b  c\x1cd\te ') == ['a\xa0b', 'c\x1cd', 'e']
    assert py2_split(' \t ') == [] and py2_split('') == []
    assert py2_lower('TCP\xc0Outside') == 'tcp\xc0outside'
    assert py2_int(' 42\n') == 42 and py2_int('-7') == -7 and py2_int(5) == 5
    for bad in ('1_000', '42\xa0', '\xb2', '', '4 2', '0x10'):
        with pytest.raises(ValueError):
            py2_int(bad)
    assert py2_isdigit('0123') and not py2_isdigit('\xb9') and not py2_isdigit('')


ASA_CFG = ('hostname fw\x85\n'
           'access-list outside_in remark first\n'
           'access-list outside_in extended permit tcp any host 10.0.0.1 eq www\n'
           'access-list outside_in remark\xa0not a remark token\n'
           'access-list outside_in extended permit udp any host 10.0.0.2 eq 53\n'
           'access-list outside_in extended deny ip any any\n'
           'access-group outside_in in interface outside\n')


def test_asa_keeps_non_ascii_whitespace_in_tokens():
    db = asa.build_db(ASA_CFG)
    assert list(db.firewalls) == ['fw\x85']
    rules = db.accesslists['fw\x85']['outside_in']['rules']
    assert len(rules) == 3
    # 'remark\xa0not...' is one token: not a remark line for the comment logic
    # (parts[2] != 'remark'), and the entry parser skips it as a remark; the
    # udp rule keeps the first block's comments
    assert rules[0].comments == ['access-list outside_in remark first']
    assert rules[1].comments == ['access-list outside_in remark first']


def test_asa_port_with_nbsp_is_a_parse_error():
    bad = ASA_CFG.replace('eq 53\n', 'eq 53\xa0\n')
    logs = []
    with pytest.raises(SystemExit):
        asa.build_db(bad, log=logs.append)
    assert 'Unable to parse one of the lines' in ''.join(logs)


def test_fortigate_keeps_nbsp_in_values():
    text = EDGES.replace('set srcintf "DMZ"', 'set srcintf "Outside"\xa0').replace(
        'set comments "guests"', 'set comments "guests\xa0only"')
    db = fortigate.build_db(text, resolve=recorded_resolver({'localhost': ['127.0.0.1']}))
    acls = db.accesslists['FG-EDGE9']
    # '"Outside"\xa0' is not '"Outside"': the policy stays in ACL ''
    assert any(r.original.startswith('access-list outside\xa0-in permit') for r in acls['']['rules'])
    assert acls['inside-in']['rules'][0].comments == ['access-list guest-inside-in remark Guest: guests\xa0only']


def test_fortigate_lines_end_at_newline_only():
    # '\x0c' and '\x1c' are line breaks for str.splitlines() but not for readlines()
    # (with readlines() the object is named '"web2"\x1c    set comment "x"', so
    # the group member "web2" is unknown: the reference's KeyError)
    text = EDGES.replace('    edit "web2"\n', '    edit "web2"\x1c    set comment "x"\n')
    with pytest.raises(KeyError) as ei:
        fortigate.build_db(text, resolve=recorded_resolver({'localhost': ['127.0.0.1']}))
    assert ei.value.args == ('"web2"',)


def test_firewallrule_string_ports_are_python2_ints():
    r = FirewallRule(True, 'tcp', 'x', 'any', 'any', ' 80', '443')
    assert r.sport == [80] and r.dport == [443]
    with pytest.raises(ValueError):
        FirewallRule(True, 'tcp', 'x', 'any', 'any', '8_0', '443')
