"""Known-answer tests of the rule predicate — the reference's only unit test,
``firewallrule.py:177-220`` — run against the oracle restatement AND the
product's drop-in ``FirewallRule``, plus IPy-semantics edge cases the path
depends on."""
import pytest

import oracle.firewallrule as ofr
import oracle.ipy as oipy
from ruleset_analysis_amd import firewallrule as pfr
from ruleset_analysis_amd import ipaddr as pip

IMPLS = [pytest.param((ofr.FirewallRule, oipy.IP), id='oracle'),
         pytest.param((pfr.FirewallRule, pip.IP), id='product')]


@pytest.mark.parametrize('impl', IMPLS)
def test_reference_testcases(impl):
    FR, _IP = impl
    orig = 'original line unknown'
    rule1 = FR(True, 'ip', orig, 'any', 'any')
    rule2 = FR(True, 'tcp', orig, '198.51.100.0/24', '192.0.2.14/32', dport=80)
    rule3 = FR(True, 'ip', orig, '198.51.100.0/24', '192.0.2.14/32')
    rule4 = FR(True, 'tcp', orig, '198.51.100.0/24', 'any', dport=80)
    conn1 = FR(True, 'tcp', orig, '198.51.100.247', '174.35.64.57', sport=54742, dport=80)
    conn2 = FR(True, 'tcp', orig, '203.0.113.247', '174.35.64.57', sport=54742, dport=80)
    conn3 = FR(True, 'tcp', orig, '198.51.100.247', '174.35.64.57', sport=54742, dport=81)
    conn4 = FR(True, 'udp', orig, '198.51.100.247', '174.35.64.57', sport=54742, dport=80)
    # firewallrule.py:194 — repr round trip
    ns = {'FirewallRule': FR}
    assert rule1 == eval(repr(rule1), ns)
    # firewallrule.py:200-202
    cases = [(rule2, rule1, True), (rule2, rule3, True), (rule3, rule2, False), (conn1, rule4, True),
             (conn2, rule4, False), (conn3, rule4, False), (conn4, rule4, False)]
    for inner, outer, expected in cases:
        assert (inner in outer) is expected, (str(inner), str(outer))


@pytest.mark.parametrize('impl', IMPLS)
def test_str_format(impl):
    FR, _ = impl
    r = FR(True, 'tcp', 'x', '10.0.0.0/255.255.255.0', '1.2.3.4', dport=80)
    assert str(r) == 'permit tcp 10.0.0.0/24 -> 1.2.3.4:[80]'
    r = FR(False, 'ip', 'x', 'any', 'any')
    assert str(r) == 'deny ip 0.0.0.0/0 -> 0.0.0.0/0'
    r = FR(True, 'udp', 'x', '10.1.2.3', '10.0.0.0/8', sport=[53], dport=[])
    assert str(r) == 'permit udp 10.1.2.3:[53] -> 10.0.0.0/8'


@pytest.mark.parametrize('impl', IMPLS)
def test_ip_semantics(impl):
    _, IP = impl
    assert str(IP('10.0.0.0/255.255.0.0')) == '10.0.0.0/16'
    assert str(IP('10.1')) == '10.1.0.0'
    assert IP('0.0.0.0/0').len() == 1 << 32
    assert IP('10.0.0.5') in IP('10.0.0.0/24')
    assert IP('10.0.1.5') not in IP('10.0.0.0/24')
    assert IP('10.0.0.0/25') in IP('10.0.0.0/24')
    assert IP('10.0.0.0/23') not in IP('10.0.0.0/24')
    assert IP('10.0.0.0-10.0.0.255') == IP('10.0.0.0/24')
    with pytest.raises(ValueError):
        IP('10.0.0.1/24')              # host bits set
    with pytest.raises(ValueError):
        IP('10.0.0.0/255.0.255.0')     # non-contiguous mask
    with pytest.raises(ValueError):
        IP('300.1.1.1')
    # IPv6 networks never contain an IPv4 host (version check)
    assert IP('1.2.3.4') not in IP('::/0')


@pytest.mark.parametrize('impl', IMPLS)
def test_constructor_normalisation(impl):
    FR, _ = impl
    r = FR(True, 'tcp', 'x', 'any', 'any', sport='80', dport=[])
    assert r.sport == [80] and r.dport == [-1]
    assert FR('False', 'tcp', 'x', 'any', 'any').action is True    # bool('False') quirk kept
    with pytest.raises(ValueError):
        FR(1, 'tcp', 'x', 'any', 'any')
    with pytest.raises(ValueError):
        FR(True, 'tcp', 'x', 'any', 'any', dport=['80'])
    with pytest.raises(ValueError):
        FR(True, 'tcp', 'x', '10.0.0.1/8', 'any')


@pytest.mark.parametrize('impl', IMPLS)
def test_port_list_semantics(impl):
    FR, _ = impl
    conn = FR(True, 'tcp', 'x', '1.1.1.1', '2.2.2.2', sport=1000, dport=443)
    assert conn in FR(True, 'tcp', 'x', 'any', 'any', dport=[80, 443])
    assert conn not in FR(True, 'tcp', 'x', 'any', 'any', dport=[80])
    assert conn not in FR(True, 'tcp', 'x', 'any', 'any', dport=[-1, -1])   # not the NO_PORT list
    assert conn in FR(True, 'tcp', 'x', 'any', 'any', sport=[-1])
    assert conn not in FR(False, 'tcp', 'x', 'any', 'any')                   # action must be equal
    assert conn in FR(True, 'ip', 'x', 'any', 'any')
    assert conn not in FR(True, 'udp', 'x', 'any', 'any')
