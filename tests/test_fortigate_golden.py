"""The FortiGate preprocessor restatements are pinned to the reference itself:
``tests/golden_fg/*`` were written by ``oracle/crosscheck_fortigate.py`` from
runs of the lib2to3-converted ``preprosess_fortigate_acl.py`` (Python-2 dict
order of the policies restored, DNS answers recorded).  Both the product's
``fortigate.build_db`` (every stored field, the stderr messages, the
exceptions) and the oracle's loop restatement (the rule columns) reproduce
them."""
import json
import os

import pytest

from conftest import ROOT
from oracle.crosscheck_fortigate import core_of_oracle, digest, dump_fg, recorded_resolver
from ruleset_analysis_amd import fortigate

GOLDEN_FG = os.path.join(ROOT, 'tests', 'golden_fg')
CASES = sorted(d for d in os.listdir(GOLDEN_FG) if os.path.isdir(os.path.join(GOLDEN_FG, d)))


def _case(name):
    d = os.path.join(GOLDEN_FG, name)
    with open(os.path.join(d, 'config.txt'), encoding='latin-1', newline='') as f:
        text = f.read()
    with open(os.path.join(d, 'dns.json')) as f:
        resolve = recorded_resolver(json.load(f))
    files = {}
    for k in ('db.sha256', 'core.sha256', 'stderr.txt', 'error.txt'):
        p = os.path.join(d, k)
        if os.path.exists(p):
            with open(p, encoding='latin-1', newline='') as f:
                files[k] = f.read()
    return text, resolve, files


def test_cases_present():
    assert {'fg_edges', 'fg_dictorder', 'fg_cfg4_small', 'fg_err_unknown_addr', 'fg_err_empty_acl'} <= set(CASES)


@pytest.mark.parametrize('name', CASES)
def test_product_equals_reference(name):
    text, resolve, files = _case(name)
    logs = []
    if 'error.txt' in files:
        with pytest.raises(Exception) as ei:
            fortigate.build_db(text, log=logs.append, resolve=resolve)
        assert '%s: %s' % (ei.type.__name__, ei.value) == files['error.txt'].strip()
        return
    db = fortigate.build_db(text, log=logs.append, resolve=resolve)
    assert digest(dump_fg(db)) == files['db.sha256'].strip()
    assert ''.join(logs) == files['stderr.txt']


@pytest.mark.parametrize('name', [c for c in CASES if not c.startswith('fg_err')])
def test_oracle_equals_reference(name):
    text, resolve, files = _case(name)
    assert digest(core_of_oracle(text, resolve)) == files['core.sha256'].strip()


def test_edges_cover_the_reference_branches():
    """What fg_edges exercises (checked on the product's DB, which equals the
    reference's): string ports from a space list, a dst:src product, 1-65535
    -> NO_PORT on either side, ICMP and IP services, a resolved fqdn, a failed
    lookup, an address without subnet, an unknown service protocol, a
    disabled policy, srcintf outside the two names (ACL ''), Guest-Inside."""
    text, resolve, files = _case('fg_edges')
    db = fortigate.build_db(text, resolve=resolve)
    acls = db.accesslists['FG-EDGE9']
    assert set(acls) == {'outside-in', 'inside-in', ''}
    rules = list(acls['outside-in']['rules'])
    ports = {(r.protocol, r.sport[0], r.dport[0]) for r in rules}
    assert ('tcp', -1, 8443) in ports and ('tcp', 1000, 2001) in ports and ('udp', 516, 514) in ports
    assert ('tcp', -1, -1) in ports and ('udp', -1, 161) in ports
    assert {'icmp', 'ip'} <= {r.protocol for r in rules}
    assert any(str(r.src) == '127.0.0.1' for r in rules)
    assert 'Unable to lookup nohost.invalid' in files['stderr.txt']
    assert 'Unable to expand address' in files['stderr.txt'] and 'Unknown protocol SCTP' in files['stderr.txt']
    assert not any('Disabled' in c for r in rules for c in r.comments)
    assert db.firewalls['FG-EDGE9'] == {'EDGE9-outside': {'in': 'outside-in'}, 'EDGE9-inside': {'in': 'inside-in'},
                                        'EDGE9-': {'in': ''}}
