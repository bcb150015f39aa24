"""ORACLE (test infrastructure only) — pin ``fortigate.py`` (the FortiGate
preprocessor restatement) and ``oracle/fortigate.py`` against the reference's
``preprosess_fortigate_acl.py`` itself.

Runs in the build container only (``/root/reference`` does not exist on the GPU
box).  For each case it converts ``preprosess_fortigate_acl.py``,
``firewallrule.py`` and ``config.py`` with ``lib2to3`` into a scratch directory
under /tmp (never committed), installs ``IPy.py`` (``oracle/ipy.py``), writes
its own ``name-number-mappings.db`` (a Python 3 shelve holding only the
``icmp_type_name_to_number`` key the script reads, :229-231 — the reference's
pickled file is never opened), and runs ``python3 preprosess_fortigate_acl.py
-f config.txt``.  Two Python-2 behaviours are restored in the converted script:

* ``obj['policy'].keys()`` (:362, SURVEY.md trap 10) iterates in CPython 2.7
  dict order: the call is wrapped in ``oracle.py2dict``'s replay of 2.7's slot
  order (``py2order.py``), fed by the Python 3 dict's insertion order;
* nothing else reaches the output in dict order (per-ACL rule lists are
  independent; firewalls/protocols are compared as mappings).

DNS: ``socket.gethostbyname_ex`` runs for real (this container has no network:
``*.invalid`` names fail into :45-46, ``localhost`` resolves from
/etc/hosts); the answers are recorded in ``dns.json`` so the CPU test replays
the same lookups.

The shelve the reference wrote is dumped (``DUMP``) and must equal
``fortigate.build_db`` on the same text (all fields, rulenum as stored — the
policy-id string), and its core columns must equal ``oracle.fortigate.expand``;
the reference's stderr must equal the product's ``log`` messages.  Cases whose
reference run raises are kept with the exception's last traceback line.
Written under ``tests/golden_fg/<case>/``: ``config.txt``, ``dns.json``,
``db.sha256`` (``dump_fg`` digest), ``core.sha256`` (``core_of`` digest),
``stderr.txt``, ``summary.json`` — or ``error.txt``.

Usage: ``python3 oracle/crosscheck_fortigate.py``.
"""

import hashlib
import json
import os
import re
import shelve
import shutil
import socket
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = '/root/reference'
OUT = os.path.join(REPO, 'tests', 'golden_fg')
sys.path.insert(0, REPO)

from oracle.crosscheck_2to3 import _convert  # noqa: E402

DUMP = r'''
import json, shelve, sys
sys.path.insert(0, '.')
db = shelve.open('accesslists.db')
acls = {h: {a: {'rules': [[r.action, r.protocol, r.original, str(r.src), str(r.dst), list(r.sport), list(r.dport),
                           list(r.comments), r.rulenum, r.ruleindex] for r in e['rules']],
                'protocols': {p: list(v) for p, v in e['protocols'].items()}}
            for a, e in hs.items()} for h, hs in db['accesslists'].items()}
json.dump({'accesslists': acls, 'firewalls': db['firewalls']}, open('dump.json', 'w'), sort_keys=True)
'''


def dump_fg(db):
    """Canonical JSON-able form of an AclDB built from a FortiGate config
    (timestamps left out; rulenum kept as stored)."""
    acls = {}
    for h, hs in db.accesslists.items():
        acls[h] = {}
        for a, e in hs.items():
            rows = []
            for r in e['rules']:
                rows.append([bool(r.action), r.protocol, r.original, str(r.src), str(r.dst),
                             [int(x) for x in r.sport], [int(x) for x in r.dport], list(r.comments), r.rulenum,
                             int(r.ruleindex)])
            acls[h][a] = {'rules': rows, 'protocols': {p: [int(x) for x in v] for p, v in e['protocols'].items()}}
    return json.loads(json.dumps({'accesslists': acls, 'firewalls': db.firewalls}, sort_keys=True))


def core_of(dump):
    """The fields ``oracle.fortigate`` computes: per ACL (action, protocol,
    src net/size, dst net/size, sport, dport) rows, protocols, firewalls."""
    from oracle.ipy import IP
    cache = {}

    def net(s):
        if s not in cache:
            a = IP(s)
            cache[s] = [a.ip, a.len()]
        return cache[s]

    acls = {}
    for h, hs in dump['accesslists'].items():
        for a, e in hs.items():
            acls[a] = {'rows': [[int(bool(r[0])), r[1]] + net(r[3]) + net(r[4]) + [r[5][0], r[6][0]]
                                for r in e['rules']],
                       'protocols': e['protocols']}
    return {'acls': acls, 'firewalls': dump['firewalls']}


def core_of_oracle(text, resolve):
    from oracle import fortigate as ofg
    host, fws, acls = ofg.expand(text, resolve=resolve)
    out = {}
    for a, A in acls.items():
        c = ofg.as_columns(A)
        rows = [[int(c['action'][i]), c['proto'][i], int(c['src'][i]), int(c['src_len'][i]), int(c['dst'][i]),
                 int(c['dst_len'][i]), int(c['sport'][i]), int(c['dport'][i])] for i in range(len(A))]
        out[a] = {'rows': rows, 'protocols': {p: list(v) for p, v in A.protocols.items()}}
    return json.loads(json.dumps({'acls': out, 'firewalls': fws}, sort_keys=True))


def digest(obj):
    return hashlib.sha256(json.dumps(obj, sort_keys=True).encode()).hexdigest()


def recorded_resolver(table):
    """``socket.gethostbyname_ex`` replayed from a {name: [ips] | null} table."""
    def resolve(name):
        ips = table.get(name)
        if ips is None:
            raise socket.gaierror(-3, 'Temporary failure in name resolution')
        return (name, [], list(ips))
    return resolve


def fqdns(text):
    return sorted(set(m.group(1) for m in re.finditer(r'set fqdn "?([^"\s]+)"?', text)))


def run_reference(work, text):
    for name in ('preprosess_fortigate_acl.py', 'firewallrule.py', 'config.py'):
        _convert(os.path.join(REF, name), os.path.join(work, name))
    with open(os.path.join(work, 'config.py')) as f:
        cfg = f.read()
    cfg = cfg.replace("ACCESSLIST_DATABASE = './input/{0}'.format(ACCESSLIST_DATABASE_FILENAME)",
                      "ACCESSLIST_DATABASE = ACCESSLIST_DATABASE_FILENAME")
    with open(os.path.join(work, 'config.py'), 'w') as f:
        f.write(cfg)
    pre = os.path.join(work, 'preprosess_fortigate_acl.py')
    with open(pre) as f:
        code = f.read()
    site = re.compile(r"for policy_id in (?:list\()?obj\['policy'\]\.keys\(\)\)?:")
    if len(site.findall(code)) != 1:
        raise RuntimeError("expected one obj['policy'].keys() loop in the converted preprocessor")
    code = site.sub("for policy_id in _py2_keys(list(obj['policy'].keys())):", code)
    code = 'from py2order import py2_keys as _py2_keys\n' + code
    with open(pre, 'w') as f:
        f.write(code)
    shutil.copy(os.path.join(HERE, 'py2dict.py'), os.path.join(work, 'py2order.py'))
    shutil.copy(os.path.join(HERE, 'ipy.py'), os.path.join(work, 'IPy.py'))
    import rsa_pkg
    rsa_pkg.load()
    from ruleset_analysis_amd.asa import ICMP_TYPES
    db = shelve.open(os.path.join(work, 'name-number-mappings.db'))
    db['icmp_type_name_to_number'] = dict(ICMP_TYPES)
    db.close()
    with open(os.path.join(work, 'config.txt'), 'w', encoding='latin-1', newline='') as f:
        f.write(text)
    env = dict(os.environ, PYTHONHASHSEED='0', LC_ALL='C', PYTHONIOENCODING='latin-1')
    r = subprocess.run([sys.executable, 'preprosess_fortigate_acl.py', '-f', 'config.txt'], cwd=work, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    err = r.stderr.decode('latin-1')
    if r.returncode != 0:
        return None, err
    with open(os.path.join(work, 'dump.py'), 'w') as f:
        f.write(DUMP)
    subprocess.run([sys.executable, 'dump.py'], cwd=work, env=env, check=True)
    with open(os.path.join(work, 'dump.json')) as f:
        ref = json.load(f)
    return ref, err


def cases():
    import rsa_pkg
    rsa_pkg.load()
    from ruleset_analysis_amd import synth_fg
    yield 'fg_edges', lambda: EDGES
    yield 'fg_dictorder', lambda: synth_fg.make_config(43, n_policies=70, n_wide=0, n_mid=0, n_syslog=3,
                                                       members=(1, 2), hostname='FG-ORDER')[0]

    def cfg4_small():
        text = synth_fg.make_config(41, n_policies=24, n_wide=1, n_mid=1, n_syslog=2, members=(2, 4),
                                    wide_members=(2, 2), hostname='FG-CFG4')[0]
        return text.replace('1024-65535', '65300-65535').replace('5000-5999', '5000-5099')
    yield 'fg_cfg4_small', cfg4_small
    yield 'fg_err_unknown_addr', lambda: EDGES.replace('set dstaddr "servers"', 'set dstaddr "nosuch"')
    # ACL "" (policies 25 and 33) ends up without rules: proto2rule[''] is never set (:427)
    yield 'fg_err_empty_acl', lambda: EDGES.replace('set srcaddr "all"\n        set dstaddr "web1"',
                                                    'set srcaddr "gone"\n        set dstaddr "web1"')


EDGES = '''config router setting
    set hostname "FG-EDGE9"
end
config firewall address
    edit "all"
        set subnet 0.0.0.0 0.0.0.0
    next
    edit "web1"
        set subnet 10.1.0.10 255.255.255.255
    next
    edit "web2"
        set subnet 10.1.0.11 255.255.255.255
    next
    edit "dbnet"
        set subnet 10.2.0.0 255.255.255.0
    next
    edit "partners"
        set comment "two words"
        set subnet 198.51.100.0 255.255.255.128
    next
    edit "lh"
        set type fqdn
        set fqdn "localhost"
    next
    edit "gone"
        set type fqdn
        set fqdn "nohost.invalid"
    next
    edit "range1"
        set type iprange
        set start-ip 10.3.0.1
        set end-ip 10.3.0.9
    next
end
config firewall addrgrp
    edit "webs"
        set member "web1" "web2"
    next
    edit "servers"
        set member "webs" "dbnet" "web1"
    next
    edit "odd"
        set member "lh" "gone" "range1" "partners"
    next
end
config firewall service custom
    edit "HTTP"
        set category "Web Access"
        set protocol TCP/UDP/SCTP
        set tcp-portrange 80
    next
    edit "WEB-LIST"
        set protocol TCP/UDP/SCTP
        set tcp-portrange 8080 8443 8000
    next
    edit "DNS"
        set protocol TCP/UDP/SCTP
        set tcp-portrange 53
        set udp-portrange 53
    next
    edit "SYSLOG"
        set protocol TCP/UDP/SCTP
        set udp-portrange 514:512-516
    next
    edit "LIST-SRC"
        set protocol TCP/UDP/SCTP
        set tcp-portrange 2000-2002:1000 1001
    next
    edit "ANY-TCP"
        set protocol TCP/UDP/SCTP
        set tcp-portrange 1-65535
    next
    edit "SNMP-ANYSRC"
        set protocol TCP/UDP/SCTP
        set udp-portrange 161-162:1-65535
    next
    edit "PING"
        set protocol ICMP
        set icmptype 8
    next
    edit "ALL"
        set protocol IP
    next
    edit "SCTP-X"
        set protocol SCTP
        set sctp-portrange 99
    next
end
config firewall service group
    edit "Web-Svcs"
        set member "HTTP" "WEB-LIST"
    next
    edit "Nested"
        set member "Web-Svcs" "DNS" "PING" "SCTP-X"
    next
end
config firewall policy
    edit 12
        set srcintf "Outside"
        set dstintf "Inside"
        set srcaddr "partners" "odd"
        set dstaddr "servers"
        set action accept
        set status enable
        set service "Nested" "SYSLOG"
        set comments "partner access"
        set global-label "Partners"
    next
    edit 3
        set srcintf "Outside"
        set dstintf "Inside"
        set srcaddr "all"
        set dstaddr "all"
        set action accept
        set status disable
        set service "ALL"
        set comments ''
        set global-label "Disabled"
    next
    edit 40
        set srcintf "Outside"
        set dstintf "Inside"
        set srcaddr "all"
        set dstaddr "webs" "dbnet"
        set action accept
        set status enable
        set service "ANY-TCP" "SNMP-ANYSRC" "LIST-SRC"
        set comments ''
        set global-label "Wide"
    next
    edit 7
        set srcintf "Guest-Inside"
        set dstintf "Outside"
        set srcaddr "dbnet"
        set dstaddr "all"
        set action accept
        set status enable
        set service "Web-Svcs" "PING"
        set comments "guests"
        set global-label "Guest"
    next
    edit 25
        set srcintf "DMZ"
        set dstintf "Inside"
        set srcaddr "all"
        set dstaddr "web1"
        set action accept
        set status enable
        set service "HTTP"
        set comments ''
        set global-label "Dmz"
    next
    edit 4
        set srcintf "Outside"
        set dstintf "Inside"
        set srcaddr "partners"
        set dstaddr "dbnet"
        set action deny
        set status enable
        set service "DNS"
        set comments ''
        set global-label "Deny"
    next
    edit 33
        set srcintf "Wan3"
        set dstintf "Inside"
        set srcaddr "gone"
        set dstaddr "all"
        set action accept
        set status enable
        set service "ALL"
    next
    edit 9
        set srcintf "Inside"
        set dstintf "Outside"
        set srcaddr "all"
        set dstaddr "all"
        set action deny
        set status enable
        set service "ALL"
        set comments ''
        set global-label "Final"
    next
    edit 1000
        set srcintf "Outside"
        set dstintf "Inside"
        set srcaddr "all"
        set dstaddr "all"
        set action deny
        set status enable
        set service "ALL"
        set comments ''
        set global-label "Final"
    next
end
'''


def main():
    import rsa_pkg
    rsa_pkg.load()
    from ruleset_analysis_amd import fortigate
    if not os.path.isdir(REF):
        sys.exit('reference not present; this script only runs in the build container')
    for name, make in cases():
        text = make()
        table = {}
        for n in fqdns(text):
            try:
                table[n] = socket.gethostbyname_ex(n)[2]
            except Exception:  # noqa: BLE001 - recorded as a failed lookup
                table[n] = None
        with tempfile.TemporaryDirectory(prefix='rsa_fg_') as work:
            ref, err = run_reference(work, text)
        resolve = recorded_resolver(table)
        logs = []
        out = os.path.join(OUT, name)
        os.makedirs(out, exist_ok=True)
        for f in os.listdir(out):
            os.remove(os.path.join(out, f))
        with open(os.path.join(out, 'config.txt'), 'w', encoding='latin-1', newline='') as f:
            f.write(text)
        with open(os.path.join(out, 'dns.json'), 'w') as f:
            json.dump(table, f, sort_keys=True, indent=1)
        if ref is None:
            last = [l for l in err.strip().split('\n') if l][-1]
            try:
                fortigate.build_db(text, log=logs.append, resolve=resolve)
                mine = 'no error'
            except Exception as e:  # noqa: BLE001 - compared with the reference's exception
                mine = '%s: %s' % (type(e).__name__, e)
            ok = last == mine
            print('%-22s reference raised %r; product %r: %s' % (name, last, mine, 'OK' if ok else 'DIFF'))
            if not ok:
                sys.exit('fortigate.py disagrees with the converted reference on case %s' % name)
            with open(os.path.join(out, 'error.txt'), 'w') as f:
                f.write(last + '\n')
            continue
        mine = dump_fg(fortigate.build_db(text, log=logs.append, resolve=resolve))
        ok_db = mine == ref
        ok_log = ''.join(logs) == err
        core = core_of(ref)
        ok_core = core_of_oracle(text, resolve) == core
        n = sum(len(e['rules']) for hs in ref['accesslists'].values() for e in hs.values())
        print('%-22s %6d expanded rules: product %s, stderr %s, oracle %s' % (
            name, n, 'OK' if ok_db else 'DIFF', 'OK' if ok_log else 'DIFF', 'OK' if ok_core else 'DIFF'))
        if not (ok_db and ok_log and ok_core):
            if not ok_log:
                print(' reference stderr: %r\n product log:      %r' % (err, ''.join(logs)))
            for h in ref['accesslists']:
                for a in ref['accesslists'][h]:
                    rr, mm = ref['accesslists'][h][a], mine['accesslists'].get(h, {}).get(a)
                    if rr != mm:
                        for i, (x, y) in enumerate(zip(rr['rules'], (mm or {'rules': []})['rules'])):
                            if x != y:
                                print(' first diff', a, i, x, y)
                                break
                        else:
                            print(' diff in', a, len(rr['rules']), len((mm or {'rules': []})['rules']),
                                  rr['protocols'] == (mm or {}).get('protocols'))
            sys.exit('disagreement with the converted reference on case %s' % name)
        with open(os.path.join(out, 'db.sha256'), 'w') as f:
            f.write(digest(ref) + '\n')
        with open(os.path.join(out, 'core.sha256'), 'w') as f:
            f.write(digest(core) + '\n')
        with open(os.path.join(out, 'stderr.txt'), 'w', encoding='latin-1', newline='') as f:
            f.write(err)
        summary = {'firewalls': ref['firewalls'],
                   'acls': {a: {'n_rules': len(e['rules']), 'protocols': {p: len(v) for p, v in e['protocols'].items()},
                                'first_rules': e['rules'][:12]}
                            for h in ref['accesslists'] for a, e in ref['accesslists'][h].items()},
                   'source': 'lib2to3-converted preprosess_fortigate_acl.py, oracle/crosscheck_fortigate.py'}
        with open(os.path.join(out, 'summary.json'), 'w') as f:
            json.dump(summary, f, sort_keys=True, indent=1)


if __name__ == '__main__':
    main()
