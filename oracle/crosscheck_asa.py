"""ORACLE (test infrastructure only) — pin ``asa.py`` (the ASA preprocessor
restatement) against the reference's ``preprosess_access_lists.py`` itself.

Runs in the build container only (``/root/reference`` does not exist on the GPU
box).  For each case it converts ``preprosess_access_lists.py``,
``firewallrule.py`` and ``config.py`` with ``lib2to3`` into a scratch directory
under /tmp (never committed), installs ``IPy.py`` (``oracle/ipy.py``) and
``ciscoconfparse.py`` (``oracle/ciscoconfparse_shim.py``) next to them, writes
its OWN ``name-number-mappings.db`` (Python 3 shelve of ``asa.PORT_NAMES`` /
``asa.ICMP_TYPES``; the reference's pickled file is never opened), runs
``python3 preprosess_access_lists.py -v -f config.txt`` and dumps the shelve it
wrote.  The dump must equal ``asa.build_db`` on the same text; the case is then
written under ``tests/golden_asa/<case>/``: ``config.txt`` (input),
``db.sha256`` (digest of the canonical dump, ``dump_db``), ``summary.json``
(counts, protocols, firewalls, the first rules) and ``shadow.json`` (the
``-v`` shadowed-rule messages per ACL).

Usage: ``python3 oracle/crosscheck_asa.py``.
"""

import hashlib
import json
import os
import shelve
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = '/root/reference'
OUT = os.path.join(REPO, 'tests', 'golden_asa')
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


def dump_db(db):
    """Canonical JSON-able form of an AclDB (timestamps left out)."""
    acls = {}
    for h, hs in db.accesslists.items():
        acls[h] = {}
        for a, e in hs.items():
            rows = []
            for r in e['rules']:
                rows.append([bool(r.action), r.protocol, r.original, str(r.src), str(r.dst),
                             [int(x) for x in r.sport], [int(x) for x in r.dport], list(r.comments), int(r.rulenum),
                             int(r.ruleindex)])
            acls[h][a] = {'rules': rows, 'protocols': {p: [int(x) for x in v] for p, v in e['protocols'].items()}}
    return {'accesslists': acls, 'firewalls': db.firewalls}


def digest(obj):
    return hashlib.sha256(json.dumps(obj, sort_keys=True).encode()).hexdigest()


def run_reference(work, text):
    from ruleset_analysis_amd.asa import PORT_NAMES, ICMP_TYPES
    for name in ('preprosess_access_lists.py', 'firewallrule.py', 'config.py'):
        _convert(os.path.join(REF, name), os.path.join(work, name))
    with open(os.path.join(work, 'config.py')) as f:
        cfg = f.read()
    cfg = cfg.replace("ACCESSLIST_DATABASE = './input/{0}'.format(ACCESSLIST_DATABASE_FILENAME)",
                      "ACCESSLIST_DATABASE = ACCESSLIST_DATABASE_FILENAME")
    with open(os.path.join(work, 'config.py'), 'w') as f:
        f.write(cfg)
    import shutil
    shutil.copy(os.path.join(HERE, 'ipy.py'), os.path.join(work, 'IPy.py'))
    shutil.copy(os.path.join(HERE, 'ciscoconfparse_shim.py'), os.path.join(work, 'ciscoconfparse.py'))
    names = {p: dict(sorted(v.items(), key=lambda kv: (-len(kv[0]), kv[0]))) for p, v in PORT_NAMES.items()}
    db = shelve.open(os.path.join(work, 'name-number-mappings.db'))
    db['cisco_port_name_to_number'] = names
    db['cisco_port_number_to_name'] = {p: {n: w for w, n in v.items()} for p, v in names.items()}
    db['icmp_type_name_to_number'] = dict(ICMP_TYPES)
    db.close()
    with open(os.path.join(work, 'config.txt'), 'w', encoding='latin-1', newline='') as f:
        f.write(text)
    env = dict(os.environ, PYTHONHASHSEED='0', LC_ALL='C')
    r = subprocess.run([sys.executable, 'preprosess_access_lists.py', '-v', '-f', 'config.txt'], cwd=work, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    if r.returncode != 0:
        raise RuntimeError('reference preprocessor failed: %s' % r.stderr.decode('latin-1')[-2000:])
    with open(os.path.join(work, 'dump.py'), 'w') as f:
        f.write(DUMP)
    subprocess.run([sys.executable, 'dump.py'], cwd=work, env=env, check=True)
    with open(os.path.join(work, 'dump.json')) as f:
        ref = json.load(f)
    return ref, r.stderr.decode('latin-1')


def shadow_by_acl(stderr_text):
    """INFO triples of the -v run, grouped per ACL (the reference logs ACLs in
    its dict order; the converted run iterates in insertion order).  Python 2
    formats them 'INFO - msg' (the reference sets logging.BASIC_FORMAT before
    basicConfig); Python 3's basicConfig ignores that global and prints
    'INFO:root:msg' — both prefixes are accepted."""
    out = {}
    lines = []
    for l in stderr_text.split('\n'):
        for pre in ('INFO - ', 'INFO:root:'):
            if l.startswith(pre):
                lines.append(l[len(pre):])
    k = 0
    while k < len(lines):
        head = lines[k]
        acl = head.rsplit('access-list ', 1)[1].rstrip('.')
        out.setdefault(acl, []).extend(lines[k:k + 3])
        k += 3
    return out


def cases():
    import rsa_pkg
    rsa_pkg.load()
    from ruleset_analysis_amd import synth_asa
    yield 'asa_small', lambda: synth_asa.make_config(1, 120)[0]
    yield 'asa_groups', lambda: synth_asa.make_config(2, 300, n_net_groups=14, n_svc_groups=8)[0]
    yield 'asa_wide', lambda: synth_asa.make_config(3, 80, wide=True)[0]
    yield 'asa_edges', lambda: EDGES
    yield 'asa_ipv6', lambda: IPV6


EDGES = '''hostname edge-fw
object-group network WEB
 network-object host 10.0.0.10
 network-object 10.0.1.0 255.255.255.0
object-group network EMPTY
object-group network CLIENTS
 description nested members are not expanded by the reference
 group-object WEB
 network-object 192.168.0.0 255.255.0.0
object-group service WEBPORTS tcp
 port-object eq www
 port-object eq https
 port-object range 8000 8010
object-group service BOTH tcp-udp
 port-object eq domain
object-group service DNS udp
 port-object eq domain
 port-object eq ntp
access-list outside_in remark first block
access-list outside_in remark second line of the first block
access-list outside_in extended permit tcp any object-group WEB object-group WEBPORTS
access-list outside_in extended permit tcp any host 10.0.0.20 lt www
access-list outside_in extended permit udp object-group CLIENTS any object-group DNS
access-list dmz_in remark dmz rules
access-list outside_in extended permit tcp any eq ftp-data host 10.0.0.30 range ftp-data ftp
access-list outside_in extended permit tcp object-group EMPTY any eq ssh
access-list outside_in remark after an empty rule
access-list outside_in extended permit tcp any any gt 65530
access-list outside_in extended permit udp any any lt 10
access-list outside_in extended permit icmp any any echo-reply
access-list outside_in extended permit icmp any any
access-list dmz_in extended permit tcp 172.16.0.0 255.240.0.0 object-group WEB eq 8443
access-list dmz_in extended permit tcp any object-group WEB object-group BOTH
access-list outside_in extended deny ip any any
access-list dmz_in extended deny ip any any
access-group outside_in in interface outside
access-group dmz_in in interface dmz
access-group dmz_in out interface inside
'''


# IPv6 hosts and networks (firewallrule.py:80-93 stores any address IPy takes)
# between IPv4 rules: they keep their ruleindex, never match an IPv4
# connection, and shadow each other only within one address family
IPV6 = '''hostname v6-fw
object-group network V6HOSTS
 network-object host 2001:db8::10
 network-object 2001:db8:1::/48
 network-object host 10.0.0.10
object-group network V6WIDE
 network-object 2001:db8::/32
object-group service WEB tcp
 port-object eq www
 port-object eq https
access-list outside_in remark v4 and v6 rules interleaved
access-list outside_in extended permit tcp any host 10.0.0.10 eq www
access-list outside_in extended permit tcp host 2001:db8::1 host 10.0.0.20 eq https
access-list outside_in extended permit tcp object-group V6WIDE any object-group WEB
access-list outside_in extended permit tcp object-group V6HOSTS any eq www
access-list outside_in extended permit tcp host 2001:db8:1::5 any eq www
access-list outside_in extended permit tcp any host 10.0.0.20 range 440 450
access-list outside_in extended permit udp any host 2001:db8::53 eq domain
access-list outside_in extended permit udp any host 2001:db8::53 eq domain
access-list outside_in extended permit tcp 10.1.0.0 255.255.0.0 host 2001:db8::99 eq 22
access-list outside_in extended permit tcp host 2001:db8::1 host 2001:db8::2 eq 22
access-list outside_in extended permit tcp object-group V6WIDE object-group V6WIDE eq 22
access-list outside_in extended permit udp any any eq domain
access-list outside_in extended deny ip any any
access-list inside_in extended permit ip host fe80::1 any
access-list inside_in extended permit tcp 10.0.0.0 255.0.0.0 any eq www
access-list inside_in extended deny ip any any
access-group outside_in in interface outside
access-group inside_in in interface inside
'''


def main():
    import rsa_pkg
    rsa_pkg.load()
    from ruleset_analysis_amd import asa
    if not os.path.isdir(REF):
        sys.exit('reference not present; this script only runs in the build container')
    for name, make in cases():
        text = make()
        with tempfile.TemporaryDirectory(prefix='rsa_asa_') as work:
            ref, err = run_reference(work, text)
        mine = json.loads(json.dumps(dump_db(asa.build_db(text)), sort_keys=True))
        ok = mine == ref
        n = sum(len(e['rules']) for hs in ref['accesslists'].values() for e in hs.values())
        print('%-12s %d expanded rules: %s' % (name, n, 'OK' if ok else 'DIFF'))
        if not ok:
            for h in ref['accesslists']:
                for a in ref['accesslists'][h]:
                    rr, mm = ref['accesslists'][h][a], mine['accesslists'].get(h, {}).get(a)
                    if rr != mm:
                        for i, (x, y) in enumerate(zip(rr['rules'], (mm or {'rules': []})['rules'])):
                            if x != y:
                                print(' first diff', a, i, x, y)
                                break
            sys.exit('asa.py disagrees with the converted reference on case %s' % name)
        out = os.path.join(OUT, name)
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, 'config.txt'), 'w', encoding='latin-1', newline='') as f:
            f.write(text)
        with open(os.path.join(out, 'db.sha256'), 'w') as f:
            f.write(digest(ref) + '\n')
        summary = {'firewalls': ref['firewalls'],
                   'acls': {a: {'n_rules': len(e['rules']), 'protocols': {p: len(v) for p, v in e['protocols'].items()},
                                'first_rules': e['rules'][:20]}
                            for h in ref['accesslists'] for a, e in ref['accesslists'][h].items()},
                   'source': 'lib2to3-converted preprosess_access_lists.py, oracle/crosscheck_asa.py'}
        with open(os.path.join(out, 'summary.json'), 'w') as f:
            json.dump(summary, f, sort_keys=True, indent=1)
        with open(os.path.join(out, 'shadow.json'), 'w') as f:
            json.dump(shadow_by_acl(err), f, sort_keys=True, indent=1)


if __name__ == '__main__':
    main()
