"""FortiGate config -> ``accesslists.db`` (restates ``preprosess_fortigate_acl.py``).

What the reference does (and this module reproduces, rule for rule):

* line parser (``:296-358``): sections ``config firewall policy|address|addrgrp|
  service custom|service group`` and ``config router setting`` (hostname);
  ``edit NAME`` opens an object (NAME keeps its quotes), ``set TITLE VALUE...``
  stores ``' '.join(words[2:])`` for the section's known titles, ``next`` closes
  it; an address ``subnet`` has its space turned into ``/``;
* ``expand_addr`` (``:30-57``): every quoted name is an address (its subnet;
  an fqdn is resolved with ``socket.gethostbyname_ex`` as the reference does —
  a failed lookup is skipped with the reference's message) or an address group
  (members, recursively);
* ``expand_service`` (``:60-140``): ``TCP/UDP/SCTP`` services expand
  ``tcp-portrange`` then ``udp-portrange``; ``a-b`` expands to every port
  (``1-65535`` to NO_PORT), ``a b c`` to each port, ``dst:src`` gives the src x
  dst product; ``ICMP``/``IP`` services give one port-less rule; groups recurse;
* policies in Python 2 dict order of their ids (``:362``, SURVEY.md trap 10) —
  replayed by ``py2dict`` — with status ``enable``; srcintf ``"Outside"`` ->
  ACL ``outside-in``, ``"Inside"``/``"Guest-Inside"`` -> ``inside-in``, anything
  else -> ACL ``""``; rules nest src -> dst -> service (``:184-186``), the
  original line / comment as ``:189-198``; ``ruleindex`` = list position
  (``:375-384``), ``protocols`` per rule protocol; interface
  ``hostname.split('-')[1] + '-' + acl.split('-')[0]`` bound ``in`` (``:387-392``).

The expanded rules are built as numpy columns (``rulecols.RuleColumns``): a
policy with a wide port range is millions of rules in the reference's DB and a
handful of stepped run entries after ``compile.compress_runs``.
"""

import re
import socket

import numpy as np

from .acldb import AclDB
from .firewallrule import FirewallRule
from .ipaddr import IP
from .py2dict import iteration_order
from .py2text import py2_int, py2_lower, py2_split, py2_strip
from .rulecols import FAM_DST6, FAM_SRC6, Nets6, RuleColumns

__all__ = ['parse_config', 'build_db', 'expand_addr', 'expand_service']

TITLES = {
    'policy': ['srcintf', 'dstintf', 'srcaddr', 'dstaddr', 'action', 'status', 'service', 'comments', 'global-label'],
    'addr': ['type', 'comment', 'subnet', 'start-ip', 'end-ip', 'fqdn'],
    'addrgrp': ['comment', 'member'],
    'service': ['category', 'protocol', 'comment', 'protocol-number', 'tcp-portrange', 'udp-portrange', 'icmptype',
                'icmpcode'],
    'srvcgrp': ['comment', 'member'],
    'router': ['hostname'],
}
SECTIONS = {'config firewall policy': 'policy', 'config firewall address': 'addr',
            'config firewall addrgrp': 'addrgrp', 'config firewall service custom': 'service',
            'config firewall service group': 'srvcgrp', 'config router setting': 'router'}
_QUOTED = re.compile(r'(\".*?\")')
_EDIT = re.compile(r'edit (.*)')


def parse_config(text):
    """The reference's section/object parser (preprosess_fortigate_acl.py:296-358)."""
    obj = {}
    section = False
    elem = False
    for line in text.split('\n'):             # readlines(): lines end at '\n' only
        line = py2_strip(line)
        if line in SECTIONS:
            section = SECTIONS[line]
            obj[section] = {}
        if section and line == 'end':
            section = False
        if not section:
            continue
        if line[:4] == 'edit':
            m = _EDIT.search(line)
            if m:
                elem = str(m.groups()[0])
                obj[section][elem] = {}
        if section == 'router' and line[:12] == 'set hostname':
            obj[section]['hostname'] = py2_split(line)[2].replace("'", '').replace('"', '')
        elif line == 'next':
            elem = False
        elif line[:3] == 'set' and elem:
            words = py2_split(line)
            title = None
            for title in TITLES[section]:
                if words[1] == title:
                    obj[section][elem][title] = ' '.join(words[2:])
                    break
            if section == 'addr' and words[1] == 'subnet':
                obj[section][elem][title] = obj[section][elem][title].replace(' ', '/')
    return obj


def expand_addr(entry, obj, log=None, resolve=socket.gethostbyname_ex):
    """Subnet strings of every quoted address / address group name in ``entry``
    (``resolve``: the DNS lookup of fqdn objects, ``socket.gethostbyname_ex``'s
    contract; any exception is a failed lookup, :43-46)."""
    res = []
    for m in _QUOTED.finditer(entry):
        name = m.groups()[0]
        if name in obj['addr']:
            a = obj['addr'][name]
            if 'subnet' in a:
                res.append(a['subnet'])
            elif 'fqdn' in a:
                fqdn = a['fqdn'].replace('"', '')
                found = None
                try:
                    found = resolve(fqdn)
                except Exception:  # noqa: BLE001 - the reference's bare except (:45)
                    if log is not None:
                        log('Unable to lookup {0}. Skipping it. \n'.format(fqdn))
                if found:
                    res.extend(found[2])
            elif log is not None:
                log('Unable to expand address "{}" to a subnet. Skipping it.\n'.format(name))
        else:
            for member in _QUOTED.finditer(obj['addrgrp'][name]['member']):
                res.extend(expand_addr(member.groups()[0], obj, log, resolve))
    return res


def _port_values(spec):
    """One side of a port spec -> int64 array of ports (-1 = NO_PORT), in the
    reference's order (range ascending, list in text order)."""
    if spec.find('-') != -1:
        start, end = spec.split('-')
        if py2_int(start) == 1 and py2_int(end) == 65535:
            return np.array([FirewallRule.NO_PORT], np.int64)
        return np.arange(py2_int(start), py2_int(end) + 1, dtype=np.int64)
    if spec.find(' ') != -1:
        return np.array([py2_int(p) for p in spec.split(' ')], np.int64)
    return np.array([py2_int(spec)], np.int64)


def expand_service(entry, obj, log=None):
    """Service segments ``(protocol, sports, dports)`` in the reference's order;
    a segment stands for ``len(sports)`` rules (port arrays of equal length)."""
    res = []
    if entry in obj['service']:
        o = obj['service'][entry]
        if o['protocol'] == 'TCP/UDP/SCTP':
            for key in ('tcp-portrange', 'udp-portrange'):
                if key not in o:
                    continue
                protocol = key[:3]
                if o[key].find(':') != -1:
                    dspec, sspec = o[key].split(':')
                else:
                    dspec, sspec = o[key], False
                dst = _port_values(dspec) if dspec else np.zeros(0, np.int64)
                if sspec:
                    src = _port_values(sspec)
                    # for src in srcobj: for dst in dstobj (:115-118)
                    res.append((protocol, np.repeat(src, len(dst)), np.tile(dst, len(src))))
                else:
                    res.append((protocol, np.full(len(dst), FirewallRule.NO_PORT, np.int64), dst))
        elif o['protocol'] in ('ICMP', 'IP'):
            res.append((py2_lower(o['protocol']), np.array([FirewallRule.NO_PORT], np.int64),
                        np.array([FirewallRule.NO_PORT], np.int64)))
        elif log is not None:
            log('Unknown protocol {} in service object {}, skipping it.\n'.format(o['protocol'], entry))
    elif entry in obj['srvcgrp']:
        for member in obj['srvcgrp'][entry]['member'].split(' '):
            res.extend(expand_service(member, obj, log))
    return res


class _AclBuilder(object):
    def __init__(self):
        self.parts = []           # per policy: dict of column arrays
        self.n = 0
        self.originals, self.comments, self.rulenums = [], [], []
        self.proto_names = []
        self.nets6 = Nets6()

    def proto_id(self, name):
        if name not in self.proto_names:
            self.proto_names.append(name)
        return self.proto_names.index(name)

    def add_policy(self, p, srcs, dsts, svcs):
        """Rules of one policy, nested src -> dst -> svc (preprosess_fortigate_acl.py:184-215).
        The original line and comment are built inside the innermost loop
        there, so a policy without rules never reads its fields."""
        if not srcs or not dsts or not svcs:
            return
        original = 'access-list {}-in {} {} to {} service {}'.format(py2_lower(p['srcintf']), p['action'], p['srcaddr'],
                                                                    p['dstaddr'], p['service'])
        original = original.replace('"', '').replace('accept', 'permit')
        if p['comments'] != "''":
            comment = 'access-list {}-in remark {}: {}'.format(py2_lower(p['srcintf']), p['global-label'], p['comments'])
        else:
            comment = 'access-list {}-in remark {}'.format(py2_lower(p['srcintf']), p['global-label'])
        comment = comment.replace('"', '')
        permit = p['action'] == 'accept'
        # per service segment: protocol id and ports; a segment of k rules
        sv_proto = np.concatenate([np.full(len(sp), self.proto_id(pr), np.int64) for pr, sp, _dp in svcs])
        sv_sport = np.concatenate([sp for _pr, sp, _dp in svcs])
        sv_dport = np.concatenate([dp for _pr, _sp, dp in svcs])
        v = len(sv_proto)
        if v == 0:
            return
        # an IPv6 subnet keeps its rules' positions; its value is a nets6 id
        # (rulecols: it never matches an IPv4 connection)
        sa = [(t, IP(t)) for t in srcs]
        da = [(t, IP(t)) for t in dsts]
        S, D = len(sa), len(da)
        s_ip = np.array([a.ip if a._ipversion == 4 else self.nets6(t) for t, a in sa], np.uint32)
        s_len = np.array([a._prefixlen for _t, a in sa], np.uint8)
        s_v6 = np.array([a._ipversion != 4 for _t, a in sa], np.uint8)
        d_ip = np.array([a.ip if a._ipversion == 4 else self.nets6(t) for t, a in da], np.uint32)
        d_len = np.array([a._prefixlen for _t, a in da], np.uint8)
        d_v6 = np.array([a._ipversion != 4 for _t, a in da], np.uint8)
        si = np.repeat(np.arange(S), D * v)
        di = np.tile(np.repeat(np.arange(D), v), S)
        vi = np.tile(np.arange(v), S * D)
        self.originals.append(original)
        self.comments.append([comment])
        self.rulenums.append(p['policy_id'])
        m = S * D * v
        self.parts.append({
            'action': np.full(m, permit, bool), 'proto': sv_proto[vi].astype(np.uint8),
            'src': s_ip[si], 'src_len': s_len[si], 'dst': d_ip[di], 'dst_len': d_len[di],
            'sport': sv_sport[vi].astype(np.int32), 'dport': sv_dport[vi].astype(np.int32),
            'orig': np.full(m, len(self.originals) - 1, np.int32),
            'comment': np.full(m, len(self.comments) - 1, np.int32),
            'rulenum': np.full(m, len(self.rulenums) - 1, np.int32),
            'fam': s_v6[si] * FAM_SRC6 | d_v6[di] * FAM_DST6})
        self.n += m

    def build(self):
        cols = {}
        for k in ('action', 'proto', 'src', 'src_len', 'dst', 'dst_len', 'sport', 'dport', 'orig', 'comment',
                  'rulenum', 'fam'):
            cols[k] = np.concatenate([p[k] for p in self.parts]) if self.parts else np.zeros(0)
        return RuleColumns(cols['action'], cols['proto'], self.proto_names, cols['src'], cols['src_len'], cols['dst'],
                           cols['dst_len'], cols['sport'], cols['dport'], cols['orig'], self.originals or [''],
                           cols['comment'], self.comments or [[]], cols['rulenum'], self.rulenums or [-1],
                           fam=cols['fam'], nets6=self.nets6.texts)


def build_db(text, timestamp=0.0, firewalls=None, accesslists=None, log=None, resolve=socket.gethostbyname_ex):
    """The reference's ``main`` (preprosess_fortigate_acl.py:220-434) on config
    text: returns the ``AclDB`` it would store (merged into ``firewalls`` /
    ``accesslists`` of an existing DB when given).  ``log`` receives the
    reference's stderr messages; ``resolve`` does the fqdn lookups."""
    obj = parse_config(text)
    firewalls = {} if firewalls is None else firewalls
    acldb = {} if accesslists is None else accesslists
    builders = {}
    order = list(obj['policy'].keys())
    for k in iteration_order(order):
        policy_id = order[k]
        p = obj['policy'][policy_id]
        if p['status'] != 'enable':
            continue
        acl = ''
        if p['srcintf'] == '"Outside"':
            acl = 'outside-in'
        elif p['srcintf'] == '"Inside"' or p['srcintf'] == '"Guest-Inside"':
            acl = 'inside-in'
        b = builders.setdefault(acl, _AclBuilder())
        p = dict(p, policy_id=policy_id)
        data = {'srcaddr': [], 'dstaddr': []}
        for key in p:
            if key.find('addr') != -1:
                for m in _QUOTED.finditer(p[key]):
                    data[key] = data[key] + expand_addr(m.groups()[0], obj, log, resolve)
        svcs = []
        if 'service' in p:
            for part in p['service'].split(' '):
                svcs.extend(expand_service(part, obj, log))
        elif data['srcaddr'] and data['dstaddr']:
            raise KeyError('service')    # data['service'] is read inside the src/dst loops (:184-186)
        b.add_policy(p, data['srcaddr'], data['dstaddr'], svcs)
    hostname = obj['router']['hostname']
    firewalls.setdefault(hostname, {})
    for acl in builders:
        intf = '-'.join([hostname.split('-')[1], acl.split('-')[0]])
        firewalls[hostname][intf] = {'in': acl}
    acldb.setdefault(hostname, {})
    for acl, b in builders.items():
        if b.n == 0:
            raise KeyError(acl)          # proto2rule[acl] was never created (:427)
        rules = b.build()
        acldb[hostname].setdefault(acl, {})
        acldb[hostname][acl]['rules'] = rules
        acldb[hostname][acl]['timestamp'] = timestamp
        acldb[hostname][acl]['protocols'] = rules.protocols()
    return AclDB(firewalls, acldb)
