"""ORACLE (test infrastructure only) — restatement of the FortiGate preprocessor
``preprosess_fortigate_acl.py`` producing the expanded rules of each ACL as
per-rule arrays for ``coracle`` (the reference stores one ``FirewallRule`` per
row; these are that object's fields).  Written close to the reference's loops:

* config parser ``:296-358`` (sections, ``edit``/``set``/``next``, subnet
  ``' '`` -> ``'/'``);
* ``expand_addr`` ``:30-57`` (an fqdn goes to ``resolve``, the contract of
  ``socket.gethostbyname_ex``; a failed lookup is skipped as the reference
  skips it);
* ``expand_service`` ``:60-140`` (``tcp-portrange`` then ``udp-portrange``;
  ``a-b`` one rule per port, ``1-65535`` NO_PORT; ``a b c``; ``dst:src`` product
  src-major; ICMP/IP port-less);
* policies in Python 2 dict order of the policy ids (``:362``, replayed by
  ``oracle.py2dict``), status ``enable``; srcintf -> ACL (``:365-368``); rules
  ``for src: for dst: for svc`` (``:184-186``); ruleindex = position; proto2rule
  (``:375-384``); interfaces (``:387-392``).

Independent of the product's ``fortigate.py`` (which builds numpy columns
vectorised); this one appends rule by rule.
"""

import re
import socket
from array import array

import numpy as np

from .ipy import IP
from .py2dict import py2_keys

NO_PORT = -1
TITLES = {
    'policy': ['srcintf', 'dstintf', 'srcaddr', 'dstaddr', 'action', 'status', 'service', 'comments', 'global-label'],
    'addr': ['type', 'comment', 'subnet', 'start-ip', 'end-ip', 'fqdn'],
    'addrgrp': ['comment', 'member'],
    'service': ['category', 'protocol', 'comment', 'protocol-number', 'tcp-portrange', 'udp-portrange', 'icmptype',
                'icmpcode'],
    'srvcgrp': ['comment', 'member'],
    'router': ['hostname'],
}


def parse(text):
    obj = {}
    elem = False
    section = False
    for line in text.split('\n'):
        line = line.strip()
        if line == 'config firewall policy':
            section = 'policy'
            obj[section] = {}
        elif line == 'config firewall address':
            section = 'addr'
            obj[section] = {}
        elif line == 'config firewall addrgrp':
            section = 'addrgrp'
            obj[section] = {}
        elif line == 'config firewall service custom':
            section = 'service'
            obj[section] = {}
        elif line == 'config firewall service group':
            section = 'srvcgrp'
            obj[section] = {}
        elif line == 'config router setting':
            section = 'router'
            obj[section] = {}
        if section and line == 'end':
            section = False
        if not section:
            continue
        if line[:4] == 'edit':
            match = re.search(r'edit (.*)', line)
            if match:
                elem = str(match.groups()[0])
                obj[section][elem] = {}
        if section == 'router' and line[:12] == 'set hostname':
            contents = line.split()[2]
            obj[section]['hostname'] = contents.replace("'", '').replace('"', '')
        elif line == 'next':
            elem = False
        elif line[:3] == 'set' and elem:
            for title in TITLES[section]:
                if line.split()[1] == title:
                    obj[section][elem][title] = ' '.join(line.split()[2:])
                    break
            if section == 'addr' and line.split()[1] == 'subnet':
                obj[section][elem][title] = obj[section][elem][title].replace(' ', '/')
    return obj


def expand_addr(entry, obj, resolve):
    res = []
    for match in re.finditer(r'(\".*?\")', entry):
        name = match.groups()[0]
        if name in obj['addr']:
            if 'subnet' in obj['addr'][name]:
                res.append(obj['addr'][name]['subnet'])
            elif 'fqdn' in obj['addr'][name]:
                try:
                    res = res + list(resolve(obj['addr'][name]['fqdn'].replace('"', ''))[2])
                except Exception:  # noqa: BLE001 - a failed lookup is skipped
                    pass
        else:
            for member in re.finditer(r'(\".*?\")', obj['addrgrp'][name]['member']):
                res = res + expand_addr(member.groups()[0], obj, resolve)
    return res


def expand_service(entry, obj):
    res = []
    if entry in obj['service']:
        o = obj['service'][entry]
        if o['protocol'] == 'TCP/UDP/SCTP':
            for key in ['tcp-portrange', 'udp-portrange']:
                if key in o:
                    protocol = key[:3]
                    data = {'src': False, 'dst': False, 'srcobj': [], 'dstobj': []}
                    if o[key].find(':') != -1:
                        data['dst'], data['src'] = o[key].split(':')
                    else:
                        data['dst'] = o[key]
                    for direction in ['src', 'dst']:
                        if data[direction]:
                            if data[direction].find('-') != -1:
                                start, end = data[direction].split('-')
                                if int(start) == 1 and int(end) == 65535:
                                    data[direction + 'obj'].append(NO_PORT)
                                else:
                                    for port in range(int(start), int(end) + 1):
                                        data[direction + 'obj'].append(port)
                            elif data[direction].find(' ') != -1:
                                for port in data[direction].split(' '):
                                    data[direction + 'obj'].append(int(port))
                            else:
                                data[direction + 'obj'].append(int(data[direction]))
                    if data['src']:
                        for src in data['srcobj']:
                            for dst in data['dstobj']:
                                res.append((protocol, src, dst))
                    else:
                        for dst in data['dstobj']:
                            res.append((protocol, NO_PORT, dst))
        elif o['protocol'] == 'ICMP' or o['protocol'] == 'IP':
            res.append((o['protocol'].lower(), NO_PORT, NO_PORT))
    elif entry in obj['srvcgrp']:
        for member in obj['srvcgrp'][entry]['member'].split(' '):
            res = res + expand_service(member, obj)
    return res


class Acl(object):
    """One ACL's expanded rules as per-rule arrays (the fields coracle needs)."""

    def __init__(self):
        self.action = array('B')
        self.proto = []            # protocol name per rule
        self.src = array('L')
        self.src_len = array('Q')
        self.dst = array('L')
        self.dst_len = array('Q')
        self.sport = array('l')
        self.dport = array('l')
        self.protocols = {}

    def __len__(self):
        return len(self.action)


def expand(text, resolve=socket.gethostbyname_ex):
    """-> (hostname, firewalls, {acl: Acl})."""
    obj = parse(text)
    acls = {}
    ip_cache = {}

    def ip(s):
        if s not in ip_cache:
            a = IP(s)
            assert a.version() == 4
            ip_cache[s] = (a.ip, a.len())
        return ip_cache[s]

    for policy_id in py2_keys(list(obj['policy'].keys())):
        p = obj['policy'][policy_id]
        if p['status'] != 'enable':
            continue
        acl = ''
        if p['srcintf'] == '"Outside"':
            acl = 'outside-in'
        elif p['srcintf'] == '"Inside"' or p['srcintf'] == '"Guest-Inside"':
            acl = 'inside-in'
        if acl not in acls:
            acls[acl] = Acl()
        A = acls[acl]
        srcs, dsts = [], []
        for m in re.finditer(r'(\".*?\")', p.get('srcaddr', '')):
            srcs = srcs + expand_addr(m.groups()[0], obj, resolve)
        for m in re.finditer(r'(\".*?\")', p.get('dstaddr', '')):
            dsts = dsts + expand_addr(m.groups()[0], obj, resolve)
        svcs = []
        for part in p['service'].split(' '):
            svcs = svcs + expand_service(part, obj)
        permit = 1 if p['action'] == 'accept' else 0
        for src in srcs:
            s_ip, s_len = ip(src)
            for dst in dsts:
                d_ip, d_len = ip(dst)
                for proto, sp, dp in svcs:
                    i = len(A)
                    A.action.append(permit)
                    A.proto.append(proto)
                    A.src.append(s_ip)
                    A.src_len.append(s_len)
                    A.dst.append(d_ip)
                    A.dst_len.append(d_len)
                    A.sport.append(sp)
                    A.dport.append(dp)
                    A.protocols.setdefault(proto, []).append(i)
    hostname = obj['router']['hostname']
    firewalls = {hostname: {}}
    for acl in acls:
        intf = '-'.join([hostname.split('-')[1], acl.split('-')[0]])
        firewalls[hostname][intf] = {'in': acl}
    return hostname, firewalls, acls


def as_columns(A):
    """numpy views of an Acl's arrays."""
    return {'action': np.frombuffer(A.action, np.uint8), 'src': np.frombuffer(A.src, np.uint32 if A.src.itemsize == 4
                                                                                 else np.uint64).astype(np.uint32),
            'src_len': np.frombuffer(A.src_len, np.uint64), 'dst': np.frombuffer(A.dst, np.uint32 if A.dst.itemsize == 4
                                                                                 else np.uint64).astype(np.uint32),
            'dst_len': np.frombuffer(A.dst_len, np.uint64),
            'sport': np.frombuffer(A.sport, np.int32 if A.sport.itemsize == 4 else np.int64).astype(np.int32),
            'dport': np.frombuffer(A.dport, np.int32 if A.dport.itemsize == 4 else np.int64).astype(np.int32),
            'proto': A.proto}
