"""Cisco ASA/FWSM config -> ``accesslists.db`` (restates ``preprosess_access_lists.py``).

What the reference does and this module reproduces, rule for rule:

* first pass over the config lines (``:356-383``): ``object-group network|service``
  names (service groups keyed by their protocol word), ``hostname``, and
  ``access-group ACL DIR interface IFC`` -> ``firewalls[host][IFC][DIR] = ACL``;
* object-group members (``:391-419``) through CiscoConfParse's
  ``find_all_children('^object-group network GRP$')``: ``network-object host A``
  -> ``A``, ``network-object A M`` -> ``A/M``; ``port-object SPEC`` with port
  names replaced by numbers (``tcp-udp`` groups: tcp and udp names);
* second pass (``:431-480``): every ``access-list `` line counts towards its
  ACL's ``rulenum``; ``remark`` lines build the comment list the following
  rules share; other lines are parsed by ``parse_cisco_fw_access_list_entry``
  (``:94-291``: ``access-list NAME extended permit|deny PROTO ...``; source
  ``any``/``host A``/``object-group G``/``A M``, optional source ports, the
  same for the destination; ports ``eq/neq/gt/lt/range`` expanded by
  ``parse_port_spec_to_list`` ``:28-91``) and expanded dport -> dst -> sport ->
  src (``:256-276``); ``ruleindex`` = list position, ``protocols`` per rule
  protocol;
* the DB write (``:525-550``): ``firewalls`` and ``accesslists[host][acl] =
  {rules, timestamp, protocols}`` merged into an existing DB.

Error behaviour follows the reference: a line its regex cannot parse, a port
that is neither a number nor a known name -> ``ValueError`` handling that logs
and exits 1 (``SystemExit(1)`` here); an address FirewallRule rejects -> the
same; an unknown object-group name -> ``KeyError``; a config without a
hostname -> exit 1; an ACL with remarks only -> ``KeyError`` at the DB write
(its ``proto2rule`` entry never exists, ``:544``).

Third-party / data the reference needs that are absent here:

* ``ciscoconfparse`` (not installed, version unpinned): only
  ``find_all_children`` is used; restated from its published behaviour — the
  lines matching the pattern and every line indented below them, in file
  order (``find_all_children``);
* ``name-number-mappings.db`` (a pickle, never loaded here): replaced by the
  Cisco ASA port-name and ICMP-type literals of the ASA command reference
  (``PORT_NAMES``, ``ICMP_TYPES``); a name outside these tables is parsed as a
  number (ValueError -> exit 1), as the reference does for names missing from
  its DB.  Parity of the name table itself is unpinned.  Port-object name
  substitution tries longer names first (the reference's order is the Python 2
  dict order of the pickled table).

Rules are built as numpy columns (``rulecols.RuleColumns``): a ``neq`` or a
wide ``range`` expands to tens of thousands of rules per line.
"""

import re

import numpy as np

from .acldb import AclDB
from .ipaddr import IP
from .py2dict import iteration_order
from .py2text import py2_int, py2_split, py2_strip
from .rulecols import FAM_DST6, FAM_SRC6, Nets6, RuleColumns

__all__ = ['PORT_NAMES', 'ICMP_TYPES', 'parse_port_spec', 'parse_acl_entry', 'find_all_children', 'build_db']

_TCP = {'aol': 5190, 'bgp': 179, 'chargen': 19, 'cifs': 3020, 'citrix-ica': 1494, 'cmd': 514, 'ctiqbe': 2748,
        'daytime': 13, 'discard': 9, 'domain': 53, 'echo': 7, 'exec': 512, 'finger': 79, 'ftp': 21, 'ftp-data': 20,
        'gopher': 70, 'h323': 1720, 'hostname': 101, 'http': 80, 'https': 443, 'ident': 113, 'imap4': 143,
        'irc': 194, 'kerberos': 750, 'klogin': 543, 'kshell': 544, 'ldap': 389, 'ldaps': 636, 'login': 513,
        'lotusnotes': 1352, 'lpd': 515, 'netbios-ssn': 139, 'nfs': 2049, 'nntp': 119, 'pcanywhere-data': 5631,
        'pim-auto-rp': 496, 'pop2': 109, 'pop3': 110, 'pptp': 1723, 'rsh': 514, 'rtsp': 554, 'sip': 5060,
        'smtp': 25, 'sqlnet': 1521, 'ssh': 22, 'sunrpc': 111, 'tacacs': 49, 'talk': 517, 'telnet': 23, 'uucp': 540,
        'whois': 43, 'www': 80}
_UDP = {'biff': 512, 'bootpc': 68, 'bootps': 67, 'cifs': 3020, 'discard': 9, 'dnsix': 195, 'domain': 53, 'echo': 7,
        'http': 80, 'isakmp': 500, 'kerberos': 750, 'mobile-ip': 434, 'nameserver': 42, 'netbios-dgm': 138,
        'netbios-ns': 137, 'nfs': 2049, 'ntp': 123, 'pcanywhere-status': 5632, 'pim-auto-rp': 496, 'radius': 1645,
        'radius-acct': 1646, 'rip': 520, 'secureid-udp': 5510, 'sip': 5060, 'snmp': 161, 'snmptrap': 162,
        'sunrpc': 111, 'syslog': 514, 'tacacs': 49, 'talk': 517, 'tftp': 69, 'time': 37, 'vxlan': 4789, 'who': 513,
        'www': 80, 'xdmcp': 177}
PORT_NAMES = {'tcp': _TCP, 'udp': _UDP}
ICMP_TYPES = {'echo-reply': 0, 'unreachable': 3, 'source-quench': 4, 'redirect': 5, 'alternate-address': 6,
              'echo': 8, 'router-advertisement': 9, 'router-solicitation': 10, 'time-exceeded': 11,
              'parameter-problem': 12, 'timestamp-request': 13, 'timestamp-reply': 14, 'information-request': 15,
              'information-reply': 16, 'mask-request': 17, 'mask-reply': 18, 'traceroute': 30,
              'conversion-error': 31, 'mobile-redirect': 32}

_RE_ACL = re.compile(r'access-list ([A-Za-z0-9_-]+) extended (permit|deny) ([a-zA-Z0-9]+) (.+)')
NO_PORT = -1


def _num(word, names):
    return names[word] if word in names else py2_int(word)


def parse_port_spec(parts, protocol, name2num):
    """parse_port_spec_to_list (:28-91): a port spec -> list of ports."""
    if len(parts) < 2:
        return []
    if protocol not in name2num:
        name2num[protocol] = {}
    names = name2num[protocol]
    op = parts[0]
    if op == 'eq':
        return [_num(parts[1], names)]
    if op == 'neq':
        ports = list(range(0, 65536))
        ports.remove(_num(parts[1], names))       # ValueError when the port is outside 0..65535
        return ports
    if op in ('range', 'gt', 'lt'):
        if op == 'range':
            start, end = _num(parts[1], names), _num(parts[2], names)
        elif op == 'gt':
            start, end = _num(parts[1], names), 65535
        else:
            start, end = 0, _num(parts[1], names)
        return list(range(start, end + 1))
    return []


def parse_acl_entry(line, name2num, icmptype2num, networkgroups, servicegroups):
    """parse_cisco_fw_access_list_entry (:94-291) up to the FirewallRule
    construction: (allow, protocol, original, src list, dst list, sport list,
    dport list), False for a remark, ValueError for anything else."""
    line = py2_strip(line)
    m = _RE_ACL.search(line)
    if not m:
        if line.find('remark') != -1:
            return False
        raise ValueError('Unable to parse access-list entry: ' + line)
    _name, action, protocol, rest = m.groups()
    allow = action == 'permit'
    parts = py2_split(rest)
    sourceports, destinationports = [], []
    if parts[0] == 'any':
        src, parts = [parts[0]], parts[1:]
    elif parts[0] == 'host':
        src, parts = [parts[1]], parts[2:]
    elif parts[0] == 'object-group':
        src, parts = networkgroups[parts[1]], parts[2:]
    else:
        src, parts = ['/'.join(parts[0:2])], parts[2:]
    # source ports (a service group found here is not consumed: the reference
    # then reads the same words as the destination, :163-170)
    if parts[0] == 'object-group':
        if protocol in servicegroups and parts[1] in servicegroups[protocol]:
            for item in servicegroups[protocol][parts[1]]:
                sourceports.append(py2_split(item))
    elif parts[0] in ('eq', 'neq', 'gt', 'lt'):
        sourceports.append(parts[0:2])
        parts = parts[2:]
    elif parts[0] == 'range':
        sourceports.append(parts[0:3])
        parts = parts[3:]
    elif protocol == 'icmp':
        if parts[0] in icmptype2num:
            sourceports.append(icmptype2num[parts[0]])
            parts = parts[1:]
    if parts[0] == 'any':
        dst, parts = [parts[0]], parts[1:]
    elif parts[0] == 'host':
        dst, parts = [parts[1]], parts[2:]
    elif parts[0] == 'object-group':
        dst, parts = networkgroups[parts[1]], parts[2:]
    else:
        dst, parts = ['/'.join(parts[0:2])], parts[2:]
    if len(parts) > 1:
        if parts[0] == 'object-group':
            if protocol in servicegroups and parts[1] in servicegroups[protocol]:
                for item in servicegroups[protocol][parts[1]]:
                    destinationports.append(py2_split(item))
            parts = parts[2:]
        elif parts[0] in ('eq', 'neq', 'gt', 'lt'):
            destinationports.append(parts[0:2])
            parts = parts[2:]
        elif parts[0] == 'range':
            destinationports.append(parts[0:3])
            parts = parts[3:]
    elif protocol == 'icmp' and len(parts) == 1:
        if parts[0] in icmptype2num:
            destinationports.append(icmptype2num[parts[0]])
            parts = parts[1:]
    if protocol != 'icmp':
        sport = [p for spec in sourceports for p in parse_port_spec(spec, protocol, name2num)]
        dport = [p for spec in destinationports for p in parse_port_spec(spec, protocol, name2num)]
    else:
        sport, dport = sourceports, destinationports
    return allow, protocol, line, src, dst, sport, dport


def find_all_children(lines, pattern):
    """CiscoConfParse.find_all_children: every line matching ``pattern`` and all
    the lines indented below it (children of children too), in file order."""
    rx = re.compile(pattern)
    out = []
    taken = set()
    for i, l in enumerate(lines):
        if not rx.search(l):
            continue
        ind = len(l) - len(l.lstrip(' '))
        for j in [i] + list(_descendants(lines, i, ind)):
            if j not in taken:
                taken.add(j)
                out.append(j)
    return [lines[j] for j in sorted(out)]


def _descendants(lines, i, ind):
    j = i + 1
    while j < len(lines):
        l = lines[j]
        if py2_strip(l) == '' or len(l) - len(l.lstrip(' ')) <= ind:
            break
        yield j
        j += 1


def _addr(text, side, nets6):
    """FirewallRule's address conversion (firewallrule.py:80-92) -> (value,
    prefix length, IPv6?); an IPv6 network's value is its ``nets6`` id."""
    if text == 'any':
        return 0, 0, 0
    try:
        ip = IP(text)
    except ValueError as e:
        raise ValueError('argument "%s" must be a valid IP address or network. Error: %s' % (side, e))
    if ip._ipversion != 4:
        return nets6(text), int(ip._prefixlen), 1
    return int(ip.ip), int(ip._prefixlen), 0


class _Acl(object):
    """Columns of one ACL's expanded rules, in ruleindex order."""

    def __init__(self):
        self.parts = []
        self.n = 0
        self.proto_names = []
        self.originals, self.comments, self.comment_ids, self.rulenums = [], [], {}, []
        self.nets6 = Nets6()

    def add(self, allow, protocol, original, src, dst, sport, dport, comments, rulenum):
        # nesting dport -> dst -> sport -> src (:256-276); an empty port list is NO_PORT
        if not src or not dst:
            return 0                      # no FirewallRule is built (no validation either)
        dp = np.array(dport if dport else [NO_PORT], np.int64)
        sp = np.array(sport if sport else [NO_PORT], np.int64)
        s = [_addr(a, 'src', self.nets6) for a in src]
        d = [_addr(a, 'dst', self.nets6) for a in dst]
        if protocol not in self.proto_names:
            self.proto_names.append(protocol)
        pid = self.proto_names.index(protocol)
        S, D, P, Q = len(s), len(d), len(sp), len(dp)
        m = S * D * P * Q
        qi = np.repeat(np.arange(Q), D * P * S)
        di = np.tile(np.repeat(np.arange(D), P * S), Q)
        pi = np.tile(np.repeat(np.arange(P), S), Q * D)
        si = np.tile(np.arange(S), Q * D * P)
        s_ip = np.array([a for a, _, _ in s], np.uint32)
        s_len = np.array([b for _, b, _ in s], np.uint8)
        s_v6 = np.array([v for _, _, v in s], np.uint8)
        d_ip = np.array([a for a, _, _ in d], np.uint32)
        d_len = np.array([b for _, b, _ in d], np.uint8)
        d_v6 = np.array([v for _, _, v in d], np.uint8)
        self.originals.append(original)
        key = id(comments)
        if key not in self.comment_ids:
            self.comment_ids[key] = len(self.comments)
            self.comments.append(comments)
        self.rulenums.append(rulenum)
        self.parts.append({
            'action': np.full(m, allow, bool), 'proto': np.full(m, pid, np.uint8),
            'src': s_ip[si], 'src_len': s_len[si], 'dst': d_ip[di], 'dst_len': d_len[di],
            'sport': sp[pi].astype(np.int32), 'dport': dp[qi].astype(np.int32),
            'orig': np.full(m, len(self.originals) - 1, np.int32),
            'comment': np.full(m, self.comment_ids[key], np.int32),
            'rulenum': np.full(m, len(self.rulenums) - 1, np.int32),
            'fam': s_v6[si] * FAM_SRC6 | d_v6[di] * FAM_DST6})
        self.n += m
        return m

    def build(self):
        cols = {}
        for k in ('action', 'proto', 'src', 'src_len', 'dst', 'dst_len', 'sport', 'dport', 'orig', 'comment',
                  'rulenum', 'fam'):
            cols[k] = np.concatenate([p[k] for p in self.parts]) if self.parts else np.zeros(0)
        return RuleColumns(cols['action'], cols['proto'], self.proto_names, cols['src'], cols['src_len'], cols['dst'],
                           cols['dst_len'], cols['sport'], cols['dport'], cols['orig'], self.originals or [''],
                           cols['comment'], self.comments or [[]], cols['rulenum'], self.rulenums or [-1],
                           fam=cols['fam'], nets6=self.nets6.texts)


def _exit(log, *msgs):
    for m in msgs:
        log('ERROR - ' + m + '\n')
    raise SystemExit(1)


def build_db(text, timestamp=0.0, firewalls=None, accesslists=None, log=None, name2num=None, icmptype2num=None):
    """The reference's ``main`` (:294-550) on config text: the AclDB it would
    store (merged into ``firewalls`` / ``accesslists`` of an existing DB)."""
    log = log or (lambda m: None)
    name2num = {p: dict(v) for p, v in (PORT_NAMES if name2num is None else name2num).items()}
    icmptype2num = dict(ICMP_TYPES if icmptype2num is None else icmptype2num)
    firewalls = {} if firewalls is None else firewalls
    raw = text.split('\n')
    file_lines = [l + '\n' for l in raw[:-1]] + ([raw[-1]] if raw[-1] else [])
    conf_lines = [l.rstrip('\r\n') for l in file_lines]
    networkgroups, servicegroups, hostname = {}, {}, ''
    for line in file_lines:
        if line[:12] == 'object-group':
            parts = py2_split(line)
            if len(parts) < 3:
                continue
            if parts[1] == 'network':
                networkgroups[parts[2]] = []
            elif parts[1] == 'service':
                servicegroups.setdefault(parts[3], {})[parts[2]] = []
        elif line[:8] == 'hostname':
            hostname = py2_strip(line[9:])
        elif line[:12] == 'access-group':
            parts = py2_split(line)
            if hostname != '':
                firewalls.setdefault(hostname, {}).setdefault(parts[4], {})[parts[2]] = parts[1]
            else:
                log('WARNING - Hostname unknown when parsing access-group line, unable to parse line. This may '
                    'result in incomplete info about which access-list is used on which interface.\n')
    if hostname == '':
        _exit(log, 'Config file does not contain hostname of firewall')
    for grp in networkgroups:
        for line in find_all_children(conf_lines, '^object-group network ' + grp + '$'):
            line = py2_strip(line)
            if line.find('network-object') != -1:
                address = line[15:]
                networkgroups[grp].append(address[5:] if address[:4] == 'host' else address.replace(' ', '/'))
    for protocol in servicegroups:
        for grp in servicegroups[protocol]:
            for line in find_all_children(conf_lines, '^object-group service ' + grp + ' ' + protocol + '$'):
                line = py2_strip(line)
                if line.find('port-object') != -1:
                    obj = line[12:]
                    for p in (['tcp', 'udp'] if protocol == 'tcp-udp' else [protocol]):
                        for portname in sorted(name2num[p], key=lambda w: (-len(w), w)):
                            if obj.find(portname) != -1:
                                obj = obj.replace(portname, str(name2num[p][portname]))
                    servicegroups[protocol][grp].append(obj)
    acls = {}
    order = []
    comments, comments_used = [], False
    linecount = {}
    for line in file_lines:
        if line[:12] != 'access-list ':
            continue
        parts = py2_split(line)
        acl = parts[1]
        if acl not in acls:
            acls[acl] = _Acl()
            order.append(acl)
        linecount[acl] = linecount.get(acl, 0) + 1
        if acl == 'ip' and parts[2] != 'remark':
            # proto2rule starts as {'ip': []} (:429): a rule of an ACL named 'ip'
            # indexes that list with its protocol name (:471-474)
            raise TypeError('list indices must be integers or slices, not str')
        if parts[2] == 'remark':
            if comments_used:
                comments, comments_used = [py2_strip(line)], False
            else:
                comments.append(py2_strip(line))
        try:
            parsed = parse_acl_entry(line, name2num, icmptype2num, networkgroups, servicegroups)
        except ValueError:
            _exit(log, 'Unable to parse one of the lines in the config, aborting.', 'The line is: {0}'.format(py2_strip(line)))
        if parsed:
            allow, protocol, original, src, dst, sport, dport = parsed
            try:
                n = acls[acl].add(allow, protocol, original, src, dst, sport, dport, comments, linecount[acl])
            except ValueError as e:
                _exit(log, 'Unable to convert line to FirewallRule object. Reason: {0}'.format(e),
                      'The line is: {0}'.format(original))
            if n:
                comments_used = True
    acldb = {} if accesslists is None else accesslists
    acldb.setdefault(hostname, {})
    for k in iteration_order(order):
        acl = order[k]
        b = acls[acl]
        if b.n == 0:
            raise KeyError(acl)          # proto2rule[acl] never created (:544)
        rules = b.build()
        acldb[hostname].setdefault(acl, {})
        acldb[hostname][acl]['rules'] = rules
        acldb[hostname][acl]['timestamp'] = timestamp
        acldb[hostname][acl]['protocols'] = rules.protocols()
    return AclDB(firewalls, acldb)
