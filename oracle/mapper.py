"""ORACLE (test infrastructure only) — restatement of the mapper, ``mapper.py:107-189``.

``map_lines`` consumes log lines exactly as ``for line in sys.stdin`` yields them
(each still carrying its ``'\\n'``) and appends the mapper's stdout text, chunk
by chunk, to ``out``.  Exceptions the reference would die with (``KeyError`` on
a missing ``'in'`` binding or protocol list, ``ValueError`` from rule
construction) propagate unchanged after the output produced so far is in
``out`` — as a crashed Hadoop task's flushed stdout would be.
"""

from .firewallrule import FirewallRule
from .fwregex import get_builtconn


class HostMissing(Exception):
    """``mapper.py:115-117``: prints the message on stdout and exits 1."""


def map_lines(lines, hostname, accesslists, firewalls, out):
    # mapper.py:115-117 — validate prerequisites
    if hostname not in firewalls or hostname not in accesslists:
        out.append('Firewall {0} not present in data structure. Aborting.\n'.format(hostname))
        raise HostMissing(hostname)
    fw = firewalls[hostname]
    acls = accesslists[hostname]
    for line in lines:
        data = get_builtconn(line)                                   # mapper.py:124
        if not data:
            continue
        protocol = data['protocol'].lower()                          # mapper.py:135
        # Connection.__init__ -> FirewallRule.__init__ (mapper.py:44-51, 138-142)
        conn = FirewallRule(True, protocol, line, data['src'], data['dst'], data['sport'], data['dport'])
        ifc = data['interface_in']
        if ifc not in fw:                                            # mapper.py:145-149
            continue
        acl = fw[ifc]['in']
        if acl not in acls:                                          # mapper.py:152-156
            out.append('Unable to process line because access-list {0} is missing from data '
                       'structure for host {1}, skipping line.\n'.format(acl, hostname))
            out.append('The skipped line is: {0}\n'.format(line))
            continue
        protos = acls[acl]['protocols']
        if protocol in ('tcp', 'udp'):                               # mapper.py:159-166
            if protocol in protos:
                candidates = sorted(protos[protocol] + protos['ip'])
            else:
                candidates = protos['ip']
        else:
            candidates = protos[protocol]
        rules = acls[acl]['rules']
        for ruleindex in candidates:                                 # mapper.py:168-189
            if conn in rules[ruleindex]:
                out.append(';'.join([hostname, acl, str(ruleindex)]) + '\t' + line + '\n')
                break
    return out
