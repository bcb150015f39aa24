"""Seeded synthetic FortiGate configs and traffic — BASELINE config 4, the
long-scan worst case: policies with 4-16 address-group members
per side, services with wide port ranges (``1024-65535``), ``dst:src`` source
port ranges and port lists, giving >= 1M expanded rules, and traffic biased to
late or no match.

``make_config`` writes FortiOS config text in the syntax
``preprosess_fortigate_acl.py`` parses (``config firewall address``/``addrgrp``/
``service custom``/``service group``/``policy``, ``config router setting`` with
``set hostname``); ``fortigate.build_db`` turns it into the rule DB.
``make_traffic`` returns the same traffic dict as ``synth.make_traffic`` (so
``synth.pack`` / ``synth.render_lines`` apply), with the ACL and interface
names of the FortiGate DB (``<host part>-outside`` bound to ``outside-in``).
"""

import numpy as np

from .py2dict import iteration_order
from .synth import F_OUTBOUND, _dotted

__all__ = ['make_config', 'make_traffic', 'SERVICES']

# name -> list of (protocol, dst spec, src spec or None); None protocol = IP / ICMP
SERVICES = {
    'HTTP': [('tcp', '80', None)],
    'HTTPS': [('tcp', '443', None)],
    'SSH': [('tcp', '22', None)],
    'SMTP': [('tcp', '25', None)],
    'DNS': [('tcp', '53', None), ('udp', '53', None)],
    'NTP': [('udp', '123', None)],
    'LDAP': [('tcp', '389', None)],
    'RDP': [('tcp', '3389', None)],
    'MYSQL': [('tcp', '3306', None)],
    'PGSQL': [('tcp', '5432', None)],
    'WEB-ALT': [('tcp', '8080 8443 8000', None)],
    'SYSLOG': [('udp', '514', '512-1023')],
    'RPC-RANGE': [('tcp', '5000-5999', None)],
    'HIGH-TCP': [('tcp', '1024-65535', None)],
    'HIGH-UDP': [('udp', '1024-65535', None)],
    'ALL-TCP': [('tcp', '1-65535', None)],
}
SINGLE = ['HTTP', 'HTTPS', 'SSH', 'SMTP', 'DNS', 'NTP', 'LDAP', 'RDP', 'MYSQL', 'PGSQL', 'WEB-ALT']
NOMATCH_PORTS = np.array([p for p in range(1, 1024) if p not in (22, 25, 53, 80, 123, 389, 443, 514)], np.int64)


def _spec_ports(spec):
    if '-' in spec:
        a, b = spec.split('-')
        return int(a), int(b)
    return None


def make_config(seed, n_policies=160, n_wide=3, n_mid=2, n_syslog=4, hostname='FG-EDGE1', members=(4, 16),
                wide_members=(4, 4)):
    """FortiGate config text + metadata (policies with their member networks
    and services) for ``make_traffic``."""
    rng = np.random.default_rng(seed)
    clients = np.unique(rng.integers(0x0B000000, 0xDF000000, size=20000, dtype=np.int64))
    rng.shuffle(clients)
    servers = np.unique(rng.integers(0x0A000000, 0x0AFFFFFF, size=20000, dtype=np.int64))
    rng.shuffle(servers)
    addr_lines, grp_lines = [], []
    addrs = {}

    def new_addr(pool, kind):
        base = int(pool[rng.integers(len(pool))])
        plen = int(rng.choice([32, 32, 32, 24, 28]))
        net = base & ~((1 << (32 - plen)) - 1) & 0xFFFFFFFF
        name = '%s-%s-%d' % (kind, _dotted(net), plen)
        if name not in addrs:
            mask = (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF
            addr_lines.extend(['    edit "%s"' % name, '        set subnet %s %s' % (_dotted(net), _dotted(mask)),
                               '    next'])
            addrs[name] = (net, plen)
        return name

    def new_group(pool, kind, k):
        names = list(dict.fromkeys(new_addr(pool, kind) for _ in range(k)))
        g = 'grp-%s-%d' % (kind, len(grp_lines))
        grp_lines.extend(['    edit "%s"' % g, '        set member %s' % ' '.join('"%s"' % n for n in names),
                          '    next'])
        return g, [addrs[n] for n in names]

    addr_lines.extend(['    edit "all"', '        set subnet 0.0.0.0 0.0.0.0', '    next'])
    addrs['all'] = (0, 0)
    svc_lines = []
    for name, parts in SERVICES.items():
        svc_lines.extend(['    edit "%s"' % name, '        set protocol TCP/UDP/SCTP'])
        for proto, dspec, sspec in parts:
            svc_lines.append('        set %s-portrange %s' % (proto, dspec if sspec is None else dspec + ':' + sspec))
        svc_lines.append('    next')
    svc_lines.extend(['    edit "ALL"', '        set protocol IP', '    next',
                      '    edit "PING"', '        set protocol ICMP', '    next'])
    srvgrp = ['    edit "Web-Svcs"', '        set member "HTTP" "HTTPS" "WEB-ALT"', '    next']
    policies = []        # (id, srcintf, action, srcgrp, srcnets, dstgrp, dstnets, [service names])
    pid = 0
    kinds = (['wide'] * n_wide + ['mid'] * n_mid + ['syslog'] * n_syslog
             + ['single'] * max(n_policies - n_wide - n_mid - n_syslog, 0))
    kinds = [kinds[i] for i in rng.permutation(len(kinds))]
    for kind in kinds:
        pid += 1
        lo, hi = wide_members if kind == 'wide' else members
        sg, snets = new_group(clients, 'c', int(rng.integers(lo, hi + 1)))
        dg, dnets = new_group(servers, 's', int(rng.integers(lo, hi + 1)))
        if kind == 'wide':
            svcs = [str(rng.choice(['HIGH-TCP', 'HIGH-UDP']))]
        elif kind == 'mid':
            svcs = ['RPC-RANGE']
        elif kind == 'syslog':
            svcs = ['SYSLOG']
        else:
            k = int(rng.integers(1, 4))
            svcs = list(dict.fromkeys(str(x) for x in rng.choice(SINGLE + ['Web-Svcs'], size=k)))
        action = 'accept' if rng.random() < 0.9 else 'deny'
        policies.append((str(pid), 'Outside', action, sg, snets, dg, dnets, svcs))
    # inside policies (outbound connections) and a DMZ policy (ACL "")
    for _ in range(6):
        pid += 1
        sg, snets = new_group(servers, 's', int(rng.integers(2, 6)))
        policies.append((str(pid), 'Inside', 'accept', sg, snets, 'all', [(0, 0)], ['Web-Svcs', 'DNS']))
    pid += 1
    dg, dnets = new_group(servers, 's', 3)
    policies.append((str(pid), 'DMZ', 'accept', 'all', [(0, 0)], dg, dnets, ['SSH']))
    # the 'ip' protocol every tcp/udp candidate list needs (mapper.py:161): deny all
    for ifc in ('Outside', 'Inside'):
        pid += 1
        policies.append((str(pid), ifc, 'deny', 'all', [(0, 0)], 'all', [(0, 0)], ['ALL']))
    pol_lines = []
    for (p, ifc, action, sg, _sn, dg, _dn, svcs) in policies:
        pol_lines.extend(['    edit %s' % p, '        set srcintf "%s"' % ifc, '        set dstintf "Inside"',
                          '        set srcaddr "%s"' % sg, '        set dstaddr "%s"' % dg,
                          '        set action %s' % action, '        set status enable',
                          '        set service %s' % ' '.join('"%s"' % x for x in svcs),
                          "        set comments ''" if int(p) % 3 else '        set comments "policy %s"' % p,
                          '        set global-label "section-%d"' % (int(p) // 20), '    next'])
    text = '\n'.join(['config router setting', '    set hostname "%s"' % hostname, 'end',
                      'config firewall address'] + addr_lines + ['end', 'config firewall addrgrp'] + grp_lines
                     + ['end', 'config firewall service custom'] + svc_lines + ['end', 'config firewall service group']
                     + srvgrp + ['end', 'config firewall policy'] + pol_lines + ['end', ''])
    ids = [p[0] for p in policies]
    rank = {ids[k]: r for r, k in enumerate(iteration_order(ids))}     # ACL order (trap 10)
    host_part = hostname.split('-')[1]
    info = {'host': hostname, 'policies': policies, 'rank': rank,
            'outside_ifc': host_part + '-outside', 'inside_ifc': host_part + '-inside'}
    return text, info


def _service_ports(name):
    """[(proto 0 tcp / 1 udp, dport lo, dport hi, sport lo or None, sport hi)] of a service."""
    if name == 'Web-Svcs':
        return sum((_service_ports(n) for n in ('HTTP', 'HTTPS', 'WEB-ALT')), [])
    out = []
    for proto, dspec, sspec in SERVICES.get(name, []):
        pr = 0 if proto == 'tcp' else 1
        for d in dspec.split(' '):
            r = _spec_ports(d) or (int(d), int(d))
            s = _spec_ports(sspec) if sspec else None
            out.append((pr, r[0], r[1], s[0] if s else None, s[1] if s else None))
    return out


def _sample_nets(rng, nets, n):
    nets = np.array(nets, np.int64).reshape(-1, 2)
    pick = nets[rng.integers(0, len(nets), size=n)]
    size = np.minimum(np.int64(1) << (32 - pick[:, 1]), 256)
    return pick[:, 0] + (rng.random(n) * size).astype(np.int64)


def make_traffic(info, n, seed, p_nomatch=0.3, late_power=3.0, form_probs=(0.86, 0.04, 0.04, 0.03, 0.02, 0.01),
                 t0=15 * 86400, span=3 * 3600, cid0=1000000):
    """Traffic dict (synth.make_traffic's layout) for a ``make_config`` DB:
    inbound lines drawn from permit Outside policies weighted by
    ``(ACL position)^late_power`` (late matches), ``p_nomatch`` of them on
    ports no service covers; outbound lines from the Inside policies."""
    rng = np.random.default_rng(seed)
    form = rng.choice(len(form_probs), size=n, p=np.asarray(form_probs) / np.sum(form_probs))
    src = np.zeros(n, np.int64)
    dst = np.zeros(n, np.int64)
    sport = rng.integers(1024, 65536, size=n)
    dport = np.zeros(n, np.int64)
    proto = (rng.random(n) < 0.3).astype(np.int64)
    for side, ifc in ((0, 'Outside'), (1, 'Inside')):
        pols = [p for p in info['policies'] if p[1] == ifc and p[2] == 'accept' and p[7] != ['ALL']]
        sel = np.nonzero((form == F_OUTBOUND) == bool(side))[0]
        if not pols or not len(sel):
            continue
        w = np.array([(info['rank'][p[0]] + 1.0) ** late_power for p in pols])
        pick = rng.choice(len(pols), size=len(sel), p=w / w.sum())
        grouped = sel[np.argsort(pick, kind='stable')]
        bounds = np.concatenate([[0], np.cumsum(np.bincount(pick, minlength=len(pols)))])
        for j, p in enumerate(pols):
            idx = grouped[bounds[j]:bounds[j + 1]]
            if not len(idx):
                continue
            src[idx] = _sample_nets(rng, p[4], len(idx))
            dst[idx] = _sample_nets(rng, p[6], len(idx))
            segs = [s for name in p[7] for s in _service_ports(name)]
            seg = rng.integers(0, len(segs), size=len(idx))
            for q, (pr, dlo, dhi, slo, shi) in enumerate(segs):
                k = idx[seg == q]
                proto[k] = pr
                dport[k] = rng.integers(dlo, dhi + 1, size=len(k))
                if slo is not None:
                    sport[k] = rng.integers(slo, shi + 1, size=len(k))
        if side == 0:
            nm = sel[rng.random(len(sel)) < p_nomatch]
            dport[nm] = NOMATCH_PORTS[rng.integers(0, len(NOMATCH_PORTS), size=len(nm))]
    # outbound: the 'for' side is the outside peer; swap so that src is the
    # inside initiator (synth.render_lines prints dst first for outbound)
    t = t0 + (np.arange(n, dtype=np.int64) * span) // max(n, 1)
    cid = cid0 + np.arange(n, dtype=np.int64)
    return {'src': src, 'dst': dst, 'sport': sport, 'dport': dport, 'proto': proto, 'ifc': np.zeros(n, np.int64),
            'form': form, 't': t, 'cid': cid, 'interfaces': [info['outside_ifc']], 'host': info['host'],
            'acl_of': ['outside-in'], 'inside_acl': 'inside-in', 'inside_ifc': info['inside_ifc']}
