"""Seeded Cisco ASA configs for the ASA preprocessor restatement (``asa.py``):
object groups (network members as hosts and masked networks; service groups
for tcp, udp and tcp-udp with named and numbered ports and ranges), remarks,
ACL lines in every source/destination/port form ``preprosess_access_lists.py``
parses (any / host / object-group / address + mask; eq, neq, gt, lt, range,
service groups, ICMP types), deny lines, and access-group bindings."""

import numpy as np

from .asa import PORT_NAMES, ICMP_TYPES

__all__ = ['make_config']


def _ip(rng, first=None):
    a = int(first if first is not None else rng.integers(1, 224))
    return '%d.%d.%d.%d' % (a, rng.integers(0, 256), rng.integers(0, 256), rng.integers(1, 255))


def _net(rng):
    plen = int(rng.choice([8, 16, 20, 24, 28]))
    v = int(rng.integers(1 << 24, 224 << 24)) & ~((1 << (32 - plen)) - 1)
    mask = (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF
    dot = lambda x: '%d.%d.%d.%d' % ((x >> 24) & 255, (x >> 16) & 255, (x >> 8) & 255, x & 255)
    return dot(v), dot(mask)


def _port_word(rng, proto):
    names = PORT_NAMES.get(proto, {})
    if names and rng.random() < 0.4:
        return str(rng.choice(sorted(names)))
    return str(int(rng.integers(1, 65536)))


def _port_spec(rng, proto, wide=False):
    r = rng.random()
    if r < 0.55:
        return 'eq ' + _port_word(rng, proto)
    if r < 0.75:
        lo = int(rng.integers(1, 60000))
        return 'range %d %d' % (lo, lo + int(rng.integers(0, 300 if wide else 20)))
    if r < 0.85:
        return 'lt %d' % int(rng.integers(1, 40))
    if r < 0.95:
        return 'gt %d' % int(rng.integers(65500, 65535))
    return 'neq %s' % _port_word(rng, proto) if wide else 'eq ' + _port_word(rng, proto)


def make_config(seed, n_lines=200, hostname='fw-asa1', n_net_groups=8, n_svc_groups=5, wide=False,
                acls=('outside_access_in', 'inside_access_in'), ifcs=('outside', 'inside')):
    """Config text and an info dict (hostname, groups, acls)."""
    rng = np.random.default_rng(seed)
    out = [': Saved', ':', 'ASA Version 9.8(2)', '!', 'hostname ' + hostname, 'domain-name example.net', '!']
    out += ['interface GigabitEthernet0/%d' % k for k in range(len(ifcs))]
    nets = []
    for g in range(n_net_groups):
        name = 'NET-%d_grp' % g
        nets.append(name)
        out.append('object-group network ' + name)
        out.append(' description network group %d' % g)
        for _ in range(int(rng.integers(1, 5))):
            if rng.random() < 0.5:
                out.append(' network-object host ' + _ip(rng))
            else:
                out.append(' network-object %s %s' % _net(rng))
    svcs = {}
    for g in range(n_svc_groups):
        proto = str(rng.choice(['tcp', 'udp', 'tcp-udp']))
        name = 'SVC-%d' % g
        svcs[name] = proto
        out.append('object-group service %s %s' % (name, proto))
        for _ in range(int(rng.integers(1, 4))):
            p = 'tcp' if proto == 'tcp-udp' else proto
            spec = _port_spec(rng, p)
            if spec.startswith('neq') or spec.startswith('lt') or spec.startswith('gt'):
                spec = 'eq ' + _port_word(rng, p)
            out.append(' port-object ' + spec)
    out.append('!')

    def addr():
        r = rng.random()
        if r < 0.2:
            return 'any'
        if r < 0.5:
            return 'host ' + _ip(rng)
        if r < 0.7 and nets:
            return 'object-group ' + str(rng.choice(nets))
        return '%s %s' % _net(rng)

    for k in range(n_lines):
        acl = acls[k % len(acls)] if rng.random() < 0.85 else acls[0]
        if rng.random() < 0.12:
            out.append('access-list %s remark rule block %d owner team-%d' % (acl, k, int(rng.integers(1, 9))))
            continue
        action = 'permit' if rng.random() < 0.85 else 'deny'
        proto = str(rng.choice(['tcp', 'tcp', 'udp', 'ip', 'icmp']))
        src, dst = addr(), addr()
        words = ['access-list', acl, 'extended', action, proto, src]
        if proto in ('tcp', 'udp'):
            if rng.random() < 0.1:
                words.append(_port_spec(rng, proto))
            words.append(dst)
            r = rng.random()
            group = [n for n, p in svcs.items() if p == proto]
            if r < 0.25 and group:
                words.append('object-group ' + str(rng.choice(group)))
            elif r < 0.9:
                words.append(_port_spec(rng, proto, wide))
        elif proto == 'icmp':
            words.append(dst)
            if rng.random() < 0.6:
                words.append(str(rng.choice(sorted(ICMP_TYPES))))
        else:
            words.append(dst)
        out.append(' '.join(words))
    for acl in acls:
        out.append('access-list %s extended deny ip any any' % acl)
    for acl, ifc in zip(acls, ifcs):
        out.append('access-group %s in interface %s' % (acl, ifc))
    out.append(': end')
    return '\n'.join(out) + '\n', {'hostname': hostname, 'nets': nets, 'svcs': svcs, 'acls': list(acls),
                                   'ifcs': list(ifcs)}
