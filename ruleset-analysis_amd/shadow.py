"""Shadowed-rule analysis: rules that can never get a hit because a rule above
them in the same access list contains them (``preprosess_access_lists.py:508-521``,
run by the ASA preprocessor with ``-v``).  The reference compares every rule
with every rule above it in Python (``rule in accesslists[acl][i]``,
``FirewallRule.__contains__`` at ``firewallrule.py:128-174``): O(R^2) per list.
Here the pairwise test runs on the GPU (``rsa_shadowed``: one lane per rule,
candidate rules staged in LDS tiles) and the host prints the reference's
three log messages per shadowed rule.

``shadow_table`` lowers a rule list (objects or ``RuleColumns``) to the 32-B
``rsa_shadow_rule`` rows: a port side is one port, ``-1`` (``[NO_PORT]``,
any) or -- for a rule whose side is a list of several ports -- a reference
``<= -2`` into a port array (``ShadowTable.ports``: count, then the ports),
where the kernel tests list containment as ``__contains__`` does
(``firewallrule.py:162-171``).

Address families: IPy answers False for an address of another version
(``firewallrule.py:154,158``), so a rule's ``v4`` byte is a family code --
1 both sides IPv4, ``2 + FAM_SRC6 + FAM_DST6`` (3, 4, 5) for IPv6 sides --
and only rules of one code compare.  IPv6 sides do not fit the kernel's
32-bit ranges; they are rewritten into a 32-bit interval space that keeps
containment exactly (``laminar_codes``: IPy networks are aligned prefixes,
so any two are nested or disjoint and a pre-order numbering of their
nesting tree turns "network a contains b" into "interval a contains b").
"""

import ctypes

import numpy as np

from .py2dict import iteration_order
from .rulecols import FAM_DST6, FAM_SRC6

__all__ = ['SHADOW_DTYPE', 'laminar_codes', 'shadow_table', 'shadowed', 'shadow_messages']

SHADOW_DTYPE = np.dtype([('src_lo', '<u4'), ('src_span', '<u4'), ('dst_lo', '<u4'), ('dst_span', '<u4'),
                         ('sport', '<i4'), ('dport', '<i4'), ('proto', '<u2'), ('action', 'u1'), ('v4', 'u1'),
                         ('reserved', '<u4')])
assert SHADOW_DTYPE.itemsize == 32


class ShadowTable(np.ndarray):
    """rsa_shadow_rule rows with the port array their list sides refer to."""
    ports = None


def _side(ports, arr):
    """One port side: the port (or -1 for [NO_PORT]), or a list reference."""
    if len(ports) == 1:
        return int(ports[0])
    at = len(arr)
    arr.append(len(ports))
    arr.extend(int(p) for p in ports)
    return -(at + 2)


def laminar_codes(nets):
    """{(value, prefix length): (lo, span)} for IPv6 prefix networks: 32-bit
    intervals with a containing b exactly when a's interval holds b's."""
    order = sorted(set(nets))            # ascending network address; at one address the wider prefix first
    out, stack, k = {}, [], 0

    def last(t):
        return t[0] + (1 << (128 - t[1])) - 1

    for t in order:
        while stack and last(stack[-1]) < t[0]:
            u = stack.pop()
            out[u] = (out[u][0], k - 1 - out[u][0])
        out[t] = (k, 0)
        stack.append(t)
        k += 1
    while stack:
        u = stack.pop()
        out[u] = (out[u][0], k - 1 - out[u][0])
    if k > 0xFFFFFFFF:
        raise OverflowError('more than 2^32 distinct IPv6 networks in one list')
    return out


def shadow_table(rules):
    """rsa_shadow_rule rows of a rule list, protocol ids with 0 = 'ip'."""
    n = len(rules)
    out = np.zeros(n, SHADOW_DTYPE).view(ShadowTable)
    out.ports = np.zeros(0, np.int32)
    names = {'ip': 0}
    cols = getattr(rules, 'proto_names', None)
    if cols is not None:                       # rulecols.RuleColumns
        from .ipaddr import IP
        pid = np.array([names.setdefault(nm, len(names)) for nm in rules.proto_names], np.uint16)
        out['proto'] = pid[rules.proto]
        out['action'] = rules.action
        fam = rules.fam
        four = ~fam.astype(bool)
        out['v4'] = np.where(four, 1, 2 + fam)
        for side, bit in (('src', FAM_SRC6), ('dst', FAM_DST6)):
            v4 = (fam & bit) == 0
            ln = getattr(rules, side + '_len').astype(np.int64)
            out[side + '_lo'] = np.where(v4, getattr(rules, side), 0)
            out[side + '_span'] = np.where(v4, (np.int64(1) << (32 - np.where(v4, ln, 32))) - 1, 0).astype(np.uint32)
        if not four.all():
            nets = [IP(t) for t in rules.nets6]
            net = [(int(a.ip), int(a._prefixlen)) for a in nets]
            codes = laminar_codes(net)
            for side, bit in (('src', FAM_SRC6), ('dst', FAM_DST6)):
                for i in np.flatnonzero(fam & bit):
                    out[i][side + '_lo'], out[i][side + '_span'] = codes[net[int(getattr(rules, side)[i])]]
        out['sport'] = rules.sport
        out['dport'] = rules.dport
        return out
    plist = []
    six = {}
    for i, r in enumerate(rules):
        f = (FAM_SRC6 if r.src._ipversion != 4 else 0) | (FAM_DST6 if r.dst._ipversion != 4 else 0)
        out[i]['proto'] = names.setdefault(r.protocol, len(names))
        out[i]['action'] = 1 if r.action == True else 0  # noqa: E712 - the reference compares with !=
        out[i]['v4'] = 2 + f if f else 1
        for side, bit in (('src', FAM_SRC6), ('dst', FAM_DST6)):
            a = getattr(r, side)
            if f & bit:
                six.setdefault((int(a.ip), int(a._prefixlen)), []).append((i, side))
            else:
                out[i][side + '_lo'], out[i][side + '_span'] = a.ip, a.len() - 1
        out[i]['sport'] = _side(r.sport, plist)
        out[i]['dport'] = _side(r.dport, plist)
    if six:
        codes = laminar_codes(list(six))
        for net, uses in six.items():
            for i, side in uses:
                out[i][side + '_lo'], out[i][side + '_span'] = codes[net]
    out.ports = np.array(plist, np.int32)
    return out


def shadowed(engine, table):
    """cover[i] = smallest j < i whose rule contains rule i, or -1 (GPU)."""
    ports = getattr(table, 'ports', None)
    ports = np.ascontiguousarray(ports if ports is not None else np.zeros(0, np.int32), np.int32)
    table = np.ascontiguousarray(np.asarray(table).view(np.ndarray), SHADOW_DTYPE)
    cover = np.empty(len(table), np.int32)
    if len(table):
        engine.ctx.call('rsa_shadowed_ports', table.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(table)),
                        ports.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(ports)),
                        cover.ctypes.data_as(ctypes.c_void_p))
    return cover


def shadow_messages(engine, accesslists, acl_order=None):
    """The reference's logging.info messages (preprosess_access_lists.py:515-517)
    for one firewall's ``accesslists`` ({acl: rule list}), ACLs in Python 2 dict
    order of ``acl_order`` (their first appearance in the config) — default:
    the mapping's own iteration order."""
    names = list(accesslists) if acl_order is None else list(acl_order)
    if acl_order is not None:
        names = [names[k] for k in iteration_order(names)]
    out = []
    for acl in names:
        rules = accesslists[acl]
        cover = shadowed(engine, shadow_table(rules))
        for index in np.nonzero(cover >= 0)[0]:
            index = int(index)
            i = int(cover[index])
            out.append('Found rule which never gets hits since it is covered by a more generic rule above it in '
                       'access-list {0}.'.format(acl))
            out.append('Specific rule ' + str(index) + ': ' + str(rules[index]))
            out.append('Generic rule ' + str(i) + ': ' + str(rules[i]))
    return out

