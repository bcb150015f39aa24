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
"""

import ctypes

import numpy as np

from .py2dict import iteration_order

__all__ = ['SHADOW_DTYPE', 'shadow_table', 'shadowed', 'shadow_messages']

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


def shadow_table(rules):
    """rsa_shadow_rule rows of a rule list, protocol ids with 0 = 'ip'."""
    n = len(rules)
    out = np.zeros(n, SHADOW_DTYPE).view(ShadowTable)
    out.ports = np.zeros(0, np.int32)
    names = {'ip': 0}
    cols = getattr(rules, 'proto_names', None)
    if cols is not None:                       # rulecols.RuleColumns
        pid = np.array([names.setdefault(nm, len(names)) for nm in rules.proto_names], np.uint16)
        out['proto'] = pid[rules.proto]
        out['action'] = rules.action
        out['v4'] = 1
        out['src_lo'] = rules.src
        out['src_span'] = ((np.int64(1) << (32 - rules.src_len.astype(np.int64))) - 1).astype(np.uint32)
        out['dst_lo'] = rules.dst
        out['dst_span'] = ((np.int64(1) << (32 - rules.dst_len.astype(np.int64))) - 1).astype(np.uint32)
        out['sport'] = rules.sport
        out['dport'] = rules.dport
        return out
    plist = []
    for i, r in enumerate(rules):
        v4 = r.src._ipversion == 4 and r.dst._ipversion == 4
        out[i]['proto'] = names.setdefault(r.protocol, len(names))
        out[i]['action'] = 1 if r.action == True else 0  # noqa: E712 - the reference compares with !=
        out[i]['v4'] = 1 if v4 else 0
        if v4:
            out[i]['src_lo'], out[i]['src_span'] = r.src.ip, r.src.len() - 1
            out[i]['dst_lo'], out[i]['dst_span'] = r.dst.ip, r.dst.len() - 1
        out[i]['sport'] = _side(r.sport, plist)
        out[i]['dport'] = _side(r.dport, plist)
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

