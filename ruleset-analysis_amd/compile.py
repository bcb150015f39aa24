"""Compile ``accesslists.db`` into the packed tables the HIP kernels scan.

* Global rule ids (gid): every (host, acl) gets a contiguous gid range in
  sorted (host, acl) order; ``gid = base + i`` for the rule at list position
  ``i`` — the index the mapper prints (``mapper.py:168,184``; SURVEY.md trap 9).
* Candidate lists: one per (host, acl, protocol) that the traffic can ask for,
  built exactly as ``mapper.py:159-166`` builds them per line (tcp/udp:
  ``sorted(protocols[p] + protocols['ip'])``, or ``protocols['ip']`` when ``p``
  has no list; anything else: ``protocols[p]``; a missing key raises the same
  ``KeyError`` the mapper would die with).  Entries are then filtered by the
  parts of ``FirewallRule.__contains__`` (``firewallrule.py:128-174``) that do
  not depend on the connection: a deny rule never contains a logged connection
  (whose action is always permit, ``mapper.py:134``), a rule whose protocol is
  neither ``'ip'`` nor ``p`` never matches, an IPv6 network never contains an
  IPv4 host, and a port list with no value in 0..65535 never matches.  What is
  left is lowered to integer ranges; a port list that is not one contiguous
  range becomes several entries with the same gid (first match = min gid, so
  the result is unchanged).
"""

import numpy as np

from .firewallrule import FirewallRule

__all__ = ['RULE_DTYPE', 'TUPLE_DTYPE', 'RECORD_DTYPE', 'CompiledRules']

RULE_DTYPE = np.dtype([('src_lo', '<u4'), ('src_span', '<u4'), ('dst_lo', '<u4'), ('dst_span', '<u4'),
                       ('port_lo', '<u4'), ('port_span', '<u4'), ('gid', '<u4'), ('reserved', '<u4')])
TUPLE_DTYPE = np.dtype([('src', '<u4'), ('dst', '<u4'), ('sport', '<u2'), ('dport', '<u2'), ('list', '<u2'),
                        ('flags', 'u1'), ('pspell', 'u1')])
RECORD_DTYPE = np.dtype([('min_order', '<u8'), ('gid', '<u4'), ('for_ip', '<u4'), ('to_ip', '<u4'),
                         ('to_port', '<u2'), ('pspell', 'u1'), ('pad', 'u1'), ('count', '<u4'), ('first', '<u4'),
                         ('last', '<u4'), ('pad2', '<u4')])
assert RULE_DTYPE.itemsize == 32 and TUPLE_DTYPE.itemsize == 16 and RECORD_DTYPE.itemsize == 40

F_VALID, F_HIT, F_BUILT, F_SWAP = 0x01, 0x02, 0x04, 0x08
MAX_LISTS = 65536


def _port_ranges(ports):
    """FirewallRule port list -> list of inclusive (lo, hi) in 0..65535, or None for 'no check'."""
    if ports == [FirewallRule.NO_PORT]:
        return None
    vals = sorted({int(p) for p in ports if 0 <= int(p) <= 65535})
    out = []
    for v in vals:
        if out and v == out[-1][1] + 1:
            out[-1][1] = v
        else:
            out.append([v, v])
    return [tuple(r) for r in out]


def _addr_range(ip):
    """(lo, span) for an IPv4 network, None for IPv6 (never contains an IPv4 tuple)."""
    if ip._ipversion != 4:
        return None
    size = ip.len()
    return ip.ip, size - 1


def candidate_indices(protocols, proto):
    """mapper.py:159-166, including its KeyError behaviour."""
    if proto in ('tcp', 'udp'):
        if proto in protocols:
            return sorted(protocols[proto] + protocols['ip'])
        return protocols['ip']
    return protocols[proto]


class CompiledRules(object):
    def __init__(self, db):
        self.db = db
        self.groups = []       # [(host, acl)] in gid order
        self.base = {}
        gid = 0
        for host in sorted(db.accesslists):
            for acl in sorted(db.accesslists[host]):
                self.groups.append((host, acl))
                self.base[(host, acl)] = gid
                gid += len(db.accesslists[host][acl]['rules'])
        self.n_rules = gid
        self._group_start = np.array([self.base[g] for g in self.groups] + [gid], dtype=np.int64)
        self.list_ids = {}
        self.list_keys = []
        self._lists = []
        self._packed = None

    # ---- gid <-> (host, acl, index) -------------------------------------------
    def locate(self, gid):
        g = int(np.searchsorted(self._group_start, gid, side='right') - 1)
        host, acl = self.groups[g]
        return host, acl, int(gid - self._group_start[g])

    def rule(self, gid):
        host, acl, i = self.locate(gid)
        return self.db.accesslists[host][acl]['rules'][i]

    def key(self, gid):
        host, acl, i = self.locate(gid)
        return '%s;%s;%d' % (host, acl, i)

    # ---- candidate lists ------------------------------------------------------
    def list_id(self, host, acl, proto):
        k = (host, acl, proto)
        lid = self.list_ids.get(k)
        if lid is not None:
            return lid
        entry = self.db.accesslists[host][acl]
        idxs = candidate_indices(entry['protocols'], proto)
        rows = self._lower(entry['rules'], idxs, proto, self.base[(host, acl)])
        if len(self._lists) >= MAX_LISTS:
            raise OverflowError('more than %d (host, acl, protocol) candidate lists' % MAX_LISTS)
        lid = len(self._lists)
        self._lists.append(rows)
        self.list_ids[k] = lid
        self.list_keys.append(k)
        self._packed = None
        return lid

    @staticmethod
    def _lower(rules, idxs, proto, base):
        rows = []
        seen = set()
        for i in idxs:
            rule = rules[i]
            if i in seen:          # duplicate index in the list: same rule, same answer
                continue
            seen.add(i)
            if rule.action is not True and rule.action != True:  # noqa: E712 - reference compares with ==
                continue
            if rule.protocol != 'ip' and rule.protocol != proto:
                continue
            s = _addr_range(rule.src)
            d = _addr_range(rule.dst)
            if s is None or d is None:
                continue
            sps = _port_ranges(rule.sport)
            dps = _port_ranges(rule.dport)
            if sps == [] or dps == []:
                continue
            for slo, shi in (sps or [(0, 65535)]):
                for dlo, dhi in (dps or [(0, 65535)]):
                    rows.append((s[0], s[1], d[0], d[1], slo | (dlo << 16), (shi - slo) | ((dhi - dlo) << 16),
                                 base + i, 0))
        return rows

    def packed(self):
        """(entries RULE_DTYPE array, offsets uint32 array of n_lists+1)."""
        if self._packed is None:
            total = sum(len(r) for r in self._lists)
            ent = np.zeros(total, dtype=RULE_DTYPE)
            off = np.zeros(len(self._lists) + 1, dtype=np.uint32)
            k = 0
            for li, rows in enumerate(self._lists):
                if rows:
                    arr = np.array(rows, dtype=np.uint64)
                    for j, name in enumerate(RULE_DTYPE.names):
                        ent[name][k:k + len(rows)] = arr[:, j]
                k += len(rows)
                off[li + 1] = k
            self._packed = (ent, off)
        return self._packed

    def n_lists(self):
        return len(self._lists)

    def ensure_lists(self, protos=('tcp', 'udp')):
        """Pre-build the lists the traffic is expected to need, skipping any the
        mapper would fail on (they are raised lazily at the offending line)."""
        for host, acl in self.groups:
            for p in protos:
                try:
                    self.list_id(host, acl, p)
                except KeyError:
                    pass
