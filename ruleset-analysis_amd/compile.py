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

    def index(self):
        """Tuple-space-search index of the current lists (cached until a list is added)."""
        if getattr(self, '_index', None) is None or self._index[0] is not self._packed:
            ent, off = self.packed()
            self._index = (self._packed, build_index(ent, off))
        return self._index[1]

    def ensure_lists(self, protos=('tcp', 'udp')):
        """Pre-build the lists the traffic is expected to need, skipping any the
        mapper would fail on (they are raised lazily at the offending line)."""
        for host, acl in self.groups:
            for p in protos:
                try:
                    self.list_id(host, acl, p)
                except KeyError:
                    pass


# ---- tuple-space-search index ------------------------------------------------------
SHAPE_DTYPE = np.dtype([('src_mask', '<u4'), ('dst_mask', '<u4'), ('port_mask', '<u4'), ('min_gid', '<u4'),
                        ('table_off', '<u4'), ('table_mask', '<u4'), ('salt', '<u4'), ('reserved', '<u4')])
ISLOT_DTYPE = np.dtype([('src', '<u4'), ('dst', '<u4'), ('ports', '<u4'), ('gid', '<u4')])
assert SHAPE_DTYPE.itemsize == 32 and ISLOT_DTYPE.itemsize == 16
M32 = 0xFFFFFFFF


def index_hash(s, d, p, salt):
    """Must equal index_hash() in csrc/ruleset_hip.hip (uint32 arithmetic)."""
    s, d, p, salt = (np.asarray(x, dtype=np.uint32) for x in (s, d, p, salt))
    with np.errstate(over='ignore'):
        h = (s * np.uint32(0x9E3779B1)) ^ (d * np.uint32(0x85EBCA77)) ^ (p * np.uint32(0xC2B2AE3D)) ^ \
            (salt * np.uint32(0x27D4EB2F))
        h ^= h >> np.uint32(15)
        h *= np.uint32(0x2C1B3C6D)
        h ^= h >> np.uint32(12)
        h *= np.uint32(0x297A2D39)
        h ^= h >> np.uint32(15)
    return h


def _prefix_mask(lo, span):
    """32-bit mask if [lo, lo+span] is an aligned prefix block, else None."""
    size = int(span) + 1
    if size & (size - 1) or int(lo) % size:
        return None
    return (M32 ^ (size - 1)) & M32


def _port_mask(lo, span):
    if lo == 0 and span == 0xFFFF:
        return 0
    if span == 0:
        return 0xFFFF
    return None


def build_index(ent, off, probe_cost=8):
    """Tuple-space-search index over packed lists (rsa_load_index arrays).

    Returns (shapes, shape_off, slots, resid, resid_off).  Per list, the index is
    used only when it is cheaper than scanning (n_shapes * probe_cost + residual
    < entries); otherwise every entry of the list stays residual (a plain scan)."""
    shapes, shape_off, slot_parts, resid_parts, resid_off = [], [0], [], [], [0]
    n_slots = 0
    salt = 1
    for L in range(len(off) - 1):
        e = ent[off[L]:off[L + 1]]
        groups = {}
        resid_idx = []
        for k in range(len(e)):
            x = e[k]
            sm = _prefix_mask(x['src_lo'], x['src_span'])
            dm = _prefix_mask(x['dst_lo'], x['dst_span'])
            pl, ps = int(x['port_lo']), int(x['port_span'])
            spm = _port_mask(pl & 0xFFFF, ps & 0xFFFF)
            dpm = _port_mask(pl >> 16, ps >> 16)
            if sm is None or dm is None or spm is None or dpm is None:
                resid_idx.append(k)
                continue
            pm = spm | (dpm << 16)
            key = (int(x['src_lo']), int(x['dst_lo']), pl & pm)
            g = groups.setdefault((sm, dm, pm), {})
            if key not in g:                 # entries are gid-ascending: first = min gid
                g[key] = int(x['gid'])
        use_index = len(groups) * probe_cost + len(resid_idx) < len(e)
        if not use_index:
            resid_parts.append(e)
            resid_off.append(resid_off[-1] + len(e))
            shape_off.append(shape_off[-1])
            continue
        resid_parts.append(e[resid_idx])
        resid_off.append(resid_off[-1] + len(resid_idx))
        order = sorted(groups.items(), key=lambda kv: min(kv[1].values()))
        for (sm, dm, pm), keys in order:
            size = 2
            while size < 2 * len(keys):
                size <<= 1
            tab = np.zeros(size, dtype=ISLOT_DTYPE)
            tab['gid'] = M32
            ks = np.array(list(keys.keys()), dtype=np.uint64).astype(np.uint32).reshape(-1, 3)
            gs = np.array(list(keys.values()), dtype=np.uint32)
            hs = index_hash(ks[:, 0], ks[:, 1], ks[:, 2], salt) & np.uint32(size - 1)
            for (a, b, c), g, h in zip(ks.tolist(), gs.tolist(), hs.tolist()):
                while tab['gid'][h] != M32:
                    h = (h + 1) & (size - 1)
                tab[h] = (a, b, c, g)
            shapes.append((sm, dm, pm, min(keys.values()), n_slots, size - 1, salt, 0))
            slot_parts.append(tab)
            n_slots += size
            salt += 1
        shape_off.append(len(shapes))
    shp = np.array(shapes, dtype=SHAPE_DTYPE) if shapes else np.zeros(0, SHAPE_DTYPE)
    slots = np.concatenate(slot_parts) if slot_parts else np.zeros(0, ISLOT_DTYPE)
    resid = np.concatenate(resid_parts) if resid_parts else np.zeros(0, RULE_DTYPE)
    return (shp, np.array(shape_off, np.uint32), slots, resid, np.array(resid_off, np.uint32))
