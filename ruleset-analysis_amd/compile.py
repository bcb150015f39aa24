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

    def index(self, prefix=32):
        """Perfect-hash tuple-space index of the current lists (cached until a list is added)."""
        ent, off = self.packed()
        if getattr(self, '_index', None) is None or self._index[0] is not self._packed or self._index[1] != prefix:
            self._index = (self._packed, prefix, build_index(ent, off, prefix=prefix))
        return self._index[2]

    def ensure_lists(self, protos=('tcp', 'udp')):
        """Pre-build the lists the traffic is expected to need, skipping any the
        mapper would fail on (they are raised lazily at the offending line)."""
        for host, acl in self.groups:
            for p in protos:
                try:
                    self.list_id(host, acl, p)
                except KeyError:
                    pass


# ---- perfect-hash tuple-space index (LDS-resident on the GPU) ----------------------
#
# Per candidate list: entries [0, prefix) are scanned linearly (early exit —
# short first matches never touch the index); entries >= prefix whose address
# ranges are prefixes and whose ports are "any" or one value are grouped by
# shape (src mask, dst mask, port mask).  Each shape owns a CHD perfect-hash
# table (hash-and-displace): key (src & smask, dst & dmask, ports & pmask) ->
# one 32-bit slot word (tag16 << 16 | list-local entry index16, tag = low half of
# the key hash) holding the
# smallest entry index with that key.  Everything else (odd ranges, keys whose
# 32-bit hash collides inside a shape, lists of >= 65535 entries) is residual,
# scanned linearly.  A query takes the minimum candidate index over all shapes;
# the GPU verifies it against the full entry (a 16-bit tag can collide) and
# defers the line to an exact scan when it fails.  First match = min gid, so
# the answer is the linear scan's.
PHT_GROUP_DTYPE = np.dtype([('src_mask', '<u4'), ('dst_mask', '<u4'), ('min_idx', '<u4'), ('n_real', '<u4')] +
                           [(f, '<u4') for c in range(4) for f in ('slot_off%d' % c, 'disp_off%d' % c,
                                                                      'n_slots%d' % c, 'disp_mask%d' % c)])
PHT_LIST_DTYPE = np.dtype([('group_beg', '<u4'), ('group_end', '<u4'), ('resid_beg', '<u4'), ('resid_end', '<u4'),
                           ('prefix', '<u4'), ('reserved0', '<u4'), ('reserved1', '<u4'), ('reserved2', '<u4')])
assert PHT_GROUP_DTYPE.itemsize == 80 and PHT_LIST_DTYPE.itemsize == 32
# the four port classes of a group, probe order: key ports & mask
PORT_CLASSES = (0x00000000, 0xFFFF0000, 0x0000FFFF, 0xFFFFFFFF)    # any, dport, sport, both
M32 = 0xFFFFFFFF
PHT_EMPTY = 0xFFFFFFFF
PHT_MAX_IDX = 0xFFFE
SALT_S, SALT_D, SALT_P = 0x9E3779B9, 0x7F4A7C15, 0x2545F491


def fmix32(x):
    """murmur3 finaliser on uint32 arrays; must equal fmix32() in csrc/ruleset_hip.hip."""
    x = np.asarray(x, dtype=np.uint32).copy()
    with np.errstate(over='ignore'):
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x85EBCA6B)
        x ^= x >> np.uint32(13)
        x *= np.uint32(0xC2B2AE35)
        x ^= x >> np.uint32(16)
    return x


def pht_hash(ks, kd, kp):
    """H of masked keys (csrc: pht_hash)."""
    return fmix32(np.asarray(ks, np.uint32) ^ np.uint32(SALT_S)) ^ fmix32(np.asarray(kd, np.uint32) ^ np.uint32(SALT_D)) \
        ^ fmix32(np.asarray(kp, np.uint32) ^ np.uint32(SALT_P))


def pht_slot(H, d, n_slots):
    """slot = hi32(x * n_slots), x = (H + ((d * ((H >> 16) | 1)) << 16)) mod 2^32.
    The slot depends on the high half of H, the tag is the low half and the
    displacement bucket is (H >> 16) & disp_mask (csrc: pht_probe)."""
    H = np.asarray(H, np.uint64)
    hi = H >> np.uint64(16)
    x = (H + ((np.asarray(d, np.uint64) * (hi | np.uint64(1))) << np.uint64(16))) & np.uint64(M32)
    return ((x * np.uint64(n_slots)) >> np.uint64(32)).astype(np.int64)


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


def _pow2_at_least(x):
    p = 1
    while p < x:
        p <<= 1
    return p


def _chd(H, load=0.9, trials=4096):
    """Hash-and-displace placement of distinct 32-bit hashes H into
    m = ceil(n / load) slots.  Returns (m, disp_mask, disp uint16[r], slot_of_key int64[n])."""
    n = len(H)
    hb = (H >> np.uint32(16)).astype(np.int64)
    m = max(1, int(np.ceil(n / load)))
    r = _pow2_at_least(max(1, (n + 3) // 4))
    while True:
        b = hb & (r - 1)
        order = np.argsort(-np.bincount(b, minlength=r), kind='stable')
        members = [[] for _ in range(r)]
        for k, bb in enumerate(b.tolist()):
            members[bb].append(k)
        used = np.zeros(m, dtype=bool)
        disp = np.zeros(r, dtype=np.uint16)
        slot_of = np.full(n, -1, dtype=np.int64)
        ds = np.arange(trials, dtype=np.uint64)[:, None]
        ok_all = True
        for bb in order.tolist():
            K = members[bb]
            if not K:
                continue
            sl = pht_slot(H[K][None, :], ds, m)                                # trials x |K|
            good = ~used[sl].any(axis=1)
            if len(K) > 1:
                srt = np.sort(sl, axis=1)
                good &= (srt[:, 1:] != srt[:, :-1]).all(axis=1)
            w = np.nonzero(good)[0]
            if len(w) == 0:
                ok_all = False
                break
            d = int(w[0])
            disp[bb] = d
            slot_of[K] = sl[d]
            used[sl[d]] = True
        if ok_all:
            return m, r - 1, disp, slot_of
        m += m // 8 + 1


def build_index(ent, off, prefix=64, min_entries=96):
    """Perfect-hash tuple-space index over packed lists (rsa_load_index arrays).

    Returns (lists PHT_LIST_DTYPE[n_lists], groups PHT_GROUP_DTYPE[], image
    uint32[], resid RULE_DTYPE[]).  A group = one (src mask, dst mask) pair of a
    list with a table per port class (PORT_CLASSES; an absent class points at
    image word 0, an always-empty one-slot table).  A list shorter than
    ``min_entries`` (or of >= 65535 entries) gets no groups: everything after
    its prefix is residual."""
    n_lists = len(off) - 1
    lists = np.zeros(n_lists, dtype=PHT_LIST_DTYPE)
    groups_out, image, resid_parts = [], [np.array([PHT_EMPTY], np.uint32)], []
    n_img = 1
    n_resid = 0
    for L in range(n_lists):
        e = ent[off[L]:off[L + 1]]
        ne = len(e)
        pre = min(prefix, ne)
        lists[L]['prefix'] = pre
        lists[L]['group_beg'] = len(groups_out)
        shapes = {}
        resid_idx = []
        indexable = ne >= min_entries and ne <= PHT_MAX_IDX
        for k in range(pre, ne):
            x = e[k]
            if not indexable:
                resid_idx.append(k)
                continue
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
            g = shapes.setdefault((sm, dm, pm), {})
            if key not in g:                 # entries are gid-ascending: first = min index
                g[key] = k
        by_sd = {}
        for (sm, dm, pm) in shapes:
            by_sd.setdefault((sm, dm), {})[pm] = shapes[(sm, dm, pm)]
        for (sm, dm) in sorted(by_sd):
            rec = [sm, dm, 0xFFFFFFFF, 0]
            for pm in PORT_CLASSES:
                keys = by_sd[(sm, dm)].get(pm)
                if not keys:
                    rec += [0, 0, 1, 0]          # dummy: image word 0 is an empty slot
                    continue
                ks = np.array(list(keys.keys()), dtype=np.uint64).astype(np.uint32).reshape(-1, 3)
                idx = np.array(list(keys.values()), dtype=np.int64)
                H = pht_hash(ks[:, 0], ks[:, 1], ks[:, 2])
                # a full 32-bit hash collision between two keys of one shape: keep the
                # smaller index in the table, the other goes residual (still exact)
                o = np.lexsort((idx, H))
                H, idx = H[o], idx[o]
                dup = np.zeros(len(H), dtype=bool)
                dup[1:] = H[1:] == H[:-1]
                resid_idx.extend(idx[dup].tolist())
                H, idx = H[~dup], idx[~dup]
                nslots, dmask, disp, slot_of = _chd(H)
                nwords_disp = (dmask + 2) // 2
                disp_off = 2 * n_img                               # in uint16 units
                dwords = np.zeros(nwords_disp * 2, dtype=np.uint16)
                dwords[:dmask + 1] = disp
                image.append(dwords.view(np.uint32))
                n_img += nwords_disp
                slots = np.full(nslots, PHT_EMPTY, dtype=np.uint32)
                slots[slot_of] = ((H & np.uint32(0xFFFF)).astype(np.uint32) << np.uint32(16)) | idx.astype(np.uint32)
                rec += [n_img, disp_off, nslots, dmask]
                rec[2] = min(rec[2], int(idx.min()))
                rec[3] += 1
                image.append(slots)
                n_img += nslots
            groups_out.append(tuple(rec))
        lists[L]['group_end'] = len(groups_out)
        resid_idx = sorted(resid_idx)
        lists[L]['resid_beg'] = n_resid
        resid_parts.append(e[resid_idx])
        n_resid += len(resid_idx)
        lists[L]['resid_end'] = n_resid
    grp = np.array(groups_out, dtype=PHT_GROUP_DTYPE) if groups_out else np.zeros(0, PHT_GROUP_DTYPE)
    img = np.concatenate(image)
    resid = np.concatenate(resid_parts) if resid_parts else np.zeros(0, RULE_DTYPE)
    return lists, grp, img, resid


def pht_lookup(index, ent, off, L, src, dst, ports):
    """Host model of the GPU classifier for one tuple (tests): the first-match
    list-local index, -1, or 'defer'.  Follows the device order exactly: prefix
    scan, min candidate over the groups' port-class probes, verification,
    residual scan."""
    lists, grp, img, resid = index
    h = lists[L]
    e = ent[off[L]:off[L + 1]]

    def match(x):
        pl, ps = int(x['port_lo']), int(x['port_span'])
        return ((src - int(x['src_lo'])) & M32) <= int(x['src_span']) and \
            ((dst - int(x['dst_lo'])) & M32) <= int(x['dst_span']) and \
            ((ports & 0xFFFF) - (pl & 0xFFFF)) & 0xFFFF <= (ps & 0xFFFF) and \
            ((ports >> 16) - (pl >> 16)) & 0xFFFF <= (ps >> 16)
    for k in range(int(h['prefix'])):
        if match(e[k]):
            return k
    cand = 0xFFFF
    d16 = img.view(np.uint16)
    for g in grp[int(h['group_beg']):int(h['group_end'])]:
        for c, pm in enumerate(PORT_CLASSES):
            H = int(pht_hash(src & int(g['src_mask']), dst & int(g['dst_mask']), ports & pm))
            tag = H & 0xFFFF
            d = int(d16[int(g['disp_off%d' % c]) + ((H >> 16) & int(g['disp_mask%d' % c]))])
            slot = int(pht_slot(H, d, int(g['n_slots%d' % c])))
            w = int(img[int(g['slot_off%d' % c]) + slot])
            if (w >> 16) == tag:
                cand = min(cand, w & 0xFFFF)
    best = None
    if cand != 0xFFFF:
        if not match(e[cand]):
            return 'defer'
        best = cand
    gid_best = int(e[best]['gid']) if best is not None else None
    for x in resid[int(h['resid_beg']):int(h['resid_end'])]:
        if gid_best is not None and int(x['gid']) >= gid_best:
            break
        if match(x):
            return int(np.searchsorted(e['gid'], x['gid']))
    return -1 if best is None else best
