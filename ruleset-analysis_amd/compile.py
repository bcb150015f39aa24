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
                       ('port_lo', '<u4'), ('port_span', '<u4'), ('gid', '<u4'), ('step', '<u4')])
STEP_SPORT = 0x80000000     # rsa_rule_entry.step: the run varies the source port (else the destination port)
RUN_MIN = 16                # shorter runs stay single-port entries (the hashed index takes those)
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


def _oor_side(ports, value):
    """A rule side against a connection port past 65535: None ('no check') if
    the side is NO_PORT or names the value, else [] (never matches)."""
    if ports == [FirewallRule.NO_PORT] or value in ports:
        return None
    return []


def _addr_range(ip):
    """(lo, span) for an IPv4 network, None for IPv6 (never contains an IPv4 tuple)."""
    if ip._ipversion != 4:
        return None
    size = ip.len()
    return ip.ip, size - 1


def candidate_indices(protocols, proto):
    """mapper.py:159-166, including its KeyError behaviour (index lists may be
    Python lists or, for columnar rule stores, integer arrays)."""
    if proto in ('tcp', 'udp'):
        if proto in protocols:
            a, b = protocols[proto], protocols['ip']
            if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
                return np.sort(np.concatenate([np.asarray(a, np.int64), np.asarray(b, np.int64)]), kind='stable')
            return sorted(a + b)
        return protocols['ip']
    return protocols[proto]


def compress_runs(rows, min_run=RUN_MIN):
    """Collapse runs of single-port entries into stepped range entries (module
    docstring).  ``rows``: RULE_DTYPE entries of one candidate list in
    ascending gid order; returns the compressed list, ascending first gid."""
    if len(rows) < min_run:
        return rows
    out = rows
    for dim in (1, 0):                     # destination-port runs first, then source-port runs
        out = _compress_dim(out, dim, min_run)
    return out


def _compress_dim(rows, dim, min_run):
    n = len(rows)
    pl = rows['port_lo'].astype(np.int64)
    ps = rows['port_span'].astype(np.int64)
    shift = 16 if dim else 0
    port = (pl >> shift) & 0xFFFF
    single = ((ps >> shift) & 0xFFFF) == 0
    other_lo = (pl >> (16 - shift)) & 0xFFFF
    other_span = (ps >> (16 - shift)) & 0xFFFF
    cand = single & (rows['step'] == 0)
    if cand.sum() < min_run:
        return rows
    gid = rows['gid'].astype(np.int64)
    # class = everything but the varying port; within a class, gid order
    o = np.lexsort((gid, other_span, other_lo, rows['dst_span'], rows['dst_lo'], rows['src_span'], rows['src_lo'],
                    ~cand))
    o = o[cand[o]]
    k = len(o)
    same = np.zeros(k, bool)
    if k > 1:
        a, b = o[:-1], o[1:]
        same[1:] = ((rows['src_lo'][a] == rows['src_lo'][b]) & (rows['src_span'][a] == rows['src_span'][b])
                    & (rows['dst_lo'][a] == rows['dst_lo'][b]) & (rows['dst_span'][a] == rows['dst_span'][b])
                    & (other_lo[a] == other_lo[b]) & (other_span[a] == other_span[b]))
    d = np.zeros(k, np.int64)
    d[1:] = gid[o[1:]] - gid[o[:-1]]
    link = np.zeros(k, bool)
    link[1:] = same[1:] & (port[o[1:]] == port[o[:-1]] + 1) & (d[1:] > 0)
    prev = np.zeros(k, bool)
    prev[1:] = link[:-1]
    brk = ~link | (prev & (d != np.roll(d, 1)))
    run = np.cumsum(brk) - 1
    n_runs = int(run[-1]) + 1 if k else 0
    length = np.bincount(run, minlength=n_runs)
    start = np.flatnonzero(brk)
    long_run = length >= min_run
    if not long_run.any():
        return rows
    keep = np.ones(n, bool)
    members = o[long_run[run]]
    keep[members] = False
    heads = o[start[long_run]]
    new = rows[heads].copy()
    span = (length[long_run] - 1).astype(np.int64)
    stride = d[start[long_run] + 1]
    if dim:
        new['port_span'] = (rows['port_span'][heads].astype(np.int64) & 0xFFFF) | (span << 16)
        new['step'] = stride.astype(np.uint32)
    else:
        new['port_span'] = (rows['port_span'][heads].astype(np.int64) & 0xFFFF0000) | span
        new['step'] = (stride | STEP_SPORT).astype(np.uint32)
    assert (stride > 0).all() and (stride < STEP_SPORT).all()
    out = np.concatenate([rows[keep], new])
    return out[np.argsort(out['gid'], kind='stable')]


def entry_gid(e, sport, dport):
    """gid an entry assigns to a connection it matches (host model of the device)."""
    st = int(e['step'])
    if st == 0:
        return int(e['gid'])
    if st & STEP_SPORT:
        return int(e['gid']) + (sport - (int(e['port_lo']) & 0xFFFF)) * (st & ~STEP_SPORT)
    return int(e['gid']) + (dport - (int(e['port_lo']) >> 16)) * st


class CompiledRules(object):
    def __init__(self, db, run_min=RUN_MIN):
        self.db = db
        self.run_min = run_min           # 0: no run compression (every expanded rule its own entry)
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
        if self.run_min:
            rows = compress_runs(rows, self.run_min)
        return self._add_list(k, rows)

    def list_id_oor(self, host, acl, proto, sport=None, dport=None):
        """Candidate list of a connection whose source and/or destination port
        is past 65535: the mapper builds the ``Connection`` from ``int()`` of
        the log's digits with no range check (``mapper.py:139``,
        ``firewallrule.py:47-53``), and a rule side with ports contains it only
        if that value is in its list (``:162-171``) while a NO_PORT side always
        does.  ``sport``/``dport``: the out-of-range values (None for a side in
        range).  The derived list keeps the entries whose out-of-range sides
        can match, widened to any port there; the line's tuple carries port 0
        on such a side.  Values no rule of the list names share one list."""
        if sport is None and dport is None:
            return self.list_id(host, acl, proto)
        entry = self.db.accesslists[host][acl]
        idxs = candidate_indices(entry['protocols'], proto)        # mapper.py:159-166 KeyError first
        named = self._named_oor(host, acl)
        fold = lambda v: None if v is None else (v if v in named else -2)
        k = (host, acl, proto, fold(sport), fold(dport))
        lid = self.list_ids.get(k)
        if lid is not None:
            return lid
        rows = self._lower(entry['rules'], idxs, proto, self.base[(host, acl)], oor=(sport, dport))
        if self.run_min:
            rows = compress_runs(rows, self.run_min)
        return self._add_list(k, rows)

    def _named_oor(self, host, acl):
        """Port values past 65535 that rules of (host, acl) name."""
        cache = self.__dict__.setdefault('_oor_named', {})
        got = cache.get((host, acl))
        if got is None:
            rules = self.db.accesslists[host][acl]['rules']
            if hasattr(rules, 'sport') and hasattr(rules, 'lower'):
                got = {int(v) for col in (rules.sport, rules.dport) for v in np.unique(col) if v > 65535}
            else:
                got = {int(p) for r in rules for p in list(r.sport) + list(r.dport) if p > 65535}
            cache[(host, acl)] = got
        return got

    def _add_list(self, k, rows):
        if len(self._lists) >= MAX_LISTS:
            raise OverflowError('more than %d (host, acl, protocol) candidate lists' % MAX_LISTS)
        lid = len(self._lists)
        self._lists.append(rows)
        self.list_ids[k] = lid
        self.list_keys.append(k)
        self._packed = None
        return lid

    @staticmethod
    def _lower(rules, idxs, proto, base, oor=(None, None)):
        lower_cols = getattr(rules, 'lower', None)
        if lower_cols is not None:          # columnar rule store (rulecols.RuleColumns)
            return lower_cols(idxs, proto, base, oor=oor)
        rows = []
        seen = set()
        for i in idxs:
            i = int(i)
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
            sps = _port_ranges(rule.sport) if oor[0] is None else _oor_side(rule.sport, oor[0])
            dps = _port_ranges(rule.dport) if oor[1] is None else _oor_side(rule.dport, oor[1])
            if sps == [] or dps == []:
                continue
            for slo, shi in (sps or [(0, 65535)]):
                for dlo, dhi in (dps or [(0, 65535)]):
                    rows.append((s[0], s[1], d[0], d[1], slo | (dlo << 16), (shi - slo) | ((dhi - dlo) << 16),
                                 base + i, 0))
        out = np.zeros(len(rows), dtype=RULE_DTYPE)
        if rows:
            arr = np.array(rows, dtype=np.uint64)
            for j, name in enumerate(RULE_DTYPE.names):
                out[name] = arr[:, j]
        return out

    def packed(self):
        """(entries RULE_DTYPE array, offsets uint32 array of n_lists+1)."""
        if self._packed is None:
            ent = np.concatenate(self._lists) if self._lists else np.zeros(0, RULE_DTYPE)
            off = np.zeros(len(self._lists) + 1, dtype=np.uint32)
            off[1:] = np.cumsum([len(r) for r in self._lists])
            self._packed = (ent, off)
        return self._packed

    def n_lists(self):
        return len(self._lists)

    def index(self, prefix=0, chunk=None, kind='auto'):
        """Index of the current lists (cached until a list is added): ``kind``
        'pht' = the pruned perfect-hash tuple-space index (build_index, RSA4),
        'bucket' / 'bucket-filtered' = the partial-key bucket index
        (bucketindex.py, image RSA5) without / with LDS row filters, 'auto'
        (default) = pht while its image fits the LDS of two classifier
        workgroups per CU (AUTO_PHT_MAX_WORDS), else bucket -- from global
        memory the bucket index's fewer dependent reads win (cfg4: 0.96 vs 4.48
        ms per classification launch; at 10k rules in LDS pht 0.90 vs 1.06);
        ``chunk``: entries per chained record (default PHT_CHUNK)."""
        ent, off = self.packed()
        chunk = chunk or PHT_CHUNK
        if kind == 'auto':
            pht = self.index(prefix, chunk, 'pht')
            if len(pht[0]) <= AUTO_PHT_MAX_WORDS:
                return pht
            kind = 'bucket'
        key = (prefix, chunk, kind)
        if getattr(self, '_index', None) is None or self._index[0] is not self._packed or self._index[1] != key:
            if kind in ('bucket', 'bucket-filtered'):
                from .bucketindex import build_bucket_index
                built = build_bucket_index(ent, off, prefix=prefix, chunk=chunk, filters=kind == 'bucket-filtered')
            elif kind == 'pht':
                built = build_index(ent, off, prefix=prefix, chunk=chunk)
            else:
                raise ValueError('index kind must be bucket or pht')
            self._index = (self._packed, key, built)
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


# ---- pruned perfect-hash tuple-space index (LDS-resident on the GPU) -----------------
#
# Per candidate list: entries [0, prefix) are scanned linearly (early exit —
# short first matches never touch the index).  Entries >= prefix whose address
# ranges are prefixes and whose ports are "any" or one value are grouped by
# (src mask, dst mask); inside a group, by port class (PORT_CLASSES).  Each
# (group, class) owns a CHD perfect-hash table (hash-and-displace): key
# (src & smask, dst & dmask, ports & pmask) -> one 32-bit slot word
# (tag16 << 16 | list-local entry index16, tag = low half of the key hash)
# holding the smallest entry index with that key.  Groups are sorted by their
# smallest entry index and at most PHT_MAX_GROUPS are indexed per list.
#
# Pruning: per distinct non-zero src mask m of a list, a CHD table maps the
# prefix (src & m) to a bitmap of the groups with src mask m that hold a rule
# on that prefix (groups with src mask 0 are always candidates); likewise for
# dst masks.  A lane probes only the groups in (src bitmap & dst bitmap), in
# ascending min-index order, and stops at the first group whose smallest index
# cannot beat its best candidate.  A 16-bit tag can collide, so the GPU
# verifies the minimum candidate against the full entry; on a failure it
# repeats the probes above that candidate (a false bitmap bit only costs a
# probe).  Everything else (odd ranges, keys whose 32-bit hash collides inside
# a table, groups past the limit, lists of >= 65535 entries) is residual,
# scanned linearly.  First match = min gid, so the answer is the linear scan's.
#
# A list longer than PHT_CHUNK entries (slot values are 16-bit list-local
# indices) is indexed as a chain of records, one per chunk of PHT_CHUNK
# entries: a lane probes chunk k+1 only while its best candidate exceeds the
# smallest gid of chunk k+1 (entries are in ascending first-gid order).
#
# Everything lives in ONE uint32 image (include/ruleset_hip.h, rsa_load_index):
#   [0] 0xFFFFFFFF (the empty slot)  [1] PHT_MAGIC  [2] n_lists  [3] list_off
#   [4] n_records (>= n_lists: records n_lists.. are chained chunks)  [5..7] 0
#   list records (PHT_LIST_WORDS each), group records, mask records, bitmaps
#   (uint64, lo word first), CHD displacements (uint16) and slot words.
PHT_MAGIC = 0x34415352              # 'RSA4'
AUTO_PHT_MAX_WORDS = 19456          # csrc kImgSmallMax: the image of two 1024-thread classifier workgroups per CU
PHT_LIST_WORDS, PHT_GROUP_WORDS, PHT_MASK_WORDS = 20, 20, 4
PHT_HEADER_WORDS = 8
PHT_CHUNK = 0xF000                  # entries per chained record: a table never needs > 2^16 slots
PHT_MAX_GROUPS = 64
PHT_ATTEMPTS = 4                    # verification failures before a line is deferred
# the four port classes of a group, probe order: key ports & mask
PORT_CLASSES = (0x00000000, 0xFFFF0000, 0x0000FFFF, 0xFFFFFFFF)    # any, dport, sport, both
M32 = 0xFFFFFFFF
PHT_EMPTY = 0xFFFFFFFF
PHT_NONE = 0xFFFF
PHT_MAX_IDX = 0xFFFE
PHT_MAX_SLOTS = 0x10000              # slot index * n_slots must fit the 24-bit multiplier
MASK_NARROW = 0x80000000            # pruning record word 1: 16-bit slots (offset in uint16 units)
HDR_ALL_NARROW = 0x2                # image word 5: every pruning table has 16-bit slots
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
    """H of a group key (csrc: index_candidate)."""
    return fmix32(np.asarray(ks, np.uint32) ^ np.uint32(SALT_S)) ^ fmix32(np.asarray(kd, np.uint32) ^ np.uint32(SALT_D)) \
        ^ fmix32(np.asarray(kp, np.uint32) ^ np.uint32(SALT_P))


def field_hash(k, side):
    """H of a pruning key: one address field (side 0 src, 1 dst)."""
    return fmix32(np.asarray(k, np.uint32) ^ np.uint32(SALT_D if side else SALT_S))


def pht_slot(H, d, n_slots):
    """slot = (x * n_slots) >> 16, x = (H + d * step) mod 2^16, step = (H >> 16) | 1
    (16 bits).  The displacement bucket is (H >> 16) & disp_mask and the tag
    the low half of H.  Every product fits 24-bit multiplier operands (d and
    step < 2^16, x < 2^16, n_slots <= 2^16), so the device uses full-rate
    v_mad_u32_u24 / v_mul_u32_u24 (csrc: pht_slot); keys of one bucket differ
    in their step's bits above the bucket bits or in their low half, so they
    separate as d grows."""
    H = np.asarray(H, np.uint64)
    step = ((H >> np.uint64(16)) | np.uint64(1)) & np.uint64(0xFFFF)
    x = (H + np.asarray(d, np.uint64) * step) & np.uint64(0xFFFF)
    return ((x * np.uint64(n_slots)) >> np.uint64(16)).astype(np.int64)


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


def _chd(H, load=0.98, trials=4096):
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
        if m < PHT_MAX_SLOTS:
            m = min(PHT_MAX_SLOTS, m + m // 8 + 1)
        elif trials < 0x10000:
            trials *= 4
        else:
            raise OverflowError('CHD placement failed for %d keys' % n)


class _Image(object):
    """Append-only uint32 image; chunks stay mutable until build()."""

    def __init__(self):
        self.chunks = [np.array([PHT_EMPTY, PHT_MAGIC, 0, 0, 0, 0, 0, 0], dtype=np.uint32)]
        self.n = PHT_HEADER_WORDS
        self.all_narrow = True      # header word 5 bit 1: every pruning table has 16-bit slots

    def alloc(self, arr, align=1):
        pad = (-self.n) % align
        if pad:
            self.chunks.append(np.zeros(pad, dtype=np.uint32))
            self.n += pad
        arr = np.ascontiguousarray(arr, dtype=np.uint32)
        off = self.n
        self.chunks.append(arr)
        self.n += len(arr)
        return off, arr

    def table(self, H, vals):
        """CHD table of distinct hashes H -> 16-bit values; returns (slot_off, disp_off, n_slots, disp_mask)."""
        nslots, dmask, disp, slot_of = _chd(H)
        dwords = np.zeros(((dmask + 2) // 2) * 2, dtype=np.uint16)
        dwords[:dmask + 1] = disp
        doff, _ = self.alloc(dwords.view(np.uint32))
        slots = np.full(nslots, PHT_EMPTY, dtype=np.uint32)
        slots[slot_of] = ((H.astype(np.uint32) & np.uint32(0xFFFF)) << np.uint32(16)) | np.asarray(vals, np.uint32)
        soff, _ = self.alloc(slots)
        return (soff, 2 * doff, nslots, dmask)

    def table16(self, H, vals):
        """Pruning CHD table with 16-bit slots (8-bit tag << 8 | 8-bit value,
        values 1..255; 0 = empty, which reads as value 0 = the empty bitmap);
        offsets in uint16 units of the image."""
        nslots, dmask, disp, slot_of = _chd(H)
        dwords = np.zeros(((dmask + 2) // 2) * 2, dtype=np.uint16)
        dwords[:dmask + 1] = disp
        doff, _ = self.alloc(dwords.view(np.uint32))
        slots = np.zeros(nslots + (nslots & 1), dtype=np.uint16)
        slots[slot_of] = ((H.astype(np.uint32) & np.uint32(0xFF)) << np.uint32(8)).astype(np.uint16) | \
            np.asarray(vals, np.uint16)
        soff, _ = self.alloc(slots.view(np.uint32))
        return (2 * soff, 2 * doff, nslots, dmask)

    def table_prune(self, H, vals):
        """Pruning CHD table with 32-bit slots (16-bit tag << 16 | value, 0 =
        empty = value 0, the empty bitmap)."""
        nslots, dmask, disp, slot_of = _chd(H)
        dwords = np.zeros(((dmask + 2) // 2) * 2, dtype=np.uint16)
        dwords[:dmask + 1] = disp
        doff, _ = self.alloc(dwords.view(np.uint32))
        slots = np.zeros(nslots, dtype=np.uint32)
        slots[slot_of] = ((H.astype(np.uint32) & np.uint32(0xFFFF)) << np.uint32(16)) | np.asarray(vals, np.uint32)
        soff, _ = self.alloc(slots)
        return (soff, 2 * doff, nslots, dmask)

    def build(self):
        return np.concatenate(self.chunks)


def _list_shapes(e, pre):
    """{(sm, dm, pm): {key: min index}}, {(sm, dm, pm): [all indices]}, residual indices."""
    shapes, members, resid = {}, {}, []
    for k in range(pre, len(e)):
        x = e[k]
        sm = _prefix_mask(x['src_lo'], x['src_span'])
        dm = _prefix_mask(x['dst_lo'], x['dst_span'])
        pl, ps = int(x['port_lo']), int(x['port_span'])
        spm = _port_mask(pl & 0xFFFF, ps & 0xFFFF)
        dpm = _port_mask(pl >> 16, ps >> 16)
        if sm is None or dm is None or spm is None or dpm is None or x['step'] != 0:
            # stepped run entries stay residual: their gid depends on the port, so
            # the smallest entry index of a key need not be the smallest gid
            resid.append(k)
            continue
        pm = spm | (dpm << 16)
        key = (int(x['src_lo']), int(x['dst_lo']), pl & pm)
        g = shapes.setdefault((sm, dm, pm), {})
        if key not in g:                 # entries are gid-ascending: first = min index
            g[key] = k
        members.setdefault((sm, dm, pm), []).append(k)
    return shapes, members, resid


def _index_record(img, rec, e, pre, min_entries, max_groups):
    """Fill one list record over entries e (list-local indices; [0, pre) are the
    linear prefix).  Returns the local indices left to the residual scan."""
    ne = len(e)
    resid_idx = []
    groups = []
    if ne >= min_entries and ne <= PHT_CHUNK:
        shapes, members, resid_idx = _list_shapes(e, pre)
        by_sd = {}
        for (sm, dm, pm), keys in shapes.items():
            by_sd.setdefault((sm, dm), {})[pm] = keys
        ranked = sorted(by_sd.items(), key=lambda kv: (min(min(k.values()) for k in kv[1].values()), kv[0]))
        for (sm, dm), tabs in ranked[max_groups:]:
            for pm in tabs:
                resid_idx.extend(members[(sm, dm, pm)])
        groups = ranked[:max_groups]
    else:
        resid_idx = list(range(pre, ne))
    if groups:
        goff, grec = img.alloc(np.zeros(PHT_GROUP_WORDS * len(groups), dtype=np.uint32), align=4)
        src_sets, dst_sets = [], []
        src_any = dst_any = 0
        for j, ((sm, dm), tabs) in enumerate(groups):
            g = grec[PHT_GROUP_WORDS * j: PHT_GROUP_WORDS * (j + 1)]
            g[0], g[1] = sm, dm
            mins, real = [], 0          # real: bit c = port class c has a table
            ss, ds = set(), set()
            for c, pm in enumerate(PORT_CLASSES):
                keys = tabs.get(pm)
                if not keys:
                    g[4 + 4 * c: 8 + 4 * c] = (0, 0, 1, 0)    # image word 0: always empty
                    continue
                ks = np.array(list(keys.keys()), dtype=np.uint64).astype(np.uint32).reshape(-1, 3)
                idx = np.array(list(keys.values()), dtype=np.int64)
                ss.update(ks[:, 0].tolist())
                ds.update(ks[:, 1].tolist())
                H = pht_hash(ks[:, 0], ks[:, 1], ks[:, 2])
                # a full 32-bit hash collision between two keys of one table: keep the
                # smaller index in the table, the other goes residual (still exact)
                o = np.lexsort((idx, H))
                H, idx = H[o], idx[o]
                dup = np.zeros(len(H), dtype=bool)
                dup[1:] = H[1:] == H[:-1]
                resid_idx.extend(idx[dup].tolist())
                H, idx = H[~dup], idx[~dup]
                g[4 + 4 * c: 8 + 4 * c] = img.table(H, idx)
                mins.append(int(idx.min()))
                real |= 1 << c
            g[2] = min(mins)
            g[3] = real
            src_sets.append(ss)
            dst_sets.append(ds)
            if sm == 0:
                src_any |= 1 << j
            if dm == 0:
                dst_any |= 1 << j
        # pruning tables: per non-zero mask of each side, prefix -> group bitmap
        tables = []
        for side, sets in ((0, src_sets), (1, dst_sets)):
            by_mask = {}
            for j, ((sm, dm), _tabs) in enumerate(groups):
                m = dm if side else sm
                if m == 0:
                    continue
                bm = by_mask.setdefault(m, {})
                for k in sets[j]:
                    bm[k] = bm.get(k, 0) | (1 << j)
            for m in sorted(by_mask):
                keys = np.array(sorted(by_mask[m]), dtype=np.uint64).astype(np.uint32)
                H = field_hash(keys, side)
                merged = {}
                for h, k in zip(H.tolist(), keys.tolist()):   # full-hash collision: OR (a superset is safe)
                    merged[h] = merged.get(h, 0) | by_mask[m][k]
                tables.append((m, side, merged))
        # bitmap 0 is the empty one: an empty slot or a tag mismatch reads it
        distinct = sorted({b for _m, _s, mg in tables for b in mg.values()})
        bm_index = {b: i + 1 for i, b in enumerate(distinct)}
        if len(distinct) + 1 > PHT_MAX_IDX:
            raise OverflowError('too many distinct group bitmaps in one list')
        bm_words = np.zeros(2 * (len(distinct) + 1), dtype=np.uint32)
        for b, i in bm_index.items():
            bm_words[2 * i] = b & M32
            bm_words[2 * i + 1] = b >> 32
        bm_off, _ = img.alloc(bm_words, align=2)
        moff, mrec = img.alloc(np.zeros(PHT_MASK_WORDS * max(len(tables), 1), dtype=np.uint32), align=4)
        narrow = len(distinct) + 1 <= 0x100      # 16-bit slots: half the LDS of the pruning tables
        if not narrow:
            img.all_narrow = False
        for q, (m, side, merged) in enumerate(tables):
            H = np.array(list(merged.keys()), dtype=np.uint32)
            vals = np.array([bm_index[b] for b in merged.values()], dtype=np.uint32)
            r = mrec[PHT_MASK_WORDS * q: PHT_MASK_WORDS * (q + 1)]
            soff, doff, nslots, dmask = img.table16(H, vals) if narrow else img.table_prune(H, vals)
            r[0] = m
            r[1] = soff | (MASK_NARROW if narrow else 0)
            r[2] = doff
            r[3] = nslots | (dmask << 17)
        rec[0:4] = (goff, len(groups), moff, len(tables))
        rec[18] = sum(1 for _m, side, _mg in tables if side == 0)   # src tables come first
        rec[7] = bm_off
        rec[8], rec[9] = src_any & M32, src_any >> 32
        rec[10], rec[11] = dst_any & M32, dst_any >> 32
        rec[14] = len(distinct) + 1
    return sorted(set(resid_idx))


def build_index(ent, off, prefix=0, min_entries=96, max_groups=PHT_MAX_GROUPS, chunk=PHT_CHUNK):
    """Pruned perfect-hash tuple-space index over packed lists.

    Returns (image uint32[], resid RULE_DTYPE[]) — the rsa_load_index
    arguments.  A list shorter than ``min_entries`` gets no groups: everything
    after its prefix is residual.  A list longer than ``chunk`` entries becomes
    a chain of records (records n_lists.. of the image)."""
    n_lists = len(off) - 1
    spans = []                                     # per list: [(beg, end) local chunk ranges]
    for L in range(n_lists):
        ne = int(off[L + 1] - off[L])
        spans.append([(a, min(a + chunk, ne)) for a in range(0, max(ne, 1), chunk)] if ne > chunk else [(0, ne)])
    n_records = n_lists + sum(len(sp) - 1 for sp in spans)
    img = _Image()
    list_off, lrec = img.alloc(np.zeros(PHT_LIST_WORDS * n_records, dtype=np.uint32), align=4)
    img.chunks[0][2] = n_lists
    img.chunks[0][3] = list_off
    img.chunks[0][4] = n_records
    resid_parts, n_resid = [], 0
    next_virtual = n_lists
    for L in range(n_lists):
        e_all = ent[off[L]:off[L + 1]]
        ne = len(e_all)
        pre = min(prefix, ne)
        rec_ids = [L] + list(range(next_virtual, next_virtual + len(spans[L]) - 1))
        next_virtual += len(spans[L]) - 1
        after = int(e_all['gid'][pre:].min()) if pre < ne else PHT_EMPTY
        for q, (a, b) in enumerate(spans[L]):
            r = rec_ids[q]
            rec = lrec[PHT_LIST_WORDS * r: PHT_LIST_WORDS * (r + 1)]
            e = e_all[a:b]
            p = max(0, min(pre - a, b - a))
            rec[6] = p if q == 0 else 0
            rec[12] = int(off[L]) + a
            rec[13] = b - a
            rec[15] = after if q == 0 else (int(e['gid'].min()) if len(e) else PHT_EMPTY)
            if q + 1 < len(spans[L]):
                rec[16] = rec_ids[q + 1]
                rec[17] = int(e_all['gid'][spans[L][q + 1][0]:].min())
            else:
                rec[16] = PHT_EMPTY
                rec[17] = PHT_EMPTY
            # linear prefix entries of later chunks do not exist: the prefix lies in chunk 0
            resid_idx = _index_record(img, rec, e, p if q == 0 else 0, min_entries, max_groups)
            rec[4] = n_resid
            resid_parts.append(e[resid_idx])
            n_resid += len(resid_idx)
            rec[5] = n_resid
    if img.all_narrow:
        img.chunks[0][5] |= HDR_ALL_NARROW
    image = img.build()
    resid = np.concatenate(resid_parts) if resid_parts else np.zeros(0, RULE_DTYPE)
    return image, resid


def _records(image):
    lo, nrec = int(image[3]), int(image[4])
    return [[int(v) for v in image[lo + PHT_LIST_WORDS * r: lo + PHT_LIST_WORDS * (r + 1)]] for r in range(nrec)]


def index_stats(index):
    """Per list record: (prefix, groups, masks, residual entries) — tests and tuning."""
    image, _resid = index
    return [(r[6], r[1], r[3], r[5] - r[4]) for r in _records(image)]


def _probe(image, H, t):
    """One CHD probe (csrc: pht_probe): the slot's 16-bit value or PHT_NONE."""
    slot_off, disp_off, n_slots, disp_mask = (int(v) for v in t)
    H = int(H)
    d = int(image.view(np.uint16)[disp_off + ((H >> 16) & disp_mask)])
    w = int(image[slot_off + int(pht_slot(H, d, n_slots))])
    return (w & 0xFFFF) if (w >> 16) == (H & 0xFFFF) else PHT_NONE


def _prune_probe(image, H, t, narrow):
    """One pruning-table probe (csrc: prune_side): the bitmap index of the
    slot, 0 (the empty bitmap) on an empty slot or a tag mismatch."""
    slot_off, disp_off, n_slots, disp_mask = (int(v) for v in t)
    H = int(H)
    h16 = image.view(np.uint16)
    d = int(h16[disp_off + ((H >> 16) & disp_mask)])
    slot = int(pht_slot(H, d, n_slots))
    if narrow:
        w = int(h16[slot_off + slot])
        return (w & 0xFF) if (w >> 8) == (H & 0xFF) else 0
    w = int(image[slot_off + slot])
    return (w & 0xFFFF) if (w >> 16) == (H & 0xFFFF) else 0


def _match(x, src, dst, ports):
    pl, ps = int(x['port_lo']), int(x['port_span'])
    return ((src - int(x['src_lo'])) & M32) <= int(x['src_span']) and \
        ((dst - int(x['dst_lo'])) & M32) <= int(x['dst_span']) and \
        ((ports & 0xFFFF) - (pl & 0xFFFF)) & 0xFFFF <= (ps & 0xFFFF) and \
        ((ports >> 16) - (pl >> 16)) & 0xFFFF <= (ps >> 16)


def _scan(entries, src, dst, ports, best):
    """Linear scan with the device's early exit: stop once best <= an entry's first gid."""
    for x in entries:
        if best is not None and int(x['gid']) >= best:
            break
        if _match(x, src, dst, ports):
            g = entry_gid(x, ports & 0xFFFF, ports >> 16)
            best = g if best is None else min(best, g)
    return best


def pht_lookup(index, ent, off, L, src, dst, ports):
    """Host model of the GPU classifier for one tuple (tests): the first-match
    gid, -1, or 'defer'.  Follows the device order exactly: prefix scan, then
    per chained record the pruning bitmaps, group probes in min-index order with
    verification and retry above a failed candidate, and the residual scan."""
    image, resid = index
    recs = _records(image)
    r = recs[L]
    best = _scan(ent[off[L]:off[L] + r[6]], src, dst, ports, None)
    if best is not None and r[15] != PHT_EMPTY and best <= r[15]:
        return best
    if r[15] == PHT_EMPTY:
        return -1 if best is None else best
    while True:
        e = ent[r[12]:r[12] + r[13]]
        goff, ng, moff, nm = r[0:4]
        if ng:
            S = r[8] | (r[9] << 32)
            D = r[10] | (r[11] << 32)
            n_src = r[18]
            for q in range(nm):
                mr = [int(v) for v in image[moff + PHT_MASK_WORDS * q: moff + PHT_MASK_WORDS * (q + 1)]]
                side = 0 if q < n_src else 1
                key = (dst if side else src) & mr[0]
                t = (mr[1] & ~MASK_NARROW, mr[2], mr[3] & 0x1FFFF, mr[3] >> 17)
                v = _prune_probe(image, field_hash(key, side), t, bool(mr[1] & MASK_NARROW))
                bits = int(image[r[7] + 2 * v]) | (int(image[r[7] + 2 * v + 1]) << 32)
                if side:
                    D |= bits
                else:
                    S |= bits
            cand0 = S & D
            floor = 0
            found = None
            for _attempt in range(PHT_ATTEMPTS):
                bi = PHT_NONE
                for j in range(ng):
                    if not (cand0 >> j) & 1:
                        continue
                    g = [int(v) for v in image[goff + PHT_GROUP_WORDS * j: goff + PHT_GROUP_WORDS * (j + 1)]]
                    if g[2] >= bi:
                        break
                    for c, pm in enumerate(PORT_CLASSES):
                        H = int(pht_hash(src & g[0], dst & g[1], ports & pm))
                        v = _probe(image, H, g[4 + 4 * c: 8 + 4 * c])
                        if v >= floor:
                            bi = min(bi, v)
                if bi == PHT_NONE:
                    break
                if _match(e[bi], src, dst, ports):
                    found = entry_gid(e[bi], ports & 0xFFFF, ports >> 16)
                    break
                floor = bi + 1
            else:
                return 'defer'
            if found is not None:
                best = found if best is None else min(best, found)
        best = _scan(resid[r[4]:r[5]], src, dst, ports, best)
        if r[16] == PHT_EMPTY or (best is not None and best <= r[17]):
            break
        r = recs[r[16]]
    return -1 if best is None else best
