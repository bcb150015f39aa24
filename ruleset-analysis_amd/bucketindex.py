"""Partial-key bucket index of the candidate lists (image magic ``RSA5``).

What the device has to answer per log line is the reference's first match
(``mapper.py:168-189``): the smallest gid among the entries of the line's
candidate list that contain the connection (``firewallrule.py:128-174``).  The
index splits a list's entries into a few *tables*, each with a key template
``(src_mask, dst_mask, port_mask)``: an entry belongs to a table only if every
connection it contains agrees with it on the masked bits (its src/dst prefix
is at least as long as the template's, its port is exact on every port side
the template keys on).  Inside a table the entries are grouped into *buckets*
by their masked key; a connection computes its key for each table, probes one
bucketised cuckoo hash table per template (two independent 8-B bucket reads,
two 4-B slots each: 11-bit tag, bucket length, first entry), and verifies every
entry of the buckets whose tag matches with the full predicate.  Every entry
that contains the connection sits in exactly one probed bucket, so the minimum
over the probed buckets (and the linear prefix and residual entries) is
exactly the linear scan's answer; a tag collision only adds entries to check.

Compared with the ``RSA4`` pruned perfect-hash index (``compile.build_index``)
a lane has no pruning stage and no verification retries: one LDS level (the
bucket reads of all tables are independent) before the entry checks, and no
line is ever deferred.

The templates are chosen per list record by a greedy cover: among all
``(src length, dst length, port class)`` templates, take the one covering the
most remaining entries whose buckets stay small (mean entries a matching
connection checks, ``sum(n_b^2) / n``, under a bound that is relaxed when
nothing qualifies), at most ``MAX_TABLES`` per record; whatever is left is
residual (scanned linearly, wave-uniform).  Tables are ordered by their
smallest gid, so a lane stops probing once its best beats a table's minimum.

Image layout (uint32 words; everything the GPU indexes is validated by
``rsa_load_index``): header ``[0xFFFFFFFF, RSA5, n_lists, list_off, n_records,
0, 0, 0]``; list records (``rsa_pht_list``, 20 words: ``group_off`` = table
descriptors, ``n_groups`` = tables, the other fields as for RSA4); table
descriptors (8 words: src_mask, dst_mask, port_mask, bucket_off, n_buckets,
filter_off, min_gid, entry_base); buckets (2 words: two slots ``tag11 << 21 |
len5 << 16 | first16``, len 0 = empty; ``first`` relative to the table's
entry_base); row filters (one word per bucket row at filter_off + row:
``row_filters``), checked in LDS before a row is loaded from the residual
array.
Bucket entries are rows of the residual entry array (the ``rsa_load_index``
resid argument) after the record's linear residual rows.
"""

import numpy as np

from .compile import RULE_DTYPE, STEP_SPORT, PHT_CHUNK, PHT_EMPTY, PHT_LIST_WORDS, M32, entry_gid, fmix32, \
    _Image, _scan, _records

__all__ = ['BKT_MAGIC', 'build_bucket_index', 'bucket_lookup', 'bucket_stats', 'bkt_hash']

BKT_MAGIC = 0x35415352                   # 'RSA5'
BKT_TABLE_WORDS = 8
MAX_TABLES = 8
BKT_MAX_LEN = 31                          # slot: tag11 << 21 | len5 << 16 | first16
TAG_BITS = 11
LENGTHS = (0, 8, 16, 24, 32)
PORT_CLASSES = (0x00000000, 0xFFFF0000, 0x0000FFFF, 0xFFFFFFFF)   # none, dport, sport, both
MUL_D, MUL_P = 0x9E3779B1, 0x85EBCA77       # odd: each field's pre-mix is a bijection
SEED_KEY, SEED_ROW = 0x2545F491, 0x6A09E667     # bucket-key hash, row-filter hash
FP_BITS = 18
BKT_LOAD = 0.85


def bkt_hash(ks, kd, kp, seed):
    """Hash of a masked key (csrc: bkt_hash)."""
    with np.errstate(over='ignore'):
        x = np.asarray(ks, np.uint32) ^ (np.asarray(kd, np.uint32) * np.uint32(MUL_D)) ^ \
            (np.asarray(kp, np.uint32) * np.uint32(MUL_P)) ^ np.uint32(seed)
    return fmix32(x)


def bkt_buckets(h, nb):
    """(b1, b2, tag) of hashes h for a table of nb <= 65536 buckets: each
    half of h picks a bucket by multiply-shift (full-rate 24-bit products on
    the device), the 11-bit tag is the xor of the low bits of both halves
    (independent of either bucket's leading bits)."""
    h = np.asarray(h, np.uint32).astype(np.int64)
    b1 = ((h & 0xFFFF) * nb) >> 16
    b2 = ((h >> 16) * nb) >> 16
    tag = ((h >> 16) ^ h) & ((1 << TAG_BITS) - 1)
    return b1, b2, tag


def _mask(length):
    return (M32 << (32 - length)) & M32 if length else 0


def _masks(lengths):
    ln = np.asarray(lengths, np.int64)
    return np.where(ln > 0, (M32 << (32 - np.clip(ln, 1, 32))) & M32, 0).astype(np.uint32)


def row_filters(rows):
    """Per bucket row the 4-B LDS filter: slen6 << 26 | dlen6 << 20 | pm2 << 18
    | fp18, fp = the low 18 bits of bkt_hash over the row's own exact bits
    (src & its prefix mask, dst & its prefix mask, the exact port sides: pm2
    bit 0 sport, bit 1 dport; range or run sides are not filtered).  A
    connection the row contains always passes; most others do not."""
    sl, dl, sx, dx = _entry_shape(rows)
    pm2 = sx.astype(np.int64) | (dx.astype(np.int64) << 1)
    pm = np.where(sx, 0xFFFF, 0) | np.where(dx, 0xFFFF0000, 0)
    h = bkt_hash(rows['src_lo'] & _masks(sl), rows['dst_lo'] & _masks(dl),
                 rows['port_lo'] & pm.astype(np.uint32), SEED_ROW)
    return ((sl.astype(np.uint32) << np.uint32(26)) | (dl.astype(np.uint32) << np.uint32(20)) |
            (pm2.astype(np.uint32) << np.uint32(18)) | (h & np.uint32((1 << FP_BITS) - 1)))


def row_passes(f, src, dst, ports):
    """The device's filter test of one row word f for a connection."""
    sl, dl, pm2 = f >> 26, (f >> 20) & 63, (f >> 18) & 3
    pm = (0xFFFF if pm2 & 1 else 0) | (0xFFFF0000 if pm2 & 2 else 0)
    h = int(bkt_hash(np.uint32(src & _mask(sl)), np.uint32(dst & _mask(dl)), np.uint32(ports & pm), SEED_ROW))
    return (h & ((1 << FP_BITS) - 1)) == (f & ((1 << FP_BITS) - 1))


def _entry_shape(e):
    """Per entry: src / dst prefix length (-1: not a prefix), dport / sport exact."""
    def plen(lo, span):
        size = span.astype(np.int64) + 1
        ok = (size & (size - 1)) == 0
        ok &= (lo.astype(np.int64) % size) == 0
        ln = 32 - np.log2(size).astype(np.int64)
        return np.where(ok, ln, -1)
    sl = plen(e['src_lo'], e['src_span'])
    dl = plen(e['dst_lo'], e['dst_span'])
    step = e['step'].astype(np.int64)
    run = step != 0
    on_sport = (step & STEP_SPORT) != 0
    ps = e['port_span'].astype(np.int64)
    sport_exact = ((ps & 0xFFFF) == 0) & ~(run & on_sport)
    dport_exact = ((ps >> 16) == 0) & ~(run & ~on_sport)
    return sl, dl, sport_exact, dport_exact


def _eligible(shape, ls, ld, pm):
    sl, dl, sx, dx = shape
    ok = (sl >= ls) & (dl >= ld)
    if pm & 0xFFFF:
        ok &= sx
    if pm & 0xFFFF0000:
        ok &= dx
    return ok


def _keys(e, ls, ld, pm):
    return (e['src_lo'] & np.uint32(_mask(ls)), e['dst_lo'] & np.uint32(_mask(ld)),
            e['port_lo'] & np.uint32(pm))


def _bucket_sizes(ks, kd, kp):
    if len(ks) == 0:
        return np.zeros(0, np.int64)
    k = np.stack([ks.astype(np.int64), kd.astype(np.int64), kp.astype(np.int64)], 1)
    _u, counts = np.unique(k, axis=0, return_counts=True)
    return counts


def choose_tables(e, idx, max_tables=MAX_TABLES, costs=(2.0, 4.0, 8.0, 16.0), min_cover=4):
    """Greedy template cover of entries e[idx] -> [(ls, ld, pm, member indices)], rest."""
    shape = _entry_shape(e)
    left = np.zeros(len(e), bool)
    left[idx] = True
    chosen = []
    lens_s = sorted({l for l in LENGTHS if (shape[0][left] >= l).any()})
    lens_d = sorted({l for l in LENGTHS if (shape[1][left] >= l).any()})
    while len(chosen) < max_tables and left.sum() >= min_cover:
        best = None
        for cmax in costs:
            for ls in lens_s:
                for ld in lens_d:
                    for pm in PORT_CLASSES:
                        w = np.nonzero(left & _eligible(shape, ls, ld, pm))[0]
                        if len(w) < min_cover:
                            continue
                        c = _bucket_sizes(*_keys(e[w], ls, ld, pm))
                        if int(c.max()) > BKT_MAX_LEN:
                            continue
                        cost = float((c.astype(np.float64) ** 2).sum() / len(w))
                        if cost > cmax:
                            continue
                        score = (len(w), -cost)
                        if best is None or score > best[0]:
                            best = (score, ls, ld, pm, w)
            if best is not None:
                break
        if best is None:
            break
        _s, ls, ld, pm, w = best
        chosen.append((ls, ld, pm, w))
        left[w] = False
    return chosen, np.nonzero(left)[0]


def _cuckoo(h, seed_rng, load=BKT_LOAD, kicks=1000):
    """Place hashes h (one per key, duplicates allowed) into 2-slot buckets,
    two candidate buckets each.  Returns (n_buckets, slot index per key)."""
    n = len(h)
    nb = max(1, int(np.ceil(n / (2 * load))))
    while True:
        if nb > 0x10000:
            raise OverflowError('bucket table of %d keys does not fit 65536 buckets' % n)
        b1, b2, _tag = bkt_buckets(h, nb)
        b1, b2 = b1.tolist(), b2.tolist()
        slot = [-1] * (2 * nb)                    # slot -> key
        where = [-1] * n
        ok = True
        for k in range(n):
            cur = k
            for _kick in range(kicks):
                placed = False
                for b in (b1[cur], b2[cur]):
                    for s in (2 * b, 2 * b + 1):
                        if slot[s] < 0:
                            slot[s] = cur
                            where[cur] = s
                            placed = True
                            break
                    if placed:
                        break
                if placed:
                    break
                b = (b1[cur], b2[cur])[int(seed_rng.integers(2))]
                s = 2 * b + int(seed_rng.integers(2))
                victim = slot[s]
                slot[s] = cur
                where[cur] = s
                where[victim] = -1
                cur = victim
            else:
                ok = False
                break
        if ok:
            return nb, np.array(where, np.int64)
        nb = nb + nb // 8 + 1


def _record(img, rec, e, base_gid_order, pre, resid_rows, filters=False):
    """Tables of one list record over entries e (record-local indices; [0, pre)
    is the linear prefix).  Appends residual rows then bucket rows to
    resid_rows (list of RULE_DTYPE arrays); returns (resid_beg, resid_end) of
    the linear residual rows."""
    idx = np.arange(pre, len(e))
    chosen, rest = choose_tables(e, idx) if len(idx) else ([], idx)
    n0 = sum(len(r) for r in resid_rows)
    resid_rows.append(e[rest])
    r_beg, r_end = n0, n0 + len(rest)
    if not chosen:
        rec[0] = rec[1] = 0
        return r_beg, r_end
    tabs = []
    pos = r_end
    for ls, ld, pm, w in chosen:
        ks, kd, kp = _keys(e[w], ls, ld, pm)
        k = np.stack([ks.astype(np.int64), kd.astype(np.int64), kp.astype(np.int64)], 1)
        uk, inv = np.unique(k, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        order = np.lexsort((w, inv))          # bucket, then entry order (= first gid order)
        rows = e[w[order]]
        counts = np.bincount(inv, minlength=len(uk))
        firsts = np.concatenate([[0], np.cumsum(counts)[:-1]])      # relative to the table's first row
        resid_rows.append(rows)
        base = pos
        pos += len(rows)
        seed = SEED_KEY
        rng = np.random.default_rng(len(tabs) + 7)
        h = bkt_hash(uk[:, 0], uk[:, 1], uk[:, 2], seed)
        nb, where = _cuckoo(h, rng)
        _b1, _b2, tag = bkt_buckets(h, nb)
        words = np.zeros(2 * nb, np.uint32)                         # bucket b = slots 2b, 2b + 1
        words[where] = (tag.astype(np.uint32) << np.uint32(21)) | (counts.astype(np.uint32) << np.uint32(16)) | \
            firsts.astype(np.uint32)
        boff, _ = img.alloc(words, align=2)
        foff = img.alloc(row_filters(rows))[0] if filters else 0
        tabs.append((int(e['gid'][w].min()), _mask(ls), _mask(ld), pm, boff, nb, foff, base))
    tabs.sort()
    toff, trec = img.alloc(np.zeros(BKT_TABLE_WORDS * len(tabs), np.uint32), align=4)
    for j, (mg, sm, dm, pm, boff, nb, foff, base) in enumerate(tabs):
        trec[BKT_TABLE_WORDS * j: BKT_TABLE_WORDS * (j + 1)] = (sm, dm, pm, boff, nb, foff, mg, base)
    rec[0], rec[1] = toff, len(tabs)
    return r_beg, r_end


def build_bucket_index(ent, off, prefix=0, chunk=PHT_CHUNK, min_entries=32, filters=False):
    """Bucket index over packed lists: (image uint32[], resid RULE_DTYPE[]),
    the rsa_load_index arguments.  Lists longer than ``chunk`` entries are
    chains of records as in the RSA4 index; a record with fewer than
    ``min_entries`` entries after its prefix is all residual.  ``filters``:
    LDS row filters (image word 5 bit 0; table filter_off)."""
    n_lists = len(off) - 1
    spans = []
    for L in range(n_lists):
        ne = int(off[L + 1] - off[L])
        spans.append([(a, min(a + chunk, ne)) for a in range(0, max(ne, 1), chunk)] if ne > chunk else [(0, ne)])
    n_records = n_lists + sum(len(sp) - 1 for sp in spans)
    img = _Image()
    img.chunks[0][1] = BKT_MAGIC
    list_off, lrec = img.alloc(np.zeros(PHT_LIST_WORDS * n_records, dtype=np.uint32), align=4)
    img.chunks[0][2] = n_lists
    img.chunks[0][3] = list_off
    img.chunks[0][4] = n_records
    img.chunks[0][5] = 1 if filters else 0
    resid_rows = []
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
            p = max(0, min(pre - a, b - a)) if q == 0 else 0
            rec[6] = p
            rec[12] = int(off[L]) + a
            rec[13] = b - a
            rec[15] = after if q == 0 else (int(e['gid'].min()) if len(e) else PHT_EMPTY)
            if q + 1 < len(spans[L]):
                rec[16] = rec_ids[q + 1]
                rec[17] = int(e_all['gid'][spans[L][q + 1][0]:].min())
            else:
                rec[16] = PHT_EMPTY
                rec[17] = PHT_EMPTY
            if len(e) - p >= min_entries:
                rb, re_ = _record(img, rec, e, None, p, resid_rows, filters)
            else:
                n0 = sum(len(x) for x in resid_rows)
                resid_rows.append(e[p:])
                rb, re_ = n0, n0 + len(e) - p
            rec[4], rec[5] = rb, re_
    image = img.build()
    resid = np.concatenate(resid_rows) if resid_rows else np.zeros(0, RULE_DTYPE)
    return image, resid


def bucket_stats(index):
    """Per list record: (prefix, tables, residual entries, bucket entries) — tests and tuning."""
    image, _resid = index
    out = []
    for r in _records(image):
        nb = 0
        for j in range(r[1]):
            t = image[r[0] + BKT_TABLE_WORDS * j: r[0] + BKT_TABLE_WORDS * (j + 1)]
            w = image[int(t[3]): int(t[3]) + 2 * int(t[4])]
            nb += int(((w >> np.uint32(16)) & np.uint32(0x1F)).sum())
        out.append((r[6], r[1], r[5] - r[4], nb))
    return out


def bucket_lookup(index, ent, off, L, src, dst, ports):
    """Host model of the GPU lookup for one tuple (tests): the first-match gid
    or -1, in the device's order (prefix scan; per chained record the tables
    in ascending min gid while they can still beat the best, their matching
    buckets, then the residual scan)."""
    image, resid = index
    recs = _records(image)
    r = recs[L]
    best = _scan(ent[off[L]:off[L] + r[6]], src, dst, ports, None)
    if r[15] == PHT_EMPTY or (best is not None and best <= r[15]):
        return -1 if best is None else best
    while True:
        for j in range(r[1]):
            t = [int(v) for v in image[r[0] + BKT_TABLE_WORDS * j: r[0] + BKT_TABLE_WORDS * (j + 1)]]
            sm, dm, pm, boff, nb, foff, mg, base = t
            if best is not None and best <= mg:
                break
            h = bkt_hash(src & sm, dst & dm, ports & pm, SEED_KEY)
            b1, b2, tag = (int(x) for x in bkt_buckets(h, nb))
            for s in (2 * b1, 2 * b1 + 1, 2 * b2, 2 * b2 + 1):       # b2 == b1: the same slots twice
                w = int(image[boff + s])
                ln = (w >> 16) & 0x1F
                if ln and (w >> 21) == tag and not int(image[5]) & 1:
                    a = base + (w & 0xFFFF)
                    best = _scan(resid[a:a + ln], src, dst, ports, best)
                elif ln and (w >> 21) == tag:
                    # the first row of the bucket that passes its filter is the
                    # bucket's candidate (rows ascend in first gid)
                    for k in range(w & 0xFFFF, (w & 0xFFFF) + ln):
                        x = resid[base + k]
                        if best is not None and int(x['gid']) >= best:
                            break
                        if row_passes(int(image[foff + k]), src, dst, ports) and \
                                _scan(resid[base + k:base + k + 1], src, dst, ports, None) is not None:
                            g = entry_gid(x, ports & 0xFFFF, ports >> 16)
                            best = g if best is None else min(best, g)
                            break
        best = _scan(resid[r[4]:r[5]], src, dst, ports, best)
        if r[16] == PHT_EMPTY or (best is not None and best <= r[17]):
            break
        r = recs[r[16]]
    return -1 if best is None else best
