"""TEST INFRASTRUCTURE ONLY — a CPU model of one rank's part of the multi-GPU
job, so the distributed protocol (``ruleset-analysis_amd/dist.py``) and
``bench.py``'s rank spawning can run without a GPU (gloo, world size >= 2).

* ``classify_entries``: brute-force first match over the product's compiled
  candidate lists (minimum matching gid, numpy), the answer the HIP classifier
  gives;
* ``NumpyTable`` / ``NumpyBackend``: the semantics of the HIP
  distinct-connection table (pass-1 aggregates, pass-2 recount, export/import,
  cap resolution) behind the backend interface ``dist.merge`` drives.

Nothing in the product imports this module; ``bench.py`` loads it only under
its ``--cpu-model`` testing flag.
"""
import numpy as np
import torch

from ruleset_analysis_amd.compile import RECORD_DTYPE

NO = 0xFFFFFFFFFFFFFFFF


def classify_entries(ent, off, tup, chunk=2048):
    """First-match gid per packed tuple (-1: none) by brute force over the
    compiled lists (entry gid = base + (port - lo) * stride for run entries)."""
    n = len(tup)
    out = np.full(n, -1, np.int64)
    valid = (tup['flags'] & 1) != 0
    lists = tup['list'].astype(np.int64)
    for L in np.unique(lists[valid]):
        sel = np.nonzero(valid & (lists == L))[0]
        e = ent[off[L]:off[L + 1]]
        if len(e) == 0:
            continue
        slo, ssp = e['src_lo'].astype(np.int64), e['src_span'].astype(np.int64)
        dlo, dsp = e['dst_lo'].astype(np.int64), e['dst_span'].astype(np.int64)
        pl, ps = e['port_lo'].astype(np.int64), e['port_span'].astype(np.int64)
        gid = e['gid'].astype(np.int64)
        stride = (e['step'].astype(np.int64) & 0x7FFFFFFF)
        on_sport = (e['step'].astype(np.int64) >> 31) & 1
        for a in range(0, len(sel), chunk):
            idx = sel[a:a + chunk]
            s = tup['src'][idx].astype(np.int64)[:, None]
            d = tup['dst'][idx].astype(np.int64)[:, None]
            sp = tup['sport'][idx].astype(np.int64)[:, None]
            dp = tup['dport'][idx].astype(np.int64)[:, None]
            m = ((s - slo) & 0xFFFFFFFF) <= ssp
            m &= ((d - dlo) & 0xFFFFFFFF) <= dsp
            m &= ((sp - (pl & 0xFFFF)) & 0xFFFF) <= (ps & 0xFFFF)
            m &= ((dp - (pl >> 16)) & 0xFFFF) <= (ps >> 16)
            step = np.where(on_sport == 1, sp - (pl & 0xFFFF), dp - (pl >> 16))
            g = np.where(m, gid + step * stride, np.iinfo(np.int64).max)
            best = g.min(axis=1)
            out[idx] = np.where(best == np.iinfo(np.int64).max, -1, best)
    return out.astype(np.int32)


class NumpyTable(object):
    """(gid, key) -> [count, first, last, min_order, count2, first2, last2]."""

    def __init__(self):
        self.t = {}

    def combine(self, k, cnt, first, last, order):
        e = self.t.get(k)
        if e is None:
            self.t[k] = [cnt, first, last, order, 0, 0xFFFFFFFF, 0]
            return True
        e[0] += cnt
        e[1] = min(e[1], first)
        e[2] = max(e[2], last)
        e[3] = min(e[3], order)
        return False

    def local_thresh(self, n_rules, cap):
        """Per rule the cap-th smallest min_order of this table (NO: fewer
        than cap entries) -- the shard's own P (rsa_resolve_cap)."""
        per = {}
        for (gid, *_), e in self.t.items():
            per.setdefault(gid, []).append(e[3])
        th = np.full(n_rules, NO, np.uint64)
        for gid, orders in per.items():
            if cap > 0 and len(orders) >= cap:
                th[gid] = sorted(orders)[cap - 1]
        return th

    def distinct(self, n_rules):
        d = np.zeros(n_rules, np.int32)
        for (gid, *_) in self.t:
            d[gid] += 1
        return d

    def records(self, which, thresh=None, keep=None):
        """Rows of the k_emit mode ``which``; ``keep(gid)``: the owner filter."""
        rows = []
        for (gid, pspell, f, t, p), e in self.t.items():
            if keep is not None and not keep(gid):
                continue
            if which == 0:
                rows.append((e[3], gid, f, t, p, pspell, 0, e[0], e[1], e[2], 0))
            elif which == 3:
                # pass1_kept (k_emit mode 3): entries that can still reach the
                # report under the shard's own threshold
                P = int(thresh[gid])
                if P == NO or e[3] <= P:
                    rows.append((e[3], gid, f, t, p, pspell, 0, e[0], e[1], e[2], 0))
            elif which == 1:
                if e[4]:
                    rows.append((e[3], gid, f, t, p, pspell, 0, e[4], e[5], e[6], 0))
            else:
                P = int(thresh[gid])
                if P == NO:
                    rows.append((e[3], gid, f, t, p, pspell, 0, e[0], e[1], e[2], 0))
                elif e[3] <= P:
                    rows.append((e[3], gid, f, t, p, pspell, 0, e[4], e[5], e[6], 0))
        arr = np.array(rows, dtype=RECORD_DTYPE) if rows else np.zeros(0, RECORD_DTYPE)
        return torch.from_numpy(arr.view(np.uint8).copy())


class NumpyBackend(object):
    """``dist.merge`` backend over one rank's shard: ``shard`` = (gid, flags,
    pspell, src, dst, sport, dport, ts, order) numpy columns.  One table, as
    the HIP ctx: the shard's pass-1 entries, joined during the merge by the
    received entries of the rules this rank owns."""

    def __init__(self, n_rules, cap, shard):
        self.n_rules, self.cap, self.shard = n_rules, cap, shard
        self.local = NumpyTable()
        self.world, self.rank = 0, 0
        gid, flags, pspell, src, dst, sport, dport, ts, order = shard
        m = np.zeros(n_rules, np.int64)
        h = np.zeros(n_rules, np.int64)
        for i in range(len(gid)):
            g = int(gid[i])
            if g < 0:
                continue
            m[g] += 1
            if flags[i] & 2:
                h[g] += 1
                if flags[i] & 4:
                    self.local.combine(self._key(i), 1, int(ts[i]), int(ts[i]), int(order[i]))
        self._counters = {'matches': torch.from_numpy(m), 'hits': torch.from_numpy(h),
                          'distinct': torch.from_numpy(self.local.distinct(n_rules)),
                          'thresh': torch.full((n_rules,), -1, dtype=torch.int64)}

    @classmethod
    def from_packed(cls, n_rules, cap, gids, tup, ts, order):
        return cls(n_rules, cap, (gids, tup['flags'], tup['pspell'], tup['src'], tup['dst'], tup['sport'],
                                  tup['dport'], ts, order))

    def _key(self, i):
        gid, flags, pspell, src, dst, sport, dport, ts, order = self.shard
        if flags[i] & 8:
            return (int(gid[i]), int(pspell[i]), int(dst[i]), int(src[i]), int(sport[i]))
        return (int(gid[i]), int(pspell[i]), int(src[i]), int(dst[i]), int(dport[i]))

    def _owned(self, gid):
        return self.world == 0 or gid % self.world == self.rank

    def counters(self):
        return self._counters

    def set_owner(self, world, rank):
        self.world, self.rank = world, rank

    def _thresh_np(self):
        return self._counters['thresh'].numpy().view(np.uint64)

    def export(self, which):
        foreign = lambda g: not self._owned(g)
        if which == 0:
            # as EngineBackend.export(0): the shard resolves its own cap first
            # and exports only the entries its threshold keeps (exact: a
            # shard's P bounds the global P from above)
            self.capped = self.resolve_cap()
            self.exported_all = sum(1 for (g, *_) in self.local.t if foreign(g))
            recs = self.local.records(3, self._thresh_np(), keep=foreign)
            self.exported_kept = recs.numel() // RECORD_DTYPE.itemsize
            return self._grouped(recs)
        return self._grouped(self.local.records(1, keep=foreign))

    route_cap = None   # TESTING: rows the first export buffer holds (None: all of them)

    def _grouped(self, recs):
        """The model of rsa_export_routed: rows grouped by owner gid % world
        and the per-owner counts.  With ``route_cap`` set, the buffer holds
        only that many rows (the library drops the rows past its buffer and
        still reports the true counts) and ``again(n)`` exports once more into
        n rows."""
        from ruleset_analysis_amd.dist import Exported
        world = max(self.world, 1)
        rows = recs.numpy().view(RECORD_DTYPE)
        owner = rows['gid'].astype(np.int64) % world
        order = np.argsort(owner, kind='stable')
        grouped = rows[order]
        counts = torch.from_numpy(np.bincount(owner, minlength=world).astype(np.int64))

        def export(n):
            return torch.from_numpy(grouped[:n].view(np.uint8).reshape(-1).copy()), counts, n

        def again(n):
            self.reexports = getattr(self, 'reexports', 0) + 1
            return export(n)

        cap = len(rows) if self.route_cap is None else min(self.route_cap, len(rows))
        buf, _c, _n = export(cap)
        return Exported(buf, counts, cap, again)

    def import_records(self, buf, which):
        for r in buf.numpy().view(RECORD_DTYPE):
            k = (int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']))
            if which == 0:
                if self.local.combine(k, int(r['count']), int(r['first']), int(r['last']), int(r['min_order'])):
                    self._counters['distinct'][k[0]] += 1
            else:
                e = self.local.t[k]
                e[4] += int(r['count'])
                e[5] = min(e[5], int(r['first']))
                e[6] = max(e[6], int(r['last']))

    def table_need(self, n_received):
        return len(self.local.t) + int(n_received)

    def resolve_cap(self):
        th = self.local.local_thresh(self.n_rules, self.cap)
        self._counters['thresh'].copy_(torch.from_numpy(th.view(np.int64).copy()))
        return int((th != NO).sum())

    def set_thresh(self, thresh):
        self._counters['thresh'].copy_(thresh)

    def recount(self):
        gid, flags, pspell, src, dst, sport, dport, ts, order = self.shard
        th = self._thresh_np()
        for i in range(len(gid)):
            g = int(gid[i])
            if g < 0 or (flags[i] & 6) != 6 or int(th[g]) == NO or int(order[i]) > int(th[g]):
                continue
            e = self.local.t[self._key(i)]
            e[4] += 1
            e[5] = min(e[5], int(ts[i]))
            e[6] = max(e[6], int(ts[i]))

    def emit_final(self):
        return self.local.records(2, self._thresh_np(), keep=self._owned)
