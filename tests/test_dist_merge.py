"""The multi-GPU merge protocol (ruleset-analysis_amd/dist.py: all_reduce of
counters, all_to_all of records to owner = gid % world, threshold all_reduce,
pass-2 exchange, gather to rank 0) run with world_size 2 on CPU (gloo).  Each
rank's table is a test-only numpy model of the HIP table's semantics; the
merged result must equal the C oracle over the whole log."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rsa_pkg

rsa_pkg.load()   # spawned workers import this module without conftest

from oracle import coracle  # noqa: E402
from ruleset_analysis_amd import synth  # noqa: E402
from ruleset_analysis_amd.compile import RECORD_DTYPE  # noqa: E402

NO = 0xFFFFFFFFFFFFFFFF


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

    def records(self, which, thresh=None):
        rows = []
        for (gid, pspell, f, t, p), e in self.t.items():
            if which == 0:
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
    def __init__(self, n_rules, cap, shard):
        self.n_rules, self.cap, self.shard = n_rules, cap, shard
        self.local = NumpyTable()
        self.owner = NumpyTable()
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
        self.counters = {'matches': torch.from_numpy(m), 'hits': torch.from_numpy(h)}
        self.thresh = torch.full((n_rules,), -1, dtype=torch.int64)

    def _key(self, i):
        gid, flags, pspell, src, dst, sport, dport, ts, order = self.shard
        if flags[i] & 8:
            return (int(gid[i]), int(pspell[i]), int(dst[i]), int(src[i]), int(sport[i]))
        return (int(gid[i]), int(pspell[i]), int(src[i]), int(dst[i]), int(dport[i]))

    def local_counters(self):
        return self.counters

    def export(self, which):
        return self.local.records(which)

    def owner_reset(self, capacity):
        self.owner = NumpyTable()

    def owner_import(self, buf, which):
        for r in buf.numpy().view(RECORD_DTYPE):
            k = (int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']))
            if which == 0:
                self.owner.combine(k, int(r['count']), int(r['first']), int(r['last']), int(r['min_order']))
            else:
                e = self.owner.t[k]
                e[4] += int(r['count'])
                e[5] = min(e[5], int(r['first']))
                e[6] = max(e[6], int(r['last']))

    def owner_resolve_cap(self):
        per = {}
        for (gid, *_), e in self.owner.t.items():
            per.setdefault(gid, []).append(e[3])
        th = np.full(self.n_rules, NO, np.uint64)
        for gid, orders in per.items():
            if self.cap > 0 and len(orders) >= self.cap:
                th[gid] = sorted(orders)[self.cap - 1]
        self.owner_thresh = torch.from_numpy(th.view(np.int64).copy())
        d = np.zeros(self.n_rules, np.int32)
        for gid, orders in per.items():
            d[gid] = len(orders)
        self.owner_distinct = torch.from_numpy(d)
        return int((th != NO).sum())

    def owner_counters(self):
        return {'thresh': self.owner_thresh, 'distinct': self.owner_distinct}

    def set_local_thresh(self, thresh):
        self.thresh = thresh.clone()

    def set_owner_thresh(self, thresh):
        self.owner_thresh = thresh.clone()

    def local_recount(self):
        gid, flags, pspell, src, dst, sport, dport, ts, order = self.shard
        th = self.thresh.numpy().view(np.uint64)
        for i in range(len(gid)):
            g = int(gid[i])
            if g < 0 or (flags[i] & 6) != 6 or int(th[g]) == NO or int(order[i]) > int(th[g]):
                continue
            e = self.local.t[self._key(i)]
            e[4] += 1
            e[5] = min(e[5], int(ts[i]))
            e[6] = max(e[6], int(ts[i]))

    def owner_emit(self):
        return self.owner.records(2, self.owner_thresh.numpy().view(np.uint64))


def _worker(rank, world, port, payload, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from ruleset_analysis_amd.dist import merge
    n_rules, cap, cols = payload
    n = len(cols[0])
    cut = np.linspace(0, n, world + 1).astype(int)
    shard = tuple(c[cut[rank]:cut[rank + 1]] for c in cols)
    out = merge(NumpyBackend(n_rules, cap, shard), dist, world, rank)
    if rank == 0:
        out_q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('cap', [15, 100000])
def test_merge_world2_matches_oracle(cap):
    dbj, info = synth.make_db(51, 300)
    tr = synth.make_traffic((dbj, info), 30000, seed=52, zipf=1.2)
    R = coracle.OracleRules(dbj)
    cols, ts, order = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ts, order, cap)
    payload = (R.n_rules, cap, (ref['gid'], cols['flags'], cols['pspell'], cols['src'], cols['dst'], cols['sport'],
                                cols['dport'], ts, order))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, payload, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    out = None
    deadline = time.time() + 300
    while out is None:
        try:
            out = q.get(timeout=2)
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail('merge worker died: exit codes %s' % [p.exitcode for p in procs])
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    recs, matches, hits, distinct, thresh = out
    assert np.array_equal(matches, ref['matches'])
    assert np.array_equal(hits, ref['hits'])
    assert np.array_equal(thresh != NO, (ref['n_conns'] >= cap) & (cap > 0))
    got = sorted((int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']),
                  int(r['count']), int(r['first']), int(r['last'])) for r in recs)
    rows = ref['rows']
    want = sorted(zip(*(rows[k].astype(int).tolist() for k in ('gid', 'pspell', 'for_ip', 'to_ip', 'to_port',
                                                                  'count', 'first', 'last'))))
    assert got == want
