"""The multi-GPU merge protocol (ruleset-analysis_amd/dist.py: all_reduce of
counters, all_to_all of records to owner = gid % world, threshold all_reduce,
pass-2 exchange, gather to rank 0) run with world_size 2 on CPU (gloo).  Each
rank's table is the test-only numpy model of the HIP table's semantics
(tests/cpu_model.py); the merged result must equal the C oracle over the
whole log."""
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

from cpu_model import NO, NumpyBackend  # noqa: E402


def _worker(rank, world, port, payload, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from ruleset_analysis_amd.dist import gather_rows, merge
    n_rules, cap, cols = payload[:3]
    gather = payload[3] if len(payload) > 3 else True
    route_cap = payload[4] if len(payload) > 4 else None
    n = len(cols[0])
    cut = np.linspace(0, n, world + 1).astype(int)
    shard = tuple(c[cut[rank]:cut[rank + 1]] for c in cols)
    be = NumpyBackend(n_rules, cap, shard)
    be.route_cap = route_cap
    stats = {}
    if gather:
        out = merge(be, dist, world, rank, stats=stats)
    else:   # the owners keep their rows (bench.py's timed job); gathered afterwards
        part = merge(be, dist, world, rank, gather=False, stats=stats)
        out = gather_rows(part, dist, world, rank)
    if rank == 0:
        out_q.put((out, be.exported_all, be.exported_kept, stats, getattr(be, 'reexports', 0)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    """A free port for a rendezvous store, drawn below the kernel's ephemeral
    range (32768-60999): a port bind(0) hands out can be taken again by a
    client socket of an earlier process group before the store binds it."""
    import random
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(('127.0.0.1', p))
        except OSError:
            continue
        finally:
            s.close()
        return p
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('cap,gather,route_cap', [(15, True, None), (100000, True, None), (15, False, None),
                                                  (15, True, 1), (15, False, 3)])
def test_merge_world2_matches_oracle(cap, gather, route_cap):
    """route_cap: every export first lands in a buffer of that many rows, so
    both exchanges take the re-export path (Exported.again at the exact size,
    ADVICE r05) and must still give the oracle's result."""
    dbj, info = synth.make_db(51, 300)
    tr = synth.make_traffic((dbj, info), 30000, seed=52, zipf=1.2)
    R = coracle.OracleRules(dbj)
    cols, ts, order = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ts, order, cap)
    payload = (R.n_rules, cap, (ref['gid'], cols['flags'], cols['pspell'], cols['src'], cols['dst'], cols['sport'],
                                cols['dport'], ts, order), gather, route_cap)
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
    (recs, matches, hits, distinct, thresh), n_all, n_kept, stats, reexports = out
    # the shard-side filter (export(0) = pass1_kept) engages when rules are capped
    assert (n_kept < n_all) if cap == 15 else (n_kept == n_all)
    assert stats['route1_sent_rows'] > 0 and stats['route1_self_rows'] == 0
    assert stats['pass2'] == (cap == 15) and ('route2_sent_rows' in stats) == (cap == 15)
    if route_cap is not None:
        # both exchanges overflowed their first buffer and exported again
        assert reexports == 2 and stats['reexports'] == 2
    assert np.array_equal(matches, ref['matches'])
    assert np.array_equal(hits, ref['hits'])
    assert np.array_equal(thresh != NO, (ref['n_conns'] >= cap) & (cap > 0))
    got = sorted((int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']),
                  int(r['count']), int(r['first']), int(r['last'])) for r in recs)
    rows = ref['rows']
    want = sorted(zip(*(rows[k].astype(int).tolist() for k in ('gid', 'pspell', 'for_ip', 'to_ip', 'to_port',
                                                                  'count', 'first', 'last'))))
    assert got == want


class _OverflowBackend(NumpyBackend):
    """Rank 1's pass-1 table overflowed: export(0) fails with RSA_ERR_CAPACITY."""

    def export(self, which):
        if which == 0 and self.fail:
            from ruleset_analysis_amd.native import NativeError, RSA_ERR_CAPACITY
            raise NativeError(RSA_ERR_CAPACITY, 'distinct-connection table overflow')
        return super().export(which)


def _overflow_worker(rank, world, port, payload, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from ruleset_analysis_amd.dist import ShardOverflow, merge
    n_rules, cap, cols = payload
    be = _OverflowBackend(n_rules, cap, cols)
    be.fail = rank == 1
    try:
        merge(be, dist, world, rank)
        out_q.put((rank, 'returned'))
    except ShardOverflow as e:
        out_q.put((rank, 'overflow %d' % e.code))
    dist.barrier()
    dist.destroy_process_group()


def test_merge_overflow_raises_on_every_rank():
    """One rank's table overflow reaches every rank as ShardOverflow (code
    RSA_ERR_CAPACITY) through the routing exchange, so bench.py reruns the job
    on all ranks instead of the healthy rank waiting in a collective."""
    dbj, info = synth.make_db(53, 100)
    tr = synth.make_traffic((dbj, info), 2000, seed=54)
    R = coracle.OracleRules(dbj)
    cols, ts, order = coracle.inputs_from_traffic(R, tr)
    gid, _ev = coracle.classify(R, cols['list'], cols['proto'], cols['src'], cols['dst'], cols['sport'],
                                cols['dport'])
    payload = (R.n_rules, 10, (gid, cols['flags'], cols['pspell'], cols['src'], cols['dst'], cols['sport'],
                               cols['dport'], ts, order))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker, args=(r, 2, port, payload, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    import queue
    import time
    deadline = time.time() + 120
    while len(got) < 2:
        try:
            r, what = q.get(timeout=2)
            got[r] = what
        except queue.Empty:
            if time.time() > deadline or any(p.exitcode not in (None, 0) for p in procs):
                for p in procs:
                    p.kill()
                pytest.fail('overflow protocol stalled: %s' % got)
    for p in procs:
        p.join(timeout=60)
    assert got == {0: 'overflow -4', 1: 'overflow -4'}
