"""bench.py's full-size checks of the distributed job (dist_full_size_checks)
and its exchange summary, run by two gloo ranks on CPU with the CPU model of
the HIP table (tests/cpu_model.py) standing in for the engine: every rank must
take part in the same collectives with the same flag vector, the flags must be
green on a correct merge, and a corrupted owner row must turn them red."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rsa_pkg

rsa_pkg.load()   # spawned workers import this module without conftest


class _Batch(object):
    def __init__(self, tup):
        self.tuples = torch.from_numpy(np.ascontiguousarray(tup).view(np.int32).reshape(-1, 4).copy())


class _Eng(object):
    """What dist_full_size_checks asks of the engine: the linear-scan switch
    and classify_only (the CPU model's gids either way)."""

    def __init__(self, gids):
        self.gids = gids

    def use_index(self, on):
        pass

    def classify_only(self, batch):
        return self.gids.clone()


def _worker(rank, world, port, corrupt, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, 'tests'))
    import bench
    import cpu_model
    from ruleset_analysis_amd.dist import gather_rows, merge
    wl = bench.Workload('cfg3', rules=300, cap=15)
    ent, off = wl.compiled.packed()
    parts = list(bench.shard_chunks(wl, 12000, rank, world))
    tup = np.concatenate([p[2] for p in parts])
    ts = np.concatenate([p[3] for p in parts])
    order = np.concatenate([p[4] for p in parts])
    gids = cpu_model.classify_entries(ent, off, tup)
    last = {}

    def step(_timed):
        be = cpu_model.NumpyBackend.from_packed(wl.compiled.n_rules, 15, gids, tup, ts, order)
        st = {}
        last['part'] = merge(be, dist, world, rank, gather=False, stats=st)
        last['merge_stats'] = st
        part = last['part']
        if corrupt and rank == 1:
            # the count of one row of an uncapped rule (every job alike)
            rows = part.final.view(-1, 40)
            rg = rows[:, 8:12].contiguous().view(torch.int32).view(-1).long()
            k = int(torch.nonzero(part.thresh[rg] == -1)[0, 0])
            part.final[40 * k + 24] ^= 1
        return 0

    step(False)
    last['merged'] = gather_rows(last['part'], dist, world, rank, to_host=False)
    g = torch.from_numpy(gids.astype(np.int32))
    checks = bench.dist_full_size_checks(_Eng(g), _Batch(tup), g, wl.compiled.n_rules, 15, last, step, dist, world,
                                         rank)
    ex = bench.merge_exchange_summary(last, dist, world, type('E', (), {'device': torch.device('cpu')})())
    if rank == 0:
        out_q.put((checks, ex))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('corrupt', [False, True])
def test_dist_full_size_checks_two_ranks(corrupt):
    from test_dist_merge import _free_port
    import queue
    import time
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, corrupt, q)) for r in range(2)]
    for p in procs:
        p.start()
    out, deadline = None, time.time() + 300
    while out is None:
        try:
            out = q.get(timeout=2)
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail('worker died: %s' % [p.exitcode for p in procs])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    checks, ex = out
    if corrupt:
        # rank 1's corrupted row: its rule's counts no longer sum to its lines
        assert not checks['ok'] and not checks['uncapped_count_sum_eq_hit_built_lines']
        assert checks['matches_eq_gid_histogram'] and checks['rerun_identical_records']
    else:
        assert checks['ok'], checks
        assert checks['uncapped_rules_checked'] > 0
        assert checks['gathered_rows_eq_owner_rows'] and checks['rerun_identical_records']
    assert ex['route1_sent_bytes_total'] == ex['route1_recv_bytes_total'] > 0
    assert ex['pass2_exchange'] is True
