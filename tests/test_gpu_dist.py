"""The multi-GPU merge with the real HIP tables: two ranks on the box's one
GPU (gloo, tensors staged through host memory; the bench uses RCCL), each
classifying and aggregating its half of the log; rank 0's merged result must
equal the C oracle over the whole log.  The merge runs inside the library
(rsa_merge, csrc/merge.hip; impl 'lib', the product path) and, as a cross-check,
as the Python protocol of dist.py over the same engines (impl 'python')."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

import rsa_pkg

rsa_pkg.load()

from oracle import coracle  # noqa: E402
from ruleset_analysis_amd import acldb, synth  # noqa: E402

pytestmark = pytest.mark.gpu
NO = 0xFFFFFFFFFFFFFFFF


def _worker(rank, world, port, args, out_q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    opts = dict(args[5]) if len(args) > 5 else {}
    backend = opts.pop('backend', 'gloo')
    if backend == 'nccl':
        torch.cuda.set_device(0)
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
    else:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    from ruleset_analysis_amd.compile import CompiledRules
    from ruleset_analysis_amd.dist import EngineBackend, merge
    from ruleset_analysis_amd.engine import DeviceBatch, Engine
    from ruleset_analysis_amd.pipeline import built_hit_count
    seed, n_rules, n_lines, cap, zipf = args[:5]
    route_cap = opts.pop('route_cap', None)
    impl = opts.pop('impl', 'lib')
    force = opts.pop('force_exchange', False)
    dbj, info = synth.make_db(seed, n_rules)
    tr = synth.make_traffic((dbj, info), n_lines, seed=seed + 1, zipf=zipf)
    compiled = CompiledRules(acldb.load_json(dbj))
    compiled.ensure_lists()
    tup, ts, order = synth.pack(tr, compiled)
    cut = np.linspace(0, n_lines, world + 1).astype(int)
    a, b = cut[rank], cut[rank + 1]
    local = Engine(0)
    local.load_compiled(compiled)
    from ruleset_analysis_amd import native
    for k, v in opts.items():
        local.set_option(getattr(native, k), v)
    batch = DeviceBatch.from_numpy(tup[a:b], ts[a:b], order[a:b], local.device)
    local.reset(max(built_hit_count(tup[a:b]), 1), cap)
    g = torch.empty(batch.n, dtype=torch.int32, device=local.device)
    local.pass1(batch, g)
    if route_cap is not None:
        # every export first lands in a buffer of route_cap rows: the library
        # drops the rows past it and the exchange exports again at the exact
        # size (rsa_merge: RSA_OPT_ROUTE_ROWS; the Python protocol:
        # dist.route_records -> Exported.again)
        if impl == 'lib':
            local.set_option(native.RSA_OPT_ROUTE_ROWS, route_cap)
        else:
            orig = local.export_routed
            local.export_routed = lambda mode, world, capacity=None: orig(mode, world, capacity=capacity or route_cap)
            local._route_buf, local._route_cap = None, 0
    stats = {}
    out = merge(EngineBackend(local, [batch], [g], cap), dist, world, rank, stats=stats, impl=impl,
                force_exchange=force)
    if force:
        # the same job on the single-GPU path: the forced exchange must not change it
        single = local.run([batch], cap, max(built_hit_count(tup[a:b]), 1))
        assert np.array_equal(single.matches, out[1]) and np.array_equal(single.hits, out[2])
        key = lambda r: sorted(map(tuple, r.view(np.uint8).reshape(len(r), -1).tolist()))  # noqa: E731
        assert key(single.records) == key(out[0])
        assert stats['allreduce_bytes'] > 0, stats
    if route_cap is not None:
        assert stats.get('reexports', 0) >= 1, stats
    if rank == 0:
        out_q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def _run_two_ranks(args, world=2):
    from test_dist_merge import _free_port
    import queue
    import time
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out, deadline = None, time.time() + 400
    while out is None:
        try:
            out = q.get(timeout=2)
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail('worker died: %s' % [p.exitcode for p in procs])
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return out


def _oracle_inputs(seed, n_rules, n_lines, zipf):
    dbj, info = synth.make_db(seed, n_rules)
    tr = synth.make_traffic((dbj, info), n_lines, seed=seed + 1, zipf=zipf)
    R = coracle.OracleRules(dbj)
    return (R,) + tuple(coracle.inputs_from_traffic(R, tr))


def _check(out, R, cols, ots, oorder, cap):
    recs, matches, hits, distinct, thresh = out
    ref = coracle.run(R, cols, ots, oorder, cap)
    assert np.array_equal(matches, ref['matches'])
    assert np.array_equal(hits, ref['hits'])
    assert np.array_equal(thresh != NO, (ref['n_conns'] >= cap) & (cap > 0))
    got = sorted((int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']),
                  int(r['count']), int(r['first']), int(r['last'])) for r in recs)
    rows = ref['rows']
    want = sorted(zip(*(rows[k].astype(int).tolist() for k in ('gid', 'pspell', 'for_ip', 'to_ip', 'to_port',
                                                                  'count', 'first', 'last'))))
    assert got == want
    return ref


@pytest.mark.parametrize('cap,impl', [(12, 'lib'), (1000, 'lib'), (12, 'python')])
def test_two_ranks_one_gpu(cap, impl):
    args = (61, 700, 120000, cap, 1.2, {'impl': impl})
    out = _run_two_ranks(args)
    _check(out, *_oracle_inputs(61, 700, 120000, 1.2), cap)


@pytest.mark.parametrize('backend', ['nccl', 'gloo'])
def test_one_rank_forced_exchange(backend):
    """rsa_merge with RSA_MERGE_ALWAYS_EXCHANGE at world 1: every collective
    runs over the transport anyway -- over RCCL (rsa_merge_rccl: the library's
    own communicator, all_reduce and grouped send/recv to itself, the gathered
    rows included) or the host-buffer callbacks (gloo).  The result must equal
    the single-GPU job and the C oracle (the box has one GPU: RCCL refuses two
    ranks on one device, so this is where the RCCL transport runs here)."""
    args = (61, 700, 120000, 12, 1.2, {'backend': backend, 'force_exchange': True})
    out = _run_two_ranks(args, world=1)
    _check(out, *_oracle_inputs(61, 700, 120000, 1.2), 12)


def test_four_ranks_one_gpu():
    """Four ranks sharing the box's GPU, each with its own HIP table, cap 12
    engaged (Zipf traffic): the owner-routed exports (rsa_export_routed), the
    owners' imports and the global thresholds give the C oracle's result."""
    args = (71, 700, 160000, 12, 1.2)
    out = _run_two_ranks(args, world=4)
    ref = _check(out, *_oracle_inputs(71, 700, 160000, 1.2), 12)
    assert (ref['n_conns'] >= 12).sum() > 20


def test_two_ranks_atomic_import():
    """RSA_OPT_REGION_IMPORT=0: the owners merge the received entries with the
    per-record atomic import (CAS claims on empty keys).  A fresh table is
    written with empty keys only for this path (the region paths never read a
    slot they did not claim), so the option is set before the reset."""
    out = _run_two_ranks((61, 700, 120000, 12, 1.2, {'RSA_OPT_REGION_IMPORT': 0}))
    _check(out, *_oracle_inputs(61, 700, 120000, 1.2), 12)


@pytest.mark.parametrize('impl', ['lib', 'python'])
def test_two_ranks_export_overflow_reexport(impl):
    """The exports of both exchanges overflow a 1-row first buffer: the
    library drops the rows past it and reports the true per-owner counts, the
    exchange exports again at the exact size (reallocating the route buffer
    after the counts were exchanged) -- the result must still be the C
    oracle's."""
    out = _run_two_ranks((61, 700, 120000, 12, 1.2, {'route_cap': 1, 'impl': impl}))
    _check(out, *_oracle_inputs(61, 700, 120000, 1.2), 12)


def test_two_ranks_capped_only_after_merge():
    """Uniform traffic and a cap above every shard's own distinct count but
    below the merged count of some rules: no rank caps a rule locally, so each
    rank's own cap resolution finds nothing, yet the merge caps rules -- every
    rank's recount must still run under the global thresholds (ADVICE r04:
    a device-side 'nothing capped' skip keyed on the local count dropped the
    non-owners' pass-2 sums)."""
    seed, n_rules, n_lines = 67, 120, 60000
    R, cols, ots, oorder = _oracle_inputs(seed, n_rules, n_lines, None)
    cut = np.linspace(0, n_lines, 3).astype(int)
    big = n_lines + 1   # no rule capped (the oracle sizes its per-rule table from the cap)
    shard_max = 0
    for a, b in zip(cut[:-1], cut[1:]):
        sub = {k: v[a:b] for k, v in cols.items()}
        shard_max = max(shard_max, int(coracle.run(R, sub, ots[a:b], oorder[a:b], big)['n_conns'].max()))
    whole = coracle.run(R, cols, ots, oorder, big)['n_conns']
    cap = shard_max + 1
    assert (whole >= cap).sum() >= 1, 'workload does not cap any rule only after the merge'
    out = _run_two_ranks((seed, n_rules, n_lines, cap, None))
    ref = _check(out, R, cols, ots, oorder, cap)
    assert (ref['n_conns'] >= cap).any()


@pytest.mark.parametrize('backend', ['nccl', 'gloo'])
def test_bench_force_dist_one_gpu(tmp_path, backend):
    """bench.py's distributed step at world 1 on the box's GPU: RCCL (nccl) moves
    the device tensors itself (all_reduce, all_to_all_single with split sizes,
    all_gather), gloo stages them through host memory; the merged result must
    equal the C oracle."""
    from test_bench_spawn import check_dump_against_oracle, run_bench
    rules, lines, cap = 800, 400000, 40
    line, got = run_bench(tmp_path, ['--gpus', '1', '--force-dist', '--backend', backend, '--rules', str(rules),
                                     '--lines', str(lines), '--cap', str(cap), '--no-check'], timeout=400)
    assert line['n_gpus'] == 1 and line['config']['backend'] == backend
    check_dump_against_oracle(got, 1, rules, lines, cap)


def test_bench_capacity_rerun(tmp_path):
    """bench.py's table sizing: a job whose table is too small overflows
    (RSA_ERR_CAPACITY), is rerun at the exact bound, and the result still equals
    the C oracle."""
    from test_bench_spawn import check_dump_against_oracle, run_bench
    rules, lines, cap = 800, 400000, 40
    line, got = run_bench(tmp_path, ['--rules', str(rules), '--lines', str(lines), '--cap', str(cap),
                                     '--capacity', '2000', '--no-check'], timeout=400)
    assert line['config']['capacity_reruns'] == 1
    assert line['config']['table_capacity'] == line['config']['capacity_bound']
    check_dump_against_oracle(got, 1, rules, lines, cap)


def test_bench_learned_capacity(tmp_path):
    """The default sizing (4x the warmup job's distinct entries, at least the
    floor, at most the bound) gives the same result as the oracle, with the
    full-size checks of the bench green.  The floor is lowered so the learned
    size is really below the bound, and the log is long enough (4.5M lines:
    filter steps after 1M and 4M lines) that the capped rules stop adding
    entries, so 4x the used entries stays under the hit+BUILT bound (at 400k
    lines ~65% of the lines are distinct entries and 4x reaches the bound)."""
    from test_bench_spawn import check_dump_against_oracle, run_bench
    rules, lines, cap = 800, 4500000, 40
    line, got = run_bench(tmp_path, ['--rules', str(rules), '--lines', str(lines), '--cap', str(cap),
                                     '--capacity-floor', '4096'], timeout=400)
    assert line['config']['table_capacity'] < line['config']['capacity_bound']
    assert line['config']['capacity_reruns'] == 0
    assert line['checks']['ok']
    check_dump_against_oracle(got, 1, rules, lines, cap)


def test_bench_two_ranks_share_gpu_checks(tmp_path):
    """bench.py's N = 2 job (two rank processes on the box's one GPU, gloo):
    the full-size checks of the distributed job (the merged counters equal the
    all-reduced gid histograms, uncapped row counts equal the hit+BUILT lines on
    their owners, gathered rows = owner rows, index = linear scan, a rerun gives
    identical rows) are green, the gather to rank 0 is timed (gather_ms) and the
    exchange volume is reported -- and the dumped result equals the C oracle."""
    from test_bench_spawn import check_dump_against_oracle, run_bench
    rules, lines, cap = 800, 400000, 40
    line, got = run_bench(tmp_path, ['--gpus', '2', '--share-gpu', '--backend', 'gloo', '--rules', str(rules),
                                     '--lines', str(lines), '--cap', str(cap)], timeout=600)
    assert line['n_gpus'] == 2
    c = line['checks']
    assert c['ok'], c
    for k in ('matches_eq_gid_histogram', 'hits_eq_gid_histogram', 'uncapped_count_sum_eq_hit_built_lines',
              'gathered_rows_eq_owner_rows', 'index_gids_eq_linear_scan', 'rerun_identical_records',
              'owner_rows_only_own_rules'):
        assert c[k] is True, k
    assert c['uncapped_rules_checked'] > 0
    assert line['gather']['gather_ms'] > 0 and line['gather']['bytes_to_rank0'] > 0
    mx = line['merge_exchange']
    assert mx['route1_sent_bytes_total'] > 0 and mx['route1_sent_bytes_total'] == mx['route1_recv_bytes_total']
    check_dump_against_oracle(got, 2, rules, lines, cap)


def test_loopback_forced_exchange_in_process(engine):
    """rsa_merge at world 1 without a process group: every collective forced
    through the loopback transport (identity all_reduce, self copy) -- the
    records, counters and capped set equal the C oracle's."""
    from ruleset_analysis_amd.compile import CompiledRules
    from ruleset_analysis_amd.dist import EngineBackend, merge
    from ruleset_analysis_amd.engine import DeviceBatch
    from ruleset_analysis_amd.pipeline import built_hit_count
    import torch
    seed, n_rules, n_lines, cap = 63, 600, 90000, 15
    dbj, info = synth.make_db(seed, n_rules)
    tr = synth.make_traffic((dbj, info), n_lines, seed=seed + 1, zipf=1.2)
    compiled = CompiledRules(acldb.load_json(dbj))
    compiled.ensure_lists()
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    g = torch.empty(b.n, dtype=torch.int32, device=engine.device)
    for _ in range(2):   # twice: the second merge reuses the library's buffers
        engine.reset(max(built_hit_count(tup), 1), cap)
        engine.pass1(b, g)
        stats = {}
        out = merge(EngineBackend(engine, [b], [g], cap), None, 1, 0, force_exchange=True, stats=stats)
        ref = _check(out, *_oracle_inputs(seed, n_rules, n_lines, 1.2), cap)
        assert stats['allreduce_bytes'] > 0 and stats['pass2'] == bool((ref['n_conns'] >= cap).any())


def test_three_ranks_one_gpu_uneven_owners():
    """Three ranks sharing the GPU (owners gid % 3: uneven rule shares and
    shard sizes from a 3-way split) through rsa_merge, cap engaged."""
    args = (73, 701, 150001, 12, 1.2)
    out = _run_two_ranks(args, world=3)
    _check(out, *_oracle_inputs(73, 701, 150001, 1.2), 12)


def test_merge_abi_errors(engine):
    """The merge entry points' error behaviour through the C ABI: a transport
    with an out-of-range world or rank, missing callbacks at world 2, unknown
    flags, rsa_gather / rsa_merge_rows before any merge, and rows that do not
    fit the caller's buffer (RSA_ERR_CAPACITY with the count)."""
    import ctypes
    import torch
    from ruleset_analysis_amd import native
    from ruleset_analysis_amd.compile import CompiledRules
    from ruleset_analysis_amd.engine import DeviceBatch
    from ruleset_analysis_amd.pipeline import built_hit_count
    lib, h = engine.ctx.lib, engine.ctx.h
    dbj, info = synth.make_db(5, 200)
    tr = synth.make_traffic((dbj, info), 20000, seed=6)
    compiled = CompiledRules(acldb.load_json(dbj))
    compiled.ensure_lists()
    tup, ts, order = synth.pack(tr, compiled)
    engine.load_compiled(compiled)
    b = DeviceBatch.from_numpy(tup, ts, order, engine.device)
    g = torch.empty(b.n, dtype=torch.int32, device=engine.device)
    engine.reset(max(built_hit_count(tup), 1), 10)
    engine.pass1(b, g)
    info_ = native.MergeInfo()
    nores = native.ALL_REDUCE_FN(), native.ALL_TO_ALLV_FN()
    rows = ctypes.c_uint64(0)
    # a fresh context: nothing merged yet
    fresh = native.Ctx(0)
    assert lib.rsa_merge_rows(fresh.h, 0, None, 0, ctypes.byref(rows)) == native.RSA_ERR_STATE
    t1 = native.Transport(None, 1, 0, 1, *nores)
    assert lib.rsa_gather(fresh.h, ctypes.byref(t1), ctypes.byref(info_)) == native.RSA_ERR_STATE
    fresh.close()
    for world, rank in ((0, 0), (2, 2), (257, 0), (2, -1)):
        t = native.Transport(None, world, rank, 1, *nores)
        assert lib.rsa_merge(h, ctypes.byref(t), None, 0, 0, ctypes.byref(info_)) == native.RSA_ERR_ARG
    t2 = native.Transport(None, 2, 0, 1, *nores)
    assert lib.rsa_merge(h, ctypes.byref(t2), None, 0, 0, ctypes.byref(info_)) == native.RSA_ERR_ARG
    assert lib.rsa_merge(h, ctypes.byref(t1), None, 0, 8, ctypes.byref(info_)) == native.RSA_ERR_ARG
    # world 1 without collectives: the single-GPU job; its rows through rsa_merge_rows
    sb = native.ShardBatch(b.tuples.data_ptr(), b.ts.data_ptr(), b.order.data_ptr(), g.data_ptr(), b.n)
    assert lib.rsa_merge(h, ctypes.byref(t1), ctypes.byref(sb), 1, native.RSA_MERGE_GATHER,
                         ctypes.byref(info_)) == 0
    n = int(info_.n_rows)
    assert n > 1 and info_.owner_rows == n and info_.gather_rows == 0
    small = torch.empty((n - 1) * 40, dtype=torch.uint8, device=engine.device)
    assert lib.rsa_merge_rows(h, 1, ctypes.c_void_p(small.data_ptr()), n - 1, ctypes.byref(rows)) == \
        native.RSA_ERR_CAPACITY and rows.value == n
    full = torch.empty(n * 40, dtype=torch.uint8, device=engine.device)
    assert lib.rsa_merge_rows(h, 0, ctypes.c_void_p(full.data_ptr()), n, ctypes.byref(rows)) == 0
    res = engine.run([b], 10, capacity=max(built_hit_count(tup), 1))
    got = sorted(map(bytes, full.cpu().numpy().reshape(n, 40)))
    assert got == sorted(map(bytes, res.records.view(np.uint8).reshape(-1, 40)))
