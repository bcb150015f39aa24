#!/usr/bin/env python3
"""Benchmark of the ruleset-analysis hot path on MI355X.

Metric (BASELINE.json): log lines/sec classified (node) at 10k rules; % of the
HBM/VALU roofline.  Workload = BASELINE config 3 per GPU: a 10k-rule ACL
(replicated; no catch-all permit, so first matches spread over the whole
list), 125M synthetic ASA connection tuples per GPU (weak scaling: N GPUs
process N x 125M lines of one global log, order keys global), cap 1000.

One step = the whole job over the resident batch: pass 1 (first-match
classification fused with per-rule counters and the distinct-connection
table), cap resolution, pass 2 when any rule is capped, and emission of the
final connection records into HBM; for N > 1 also the merge (all_reduce of
counters, all_to_all of records to owner ranks, threshold all_reduce, pass-2
exchange, gather of the owners' records to rank 0).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import rsa_pkg  # noqa: E402

rsa_pkg.load()

from ruleset_analysis_amd import acldb, synth  # noqa: E402
from ruleset_analysis_amd.compile import CompiledRules  # noqa: E402
from ruleset_analysis_amd.engine import DeviceBatch, Engine  # noqa: E402
from ruleset_analysis_amd.pipeline import built_hit_count  # noqa: E402

BYTES_PER_LINE = 28          # 16 B tuple + 4 B timestamp code + 8 B order key
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
# int32 VALU lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes/cycle x 2.4 GHz (MI355X_MICROARCH.md:
# a wave issues one VALU instruction over 2 cycles, 32 lanes per cycle)
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9
SCATTER_ATOMIC_PEAK = 0.08e12 / 4   # 4-B device atomics/s, 64 lanes in 64 rows (MI355X_MICROARCH.md)
OPS_PER_EVAL = 8             # 2 per address range test x 2 + 2 per port range test x 2
CONFIGS = {
    # name: (rules, lines per GPU, cap, seed, zipf, interfaces, broad)
    'cfg3': (10000, 125_000_000, 1000, 3, None, ('outside',), False),
    'cfg3_broad': (10000, 125_000_000, 1000, 3, None, ('outside',), True),
    'cfg2': (1000, 100_000_000, 1000, 2, None, ('outside',), False),
    'cfg5': (2500, 100_000_000, 1000, 5, 1.1, ('outside', 'partner', 'vpn', 'extranet'), False),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_shard(dbj, info, compiled, n, rank, seed, zipf, device, chunk=8_000_000, world=1):
    """Generate this rank's contiguous slice of the global synthetic log straight
    into HBM, in chunks (host memory stays bounded)."""
    import torch
    tuples = torch.empty((n, 4), dtype=torch.int32, device=device)
    ts = torch.empty(n, dtype=torch.int32, device=device)
    order = torch.empty(n, dtype=torch.int64, device=device)
    n_hb = 0
    span_total = 3 * 3600 * world
    for k, a in enumerate(range(0, n, chunk)):
        m = min(chunk, n - a)
        g0 = rank * n + a                                # global line index of the chunk
        t0 = 15 * 86400 + (g0 * span_total) // (n * world)
        t1 = 15 * 86400 + ((g0 + m) * span_total) // (n * world)
        tr = synth.make_traffic((dbj, info), m, seed=seed * 1_000_003 + rank * 1009 + k, zipf=zipf, t0=t0,
                                span=max(t1 - t0, 1), cid0=1_000_000 + g0)
        tup, t, o = synth.pack(tr, compiled)
        n_hb += built_hit_count(tup)
        tuples[a:a + m].copy_(torch.from_numpy(tup.view(np.int32).reshape(-1, 4)))
        ts[a:a + m].copy_(torch.from_numpy(t.view(np.int32)))
        order[a:a + m].copy_(torch.from_numpy(o.view(np.int64)))
        log('shard: %d / %d lines generated' % (a + m, n))
    return DeviceBatch(tuples, ts, order), n_hb


def cpu_baseline(dbj, info, seconds=15.0):
    """The oracle's restatement of the reference pipeline (mapper | sort | reducer,
    pure Python like the reference) on a bounded sample of the same workload,
    one core."""
    from oracle import pipeline as op
    from oracle.crosscheck_2to3 import oracle_db
    acls, fws = oracle_db(dbj)
    tr = synth.make_traffic((dbj, info), 200_000, seed=99)
    lines = synth.render_lines(tr)
    # calibrate on a small prefix, then size the timed sample to ~`seconds`
    probe = 200
    t = time.perf_counter()
    op.run_pipeline(''.join(l + '\n' for l in lines[:probe]), 'fw1', acls, fws, cap=1000)
    per = (time.perf_counter() - t) / probe
    n = int(min(len(lines), max(probe, seconds / max(per, 1e-7))))
    text = ''.join(l + '\n' for l in lines[:n])
    t = time.perf_counter()
    op.run_pipeline(text, 'fw1', acls, fws, cap=1000)
    dt = time.perf_counter() - t
    return {'value': n / dt, 'unit': 'lines/s', 'cores': 1, 'kind': 'port',
            'sample': '%d lines of the same 10k-rule workload through oracle/pipeline.py '
                      '(mapper | LC_ALL=C sort | reducer restated in Python, 1 process), %.1f s' % (n, dt)}


def scan_work(compiled, batch, gids):
    """Sum over lines of E(t): the 1-based position of the
    first match in the line's compiled permit-only candidate list, or the list
    length when nothing matches; 0 for lines that are not classified.  Computed
    on the GPU from the pass-1 gids (a searchsorted per line)."""
    import torch
    ent, off = compiled.packed()
    dev = gids.device
    lists = (batch.tuples[:, 3] & 0xFFFF).long()
    valid = ((batch.tuples[:, 3] >> 16) & 1) == 1
    off_t = torch.from_numpy(off.astype(np.int64)).to(dev)
    length = (off_t[1:] - off_t[:-1])[lists]
    key = torch.from_numpy((np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off).astype(np.int64)) << 32)
                           | ent['gid'].astype(np.int64)).to(dev)
    q = (lists << 32) | gids.long().clamp(min=0)
    pos = torch.searchsorted(key, q) - off_t[lists] + 1
    e = torch.where(gids >= 0, pos, length)
    e = torch.where(valid, e, torch.zeros_like(e))
    return int(e.sum().item())


def read_traffic(name):
    """HBM bytes of the pass-1 kernel launches of one step (the 1/16 slice and the
    rest, summed like `achieved`) from a committed rocprofv3 PMC summary
    (profiles/<name>, written by tools/pmc_summary.py with the gfx950 FETCH_SIZE
    correction of MI355X_MICROARCH.md §HBM), if present for this workload."""
    path = os.path.join(ROOT, 'profiles', name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get('hbm_bytes_per_step')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--config', default='cfg3', choices=sorted(CONFIGS))
    ap.add_argument('--lines', type=int, default=0, help='override lines per GPU')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--filter-slice', type=int, default=0, help='override RSA_OPT_FILTER_SLICE')
    ap.add_argument('--opt', action='append', default=[], help='NAME=VALUE library option (e.g. FILTER_STEPS=3)')
    ap.add_argument('--no-index', action='store_true', help='classify with the plain linear scan')
    ap.add_argument('--prefix', type=int, default=0, help='entries per list scanned before the index')
    args = ap.parse_args()

    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    rules, lines, cap, seed, zipf, ifcs, broad = CONFIGS[args.config]
    if args.lines:
        lines = args.lines
    t_setup = time.perf_counter()
    dbj, info = synth.make_db(seed, rules, interfaces=ifcs, broad=broad)
    compiled = CompiledRules(acldb.load_json(dbj))
    compiled.ensure_lists()
    eng = Engine(local)
    eng.load_compiled(compiled, index=not args.no_index, prefix=args.prefix)
    from ruleset_analysis_amd import native
    if args.filter_slice:
        eng.set_option(native.RSA_OPT_FILTER_SLICE, args.filter_slice)
    for kv in args.opt:
        k, v = kv.split('=')
        eng.set_option(getattr(native, 'RSA_OPT_' + k), int(v))
    ent, _off = compiled.packed()
    batch, n_hb = build_shard(dbj, info, compiled, lines, rank, seed, zipf, eng.device, world=world)
    owner = None
    if world > 1:
        owner = Engine(local)
        owner.set_rule_count(compiled.n_rules)
    gbuf = torch.empty(lines, dtype=torch.int32, device=eng.device)
    torch.cuda.synchronize()
    log('rank %d setup %.1fs: %d rules, %d lists, %d entries, %d lines, %d hit+built' % (
        rank, time.perf_counter() - t_setup, compiled.n_rules, compiled.n_lists(), len(ent), lines, n_hb))

    # table capacity: the exact upper bound (every hit line a new connection);
    # only the slots a job uses are cleared between jobs
    capacity = max(n_hb, 1)
    pass1_launch_ms = []

    def step(timed):
        eng.reset(capacity, cap)
        eng.pass1(batch, gbuf)
        if timed:
            pass1_launch_ms.append(eng.last_pass1_times())
        if world == 1:
            if eng.resolve_cap():
                eng.pass2(batch, gbuf)
            recs = eng.emit_device('final')
            return recs.numel()
        from ruleset_analysis_amd.dist import EngineBackend, merge
        out = merge(EngineBackend(eng, owner, [batch], [gbuf], cap), dist, world, rank)
        return 0 if out is None else len(out[0])

    for _ in range(args.warmup):
        step(False)

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_rec = step(True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=eng.device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    classify_ms = float(np.mean([a for a, _b in pass1_launch_ms]))
    aggregate_ms = float(np.mean([b for _a, b in pass1_launch_ms]))
    pass1_ms = classify_ms + aggregate_ms
    # table-work counters of one more (untimed) step: lines combined, slot atomics
    eng.set_option(native.RSA_OPT_STATS, 1)
    eng.stats()
    step(False)
    torch.cuda.synchronize()
    tstats = eng.stats()
    eng.set_option(native.RSA_OPT_STATS, 0)
    sum_e = scan_work(compiled, batch, gbuf) if rank == 0 else 0
    if rank == 0:
        total_lines = lines * world * args.steps
        value = total_lines / dt
        achieved = BYTES_PER_LINE * lines / (pass1_ms * 1e-3) / 1e9
        traffic = read_traffic('%s_pass1_pmc.json' % args.config)
        res = {
            'metric': 'log lines/sec classified (node) at %d rules; %% of HBM roofline' % rules,
            'value': value, 'unit': 'lines/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'u32', 'data': 'synthetic (seeded ASA connection tuples, pre-parsed, '
                                                          'resident in HBM; seeded ACL, %s)' % (
                                                              'catch-all permits allowed' if broad else
                                                              'no catch-all permit'),
            'config': {'workload': '%s: %d-rule ACL, %d lines per GPU, cap %d' % (args.config, compiled.n_rules,
                                                                                  lines, cap),
                       'rules': compiled.n_rules, 'lines_per_gpu': lines, 'cap': cap, 'parallelism': 'dp%d' % world,
                       'records': n_rec},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'kernel': 'pass 1 = k_classify + k_tail + aggregation (k_aggregate, k_part_hist/scan/k_part_scatter, '
                                   'k_reduce<1>) over the filter slices + rest of one step',
                         'kernel_ms': pass1_ms, 'bytes_per_line': BYTES_PER_LINE,
                         'kernels': {
                             'classify_ms': classify_ms,
                             'aggregate_ms': aggregate_ms,
                             'classify_gbs': BYTES_PER_LINE * lines / (classify_ms * 1e-3) / 1e9,
                             'aggregate_table_lines': tstats[0],
                             'aggregate_slot_atomics': tstats[3],
                             'note': 'aggregation = record append in line order, counting sort by table region, '
                                     'per-region LDS reduction merged into region-owned slots with plain stores; '
                                     'table counters are collected only in the untimed stats step'},
                         'valu': {'achieved': OPS_PER_EVAL * sum_e / (pass1_ms * 1e-3) / 1e12,
                                  'peak': VALU_PEAK_OPS / 1e12, 'unit': 'Tops/s',
                                  'frac': OPS_PER_EVAL * sum_e / (pass1_ms * 1e-3) / VALU_PEAK_OPS,
                                  'mean_scan_position': sum_e / lines,
                                  'definition': 'SURVEY.md 8d linear-scan work: 8 int ops x E(t) per line, E = '
                                                '1-based first-match position in the permit-only candidate list '
                                                '(list length if unmatched); the index does less work than this, '
                                                'so frac > 1 is possible'}},
        }
        if world == 1 and not args.no_cpu_baseline:
            res['cpu_baseline'] = cpu_baseline(dbj, info)
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
