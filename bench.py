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
exchange, gather of the owners' records to rank 0) -- the MI355X replacement of
the Hadoop shuffle (runAnalysis.sh:12,42-56).

Ranks: ``--gpus N`` spawns N rank processes (one per GPU, torch
multiprocessing, spawn context, before any GPU call in the parent); under
``torch.distributed.run`` the ranks come from RANK/WORLD_SIZE/LOCAL_RANK and
must agree with ``--gpus``.  Backend nccl (= RCCL over xGMI); ``--force-dist``
runs the distributed merge even at N = 1.  ``--cpu-model`` (TESTING, no GPU)
replaces the HIP library by tests/cpu_model.py so the spawn + merge path runs
on CPU with gloo.

Prints ONE JSON line on rank 0; after the timed
steps, untimed full-size checks (``checks``) unless ``--no-check``.
"""
import argparse
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import rsa_pkg  # noqa: E402

rsa_pkg.load()

from ruleset_analysis_amd import acldb, synth  # noqa: E402
from ruleset_analysis_amd.compile import CompiledRules, RECORD_DTYPE, TUPLE_DTYPE  # noqa: E402
from ruleset_analysis_amd.pipeline import built_hit_count  # noqa: E402

BYTES_PER_LINE = 28          # 16 B tuple + 4 B timestamp code + 8 B order key
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
N_SIMD = 256 * 4             # 256 CUs x 4 SIMDs
# int32 VALU lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes/cycle x 2.4 GHz (MI355X_MICROARCH.md:
# a wave64 VALU instruction occupies its SIMD for 2 cycles)
VALU_PEAK_OPS = N_SIMD * 32 * 2.4e9
OPS_PER_EVAL = 8             # 2 per address range test x 2 + 2 per port range test x 2
CONFIGS = {
    # ASA-shaped expanded ACLs (synth.make_db): rules, lines per GPU, cap, seed, zipf, interfaces, broad
    'cfg3': dict(kind='asa', rules=10000, lines=125_000_000, cap=1000, seed=3, zipf=None, ifcs=('outside',),
                 broad=False),
    'cfg3_broad': dict(kind='asa', rules=10000, lines=125_000_000, cap=1000, seed=3, zipf=None, ifcs=('outside',),
                       broad=True),
    'cfg2': dict(kind='asa', rules=1000, lines=100_000_000, cap=1000, seed=2, zipf=None, ifcs=('outside',),
                 broad=False),
    # 4 interfaces x 2.5k-rule ACLs; (src, dst, dport) Zipf s=1.1 over a population of 1e8 connections
    'cfg5': dict(kind='asa', rules=2500, lines=100_000_000, cap=1000, seed=5, zipf=1.1, population=10 ** 8,
                 ifcs=('outside', 'partner', 'vpn', 'extranet'), broad=False),
    # FortiGate policy set (synth_fg.make_config): 160 policies, 3 with 1024-65535 ranges, >= 3M expanded rules,
    # traffic biased to late or no match (BASELINE config 4, the long-scan worst case)
    'cfg4': dict(kind='fortigate', policies=160, wide=3, lines=100_000_000, cap=1000, seed=4, zipf=None),
}


class Workload(object):
    """A benchmark configuration: the rule DB, its compiled lists, and a
    generator of the global synthetic log."""

    def __init__(self, name, rules=0, cap=None):
        spec = dict(CONFIGS[name])
        self.name, self.kind = name, spec['kind']
        self.lines, self.seed, self.zipf = spec['lines'], spec['seed'], spec.get('zipf')
        self.population = spec.get('population')
        self.cap = spec['cap'] if cap is None else cap
        if self.kind == 'asa':
            self.rules = rules or spec['rules']
            self.dbj, self.info = synth.make_db(self.seed, self.rules, interfaces=spec['ifcs'], broad=spec['broad'])
            self.db = acldb.load_json(self.dbj)
            self.describe = '%d-rule ACL' % self.rules
            self.data = 'seeded ASA-shaped ACL, %s' % ('catch-all permits allowed' if spec['broad']
                                                        else 'no catch-all permit')
        else:
            from ruleset_analysis_amd import fortigate, synth_fg
            self.text, self.info = synth_fg.make_config(self.seed, n_policies=rules or spec['policies'],
                                                        n_wide=spec['wide'])
            self.db = fortigate.build_db(self.text)
            self.describe = 'FortiGate %d-policy set' % (rules or spec['policies'])
            self.data = 'seeded FortiGate config through the restated preprocessor; late/no-match traffic'
        self.compiled = CompiledRules(self.db)
        self.compiled.ensure_lists()

    def traffic(self, m, seed, t0, span, cid0):
        if self.kind == 'asa' and self.population:
            return synth.make_traffic_population((self.dbj, self.info), m, seed=seed, s=self.zipf,
                                                 population=self.population, t0=t0, span=span, cid0=cid0,
                                                 pop_seed=self.seed)
        if self.kind == 'asa':
            return synth.make_traffic((self.dbj, self.info), m, seed=seed, zipf=self.zipf, t0=t0, span=span,
                                      cid0=cid0)
        from ruleset_analysis_amd import synth_fg
        return synth_fg.make_traffic(self.info, m, seed=seed, t0=t0, span=span, cid0=cid0)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def die(msg, code=2):
    log('bench.py: ' + msg)
    sys.exit(code)


def shard_chunks(wl, n, rank, world=1, chunk=8_000_000):
    """This rank's contiguous slice of the global synthetic log, in chunks:
    yields (offset, traffic dict, packed tuples, ts codes, order keys)."""
    span_total = 3 * 3600 * world
    for k, a in enumerate(range(0, n, chunk)):
        m = min(chunk, n - a)
        g0 = rank * n + a                                # global line index of the chunk
        t0 = 15 * 86400 + (g0 * span_total) // (n * world)
        t1 = 15 * 86400 + ((g0 + m) * span_total) // (n * world)
        tr = wl.traffic(m, wl.seed * 1_000_003 + rank * 1009 + k, t0, max(t1 - t0, 1), 1_000_000 + g0)
        tup, t, o = synth.pack(tr, wl.compiled)
        yield a, tr, tup, t, o


def build_shard(wl, n, rank, device, world=1):
    """Generate this rank's shard straight into device memory (host memory stays bounded)."""
    import torch
    from ruleset_analysis_amd.engine import DeviceBatch
    tuples = torch.empty((n, 4), dtype=torch.int32, device=device)
    ts = torch.empty(n, dtype=torch.int32, device=device)
    order = torch.empty(n, dtype=torch.int64, device=device)
    n_hb = 0
    for a, _tr, tup, t, o in shard_chunks(wl, n, rank, world):
        m = len(tup)
        n_hb += built_hit_count(tup)
        tuples[a:a + m].copy_(torch.from_numpy(tup.view(np.int32).reshape(-1, 4)))
        ts[a:a + m].copy_(torch.from_numpy(t.view(np.int32)))
        order[a:a + m].copy_(torch.from_numpy(o.view(np.int64)))
        log('rank %d shard: %d / %d lines generated' % (rank, a + m, n))
    return DeviceBatch(tuples, ts, order), n_hb


def cpu_baseline(wl, seconds=15.0):
    """The reference pipeline restated on the CPU, timed on a bounded sample of
    the same workload.  ASA configs: the oracle's pure-Python mapper | sort |
    reducer (like the reference, one process).  FortiGate config: the expanded
    DB has millions of rules (no Python objects for them), so the C oracle
    (classify = the mapper's first-match scan, OpenMP over lines; reduce = the
    reducer loop) is timed instead."""
    if wl.kind != 'asa':
        from oracle import coracle
        R = coracle.OracleRules.from_fortigate(wl.text)
        n = 20000
        tr = wl.traffic(n, 99, 15 * 86400, 3 * 3600, 1_000_000)
        cols, ts, order = coracle.inputs_from_traffic(R, tr)
        t = time.perf_counter()
        coracle.run(R, cols, ts, order, wl.cap)
        dt = time.perf_counter() - t
        threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
        return {'value': n / dt, 'unit': 'lines/s', 'cores': threads, 'kind': 'port', 'host_cpus': os.cpu_count(),
                'sample': '%d lines of the same workload through oracle/rsa_oracle.c (linear first-match scan of the '
                          'expanded rules, OpenMP over lines, + reducer loop), %.1f s' % (n, dt)}
    from oracle import pipeline as op
    from oracle.crosscheck_2to3 import oracle_db
    acls, fws = oracle_db(wl.dbj)
    tr = synth.make_traffic((wl.dbj, wl.info), 200_000, seed=99)
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
    return {'value': n / dt, 'unit': 'lines/s', 'cores': 1, 'kind': 'port', 'host_cpus': os.cpu_count(),
            'sample': '%d lines of the same 10k-rule workload through oracle/pipeline.py '
                      '(mapper | LC_ALL=C sort | reducer restated in Python, 1 process), %.1f s' % (n, dt)}


def _hadoop_partition(key, n):
    """org.apache.hadoop.mapred.lib.HashPartitioner over a streaming Text key:
    (WritableComparator.hashBytes(key) & Integer.MAX_VALUE) % n, hashBytes =
    31 * h + (signed) byte from h = 1, 32-bit wrap (runAnalysis.sh:44 uses 4
    reducers)."""
    h = 1
    for b in key:
        h = (31 * h + (b - 256 if b > 127 else b)) & 0xFFFFFFFF
    return (h & 0x7FFFFFFF) % n


def reference_pipeline_baseline(n_lines=1_000_000, rules=200, seed=1, procs=None, reducers=4, broad=True,
                                single=True):
    """SURVEY.md §8d CPU baseline, BASELINE config 1: a 200-rule ACL and 1M
    synthetic ASA log lines through the reference's job restated in Python
    (oracle.cli: mapper.py / connlist-reducer.py as Unix filters), run as real
    processes on this host:

    (1) ``mapper | LC_ALL=C sort | reducer`` (one process each;
        skipped with single=False);
    (2) Hadoop-like: ``procs`` mappers over contiguous splits, map output
        partitioned by Hadoop's key hash into ``reducers`` parts
        (runAnalysis.sh:12,44), ``LC_ALL=C sort --parallel``, one reducer per part.

    ``rules``/``seed``/``broad`` pick the synth.make_db workload (the bench's
    own configuration for the same-workload baseline)."""
    import shutil
    import subprocess
    import tempfile
    # nproc mappers: the CPUs this job may use -- on the GPU box the job of one
    # GPU gets 16 of the host's CPUs (OMP_NUM_THREADS=16 there), although
    # os.cpu_count() shows the whole machine
    procs = procs or int(os.environ.get('OMP_NUM_THREADS') or len(os.sched_getaffinity(0)) or 1)
    dbj, info = synth.make_db(seed, rules, broad=broad)
    tr = synth.make_traffic((dbj, info), n_lines, seed=seed + 100)
    text = ''.join(l + '\n' for l in synth.render_lines(tr))
    work = tempfile.mkdtemp(prefix='rsa_cpu_baseline_')
    try:
        with open(os.path.join(work, 'db.json'), 'w') as f:
            json.dump(dbj, f)
        with open(os.path.join(work, 'log.txt'), 'w', encoding='latin-1', newline='') as f:
            f.write(text)
        env = dict(os.environ, LC_ALL='C', mapred_input_dir='/logs/fw1/part-00000', PYTHONPATH=ROOT,
                   OMP_NUM_THREADS='1')
        py = sys.executable
        t_single = None
        if single:
            t = time.perf_counter()
            subprocess.run('%s -m oracle.cli map db.json < log.txt | LC_ALL=C sort | %s -m oracle.cli reduce db.json '
                           '1000 > report.txt' % (py, py), shell=True, cwd=work, env=env, check=True)
            t_single = time.perf_counter() - t
        # Hadoop-like job
        lines = text.splitlines(True)
        cuts = np.linspace(0, len(lines), procs + 1).astype(int)
        for k in range(procs):
            with open(os.path.join(work, 'split%d.txt' % k), 'w', encoding='latin-1', newline='') as f:
                f.write(''.join(lines[cuts[k]:cuts[k + 1]]))
        t = time.perf_counter()
        mappers = [subprocess.Popen('%s -m oracle.cli map db.json < split%d.txt > map%d.txt' % (py, k, k), shell=True,
                                    cwd=work, env=env) for k in range(procs)]
        for m in mappers:
            if m.wait() != 0:
                raise RuntimeError('mapper failed')
        parts = [[] for _ in range(reducers)]
        for k in range(procs):
            with open(os.path.join(work, 'map%d.txt' % k), 'rb') as f:
                for rec in f:
                    body = rec[:-1] if rec.endswith(b'\n') else rec
                    tab = body.find(b'\t')
                    parts[_hadoop_partition(body if tab < 0 else body[:tab], reducers)].append(rec)
        for r in range(reducers):
            with open(os.path.join(work, 'part%d.txt' % r), 'wb') as f:
                f.write(b''.join(parts[r]))
        red = [subprocess.Popen('LC_ALL=C sort --parallel=%d part%d.txt | %s -m oracle.cli reduce db.json 1000 > '
                                'red%d.txt' % (max(procs // reducers, 1), r, py, r), shell=True, cwd=work, env=env)
               for r in range(reducers)]
        for m in red:
            if m.wait() != 0:
                raise RuntimeError('reducer failed')
        t_hadoop = time.perf_counter() - t
        hits = lambda txt: sum(int(l.split(': ')[1]) for l in txt.splitlines() if l.startswith('Total number of hits'))
        h2 = 0
        for r in range(reducers):
            with open(os.path.join(work, 'red%d.txt' % r), encoding='latin-1') as f:
                h2 += hits(f.read())
        h1 = h2
        if single:
            with open(os.path.join(work, 'report.txt'), encoding='latin-1') as f:
                h1 = hits(f.read())
            if h1 != h2:
                raise RuntimeError('the partitioned job disagrees with the single pipeline (%d vs %d hits)' % (h1, h2))
    finally:
        shutil.rmtree(work, ignore_errors=True)
    return {'config': '%d-rule ACL, %d synthetic ASA lines, seed %d' % (rules, n_lines, seed),
            'single': None if t_single is None else {
                'value': n_lines / t_single, 'unit': 'lines/s', 'wall_s': t_single, 'cores': 1, 'kind': 'port',
                'pipeline': 'oracle.cli map | LC_ALL=C sort | oracle.cli reduce'},
            'hadoop_like': {'value': n_lines / t_hadoop, 'unit': 'lines/s', 'wall_s': t_hadoop, 'cores': procs,
                            'kind': 'port', 'pipeline': '%d mappers, Hadoop HashPartitioner to %d parts, '
                                                        'sort --parallel, %d reducers' % (procs, reducers, reducers)},
            'host_cpus': os.cpu_count(), 'total_hits': h1}


def scan_work(compiled, batch, gids):
    """Sum over lines of E(t): the 1-based position of the
    first match in the line's permit-only candidate list of EXPANDED rules, or
    the list length when nothing matches; 0 for lines that are not classified.
    Computed on the GPU from the pass-1 gids: the expanded rules of a list at or
    before gid g are, per entry, the rules of its run with gid <= g."""
    import torch
    ent, off = compiled.packed()
    dev = gids.device
    lists = (batch.tuples[:, 3] & 0xFFFF).long()
    valid = ((batch.tuples[:, 3] >> 16) & 1) == 1
    step = ent['step'].astype(np.int64)
    stride = step & 0x7FFFFFFF
    span = np.where(step >> 31, ent['port_span'].astype(np.int64) & 0xFFFF, ent['port_span'].astype(np.int64) >> 16)
    count = np.where(stride > 0, span + 1, 1)
    # expanded gids of every list, ascending (runs unrolled)
    L = np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off).astype(np.int64))
    Lx = np.repeat(L, count)
    base = np.repeat(ent['gid'].astype(np.int64), count)
    k = np.arange(len(base)) - np.repeat(np.cumsum(count) - count, count)
    g = base + k * np.repeat(stride, count)
    key_np = np.unique((Lx << 32) | g)
    lens = np.bincount(key_np >> 32, minlength=len(off) - 1)
    starts = np.concatenate([[0], np.cumsum(lens)])
    key = torch.from_numpy(key_np).to(dev)
    st = torch.from_numpy(starts.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.astype(np.int64)).to(dev)
    q = (lists << 32) | gids.long().clamp(min=0)
    pos = torch.searchsorted(key, q) - st[lists] + 1
    e = torch.where(gids >= 0, pos, ln[lists])
    e = torch.where(valid, e, torch.zeros_like(e))
    return int(e.sum().item())


def read_profile(name):
    path = os.path.join(ROOT, 'profiles', name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def valu_busy(sq, kernel_prefix):
    """VALU busy of one kernel from a committed rocprofv3 SQ-counter summary:
    2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md cycle table) x
    SQ_INSTS_VALU / (SIMDs x per-XCD active cycles, GRBM_GUI_ACTIVE / 8)."""
    if not sq:
        return None
    # the kernel of that name that ran longest (the emitting classifier, not the
    # classify-only launches of the untimed checks; k_classify_pair for cfg4)
    best = None
    for name, c in sq.items():
        if name.startswith(kernel_prefix) and c.get('GRBM_GUI_ACTIVE'):
            if best is None or c['GRBM_GUI_ACTIVE'] > best['GRBM_GUI_ACTIVE']:
                best = c
    return None if best is None else 2.0 * best['SQ_INSTS_VALU'] / (N_SIMD * best['GRBM_GUI_ACTIVE'] / 8.0)


def record_checksum(recs_u8):
    """Order-independent checksum of a record set (sum of a 64-bit mix of each
    40-B row, mod 2^64) on the device."""
    import torch
    if recs_u8.numel() == 0:
        return 0
    w = recs_u8.view(-1, 40)[:, :40].contiguous().view(torch.int64).view(-1, 5)
    x = w[:, 0] * 0x100000001B3 + w[:, 1] * 0x9E3779B1 + w[:, 2] * 0x7F4A7C15 + w[:, 3] * 0x2545F491 + w[:, 4]
    x = x ^ (x >> 29)
    x = x * 0x5DEECE66D
    x = x ^ (x >> 31)
    return int(x.sum().item()) & 0xFFFFFFFFFFFFFFFF


def roofline_block(lines, classify_ms, aggregate_ms, launches, step_ms, pmc, sq, config):
    """Roofline of the dominant kernel, k_classify (+ its k_tail): algorithmic
    bytes per launch (28 B per line of the launch's filter slice, SURVEY.md
    8d) / its average launch time, both from the HIP events the library
    records on its own stream; traffic = the committed rocprofv3 FETCH_SIZE +
    WRITE_SIZE bytes of k_classify per launch.  Pass 1 as a whole and the
    whole step are reported beside it at the same 28 B per line."""
    launches = max(launches, 1.0)
    per_launch_bytes = BYTES_PER_LINE * lines / launches
    ms_launch = classify_ms / launches
    achieved = per_launch_bytes / (ms_launch * 1e-3) / 1e9
    traffic = None
    if pmc and 'k_classify' in pmc.get('kernels', {}):
        k = pmc['kernels']['k_classify']
        traffic = (k['read_bytes_per_step'] + k['write_bytes_per_step']) / launches
    pass1_ms = classify_ms + aggregate_ms
    return {
        'bound': 'hbm', 'kernel': 'k_classify', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
        'traffic_unit': 'HBM bytes per k_classify launch (rocprofv3 FETCH_SIZE x2, calibrated for its streaming reads in profiles/r03l_fetch_calibration.json, + WRITE_SIZE)',
        'traffic_source': 'profiles/%s_pass1_pmc.json' % config if traffic is not None else None,
        'launches_per_step': launches, 'ms_per_launch': ms_launch, 'algorithmic_bytes_per_launch': per_launch_bytes,
        'bytes_per_line': BYTES_PER_LINE,
        'valu_busy': valu_busy(sq, 'k_classify'),
        'valu_source': 'profiles/%s_sq.json' % config if sq else None,
        'valu_definition': '2 cycles x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)',
        'pass1': {'ms': pass1_ms, 'classify_ms': classify_ms, 'aggregate_ms': aggregate_ms,
                  'achieved': BYTES_PER_LINE * lines / (pass1_ms * 1e-3) / 1e9,
                  'frac': BYTES_PER_LINE * lines / (pass1_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                  'traffic_per_step': pmc.get('hbm_bytes_per_step') if pmc else None},
        'step': {'ms': step_ms, 'achieved': BYTES_PER_LINE * lines / (step_ms * 1e-3) / 1e9,
                 'frac': BYTES_PER_LINE * lines / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
    }


def full_size_checks(eng, batch, gbuf, n_rules, cap, recs_final, owner_rows=None):
    """Untimed properties of the benched job at full size (no oracle: too large):
    matches == per-rule line counts of the gids, hits likewise over hit lines,
    every uncapped rule's connection counts sum to its hit+BUILT lines, and the
    index-classified gids equal a linear scan of the whole lists."""
    import torch
    out = {}
    flags = (batch.tuples[:, 3] >> 16) & 0xFF
    g = gbuf.long()
    ok = g >= 0
    m = torch.bincount(g[ok], minlength=n_rules)[:n_rules]
    hitm = ok & ((flags & 2) != 0)
    h = torch.bincount(g[hitm], minlength=n_rules)[:n_rules]
    out['matches_eq_gid_histogram'] = bool(torch.equal(m, eng.counters['matches'][:n_rules]))
    out['hits_eq_gid_histogram'] = bool(torch.equal(h, eng.counters['hits'][:n_rules]))
    out['sum_matches_eq_classified_lines'] = int(eng.counters['matches'][:n_rules].sum().item()) == int(ok.sum().item())
    hb = hitm & ((flags & 4) != 0)
    need = torch.bincount(g[hb], minlength=n_rules)[:n_rules]
    rows = recs_final.view(-1, 40)
    rg = rows[:, 8:12].contiguous().view(torch.int32).view(-1).long()
    rc = rows[:, 24:28].contiguous().view(torch.int32).view(-1).long()
    got = torch.zeros(n_rules, dtype=torch.int64, device=g.device).index_add_(0, rg, rc)
    unc = eng.counters['thresh'][:n_rules] == -1
    if cap == 0:
        unc = torch.zeros_like(unc)
    out['uncapped_rules_checked'] = int(unc.sum().item())
    out['uncapped_count_sum_eq_hit_built_lines'] = bool(torch.equal(got[unc], need[unc]))
    # the index vs the plain linear scan of the compiled lists, every line
    eng.use_index(False)
    g2 = eng.classify_only(batch)
    eng.use_index(True)
    out['index_gids_eq_linear_scan'] = bool(torch.equal(g2, gbuf))
    out['ok'] = all(v for k, v in out.items() if isinstance(v, bool))
    return out


def dist_full_size_checks(eng, batch, gbuf, n_rules, cap, last, step, dist, world, rank):
    """The N = 1 full-size properties (full_size_checks) over the distributed
    job's merged result, untimed, every rank taking part: the merged line and
    hit counters equal the gid histograms of all shards (all_reduced), every
    uncapped rule's row counts (on its owner) sum to its hit+BUILT lines of all
    shards, each owner keeps only its own rules' rows, rank 0's gathered rows
    are every owner's rows (checksum), the index gids equal a linear scan on
    every shard, and a rerun of the whole job gives every owner the identical
    rows.  Flags are AND-ed over the ranks; returned on rank 0 (None elsewhere)."""
    import torch
    from ruleset_analysis_amd.dist import _all_reduce
    dev = gbuf.device
    part = last['part']
    flags = (batch.tuples[:, 3] >> 16) & 0xFF
    g = gbuf.long()
    ok = g >= 0
    hitm = ok & ((flags & 2) != 0)
    hb = hitm & ((flags & 4) != 0)
    hist = torch.cat([torch.bincount(g[ok], minlength=n_rules)[:n_rules],
                      torch.bincount(g[hitm], minlength=n_rules)[:n_rules],
                      torch.bincount(g[hb], minlength=n_rules)[:n_rules],
                      ok.sum().view(1)]).to(torch.int64)
    _all_reduce(hist, dist, None)
    m, h, need, n_cls = hist[:n_rules], hist[n_rules:2 * n_rules], hist[2 * n_rules:3 * n_rules], hist[-1]
    out = {}
    out['matches_eq_gid_histogram'] = bool(torch.equal(m, part.matches[:n_rules]))
    out['hits_eq_gid_histogram'] = bool(torch.equal(h, part.hits[:n_rules]))
    out['sum_matches_eq_classified_lines'] = int(part.matches[:n_rules].sum().item()) == int(n_cls.item())
    rows = part.final.view(-1, 40)
    rg = rows[:, 8:12].contiguous().view(torch.int32).view(-1).long()
    rc = rows[:, 24:28].contiguous().view(torch.int32).view(-1).long()
    got = torch.zeros(n_rules, dtype=torch.int64, device=dev).index_add_(0, rg, rc)
    own = (torch.arange(n_rules, device=dev) % world) == rank
    unc = own & (part.thresh[:n_rules] == -1)
    if cap == 0:
        unc = torch.zeros_like(unc)
    out['owner_rows_only_own_rules'] = bool(((rg % world) == rank).all().item())
    out['uncapped_count_sum_eq_hit_built_lines'] = bool(torch.equal(got[unc], need[unc]))
    n_unc = torch.tensor([int(unc.sum().item())], dtype=torch.int64, device=dev)
    _all_reduce(n_unc, dist, None)
    out['uncapped_rules_checked'] = int(n_unc.item())
    # rank 0's gathered rows = every owner's rows (the checksum is a sum over rows)
    c_own = record_checksum(part.final)
    cs = torch.tensor([c_own - (1 << 64) if c_own >= 1 << 63 else c_own], dtype=torch.int64, device=dev)
    _all_reduce(cs, dist, None)
    c_sum = int(cs.item()) & 0xFFFFFFFFFFFFFFFF
    out['gathered_rows_eq_owner_rows'] = True   # (decided on rank 0, which holds the gathered rows)
    if rank == 0:
        c_merged = record_checksum(last['merged'][0])
        out['gathered_rows_eq_owner_rows'] = c_merged == c_sum
        out['merged_record_checksum'] = '%016x' % c_merged
    eng.use_index(False)
    g2 = eng.classify_only(batch)
    eng.use_index(True)
    out['index_gids_eq_linear_scan'] = bool(torch.equal(g2, gbuf))
    # a rerun of the whole distributed job: the identical rows on every owner
    step(False)
    out['rerun_identical_records'] = record_checksum(last['part'].final) == c_own
    flags_ok = sorted(k for k, v in out.items() if isinstance(v, bool))   # the same keys on every rank
    f = torch.tensor([int(out.get(k, True)) for k in flags_ok], dtype=torch.int64, device=dev)
    _all_reduce(f, dist, None, op=dist.ReduceOp.MIN)
    for k, v in zip(flags_ok, f.tolist()):
        out[k] = bool(v)
    out['ok'] = all(out[k] for k in flags_ok)
    return out if rank == 0 else None


def merge_exchange_summary(last, dist, world, eng):
    """The rows the last timed job's merge moved (dist.merge stats), summed
    and maxed over the ranks, in bytes of 40-B rows; projected per rank for
    other world sizes in DESIGN.md section 6."""
    import torch
    from ruleset_analysis_amd.dist import _all_reduce
    st = last.get('merge_stats') or {}
    keys = ['route1_sent_rows', 'route1_recv_rows', 'route2_sent_rows', 'route2_recv_rows', 'owner_rows']
    v = torch.tensor([int(st.get(k, 0)) for k in keys], dtype=torch.int64, device=eng.device)
    vmax = v.clone()
    _all_reduce(v, dist, None)
    _all_reduce(vmax, dist, None, op=dist.ReduceOp.MAX)
    rec = RECORD_DTYPE.itemsize
    out = {'row_bytes': rec, 'allreduce_bytes_per_rank': int(st.get('allreduce_bytes', 0)),
           'pass2_exchange': bool(st.get('pass2', False))}
    for k, a, b in zip(keys, v.tolist(), vmax.tolist()):
        out[k.replace('_rows', '_bytes') + '_total'] = a * rec
        out[k.replace('_rows', '_bytes') + '_max_rank'] = b * rec
    return out


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


class ResultOut(object):
    """This process's real stdout, kept for the ONE result line.  Everything
    else written to fd 1 -- RCCL's version banner at communicator init (seen
    at world 1 with --force-dist), prints of the libraries -- goes to stderr
    instead, so the driver reads exactly one JSON line from stdout."""

    def __init__(self):
        sys.stdout.flush()
        self.fd = os.dup(1)
        os.dup2(2, 1)

    def line(self, obj):
        sys.stdout.flush()
        os.write(self.fd, (json.dumps(obj) + '\n').encode())


def rank_main(args, rank, world, local):
    import torch
    result_out = ResultOut()
    dist = None
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        if args.backend == 'nccl':
            torch.cuda.set_device(local)
            dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', local))
        else:
            dist.init_process_group('gloo', rank=rank, world_size=world)
    t_setup = time.perf_counter()
    wl = Workload(args.config, rules=args.rules, cap=args.cap)
    lines = args.lines or wl.lines
    cap = wl.cap
    compiled = wl.compiled
    if args.cpu_model:
        return _cpu_model_rank(args, wl, lines, cap, rank, world, dist, result_out)

    from ruleset_analysis_amd import native
    from ruleset_analysis_amd.dist import EngineBackend, ShardOverflow, gather_rows, merge
    from ruleset_analysis_amd.engine import Engine
    # --share-gpu (diagnosis: several ranks on one card, gloo): rank -> card rank % cards
    eng = Engine(local % max(torch.cuda.device_count(), 1) if args.share_gpu else local)
    eng.load_compiled(compiled, index=not args.no_index, prefix=args.prefix, kind=args.index)
    if args.filter_slice:
        eng.set_option(native.RSA_OPT_FILTER_SLICE, args.filter_slice)
    for kv in args.opt:
        k, v = kv.split('=')
        eng.set_option(getattr(native, 'RSA_OPT_' + k), int(v))
    ent, _off = compiled.packed()
    batch, n_hb = build_shard(wl, lines, rank, eng.device, world=world)
    gbuf = torch.empty(lines, dtype=torch.int32, device=eng.device)
    torch.cuda.synchronize()
    log('rank %d setup %.1fs: %d rules, %d lists, %d entries, %d lines, %d hit+built' % (
        rank, time.perf_counter() - t_setup, compiled.n_rules, compiled.n_lists(), len(ent), lines, n_hb))

    # table capacity.  The exact upper bound is every hit+BUILT line a new
    # connection (clamped by the library to its largest table); the first
    # warmup job runs with it, and later jobs over the same log are sized to 4x
    # the distinct entries that job actually used (max over ranks), the way a
    # stream of similar batches is sized from the last one: a 4x smaller table
    # has 4x fewer regions and spans far fewer pages, so the slot traffic of
    # the region sort and reduction is cheaper.  A job whose
    # table overflows anyway fails with RSA_ERR_CAPACITY and is rerun at the
    # bound (the re-run is inside the timed step when it happens; with several
    # ranks the merge raises ShardOverflow on all of them and they rerun
    # together, at the largest bound of any rank).
    bound = max(n_hb, 1)
    if dist is not None:
        tb = torch.tensor([bound], dtype=torch.int64, device=eng.device)
        dist.all_reduce(tb, op=dist.ReduceOp.MAX)
        bound = int(tb.item())
    sizing = {'capacity': args.capacity or bound, 'learn': not args.capacity, 'reruns': 0}
    pass1_launch_ms = []
    pass1_launches = []
    last = {}
    pending = {'pass1_times': False}

    def read_pass1_times():
        # a timed job's pass-1 event times, read at the start of the next step
        # (or after the timed loop): that job ended in a host read, so its
        # events are complete, and no extra host round trip sits in the step
        if pending['pass1_times']:
            pass1_launch_ms.append(eng.last_pass1_times())
            pass1_launches.append(eng.last_pass1_launches())
            pending['pass1_times'] = False

    def step(timed):
        read_pass1_times()
        n_t, n_l = len(pass1_launch_ms), len(pass1_launches)
        try:
            r = job(timed)
        except (native.NativeError, ShardOverflow) as e:
            pending['pass1_times'] = False
            # multi-GPU: the merge raises ShardOverflow on every rank together,
            # with the entries the fullest owner table needs (its shard's plus
            # the imported ones: the per-shard bound does not cover those)
            need = max(bound, getattr(e, 'needed', 0))
            if e.code != native.RSA_ERR_CAPACITY or sizing['capacity'] >= need:
                raise
            del pass1_launch_ms[n_t:], pass1_launches[n_l:]
            sizing['capacity'] = need
            sizing['reruns'] += 1
            r = job(timed)
        return r

    def learn_capacity():
        used = torch.tensor([eng.table_size()], dtype=torch.int64, device=eng.device)
        if dist is not None:
            dist.all_reduce(used, op=dist.ReduceOp.MAX)
        sizing['capacity'] = min(bound, max(4 * int(used.item()), args.capacity_floor))
        sizing['learn'] = False

    def job(timed):
        eng.reset(sizing['capacity'], cap)
        eng.pass1(batch, gbuf)
        pending['pass1_times'] = timed
        if dist is None:
            # the capped-rule count stays on the device: the recount's kernels
            # skip their work there when no rule is capped
            eng.resolve_cap(sync=False)
            eng.pass2(batch, gbuf)
            recs = eng.emit_device('final')
            last['recs'] = recs
            return recs.numel() // RECORD_DTYPE.itemsize
        # each owner's final rows stay in its HBM -- the reference's job ends
        # with NUM_REDUCERS reducer outputs, separate part files of its -output
        # directory (runAnalysis.sh:12,42-56) -- and are gathered to rank 0 for
        # the checks and --dump after the timed steps (gather_rows)
        mstats = {}
        part = merge(EngineBackend(eng, [batch], [gbuf], cap), dist, world, rank, to_host=False, gather=False,
                     stats=mstats, impl=args.merge_impl, force_exchange=world == 1 and args.merge_impl == 'lib')
        last['part'], last['merge_stats'] = part, mstats
        return part.final.numel() // RECORD_DTYPE.itemsize

    cold_ms = None
    for w in range(max(args.warmup, 1 if sizing['learn'] else 0)):
        if w == 0:
            # a cold one-shot job: first table allocation + clear (k_table_init)
            # at the exact bound, nothing learned yet
            torch.cuda.synchronize()
            tc = time.perf_counter()
        step(False)
        if w == 0:
            torch.cuda.synchronize()
            cold_ms = (time.perf_counter() - tc) * 1e3
        if sizing['learn']:
            learn_capacity()

    phase_prof = os.environ.get('RSA_PHASE_PROF') == '1'   # PROFILING: a -DRSA_PHASE_PROF library variant
    if phase_prof:
        import ctypes
        ph = (ctypes.c_uint64 * 25)()
        eng.ctx.call('rsa_phase_prof', ph, ctypes.c_int(1))
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_rec = step(True)
    torch.cuda.synchronize()
    read_pass1_times()
    if phase_prof:
        eng.ctx.call('rsa_phase_prof', ph, ctypes.c_int(1))
        v = [int(x) for x in ph]
        names = ['tuple+list', 'prefix', 'pruning', 'group0', 'tasks', 'verify', 'resid+chain', 'emit']
        log('phase_prof cycles/wave-iteration: ' + json.dumps(
            {nm: round(v[k] / max(v[8], 1), 1) for k, nm in enumerate(names)}) + ' iterations %d' % v[8])
        for name, b in (('k_reduce<1>', 9), ('k_reduce<2>', 17)):
            log('phase_prof %s cycles/workgroup: ' % name + json.dumps(
                {nm: round(v[b + k] / max(v[b + 3], 1), 1) for k, nm in enumerate(('setup', 'insert', 'flush'))}) +
                ' workgroups %d; inside: ' % v[b + 3] + json.dumps(
                    {nm: round(v[b + 4 + k] / max(v[b + 3], 1), 1) for k, nm in
                     enumerate(('record_load_wait', 'lds_insert', 'flush_claims', 'flush_writes'))}))
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
    gather = None
    if dist is not None:
        # the last job's owner rows to rank 0, timed on its own
        # beside the owner-rows step (barrier + synchronize on both sides, max
        # over ranks): the reference's job also ends with separate reducer part
        # files that `hadoop dfs -getmerge` pairs afterwards (README.md:35-38)
        g_ms = []
        for _ in range(max(1, min(args.steps, 5))):
            dist.barrier()
            torch.cuda.synchronize()
            tg = time.perf_counter()
            last['merged'] = gather_rows(last['part'], dist, world, rank, to_host=False)
            torch.cuda.synchronize()
            dist.barrier()
            g_ms.append((time.perf_counter() - tg) * 1e3)
        tg = torch.tensor([float(np.mean(g_ms))], dtype=torch.float64, device=eng.device)
        dist.all_reduce(tg, op=dist.ReduceOp.MAX)
        gather = {'gather_ms': float(tg.item()), 'repeats': len(g_ms)}
        if last['merged'] is not None:   # rank 0: every owner's rows
            n_rec = last['merged'][0].numel() // RECORD_DTYPE.itemsize
        gather['bytes_to_rank0'] = int(last['merge_stats'].get('gather_rows_to_rank0', 0)) * RECORD_DTYPE.itemsize
    if args.dump and rank == 0:
        _dump(args.dump, last, eng, cap)
    checks = None
    if not args.no_check and dist is None:
        # untimed: a second job must give the bit-identical record set, then the
        # full-size properties of its result
        c1 = record_checksum(last['recs'])
        step(False)
        c2 = record_checksum(last['recs'])
        checks = {'rerun_identical_records': c1 == c2, 'record_checksum': '%016x' % c1}
        checks.update(full_size_checks(eng, batch, gbuf, compiled.n_rules, cap, last['recs']))
        checks['ok'] = checks['ok'] and checks['rerun_identical_records']
        log('checks: %s' % json.dumps(checks))
    elif not args.no_check:
        # untimed checks of the distributed job at full size, the N = 1
        # properties over the merged result (dist_full_size_checks)
        checks = dist_full_size_checks(eng, batch, gbuf, compiled.n_rules, cap, last, step, dist, world, rank)
        if world == 1 and rank == 0:
            eng.reset(sizing['capacity'], cap)
            eng.pass1(batch, gbuf)
            if eng.resolve_cap():
                eng.pass2(batch, gbuf)
            checks['merged_eq_single_gpu_records'] = record_checksum(eng.emit_device('final')) == \
                int(checks['merged_record_checksum'], 16)
            checks['ok'] = checks['ok'] and checks['merged_eq_single_gpu_records']
        if rank == 0:
            log('checks: %s' % json.dumps(checks))
    merge_exchange = merge_exchange_summary(last, dist, world, eng) if dist is not None else None
    sum_e = scan_work(compiled, batch, gbuf) if rank == 0 else 0
    if rank == 0:
        total_lines = lines * world * args.steps
        value = total_lines / dt
        pmc = read_profile('%s_pass1_pmc.json' % args.config)
        sq = read_profile('%s_sq.json' % args.config)
        res = {
            'metric': 'log lines/sec classified (node) at %d rules; %% of HBM roofline' % (
                wl.rules if wl.kind == 'asa' else compiled.n_rules),
            'value': value, 'unit': 'lines/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'u32',
            'data': 'synthetic (seeded ASA connection tuples, pre-parsed, resident in HBM; %s)' % wl.data,
            'config': {'workload': '%s: %s (%d expanded rules, %d candidate-list entries), %d lines per GPU, cap %d'
                                   % (args.config, wl.describe, compiled.n_rules, len(ent), lines, cap),
                       'rules': compiled.n_rules, 'entries': len(ent), 'lines_per_gpu': lines, 'cap': cap,
                       'parallelism': 'dp%d' % world, 'index': 'none' if args.no_index else getattr(eng, 'index_kind', args.index),
                       'backend': args.backend if dist is not None else 'none', 'records': n_rec,
                       'merge': ('rsa_merge_rccl' if args.backend == 'nccl' else 'rsa_merge (host-buffer transport)')
                                if dist is not None and args.merge_impl == 'lib' else
                                ('dist.merge (Python protocol)' if dist is not None else 'none'),
                       'table_capacity': sizing['capacity'], 'capacity_bound': bound,
                       'capacity_reruns': sizing['reruns'],
                       'cold_job_ms': cold_ms,
                       'cold_job': 'rank-local wall time of the first (untimed) job: table allocated and cleared '
                                   'at the exact bound, no learned size',
                       'capacity_policy': 'first warmup job at the bound (hit+BUILT lines), then 4x the distinct '
                                          'entries it used; rerun at the bound on overflow'},
            'roofline': roofline_block(lines, classify_ms, aggregate_ms, float(np.mean(pass1_launches)),
                                       dt / args.steps * 1e3, pmc, sq, args.config),
            'scan_work': {'mean_scan_position': sum_e / lines,
                          'linear_scan_equivalent_tops': OPS_PER_EVAL * sum_e / (pass1_ms * 1e-3) / 1e12,
                          'valu_peak_tops': VALU_PEAK_OPS / 1e12,
                          'definition': 'SURVEY.md 8d linear-scan work: 8 int ops x E(t) per line, E = 1-based '
                                        'first-match position in the permit-only candidate list (list length if '
                                        'unmatched); the index does far less work than this, so this is a '
                                        'scan-equivalent rate, not a utilisation'},
            'checks': checks,
        }
        if dist is not None:
            res['gather'] = dict(gather, ms_per_step_with_gather=dt / args.steps * 1e3 + gather['gather_ms'],
                                 value_with_gather=total_lines / (dt + args.steps * gather['gather_ms'] * 1e-3),
                                 definition='the owners\' final rows gathered to rank 0 (dist.gather_rows), timed '
                                            'after the timed steps on its own; value/ms_per_step leave each owner\'s '
                                            'rows in its HBM like the reference\'s reducer part files')
            res['merge_exchange'] = merge_exchange
        if world == 1 and not args.no_cpu_baseline:
            res['cpu_baseline'] = cpu_baseline(wl)
            spec = CONFIGS[args.config]
            if wl.kind == 'asa' and not spec.get('zipf') and len(spec['ifcs']) == 1 and args.baseline_same_lines:
                # the same workload through the restated reference JOB on the
                # host's cores, Hadoop-like (mappers over splits, key-hash
                # partition to 4 reducers, sort): the headline CPU baseline,
                # the single-core sample beside it
                t = time.perf_counter()
                par = reference_pipeline_baseline(n_lines=args.baseline_same_lines, rules=wl.rules, seed=wl.seed,
                                                  broad=spec['broad'], single=False,
                                                  procs=args.baseline_procs or None)
                hl = par['hadoop_like']
                one = res['cpu_baseline']
                res['cpu_baseline'] = {
                    'value': hl['value'], 'unit': 'lines/s', 'cores': hl['cores'], 'kind': 'port',
                    'host_cpus': os.cpu_count(),
                    'sample': '%d lines of the same %d-rule workload (synth seed %d, %s) through the restated '
                              'reference job as real processes: %s; wall %.1f s' % (
                                  args.baseline_same_lines, wl.rules, wl.seed, wl.data, hl['pipeline'], hl['wall_s']),
                    'single_core': one, 'measure_s': time.perf_counter() - t}
            if not args.no_config1:
                # SURVEY.md 8d's config-1 job (BASELINE config 1: 1M lines, 200
                # rules; the single pipeline and the Hadoop-like variant), run
                # here on this host as real processes (~30 s)
                t = time.perf_counter()
                c1 = reference_pipeline_baseline(n_lines=args.baseline_lines, procs=args.baseline_procs or None)
                c1['source'] = 'measured in this bench run (bench.py reference_pipeline_baseline)'
                c1['measure_s'] = time.perf_counter() - t
                res['cpu_baseline']['config1'] = c1
        result_out.line(res)
    if dist is not None:
        dist.destroy_process_group()
    return 0


_TEXT_WL = None


def _render_chunk(job):
    """(offset, m, rank) -> the rendered log bytes of that chunk (fork worker)."""
    a, m, k = job
    wl = _TEXT_WL
    t0 = 15 * 86400 + a // 2000
    tr = wl.traffic(m, wl.seed * 1_000_003 + 7919 + k, t0, max(m // 2000, 1), 1_000_000 + a)
    return ('\n'.join(synth.render_lines(tr)) + '\n').encode('latin-1'), a


def text_main(args):
    """--text: the fused job from log TEXT resident in HBM:
    line split + parse + order keys (textparse.hip) + classify + aggregate.
    The text is rendered on the host by forked workers before the GPU is
    touched (not timed)."""
    global _TEXT_WL
    import multiprocessing
    result_out = ResultOut()
    wl = Workload(args.config, rules=args.rules, cap=args.cap)
    if wl.kind != 'asa':
        die('--text renders ASA log lines: use an ASA config')
    lines = args.lines or 16_000_000
    chunk = 500_000
    _TEXT_WL = wl
    t_r = time.perf_counter()
    jobs = [(a, min(chunk, lines - a), k) for k, a in enumerate(range(0, lines, chunk))]
    with multiprocessing.get_context('fork').Pool(min(16, len(jobs))) as pool:
        parts = sorted(pool.map(_render_chunk, jobs), key=lambda x: x[1])
    data = b''.join(p for p, _a in parts)
    del parts
    log('rendered %d lines, %.2f GB of text in %.1fs' % (lines, len(data) / 1e9, time.perf_counter() - t_r))
    import ctypes
    import torch
    from ruleset_analysis_amd import textparse
    from ruleset_analysis_amd.engine import DeviceBatch, Engine
    compiled = wl.compiled
    eng = Engine(0)
    ifcs, _names = textparse.interface_table(wl.db, compiled, wl.info['host'])
    spells = textparse.spell_table(list(textparse.DEFAULT_SPELLS))
    eng.load_compiled(compiled, index=not args.no_index, prefix=args.prefix, kind=args.index)
    from ruleset_analysis_amd import native
    for kv in args.opt:
        k, v = kv.split('=')
        eng.set_option(getattr(native, 'RSA_OPT_' + k), int(v))
    dev = eng.device
    text = textparse._device_bytes(torch, data, dev)
    n = lines
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    tup = torch.empty((n, 4), dtype=torch.int32, device=dev)
    ts = torch.empty(n, dtype=torch.int32, device=dev)
    disp = torch.empty(n, dtype=torch.int32, device=dev)
    order = torch.empty(n, dtype=torch.int64, device=dev)
    gbuf = torch.empty(n, dtype=torch.int32, device=dev)
    v = lambda t: ctypes.c_void_p(t.data_ptr())
    hp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ctx = eng.ctx
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    phases = []
    last = {}
    group = torch.empty(n, dtype=torch.int32, device=dev)

    def step(timed):
        # split -> parse -> classify -> order keys within each rule (the reducer
        # only compares one rule's lines: pipeline.analyze_text) -> aggregate
        ev[0].record()
        # one pass over the text: offsets and the line count (the offset
        # buffer is sized for the lines the generator rendered)
        nl = ctypes.c_uint64(0)
        ctx.call('rsa_text_split', v(text), ctypes.c_uint64(len(data)), v(off), ctypes.c_uint64(n), ctypes.byref(nl))
        if nl.value != n:
            die('line count %d != %d' % (nl.value, n))
        ev[1].record()
        ctx.call('rsa_parse_text', v(text), v(off), ctypes.c_uint64(n), hp(ifcs), ctypes.c_uint32(len(ifcs)),
                 hp(spells), ctypes.c_uint32(len(spells)), v(tup), v(ts), v(disp))
        ev[2].record()
        ctx.call('rsa_classify_only', v(tup), ctypes.c_uint64(n), v(gbuf))
        flags = (tup[:, 3] >> 16) & 0xFF
        both = 0x06
        hb = (flags & both) == both
        torch.where(hb & (gbuf >= 0), gbuf, torch.full_like(gbuf, -1), out=group)
        ev[3].record()
        ctx.call('rsa_order_keys_grouped', v(text), v(off), ctypes.c_uint64(n), v(group), ctypes.c_uint64(0), v(order))
        ev[4].record()
        n_host = int(((disp & 0xFF) == textparse.LINE_HOST).sum().item())
        if n_host:
            die('%d synthetic lines outside the device grammar' % n_host)
        n_hb = int(hb.sum().item())
        b = DeviceBatch(tup, ts, order, gbuf)
        eng.reset(max(n_hb, 1), wl.cap)
        eng.pass1(b)
        if eng.resolve_cap():
            eng.pass2(b)
        last['recs'] = eng.emit_device('final')
        ev[5].record()
        if timed:
            torch.cuda.synchronize()
            phases.append([ev[k].elapsed_time(ev[k + 1]) for k in range(5)])

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ph = np.mean(np.array(phases), axis=0)
    checks = None
    if not args.no_check:
        # untimed: the device parse equals the generator's packed form, order
        # keys rank the line bytes (sampled adjacent pairs), and the job's
        # records equal those of the same job from the packed tuples
        ok = True
        h_off = off.cpu().numpy()
        gt = tup.cpu().numpy().reshape(-1).view(np.uint8).view(TUPLE_DTYPE)
        pk = []
        for (a, m, k) in jobs:
            tr = wl.traffic(m, wl.seed * 1_000_003 + 7919 + k, 15 * 86400 + a // 2000, max(m // 2000, 1),
                            1_000_000 + a)
            pk.append(synth.pack(tr, compiled)[0])
        pk = np.concatenate(pk)
        cls = (disp & 0xFF).cpu().numpy() == textparse.LINE_CLASSIFY
        same_tuples = bool(np.array_equal(gt[cls].view(np.uint8), pk[cls].view(np.uint8))) and \
            not pk['flags'][~cls].any()
        perm = torch.argsort(order).cpu().numpy()
        grp = group.cpu().numpy()
        rng = np.random.default_rng(0)
        sample = rng.integers(0, n - 1, 100_000)
        line = lambda i: data[h_off[i]:h_off[i + 1] - 1]
        # adjacent ranks of one rule's lines are in byte order (ranks are grouped by rule)
        sorted_pairs = all(line(perm[j]) <= line(perm[j + 1]) for j in sample
                           if grp[perm[j]] >= 0 and grp[perm[j]] == grp[perm[j + 1]])
        distinct = bool(torch.unique(order).numel() == n)
        c_text = record_checksum(last['recs'])
        b2 = DeviceBatch.from_numpy(pk, ts.cpu().numpy().view(np.uint32), order.cpu().numpy().view(np.uint64), dev)
        eng.reset(max(built_hit_count(pk), 1), wl.cap)
        eng.pass1(b2, gbuf)
        if eng.resolve_cap():
            eng.pass2(b2, gbuf)
        c_packed = record_checksum(eng.emit_device('final'))
        ok = same_tuples and sorted_pairs and distinct and c_text == c_packed
        checks = {'tuples_eq_generator': same_tuples, 'order_sorted_sampled_pairs': bool(sorted_pairs),
                  'order_keys_distinct': distinct, 'records_eq_packed_job': c_text == c_packed, 'ok': bool(ok)}
        log('checks: %s' % json.dumps(checks))
    text_bytes = len(data)
    parse_gbs = (text_bytes + 32 * n) / (ph[1] * 1e-3) / 1e9
    res = {
        'metric': 'log lines/sec from TEXT in HBM: line split + parse + classify + order keys + aggregate (1 GPU)',
        'value': n * args.steps / dt, 'unit': 'lines/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'u8',
        'data': 'synthetic ASA log text rendered on the host (%s), resident in HBM' % wl.data,
        'config': {'workload': '%s text: %d lines, %.2f GB, %d expanded rules, cap %d'
                               % (args.config, n, text_bytes / 1e9, compiled.n_rules, wl.cap),
                   'lines': n, 'text_bytes': text_bytes, 'parallelism': 'dp1'},
        'phases_ms': {'split': ph[0], 'parse': ph[1], 'classify': ph[2], 'order_keys_within_rules': ph[3],
                      'aggregate_job': ph[4]},
        'roofline': {'bound': 'hbm', 'kernel': 'k_parse', 'achieved': parse_gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': parse_gbs / HBM_PEAK_GBS, 'traffic': None,
                     'bytes': 'text bytes read + 32 B/line (off 8, tuple 16, ts 4, disp 4)'},
        'checks': checks,
    }
    result_out.line(res)
    return 0


def _dump(path, last, eng, cap):
    """TESTING: rank 0 writes the merged (or single-GPU) result as npz."""
    if 'merged' in last:
        from ruleset_analysis_amd.dist import merged_to_host
        recs, matches, hits, distinct, thresh = merged_to_host(last['merged'])
    else:
        res = eng.results(cap)
        recs, matches, hits, distinct, thresh = res.records, res.matches, res.hits, res.distinct, res.thresh
    np.savez(path, records=recs.view(np.uint8), matches=matches, hits=hits, distinct=distinct, thresh=thresh)


def _cpu_model_rank(args, wl, lines, cap, rank, world, dist, result_out):
    """TESTING: one rank of the spawn + merge path with the CPU model of
    tests/cpu_model.py in place of the HIP library (no GPU)."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import cpu_model
    from ruleset_analysis_amd.dist import merge
    compiled = wl.compiled
    ent, off = compiled.packed()
    parts = list(shard_chunks(wl, lines, rank, world))
    tup = np.concatenate([p[2] for p in parts])
    ts = np.concatenate([p[3] for p in parts])
    order = np.concatenate([p[4] for p in parts])
    gids = cpu_model.classify_entries(ent, off, tup)
    t0 = time.perf_counter()
    out = None
    for _ in range(max(args.steps, 1)):
        out = merge(cpu_model.NumpyBackend.from_packed(compiled.n_rules, cap, gids, tup, ts, order), dist, world, rank)
    dist.barrier()
    dt = time.perf_counter() - t0
    if rank == 0:
        if args.dump:
            recs, matches, hits, distinct, thresh = out
            np.savez(args.dump, records=recs.view(np.uint8), matches=matches, hits=hits, distinct=distinct,
                     thresh=thresh)
        result_out.line({'metric': 'TESTING cpu-model merge (not a measurement)', 'value': lines * world / dt,
                         'unit': 'lines/s', 'n_gpus': world, 'steps': args.steps, 'cpu_model': True,
                         'records': len(out[0])})
    dist.destroy_process_group()
    return 0


def _spawned(args, rank, world, port):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.exit(rank_main(args, rank, world, rank))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--config', default='cfg3', choices=sorted(CONFIGS))
    ap.add_argument('--lines', type=int, default=0, help='override lines per GPU')
    ap.add_argument('--rules', type=int, default=0, help='override the expanded rule count')
    ap.add_argument('--cap', type=int, default=None, help='override the per-rule connection cap')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'])
    ap.add_argument('--force-dist', action='store_true',
                    help='run the distributed merge even with one rank (every collective runs: '
                         'RSA_MERGE_ALWAYS_EXCHANGE)')
    ap.add_argument('--merge-impl', default='lib', choices=['lib', 'python'],
                    help='the merge inside the library (rsa_merge, default) or the Python protocol of dist.py')
    ap.add_argument('--cpu-model', action='store_true', help='TESTING: CPU model instead of the HIP library')
    ap.add_argument('--dump', default='', help='TESTING: rank 0 writes the final result (npz) here')
    ap.add_argument('--no-check', action='store_true', help='skip the untimed full-size checks')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--share-gpu', action='store_true',
                    help='DIAGNOSIS ONLY: let --gpus exceed the visible cards, ranks sharing them (gloo)')
    ap.add_argument('--no-config1', action='store_true',
                    help='skip the config-1 CPU pipeline (1M lines) that the default line measures beside the GPU job')
    ap.add_argument('--cpu-baseline-only', action='store_true',
                    help='run only the SURVEY.md 8d CPU baseline (config 1 through the restated reference job)')
    ap.add_argument('--baseline-lines', type=int, default=1_000_000)
    ap.add_argument('--baseline-procs', type=int, default=0)
    ap.add_argument('--baseline-same-lines', type=int, default=160_000,
                    help='lines of the headline CPU baseline (the bench workload through the Hadoop-like restated '
                         'reference job on the host cores; 0 = only the single-core sample)')
    ap.add_argument('--filter-slice', type=int, default=0, help='override RSA_OPT_FILTER_SLICE')
    ap.add_argument('--opt', action='append', default=[], help='NAME=VALUE library option (e.g. FILTER_STEPS=3)')
    ap.add_argument('--no-index', action='store_true', help='classify with the plain linear scan')
    ap.add_argument('--index', default='auto', choices=('auto', 'pht', 'bucket', 'bucket-filtered'),
                    help='classification index: auto (default: pht while its image fits LDS, else bucket), the '
                         'pruned perfect-hash index or the partial-key bucket index (without / with LDS row filters)')
    ap.add_argument('--capacity', type=int, default=0, help='EXPERIMENT: table capacity (default: hit+built lines)')
    ap.add_argument('--capacity-floor', type=int, default=1 << 20,
                    help='TESTING: smallest learned table capacity (default 2^20)')
    ap.add_argument('--prefix', type=int, default=0, help='entries per list scanned before the index')
    ap.add_argument('--text', action='store_true',
                    help='the fused job from log text in HBM (GPU parse + order keys + classify + aggregate)')
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.cpu_baseline_only:
        print(json.dumps(reference_pipeline_baseline(n_lines=args.baseline_lines, procs=args.baseline_procs or None)),
              flush=True)
        return
    if args.text:
        if args.gpus != 1 or 'WORLD_SIZE' in os.environ:
            die('--text runs on one GPU')
        sys.exit(text_main(args))
    if args.cpu_model and args.backend != 'gloo':
        die('--cpu-model runs without a GPU: use --backend gloo')
    if 'WORLD_SIZE' in os.environ and 'RANK' in os.environ:
        # launched by torch.distributed.run: one process per rank already
        world = int(os.environ['WORLD_SIZE'])
        if world != args.gpus:
            die('WORLD_SIZE=%d but --gpus %d: launch with --nproc-per-node equal to --gpus' % (world, args.gpus))
        sys.exit(rank_main(args, int(os.environ['RANK']), world, int(os.environ.get('LOCAL_RANK', '0'))))
    world = args.gpus
    if world < 1:
        die('--gpus must be >= 1')
    if not args.cpu_model:
        import torch
        n_dev = torch.cuda.device_count()   # counts devices without initialising the GPU
        if world > n_dev and not args.share_gpu:
            die('--gpus %d but %d GPU(s) visible' % (world, n_dev))
        if args.share_gpu and args.backend != 'gloo':
            die('--share-gpu runs the ranks over gloo (--backend gloo)')
    if world == 1:
        if args.force_dist:
            os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()), RANK='0', WORLD_SIZE='1',
                              LOCAL_RANK='0')
        sys.exit(rank_main(args, 0, 1, 0))
    # one process per rank; this parent never touches the GPU
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_spawned, args=(args, r, world, port)) for r in range(world)]
    for p in procs:
        p.start()
    rc = 0
    while procs:
        for p in list(procs):
            p.join(timeout=1.0)
            if p.exitcode is None:
                continue
            procs.remove(p)
            if p.exitcode != 0:
                rc = rc or (p.exitcode if p.exitcode > 0 else 1)
                log('bench.py: a rank exited with %d; stopping the others' % p.exitcode)
                for q in procs:
                    q.join(timeout=30)
                    if q.exitcode is None:
                        q.terminate()
    sys.exit(rc)


if __name__ == '__main__':
    main()
