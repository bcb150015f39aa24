#!/usr/bin/env python3
"""Throughput of the reducer drop-in (reducer_stream: GPU parse + aggregation)
on BASELINE config 1's sorted mapper stream (200-rule ACL, 1M synthetic ASA
lines, seed 1 -- the input bench.py's config-1 CPU baseline feeds to
``oracle.cli map | LC_ALL=C sort | oracle.cli reduce``), against the oracle's
restatement of connlist-reducer.py on the same bytes; the two reports must be
byte-identical.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rsa_pkg  # noqa: E402

rsa_pkg.load()
from ruleset_analysis_amd import acldb, synth  # noqa: E402
from ruleset_analysis_amd.compile import CompiledRules  # noqa: E402
from ruleset_analysis_amd.engine import Engine  # noqa: E402
from ruleset_analysis_amd.reducer_stream import ReducerStream  # noqa: E402
from ruleset_analysis_amd.report import mapper_output  # noqa: E402
from ruleset_analysis_amd.textparse import parse_text  # noqa: E402


def main():
    n_lines = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    cap = 1000
    dbj, info = synth.make_db(1, 200)
    tr = synth.make_traffic((dbj, info), n_lines, seed=101)
    text = ''.join(l + '\n' for l in synth.render_lines(tr)).encode('latin-1')
    db = acldb.load_json(dbj)
    eng = Engine(0)
    compiled = CompiledRules(db)
    compiled.ensure_lists()
    eng.load_compiled(compiled)
    parsed = parse_text(eng, 'fw1', text, db, compiled, need_order=False)
    gids = eng.classify_only(parsed.batch()).cpu().numpy()
    stream = mapper_output(parsed, gids, compiled).encode('latin-1')
    lines = stream.splitlines(True)
    lines.sort()                                   # LC_ALL=C sort: byte order
    data = b''.join(lines)
    eng.close()
    red = Engine(0)                                # the reducer's own ctx (no rule lists loaded)
    out = []
    best = None
    for rep in range(3):
        out = []
        job = ReducerStream(red, acldb.load_json(dbj), cap, out.append)
        red.torch.cuda.synchronize()
        t = time.perf_counter()
        for a in range(0, len(data), 16 << 20):
            job.feed(data[a:a + (16 << 20)])
        job.finish()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    if os.environ.get('RSA_PROFILE_HOST'):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        job = ReducerStream(red, acldb.load_json(dbj), cap, lambda t: None)
        pr.enable()
        for a in range(0, len(data), 16 << 20):
            job.feed(data[a:a + (16 << 20)])
        job.finish()
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats('cumulative').print_stats(25)
    got = ''.join(out)
    from oracle.crosscheck_2to3 import oracle_db
    from oracle.reducer import reduce_lines
    acls, _fws = oracle_db(dbj)
    t = time.perf_counter()
    want, _blocks = reduce_lines(data.decode('latin-1').splitlines(True), acls, cap)
    t_cpu = time.perf_counter() - t
    want = ''.join(l + '\n' for l in want)
    print(json.dumps({
        'metric': 'reducer drop-in lines/s (sorted mapper stream of BASELINE config 1)',
        'value': len(lines) / best, 'unit': 'lines/s', 'lines': len(lines), 'bytes': len(data), 'seconds': best,
        'what': 'ReducerStream over the stream in host memory: host->HBM copy, GPU line split + reducer parse, '
                'run decisions on the host, GPU aggregation (rsa_aggregate_gids), report text; best of 3',
        'cpu_baseline': {'value': len(lines) / t_cpu, 'unit': 'lines/s', 'seconds': t_cpu, 'cores': 1,
                         'kind': 'port', 'what': 'oracle/reducer.py (connlist-reducer.py restated), same bytes'},
        'identical_to_oracle': got == want}))


if __name__ == '__main__':
    main()
