#!/usr/bin/env python3
"""Per-stage timing of the hot path on one GPU (HIP events on the library's
stream): classify only, pass 1 (classify + aggregate), cap resolution, pass 2,
emit.  Usage: python tools/microbench.py [--lines N] [--rules R] [--reps K]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rsa_pkg  # noqa: E402

rsa_pkg.load()
import torch  # noqa: E402

from bench import build_shard  # noqa: E402
from ruleset_analysis_amd import acldb, synth  # noqa: E402
from ruleset_analysis_amd.compile import CompiledRules  # noqa: E402
from ruleset_analysis_amd.engine import Engine  # noqa: E402


def timed(fn, reps):
    out = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    out.sort()
    print('timed: %.3f ms' % out[len(out) // 2], file=sys.stderr, flush=True)
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lines', type=int, default=20_000_000)
    ap.add_argument('--rules', type=int, default=10000)
    ap.add_argument('--cap', type=int, default=1000)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--zipf', type=float, default=0.0)
    ap.add_argument('--broad', action='store_true', help='allow catch-all permits (short scans)')
    ap.add_argument('--scan', action='store_true', help='also time the plain linear scan')
    args = ap.parse_args()
    dbj, info = synth.make_db(3, args.rules, broad=args.broad)
    compiled = CompiledRules(acldb.load_json(dbj))
    compiled.ensure_lists()
    eng = Engine(0)
    eng.load_compiled(compiled)
    ent, off = compiled.packed()
    batch, n_hb = build_shard(dbj, info, compiled, args.lines, 0, 3, args.zipf or None, eng.device)
    g = torch.empty(args.lines, dtype=torch.int32, device=eng.device)
    cap = args.cap
    eng.reset(n_hb, cap)
    eng.pass1(batch, g)
    size = eng.table_size()
    res = {'lines': args.lines, 'rules': compiled.n_rules, 'entries': len(ent), 'hit_built': n_hb,
           'distinct': size}
    res['classify_only_ms'] = timed(lambda: eng.classify_only(batch, g), args.reps)
    from ruleset_analysis_amd import native
    for pre in (0, 32, 256):
        eng.load_compiled(compiled, prefix=pre)
        res['classify_prefix%d_ms' % pre] = timed(lambda: eng.classify_only(batch, g), args.reps)
    eng.load_compiled(compiled)
    if args.scan:
        eng.use_index(False)
        res['classify_scan_ms'] = timed(lambda: eng.classify_only(batch, g), args.reps)
        eng.use_index(True)

    def p1():
        eng.reset(int(size * 1.25), cap)
        eng.pass1(batch, g)
    res['reset_ms'] = timed(lambda: eng.reset(int(size * 1.25), cap), args.reps)
    res['reset_pass1_ms'] = timed(p1, args.reps)
    for mask, name in ((1, 'no_counters'), (2, 'no_table'), (3, 'no_agg')):
        eng.set_option(native.RSA_OPT_PROFILE_SKIP, mask)
        res['pass1_%s_ms' % name] = timed(p1, args.reps)
    eng.set_option(native.RSA_OPT_PROFILE_SKIP, 0)
    for steps in (1, 2, 4, 5):
        eng.set_option(native.RSA_OPT_FILTER_STEPS, steps)
        res['reset_pass1_steps%d_ms' % steps] = timed(p1, args.reps)
    eng.set_option(native.RSA_OPT_FILTER_STEPS, 3)   # library default
    eng.reset(int(size * 1.25), cap)
    eng.pass1(batch, g)
    t = time.perf_counter()
    ncap = eng.resolve_cap()
    torch.cuda.synchronize()
    res['resolve_cap_ms'] = (time.perf_counter() - t) * 1e3
    res['n_capped'] = ncap
    res['pass2_ms'] = timed(lambda: eng.pass2(batch, g), 1)
    t = time.perf_counter()
    recs = eng.emit_device('final')
    torch.cuda.synchronize()
    res['emit_ms'] = (time.perf_counter() - t) * 1e3
    res['records'] = recs.numel() // 40
    res['classify_Mlines_s'] = args.lines / res['classify_only_ms'] / 1e3
    print(json.dumps(res))


if __name__ == '__main__':
    main()
