#!/usr/bin/env python3
"""Per-stage timing of the hot path on one GPU, one line per measurement
(flushed, so a slow stage is visible while it runs).  HIP events on the
library's stream.  Usage:
  python tools/stage_probe.py [--lines N] [--rules R] [--stages a,b,...]
Stages: classify (classify only), pass1 (reset + pass 1), skip1/skip2/skip3
(pass 1 with RSA_OPT_PROFILE_SKIP, results invalid), steps<k> (pass 1 with
FILTER_STEPS=k), job (reset + pass 1 + cap + pass 2 + emit), prefix<p>
(classify only with the index rebuilt for prefix p)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rsa_pkg  # noqa: E402

rsa_pkg.load()
import torch  # noqa: E402

from bench import build_shard, CONFIGS  # noqa: E402
from ruleset_analysis_amd import acldb, native, synth  # noqa: E402
from ruleset_analysis_amd.compile import CompiledRules  # noqa: E402
from ruleset_analysis_amd.engine import Engine  # noqa: E402


def say(*a):
    print(*a, flush=True)


def timed(name, fn, reps):
    out = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
        say('  %s rep: %.3f ms' % (name, out[-1]))
    out.sort()
    say('%s: median %.3f ms' % (name, out[len(out) // 2]))
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='cfg3', choices=sorted(CONFIGS))
    ap.add_argument('--lines', type=int, default=0)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--prefix', type=int, default=64)
    ap.add_argument('--capacity', type=int, default=0, help='table capacity (default: hit+built lines)')
    ap.add_argument('--stages', default='classify,pass1,skip1,skip2,skip3,job')
    args = ap.parse_args()
    rules, lines, cap, seed, zipf, ifcs, broad = CONFIGS[args.config]
    lines = args.lines or lines
    dbj, info = synth.make_db(seed, rules, interfaces=ifcs, broad=broad)
    compiled = CompiledRules(acldb.load_json(dbj))
    compiled.ensure_lists()
    eng = Engine(0)
    eng.load_compiled(compiled, prefix=args.prefix)
    batch, n_hb = build_shard(dbj, info, compiled, lines, 0, seed, zipf, eng.device)
    g = torch.empty(lines, dtype=torch.int32, device=eng.device)
    torch.cuda.synchronize()
    say('setup done: %d lines, %d hit+built, image %d words' % (lines, n_hb, len(compiled.index(args.prefix)[0])))

    capacity = args.capacity or n_hb

    def p1():
        eng.reset(capacity, cap)
        eng.pass1(batch, g)

    def job():
        p1()
        if eng.resolve_cap():
            eng.pass2(batch, g)
        eng.emit_device('final')

    for st in args.stages.split(','):
        if st == 'classify':
            timed(st, lambda: eng.classify_only(batch, g), args.reps)
        elif st == 'pass1':
            timed(st, p1, args.reps)
            say('  pass1 library events: classify %.3f ms, aggregate %.3f ms; table entries %d (capacity %d)' % (
                eng.last_pass1_times() + (eng.table_size(), capacity)))
        elif st.startswith('rskip'):
            eng.set_option(native.RSA_OPT_PROFILE_SKIP, int(st[5:]))
            timed(st, p1, args.reps)
            say('  pass1 library events: classify %.3f ms, aggregate %.3f ms' % eng.last_pass1_times())
            eng.set_option(native.RSA_OPT_PROFILE_SKIP, 0)
        elif st.startswith('skip'):
            eng.set_option(native.RSA_OPT_PROFILE_SKIP, int(st[4:]))
            timed(st, p1, args.reps)
            eng.set_option(native.RSA_OPT_PROFILE_SKIP, 0)
        elif st.startswith('steps'):
            eng.set_option(native.RSA_OPT_FILTER_STEPS, int(st[5:]))
            timed(st, p1, args.reps)
            eng.set_option(native.RSA_OPT_FILTER_STEPS, 3)
        elif st.startswith('slice'):
            eng.set_option(native.RSA_OPT_FILTER_SLICE, int(st[5:]))
            timed(st, p1, args.reps)
            eng.set_option(native.RSA_OPT_FILTER_SLICE, 256)
        elif st.startswith('pre'):
            eng.set_option(native.RSA_OPT_PRECHECK, int(st[3:]))
            timed(st, p1, args.reps)
            eng.set_option(native.RSA_OPT_PRECHECK, 1)
        elif st == 'stats':
            eng.set_option(native.RSA_OPT_STATS, 1)
            eng.stats()
            p1()
            torch.cuda.synchronize()
            say('stats: table lines %d, extra probes %d, atomic-path probes %d, slot atomics %d' % tuple(eng.stats()))
            eng.set_option(native.RSA_OPT_STATS, 0)
        elif st == 'minlines':
            # lines that must reach the table: hit+BUILT lines of uncapped rules, and of
            # capped rules those with order <= the final threshold P
            job()
            torch.cuda.synchronize()
            th = eng.counters['thresh']
            fl = (batch.tuples[:, 3] >> 16) & 0xFF
            hb = ((fl & 6) == 6) & (g >= 0)
            gg = g.clamp(min=0).long()
            P = th[gg]
            unc = P == -1
            need = hb & (unc | (batch.order <= P))
            say('minlines: hit+built %d, uncapped-rule lines %d, needed %d, capped rules %d' % (
                int(hb.sum()), int((hb & unc).sum()), int(need.sum()), int((th[:eng.n_rules] != -1).sum())))
        elif st == 'job':
            timed(st, job, args.reps)
        elif st == 'noindex':
            eng.use_index(False)
            timed(st, lambda: eng.classify_only(batch, g), args.reps)
            eng.use_index(True)
        elif st.startswith('prefix'):
            t = time.perf_counter()
            eng.load_compiled(compiled, prefix=int(st[6:]))
            say('  index build+load %.1f s' % (time.perf_counter() - t))
            timed(st, lambda: eng.classify_only(batch, g), args.reps)
        else:
            raise SystemExit('unknown stage ' + st)


if __name__ == '__main__':
    main()
