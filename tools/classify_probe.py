#!/usr/bin/env python3
"""Classification ablations on one GPU (profiling only: most variants give
invalid results).  For each variant the library options are set, pass 1 runs
`--reps` times and the median classify time per launch (HIP events on the
library stream) is printed, plus rsa_classify_only over the whole batch.
Usage: python tools/classify_probe.py [--config cfg3] [--lines N]
       [--variants 'base;GROUP_TASKS=0;PROFILE_CLASSIFY=1;...']"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rsa_pkg  # noqa: E402

rsa_pkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import Workload, build_shard  # noqa: E402
from ruleset_analysis_amd import native  # noqa: E402
from ruleset_analysis_amd.engine import Engine  # noqa: E402

DEFAULTS = {'GROUP_TASKS': 1, 'PROFILE_CLASSIFY': 0, 'PROFILE_SKIP': 0}


def say(*a):
    print(*a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='cfg3')
    ap.add_argument('--lines', type=int, default=0)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--variants', default='base;GROUP_TASKS=0;PROFILE_CLASSIFY=1;PROFILE_CLASSIFY=2;'
                                          'PROFILE_CLASSIFY=4;GROUP_TASKS=0,PROFILE_CLASSIFY=4')
    args = ap.parse_args()
    wl = Workload(args.config)
    lines = args.lines or wl.lines
    eng = Engine(0)
    eng.load_compiled(wl.compiled)
    batch, n_hb = build_shard(wl, lines, 0, eng.device)
    g = torch.empty(lines, dtype=torch.int32, device=eng.device)
    torch.cuda.synchronize()
    say('setup: %d lines, %d hit+built' % (lines, n_hb))
    for var in args.variants.split(';'):
        opts = dict(DEFAULTS)
        if var != 'base':
            for kv in var.split(','):
                k, v = kv.split('=')
                opts[k] = int(v)
        for k, v in opts.items():
            eng.set_option(getattr(native, 'RSA_OPT_' + k), v)
        per, agg = [], []
        for _ in range(args.reps):
            eng.reset(n_hb, wl.cap)
            eng.pass1(batch, g)
            c, a = eng.last_pass1_times()
            n = max(eng.last_pass1_launches(), 1)
            per.append(c / n)
            agg.append(a)
        co = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            eng.classify_only(batch, g)
            e.record()
            torch.cuda.synchronize()
            co.append(s.elapsed_time(e))
        say('%-40s classify/launch %.3f ms (x%d)  aggregate %.3f ms  classify_only %.3f ms' % (
            var, float(np.median(per)), n, float(np.median(agg)), float(np.median(co))))
    for k, v in DEFAULTS.items():
        eng.set_option(getattr(native, 'RSA_OPT_' + k), v)


if __name__ == '__main__':
    main()
