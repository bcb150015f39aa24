"""The fused job's death and edge cases (shared by ``test_pipeline_deaths.py``
and the generator ``oracle/crosscheck_deaths.py``): lines the reference
accepts or dies on, built from one seeded synthetic log, and their committed
fixture ``tests/golden_deaths/`` -- the inputs (the base log plus each case's
replaced lines) and the stdout bytes / exit status / exception of the
lib2to3-converted reference's ``mapper | LC_ALL=C sort | reducer`` job.
"""
import gzip
import json
import os
import re

import numpy as np

from oracle import pipeline as op
from oracle.crosscheck_2to3 import oracle_db
from oracle.mapper import HostMissing, map_lines
from oracle.reducer import reduce_lines

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, 'golden_deaths')

CAP = 5


def _base(n=3000, seed=7):
    from ruleset_analysis_amd import synth
    dbj, info = synth.make_db(1, 200, broad=False)
    tr = synth.make_traffic((dbj, info), n, seed=seed, zipf=1.3)
    return dbj, [l + '\n' for l in synth.render_lines(tr)]


def _mapped(dbj, lines):
    """Oracle mapper key per line (None: no output)."""
    acls, fws = oracle_db(dbj)
    keys = []
    for l in lines:
        out = []
        map_lines([l], 'fw1', acls, fws, out)
        keys.append(out[0].split('\t', 1)[0] if out and '\t' in out[0] else None)
    return keys


def _hit_built(l):
    return '-6-302013' in l or '-6-302015' in l


def _month(l, word='Foo'):
    """The device date's month (the reducer's res[1]) replaced."""
    assert ' Jul ' in l
    return l.replace(' Jul ', ' %s ' % word, 1)


def oracle_job(dbj, inputs, cap):
    """(stdout lines, exception or None) of mapper | sort | reducer under pipefail."""
    acls, fws = oracle_db(dbj)
    out, err = [], None
    for host, lines in inputs:
        try:
            map_lines(lines, host, acls, fws, out)
        except (KeyError, ValueError, HostMissing) as exc:
            err = exc
            break
    srt = op.c_sort(''.join(out))
    red = []
    try:
        reduce_lines(op._split_nl(srt), acls, cap, out=red)
    except (KeyError, ValueError, IndexError) as exc:
        err = exc
    return red, err


def cases():
    """name -> (inputs, cap, expect a death?)."""
    dbj, lines = _base()
    keys = _mapped(dbj, lines)
    hb = [i for i, l in enumerate(lines) if _hit_built(l) and ' Jul ' in l]
    matched = [i for i in hb if keys[i] is not None]
    unmatched = [i for i in hb if keys[i] is None]
    by_key = {}
    for i in matched:
        by_key.setdefault(keys[i], []).append(i)
    busiest = max(by_key.values(), key=len)          # a rule far past the cap
    late = max(busiest, key=lambda i: lines[i])      # its last line in sort order
    quiet = min((v for v in by_key.values() if len(v) < CAP), key=len)   # a rule that never fills its dict
    out = {}

    def mut(idx, word='Foo'):
        ls = list(lines)
        for i in idx:
            ls[i] = _month(ls[i], word)
        return [('fw1', ls)]

    out['month_unmatched'] = (mut(unmatched[:3]), CAP, False)
    out['month_capped_late'] = (mut([late], 'jul'), CAP, False)
    out['month_under_cap'] = (mut([quiet[0]]), CAP, True)
    out['month_first_of_busy_rule'] = (mut([min(busiest, key=lambda i: lines[i])]), CAP, True)
    out['month_cap0'] = (mut([quiet[0]]), 0, False)
    rng = np.random.default_rng(3)
    out['month_many'] = (mut(rng.choice(hb, size=len(hb) // 50, replace=False).tolist(), 'Xyz'), CAP, None)
    out['month_many_big_cap'] = (mut(rng.choice(hb, size=len(hb) // 50, replace=False).tolist()), 1000, True)

    # ports past 65535 (kept digits), and one past a 64-bit int (the mapper dies)
    ls = list(lines)
    for k, i in enumerate(rng.choice(len(ls), size=300, replace=False).tolist()):
        if 'Built inbound' not in ls[i]:
            continue
        if k % 3 == 0:
            ls[i] = re.sub(r'(for [a-z]+:[0-9.]+)/([0-9]+)', lambda m: m.group(1) + '/%d' % (65536 + k), ls[i], 1)
        elif k % 3 == 1:
            ls[i] = re.sub(r'(to [a-z]+:[0-9.]+)/([0-9]+)', lambda m: m.group(1) + '/%d' % (99990 + k), ls[i], 1)
        else:
            ls[i] = re.sub(r'(for [a-z]+:[0-9.]+)/([0-9]+)', r'\1/0000070000', ls[i], 1)
    out['ports_past_16_bit'] = ([('fw1', ls)], CAP, False)
    out['ports_past_16_bit_cap1000'] = ([('fw1', ls)], 1000, False)
    ls2 = list(ls)
    j = hb[len(hb) // 2]
    ls2[j] = re.sub(r'(for [a-z]+:[0-9.]+)/([0-9]+)', r'\1/9223372036854775808', ls2[j], 1)
    out['port_python2_long'] = ([('fw1', ls2)], CAP, True)
    ls3 = list(lines)
    ls3[j] = re.sub(r'(for [a-z]+:[0-9.]+)/([0-9]+)', r'\1/9223372036854775807', ls3[j], 1)
    out['port_python2_maxint'] = ([('fw1', ls3)], CAP, False)

    # mapper deaths: a bad address; a firewall missing from the DB
    ls = list(lines)
    ls[j] = re.sub(r'for ([a-z]+):[0-9.]+/', r'for \1:999.0.0.1/', ls[j], 1)
    out['mapper_bad_address'] = ([('fw1', ls)], CAP, True)
    out['mapper_missing_firewall'] = ([('fw1', lines[:1500]), ('fw9', lines[1500:])], CAP, True)
    out['mapper_death_and_month'] = ([('fw1', mut([quiet[0]])[0][1][:j] + ls[j:])], CAP, True)

    # 200 protocol spellings in the reducer's BUILT match (the last "Built ..bound WORD")
    ls = list(lines)
    words = ['T' + ''.join(chr(97 + (k // 26 ** e) % 26) for e in range(3)) for k in range(200)]
    for k, i in enumerate(hb[:1200]):
        m = re.search(r'for ([a-z]+):([0-9.]+)/([0-9]+) \([^)]*\) to ([a-z]+):([0-9.]+)/([0-9]+)', ls[i])
        ls[i] = ls[i].rstrip('\n') + ' Built inbound %s x for %s:%s/%s y to %s:%s/%s\n' % (
            words[k % 200], m.group(1), m.group(2), m.group(3), m.group(4), m.group(5), m.group(6))
    out['spellings_200'] = ([('fw1', ls)], 1000, False)
    return dbj, out


NAMES = ['month_unmatched', 'month_capped_late', 'month_under_cap', 'month_first_of_busy_rule', 'month_cap0',
         'month_many', 'month_many_big_cap', 'ports_past_16_bit', 'ports_past_16_bit_cap1000', 'port_python2_long',
         'port_python2_maxint', 'mapper_bad_address', 'mapper_missing_firewall', 'mapper_death_and_month',
         'spellings_200']


# ---- the committed fixture -------------------------------------------------

def encode_inputs(base, inputs):
    """A case's [(host, lines)] as base ranges plus replaced lines."""
    enc, off = [], 0
    for host, ls in inputs:
        a = 0 if len(ls) == len(base) else off
        rep = {str(i): l for i, l in enumerate(ls) if l != base[a + i]}
        enc.append({'host': host, 'start': a, 'stop': a + len(ls), 'replace': rep})
        off = a + len(ls)
    return enc


def decode_inputs(base, enc):
    out = []
    for h in enc:
        ls = base[h['start']:h['stop']]
        for i, l in h['replace'].items():
            ls[int(i)] = l
        out.append((h['host'], ls))
    return out


def save_fixture(dbj, base, entries):
    """db.json, the base log and every case's inputs (gzip), and the
    reference's results per case (expected.json, readable)."""
    os.makedirs(FIXTURE, exist_ok=True)
    with open(os.path.join(FIXTURE, 'db.json'), 'w') as f:
        json.dump(dbj, f, sort_keys=True)
    with gzip.GzipFile(os.path.join(FIXTURE, 'base_log.txt.gz'), 'wb', mtime=0) as f:
        f.write(''.join(base).encode('latin-1'))
    inputs = {n: e['inputs'] for n, e in entries.items() if not n.startswith('_')}
    with gzip.GzipFile(os.path.join(FIXTURE, 'inputs.json.gz'), 'wb', mtime=0) as f:
        f.write(json.dumps(inputs, sort_keys=True).encode('latin-1'))
    expected = {n: ({k: v for k, v in e.items() if k != 'inputs'} if isinstance(e, dict) else e)
                for n, e in entries.items()}
    with open(os.path.join(FIXTURE, 'expected.json'), 'w') as f:
        json.dump(expected, f, sort_keys=True, indent=1)


def load_fixture():
    """(dbj, base lines, {name: (inputs, cap, reference result)}) from
    tests/golden_deaths."""
    with open(os.path.join(FIXTURE, 'db.json')) as f:
        dbj = json.load(f)
    with gzip.open(os.path.join(FIXTURE, 'base_log.txt.gz'), 'rb') as f:
        base = f.read().decode('latin-1').splitlines(True)
    with gzip.open(os.path.join(FIXTURE, 'inputs.json.gz'), 'rb') as f:
        inputs = json.loads(f.read().decode('latin-1'))
    with open(os.path.join(FIXTURE, 'expected.json')) as f:
        expected = json.load(f)
    return dbj, base, {n: (decode_inputs(base, inputs[n]), e['cap'], e['reference'])
                       for n, e in expected.items() if not n.startswith('_')}


def exc_name(err):
    """The exception name a job died with, as the reference's traceback names it."""
    if err is None:
        return None
    if isinstance(err, (HostMissing, SystemExit)):
        return 'SystemExit'
    return type(err).__name__
