"""Lines the reference accepts or dies on, through the fused job, against the
oracle's ``mapper | LC_ALL=C sort | reducer`` (``set -o pipefail``).

* month names ``months.index`` rejects: the mapper never looks at the month
  (``mapper.py:127-131``); the reducer dies only at a matched hit BUILT line
  it still inserts (``connlist-reducer.py:151-164``), after printing every
  earlier key's block -- an unmatched line, a capped rule's late line or cap 0
  change nothing;
* ports past 65535: ``int()`` with no range check (``firewallrule.py:47-53``),
  such a side matches NO_PORT rule sides only; a port past 2^63 - 1 is a
  Python 2 long, which the constructor rejects (``:67-75``) -- the mapper dies;
* a mapper death (bad address, missing firewall): the reducer's report over
  the lines before it;
* more protocol spellings and non-canonical keys than the packed form holds.

The CPU tests run ``pipeline.analyze`` over a CPU stand-in of the engine
(``cpu_engine``); the GPU tests run the same cases through the HIP library,
the GPU text parse and the drop-in CLIs.
"""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from oracle import pipeline as op
from oracle.crosscheck_2to3 import oracle_db
from oracle.mapper import HostMissing, map_lines
from oracle.reducer import reduce_lines
from ruleset_analysis_amd import acldb, synth

CAP = 5


def _base(n=3000, seed=7):
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


def product_job(dbj, inputs, cap, engine, text=False):
    from ruleset_analysis_amd.pipeline import analyze, analyze_text
    db = acldb.load_json(dbj)
    try:
        if text:
            out, _ = analyze_text([(h, ''.join(ls).encode('latin-1')) for h, ls in inputs], db, cap=cap,
                                  engine=engine)
        else:
            out, _ = analyze(inputs, db, cap=cap, engine=engine)
        return out, None
    except BaseException as exc:      # noqa: BLE001 - SystemExit is the mapper's missing-firewall death
        assert hasattr(exc, 'rsa_report'), exc
        return exc.rsa_report, exc


def _same_death(got, want):
    if want is None or got is None:
        return want is None and got is None
    if isinstance(want, HostMissing):
        return isinstance(got, SystemExit)
    # the message of an address error is IPy's text (absent from the reference,
    # restated differently by the product and the oracle; stderr only)
    return type(got) is type(want) and (str(got) == str(want) or 'valid IP address' in str(want))


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


@pytest.fixture(scope='module')
def all_cases():
    return cases()


@pytest.fixture(scope='module')
def cpu_engine():
    sys.path.insert(0, os.path.dirname(__file__))
    from cpu_engine import CpuEngine
    return CpuEngine()


NAMES = ['month_unmatched', 'month_capped_late', 'month_under_cap', 'month_first_of_busy_rule', 'month_cap0',
         'month_many', 'month_many_big_cap', 'ports_past_16_bit', 'ports_past_16_bit_cap1000', 'port_python2_long',
         'port_python2_maxint', 'mapper_bad_address', 'mapper_missing_firewall', 'mapper_death_and_month',
         'spellings_200']


@pytest.mark.parametrize('name', NAMES)
def test_oracle_job_has_teeth(all_cases, name):
    dbj, cs = all_cases
    inputs, cap, death = cs[name]
    red, err = oracle_job(dbj, inputs, cap)
    if death is not None:
        assert (err is not None) == death, err
    if name.startswith('ports_past'):
        acls, fws = oracle_db(dbj)
        mapped = []
        map_lines(inputs[0][1], 'fw1', acls, fws, mapped)
        oor = re.compile(r'/(6553[6-9]|65[6-9][0-9]{2}|[7-9][0-9]{4}|0000070000) ')
        assert sum(1 for l in mapped if oor.search(l)) >= 20        # matched (NO_PORT sides)
    if name == 'ports_past_16_bit_cap1000':
        assert sum(1 for l in red if re.search(r' (99[0-9]{3}|100[0-9]{3}) ', l)) >= 3   # TOPORT past 65535 printed
    if name == 'spellings_200':
        assert len({l.split()[1] for l in red if re.match(r' +[0-9]+ T[a-z]{3} ', l)}) > 150


@pytest.mark.parametrize('name', NAMES)
def test_cpu_engine_job_equals_oracle(all_cases, cpu_engine, name):
    dbj, cs = all_cases
    inputs, cap, _death = cs[name]
    want, werr = oracle_job(dbj, inputs, cap)
    got, gerr = product_job(dbj, inputs, cap, cpu_engine)
    assert _same_death(gerr, werr), (gerr, werr)
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize('text', [False, True])
@pytest.mark.parametrize('name', NAMES)
def test_gpu_job_equals_oracle(all_cases, engine, name, text):
    dbj, cs = all_cases
    inputs, cap, _death = cs[name]
    want, werr = oracle_job(dbj, inputs, cap)
    got, gerr = product_job(dbj, inputs, cap, engine, text=text)
    assert _same_death(gerr, werr), (gerr, werr)
    assert got == want


def _shell_case(tmp_path, dbj, lines, cap):
    (tmp_path / 'accesslists.json').write_text(json.dumps(dbj))
    (tmp_path / 'config.py').write_text("ACCESSLIST_DATABASE_FILENAME = 'accesslists.json'\n"
                                        "MAX_NUMBER_OF_CONNECTIONS_PER_RULE = %d\n" % cap)
    logdir = tmp_path / 'logs' / 'fw1'
    logdir.mkdir(parents=True)
    log = logdir / 'part-0000'
    log.write_bytes(''.join(lines).encode('latin-1'))
    return log


def _oracle_shell(tmp_path, log, cap):
    """oracle.cli map | LC_ALL=C sort | oracle.cli reduce, set -o pipefail."""
    env = dict(os.environ, mapred_input_dir=str(log.parent) + '/part-0000', LC_ALL='C', PYTHONPATH=ROOT)
    cmd = ('set -o pipefail; {py} -m oracle.cli map accesslists.json < {log} | sort | '
           '{py} -m oracle.cli reduce accesslists.json {cap}').format(py=sys.executable, log=log, cap=cap)
    return subprocess.run(['bash', '-c', cmd], cwd=tmp_path, env=env, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, timeout=600)


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['month_unmatched', 'month_under_cap', 'month_capped_late', 'ports_past_16_bit',
                                  'mapper_bad_address', 'port_python2_long'])
def test_gpu_cli_run_and_mapper_equal_oracle_shell(tmp_path, all_cases, name):
    """(a)-(d) of the round-3 review: rsa_run.py and rsa_mapper.py against the
    oracle CLIs, stdout bytes and exit status."""
    dbj, cs = all_cases
    inputs, cap, _death = cs[name]
    log = _shell_case(tmp_path, dbj, inputs[0][1], cap)
    want = _oracle_shell(tmp_path, log, cap)
    got = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_run.py'), '--db', 'accesslists.json', '--cap',
                          str(cap), str(log)], cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         timeout=600)
    assert got.stdout == want.stdout
    assert (got.returncode == 0) == (want.returncode == 0), (got.stderr[-800:], want.stderr[-800:])
    env = dict(os.environ, mapred_input_dir=str(log.parent) + '/part-0000', PYTHONPATH=ROOT)
    om = subprocess.run([sys.executable, '-m', 'oracle.cli', 'map', 'accesslists.json'], cwd=tmp_path, env=env,
                        stdin=open(log, 'rb'), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    pm = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_mapper.py')], cwd=tmp_path, env=env,
                        stdin=open(log, 'rb'), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert pm.stdout == om.stdout
    assert (pm.returncode == 0) == (om.returncode == 0), (pm.stderr[-800:], om.stderr[-800:])
