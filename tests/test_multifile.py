"""Several log files of one firewall in one job.

The reference reads ``cat f1 f2 f3 | mapper | LC_ALL=C sort | reducer`` (or
Hadoop's shuffle sort over every split, ``runAnalysis.sh:42-56``): within one
key the reducer sees the lines of all files in byte order, and the cap freeze
(``connlist-reducer.py:151``) follows that order.  The fused path must rank the
lines of all inputs together (``textparse.order_keys_global``), not per file.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from oracle import coracle
from oracle import pipeline as op
from oracle.crosscheck_2to3 import oracle_db
from ruleset_analysis_amd import synth

CAP = 17


def _workload(n=40000):
    """fw1 (two ACLs) + fw2: Zipf traffic so several rules pass the cap; the
    fw1 lines dealt at random into three files and shuffled inside each file
    (so the files' timestamps interleave)."""
    db1, info1 = synth.make_db(31, 300, interfaces=('outside', 'partner'))
    db2, info2 = synth.make_db(33, 120, host='fw2')
    tr1 = synth.make_traffic((db1, info1), n, seed=32, zipf=1.3)
    tr2 = synth.make_traffic((db2, info2), n // 4, seed=34, zipf=1.3, cid0=5000000)
    dbj = {'firewalls': dict(db1['firewalls'], **db2['firewalls']),
           'accesslists': dict(db1['accesslists'], **db2['accesslists'])}
    rng = np.random.default_rng(35)
    lines1 = synth.render_lines(tr1)
    which = rng.integers(0, 3, size=len(lines1))
    files1 = []
    for k in range(3):
        part = [lines1[i] for i in np.nonzero(which == k)[0]]
        part = [part[i] for i in rng.permutation(len(part))]
        files1.append(''.join(l + '\n' for l in part))
    lines2 = synth.render_lines(tr2)
    text2 = ''.join(lines2[i] + '\n' for i in rng.permutation(len(lines2)))
    return dbj, files1, text2, (db1, info1, tr1, which)


def _oracle_report(dbj, files1, text2, cap):
    acls, fws = oracle_db(dbj)
    _m, _s, red, _b = op.run_multi([('fw1', ''.join(files1)), ('fw2', text2)], acls, fws, cap=cap)
    return ''.join(l + '\n' for l in red)


def test_per_file_ranking_would_differ():
    """The workload has teeth: ranking each file's lines on its own (file k's
    lines all after file k-1's) changes the capped rules' tables (C oracle)."""
    _dbj, files1, _t2, (db1, info1, tr1, which) = _workload()
    R = coracle.OracleRules(db1)
    cols, ts, order = coracle.inputs_from_traffic(R, tr1)
    glob = coracle.run(R, cols, ts, order, CAP)
    per = np.empty_like(order)
    base = 0
    for k in range(3):
        idx = np.nonzero(which == k)[0]
        ranks = np.empty(len(idx), np.uint64)
        ranks[np.argsort(order[idx], kind='stable')] = np.arange(len(idx), dtype=np.uint64)
        per[idx] = ranks + np.uint64(base)
        base += len(idx)
    perfile = coracle.run(R, cols, ts, per, CAP)
    assert (glob['n_conns'] >= CAP).sum() >= 3      # several rules capped
    a, b = glob['rows'], perfile['rows']
    differ = len(a['gid']) != len(b['gid']) or any(not np.array_equal(a[k], b[k]) for k in a)
    assert differ


@pytest.mark.gpu
def test_gpu_fused_run_three_files_equals_cat_sort_pipeline(tmp_path):
    dbj, files1, text2, _ = _workload()
    (tmp_path / 'accesslists.json').write_text(json.dumps(dbj))
    paths = []
    for k, t in enumerate(files1):
        d = tmp_path / 'logs' / 'fw1'
        d.mkdir(parents=True, exist_ok=True)
        (d / ('part-%04d' % k)).write_bytes(t.encode('latin-1'))
        paths.append(str(d / ('part-%04d' % k)))
    d2 = tmp_path / 'logs' / 'fw2'
    d2.mkdir(parents=True)
    (d2 / 'part-0000').write_bytes(text2.encode('latin-1'))
    paths.insert(1, str(d2 / 'part-0000'))       # hosts interleaved on the command line
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_run.py'), '--db', 'accesslists.json', '--cap',
                        str(CAP)] + paths, cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    want = _oracle_report(dbj, files1, text2, CAP)
    assert 'NOTE: Maximum number of connections' in want
    assert r.stdout.decode('latin-1') == want


@pytest.mark.gpu
def test_gpu_analyze_text_multi_input_equals_host_analyze(engine):
    """Both product entry points agree on several inputs (analyze sorts all
    lines together on the host; analyze_text ranks them on the GPU)."""
    from ruleset_analysis_amd import acldb
    from ruleset_analysis_amd.pipeline import analyze, analyze_text
    from golden_io import split_lines
    dbj, files1, text2, _ = _workload(12000)
    db = acldb.load_json(dbj)
    ins = [('fw1', files1[0]), ('fw2', text2), ('fw1', files1[1]), ('fw1', files1[2])]
    want, _ = analyze([(h, split_lines(t)) for h, t in ins], db, cap=5, engine=engine)
    got, _ = analyze_text([(h, t.encode('latin-1')) for h, t in ins], db, cap=5, engine=engine)
    assert got == want
    assert any(l.startswith('NOTE: Maximum') for l in got)
