"""The drop-in CLIs reproduce the reference's stdout contracts on the golden
cases: rsa_mapper.py (mapper.py), LC_ALL=C sort, rsa_reducer.py
(connlist-reducer.py), and the fused rsa_run.py."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, golden_cases
from golden_io import load_case

pytestmark = pytest.mark.gpu


def _setup(tmp_path, case):
    dbj, text, report, sha, params = load_case(case)
    (tmp_path / 'accesslists.json').write_text(json.dumps(dbj))
    (tmp_path / 'config.py').write_text("ACCESSLIST_DATABASE_FILENAME = 'accesslists.json'\n"
                                        "ACCESSLIST_DATABASE = './input/{0}'.format(ACCESSLIST_DATABASE_FILENAME)\n"
                                        "MAX_NUMBER_OF_CONNECTIONS_PER_RULE = %d\n" % params['cap'])
    logdir = tmp_path / 'logs' / params['host']
    logdir.mkdir(parents=True)
    (logdir / 'part-0000').write_bytes(text.encode('latin-1'))
    return text, report, sha, params, logdir / 'part-0000'


@pytest.mark.parametrize('case', ['small_200r', 'multi_acl', 'cap1', 'empty_log'])
def test_mapper_sort_reducer_cli(tmp_path, case):
    text, report, sha, params, logfile = _setup(tmp_path, case)
    env = dict(os.environ, mapred_input_dir=str(logfile.parent) + '/part-0000', LC_ALL='C')
    m = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_mapper.py')], cwd=tmp_path, env=env,
                       input=text.encode('latin-1'), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert m.returncode == 0, m.stderr.decode()[-2000:]
    assert hashlib.sha256(m.stdout).hexdigest() == sha
    s = subprocess.run(['sort'], input=m.stdout, stdout=subprocess.PIPE, env=env, check=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_reducer.py')], cwd=tmp_path, env=env, input=s.stdout,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert r.stdout.decode('latin-1') == report


@pytest.mark.parametrize('case', ['cap5_zipf', 'multi_acl'])
def test_fused_run_cli(tmp_path, case):
    text, report, sha, params, logfile = _setup(tmp_path, case)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_run.py'), '--db', 'accesslists.json', '--cap',
                        str(params['cap']), str(logfile)], cwd=tmp_path, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert r.stdout.decode('latin-1') == report


@pytest.mark.parametrize('case', ['small_200r', 'multi_acl'])
def test_mapper_streamed_chunks(tmp_path, case):
    """The mapper drop-in streams stdin in chunks of whole lines: with 4 KiB
    chunks (hundreds of them, lines cut at every boundary, the multi_acl log
    ending without a newline) its output is still the reference's byte for byte."""
    text, report, sha, params, logfile = _setup(tmp_path, case)
    env = dict(os.environ, mapred_input_dir=str(logfile.parent) + '/part-0000', LC_ALL='C', RSA_MAPPER_CHUNK='4096')
    m = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_mapper.py')], cwd=tmp_path, env=env,
                       input=text.encode('latin-1'), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert m.returncode == 0, m.stderr.decode()[-2000:]
    assert hashlib.sha256(m.stdout).hexdigest() == sha


def test_mapper_unknown_host(tmp_path):
    text, report, sha, params, logfile = _setup(tmp_path, 'small_200r')
    env = dict(os.environ, mapred_input_dir='/logs/nosuchfw/part-0000')
    m = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_mapper.py')], cwd=tmp_path, env=env,
                       input=b'', stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert m.returncode == 1
    assert m.stdout == b'Firewall nosuchfw not present in data structure. Aborting.\n'


@pytest.mark.parametrize('case', ['small_200r', 'multi_acl'])
def test_fused_run_postprocess_cli(tmp_path, case):
    """rsa_run.py --postprocess prints what postprocess_ruleset_analysis.py
    prints for the job's Hadoop output (golden: the converted reference)."""
    text, report, sha, params, logfile = _setup(tmp_path, case)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'rsa_run.py'), '--db', 'accesslists.json', '--cap',
                        str(params['cap']), '--postprocess', '--shadowed', str(logfile)], cwd=tmp_path,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    with open(os.path.join(ROOT, 'tests', 'golden', case, 'postprocess.txt'), encoding='latin-1', newline='') as f:
        assert r.stdout.decode('latin-1') == f.read()
    assert b'INFO - Found rule which never gets hits' in r.stderr


def test_config1_rsa_run_equals_oracle_pipeline(tmp_path):
    """BASELINE config 1 exactly as bench.py's CPU baseline builds it (a
    200-rule ACL and 1M synthetic ASA lines, seed 1): the fused rsa_run.py
    report is byte-identical to ``oracle.cli map | LC_ALL=C sort | oracle.cli
    reduce`` -- the pipeline the CPU baseline times -- over the same bytes."""
    from ruleset_analysis_amd import synth
    dbj, info = synth.make_db(1, 200)
    tr = synth.make_traffic((dbj, info), 1_000_000, seed=101)
    text = ''.join(l + '\n' for l in synth.render_lines(tr)).encode('latin-1')
    (tmp_path / 'db.json').write_text(json.dumps(dbj))
    logdir = tmp_path / 'logs' / 'fw1'
    logdir.mkdir(parents=True)
    (logdir / 'part-00000').write_bytes(text)
    env = dict(os.environ, LC_ALL='C', mapred_input_dir=str(logdir) + '/part-00000', PYTHONPATH=ROOT)
    py = sys.executable
    want = subprocess.run('%s -m oracle.cli map db.json < logs/fw1/part-00000 | LC_ALL=C sort | '
                          '%s -m oracle.cli reduce db.json 1000' % (py, py), shell=True, cwd=tmp_path, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600, check=True).stdout
    r = subprocess.run([py, os.path.join(ROOT, 'rsa_run.py'), '--db', 'db.json', '--cap', '1000',
                        str(logdir / 'part-00000')], cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert r.stdout == want
    assert want.count(b'Total number of hits') > 50
