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
