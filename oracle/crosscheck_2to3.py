"""ORACLE (test infrastructure only) — pin the oracle against the reference itself.

Run in the build container only (``/root/reference`` does not exist on the GPU
box).  For each fixture case it:

1. converts the reference's ``mapper.py``, ``connlist-reducer.py``,
   ``firewallrule.py`` and ``config.py`` with ``lib2to3`` into a scratch
   directory under /tmp (the converted code is never written into the repo);
2. adds two shims next to them: ``IPy.py`` (this oracle's ``ipy`` restatement —
   IPy itself is not installed) and ``libfwregex.py`` (this oracle's
   ``get_builtconn`` — the ``lib/fw-regex`` submodule is absent); Python 3
   dicts iterate in insertion order where the reference's Python 2 dicts
   iterate in hash-slot order, so the converted reducer's ``conns.keys()``
   (``connlist-reducer.py:109,190``, the only dict whose order reaches the
   output) is wrapped in ``oracle.py2dict``'s replay of CPython 2.7's slot order
   (``py2order.py``), fed by the Python 3 dict's insertion order;
3. builds ``accesslists.db`` with Python 3 ``shelve`` from the converted
   ``FirewallRule`` class, sets the cap in ``config.py``;
4. runs ``mapred_input_dir=/x/<host>/y python3 mapper.py < log | LC_ALL=C sort |
   python3 connlist-reducer.py`` exactly as SURVEY.md §3.1's no-Hadoop form;
5. checks the oracle (``oracle.pipeline``) gives the same mapper text and the
   same reducer text, and writes the case under ``tests/golden/<case>/``:
   ``db.json`` (input), ``log.txt`` (input), ``params.json``,
   ``mapper.sha256`` and ``report.txt`` (outputs of the converted reference);
6. runs the converted ``postprocess_ruleset_analysis.py`` on the report in
   Hadoop's output form (``hadoop.txt``, input) and keeps its stdout
   (``postprocess.txt``).

Usage: ``python3 oracle/crosscheck_2to3.py [--cases NAME ...]``.
"""

import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = '/root/reference'
GOLDEN = os.path.join(REPO, 'tests', 'golden')

sys.path.insert(0, REPO)


def _convert(src, dst):
    shutil.copy(src, dst)
    subprocess.run([sys.executable, '-m', 'lib2to3', '-w', '-n', '--no-diffs', dst], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


BUILD_DB = r'''
import json, shelve, sys
from firewallrule import FirewallRule
dbj = json.load(open(sys.argv[1]))
acls = {}
for h, a in dbj['accesslists'].items():
    acls[h] = {}
    for name, e in a.items():
        rules = []
        for r in e['rules']:
            rule = FirewallRule(r['action'], r['protocol'], r['original'], r['src'], r['dst'],
                                list(r['sport']), list(r['dport']))
            rule.comments = list(r['comments']); rule.rulenum = r['rulenum']; rule.ruleindex = r['ruleindex']
            rules.append(rule)
        acls[h][name] = {'rules': rules, 'protocols': {p: list(v) for p, v in e['protocols'].items()},
                         'timestamp': e['timestamp']}
db = shelve.open('accesslists.db')
db['firewalls'] = dbj['firewalls']
db['accesslists'] = acls
db.close()
'''


def prepare_reference(work, db_json, cap):
    """Convert the reference scripts into ``work`` and build its
    ``accesslists.db`` from ``db_json``, the cap set in its ``config.py``."""
    os.makedirs(work, exist_ok=True)
    for name in ('mapper.py', 'connlist-reducer.py', 'firewallrule.py', 'config.py'):
        _convert(os.path.join(REF, name), os.path.join(work, name))
    red = os.path.join(work, 'connlist-reducer.py')
    with open(red) as f:
        code = f.read()
    n_sites = code.count('entries = list(conns.keys())')
    if n_sites != 2:
        raise RuntimeError('expected 2 conns.keys() sites in the converted reducer, found %d' % n_sites)
    code = code.replace('entries = list(conns.keys())', 'entries = _py2_keys(list(conns.keys()))')
    code = 'from py2order import py2_keys as _py2_keys\n' + code
    with open(red, 'w') as f:
        f.write(code)
    shutil.copy(os.path.join(HERE, 'py2dict.py'), os.path.join(work, 'py2order.py'))
    with open(os.path.join(work, 'config.py')) as f:
        cfg = f.read()
    cfg = cfg.replace('MAX_NUMBER_OF_CONNECTIONS_PER_RULE = 1000', 'MAX_NUMBER_OF_CONNECTIONS_PER_RULE = %d' % cap)
    with open(os.path.join(work, 'config.py'), 'w') as f:
        f.write(cfg)
    shutil.copy(os.path.join(HERE, 'ipy.py'), os.path.join(work, 'IPy.py'))
    shutil.copy(os.path.join(HERE, 'fwregex.py'), os.path.join(work, 'libfwregex.py'))
    with open(os.path.join(work, 'db.json'), 'w') as f:
        json.dump(db_json, f)
    with open(os.path.join(work, 'build_db.py'), 'w') as f:
        f.write(BUILD_DB)
    subprocess.run([sys.executable, 'build_db.py', 'db.json'], cwd=work, check=True, env=_env())


def _env():
    return dict(os.environ, PYTHONIOENCODING='latin-1', LC_ALL='C', PYTHONHASHSEED='0')


def _last_exception(stderr):
    """Name of the exception a Python traceback on stderr ends with (None: none)."""
    lines = [l for l in stderr.decode('latin-1').splitlines() if l.strip()]
    if not lines or not any(l.startswith('Traceback') for l in lines):
        return None
    return lines[-1].split(':', 1)[0].strip().rsplit('.', 1)[-1]


def run_reference_job(work, inputs):
    """The no-Hadoop job of SURVEY.md §3.1 under ``set -o pipefail`` in a work
    dir prepared by prepare_reference: for each (host, log text) in turn the
    converted mapper (host from ``mapred_input_dir``, mapper.py:107-112), its
    stdout appended to the map output; the first mapper that exits non-zero
    ends the map stage (a Hadoop job whose map task failed).  Then ``LC_ALL=C
    sort | connlist-reducer.py``.  Returns a dict: map text, reducer stdout,
    the exit status of each stage and the exception a stage died with."""
    env = _env()
    maps, m_rc, m_exc = [], 0, None
    for k, (host, text) in enumerate(inputs):
        path = os.path.join(work, 'log%d.txt' % k)
        with open(path, 'w', encoding='latin-1', newline='') as f:
            f.write(text)
        env['mapred_input_dir'] = '/logs/%s/part-0000' % host
        with open(path, 'rb') as fin:
            m = subprocess.run([sys.executable, 'mapper.py'], cwd=work, env=env, stdin=fin, stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE)
        maps.append(m.stdout)
        if m.returncode != 0:
            m_rc, m_exc = m.returncode, _last_exception(m.stderr) or 'SystemExit'
            break
    mapped = b''.join(maps)
    s = subprocess.run(['sort'], input=mapped, stdout=subprocess.PIPE, env=env, check=True)
    r = subprocess.run([sys.executable, 'connlist-reducer.py'], cwd=work, env=env, input=s.stdout,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    return {'map': mapped.decode('latin-1'), 'reduce': r.stdout.decode('latin-1'), 'map_rc': m_rc,
            'map_exc': m_exc, 'reduce_rc': r.returncode,
            'reduce_exc': _last_exception(r.stderr) if r.returncode else None}


def run_reference(work, db_json, log_text, host, cap):
    prepare_reference(work, db_json, cap)
    res = run_reference_job(work, [(host, log_text)])
    if res['map_rc'] != 0:
        raise RuntimeError('reference mapper failed: %s' % res['map_exc'])
    if res['reduce_rc'] != 0:
        raise RuntimeError('reference reducer failed: %s' % res['reduce_exc'])
    return res['map'], res['reduce']


def run_postprocess(work, hadoop_text):
    """The converted postprocess_ruleset_analysis.py (``-f`` the Hadoop-form
    reducer output) in a work dir prepared by run_reference (same DB)."""
    _convert(os.path.join(REF, 'postprocess_ruleset_analysis.py'), os.path.join(work, 'postprocess.py'))
    with open(os.path.join(work, 'config.py')) as f:
        cfg = f.read()
    cfg = cfg.replace("ACCESSLIST_DATABASE = './input/{0}'.format(ACCESSLIST_DATABASE_FILENAME)",
                      "ACCESSLIST_DATABASE = ACCESSLIST_DATABASE_FILENAME")
    with open(os.path.join(work, 'config.py'), 'w') as f:
        f.write(cfg)
    with open(os.path.join(work, 'hadoop.txt'), 'w', encoding='latin-1', newline='') as f:
        f.write(hadoop_text)
    env = dict(os.environ, PYTHONIOENCODING='latin-1', LC_ALL='C', PYTHONHASHSEED='0')
    r = subprocess.run([sys.executable, 'postprocess.py', '-f', 'hadoop.txt'], cwd=work, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    if r.returncode != 0:
        raise RuntimeError('reference postprocessor failed: %s' % r.stderr.decode('latin-1')[-2000:])
    return r.stdout.decode('latin-1')


def hadoop_part(report_text):
    """The Hadoop TextOutputFormat form (line + '\t\n') of a reducer report
    without its leading noise records (what a reduce partition that received
    no empty mapper records writes; the noise entry would stop the
    postprocessor at postprocess_ruleset_analysis.py:96)."""
    lines = report_text.split('\n')[:-1]
    if not any(': access-list ' in l for l in lines):
        return ''                  # no rule block: the postprocessor has nothing to attach (IndexError at :96)
    k = 0
    while k < len(lines) and lines[k] != '':
        k += 1
    return ''.join(l + '\t\n' for l in lines[k:])


def oracle_db(dbj):
    from oracle.firewallrule import FirewallRule
    acls = {}
    for h, a in dbj['accesslists'].items():
        acls[h] = {}
        for name, e in a.items():
            rules = []
            for r in e['rules']:
                rule = FirewallRule(r['action'], r['protocol'], r['original'], r['src'], r['dst'], list(r['sport']),
                                    list(r['dport']), comments=list(r['comments']), rulenum=r['rulenum'],
                                    ruleindex=r['ruleindex'])
                rules.append(rule)
            acls[h][name] = {'rules': rules, 'protocols': {p: list(v) for p, v in e['protocols'].items()},
                             'timestamp': e['timestamp']}
    return acls, dbj['firewalls']


def cases():
    import rsa_pkg
    rsa_pkg.load()
    from ruleset_analysis_amd import synth

    def synthetic(seed, n_rules, n_lines, cap, zipf=None, interfaces=('outside',), drop_last_nl=False,
                  missing_acl=False):
        db, info = synth.make_db(seed, n_rules, interfaces=interfaces)
        tr = synth.make_traffic((db, info), n_lines, seed=seed + 100, zipf=zipf)
        lines = synth.render_lines(tr)
        if missing_acl:
            # bind an interface to an ACL absent from the DB (mapper.py:152-156)
            db['firewalls']['fw1']['dmz'] = {'in': 'dmz_access_in'}
        text = ''.join(l + '\n' for l in lines)
        if drop_last_nl:
            text = text[:-1]
        return db, text, cap

    yield 'small_200r', lambda: synthetic(1, 200, 3000, 1000)
    yield 'cap5_zipf', lambda: synthetic(2, 120, 4000, 5, zipf=1.3)
    yield 'multi_acl', lambda: synthetic(3, 80, 3000, 40, interfaces=('outside', 'partner'), missing_acl=True,
                                         drop_last_nl=True)
    yield 'cap1', lambda: synthetic(4, 60, 1500, 1, zipf=1.5)
    yield 'empty_log', lambda: synthetic(5, 30, 0, 1000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cases', nargs='*')
    args = ap.parse_args()
    from oracle import pipeline as op
    if not os.path.isdir(REF):
        sys.exit('reference not present; this script only runs in the build container')
    for name, make in cases():
        if args.cases and name not in args.cases:
            continue
        db, text, cap = make()
        with tempfile.TemporaryDirectory(prefix='rsa_xref_') as work:
            ref_map, ref_red = run_reference(work, db, text, 'fw1', cap)
            hadoop = hadoop_part(ref_red)
            ref_post = run_postprocess(work, hadoop) if hadoop else None
        acls, fws = oracle_db(db)
        o_map, _srt, o_red, _blocks = op.run_pipeline(text, 'fw1', acls, fws, cap=cap)
        o_red_text = ''.join(l + '\n' for l in o_red)
        ok_map = o_map == ref_map
        ok_red = o_red_text == ref_red
        print('%-12s lines=%-6d mapper %s reducer %s (%d report lines)' % (
            name, text.count('\n'), 'OK' if ok_map else 'DIFF', 'OK' if ok_red else 'DIFF', ref_red.count('\n')))
        if not (ok_map and ok_red):
            sys.exit('oracle disagrees with the converted reference on case %s' % name)
        out = os.path.join(GOLDEN, name)
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, 'db.json'), 'w') as f:
            json.dump(db, f, sort_keys=True)
        with open(os.path.join(out, 'log.txt'), 'w', encoding='latin-1', newline='') as f:
            f.write(text)
        with open(os.path.join(out, 'report.txt'), 'w', encoding='latin-1', newline='') as f:
            f.write(ref_red)
        with open(os.path.join(out, 'mapper.sha256'), 'w') as f:
            f.write(hashlib.sha256(ref_map.encode('latin-1')).hexdigest() + '\n')
        if ref_post is not None:
            with open(os.path.join(out, 'hadoop.txt'), 'w', encoding='latin-1', newline='') as f:
                f.write(hadoop)
            with open(os.path.join(out, 'postprocess.txt'), 'w', encoding='latin-1', newline='') as f:
                f.write(ref_post)
        with open(os.path.join(out, 'params.json'), 'w') as f:
            json.dump({'host': 'fw1', 'cap': cap, 'source': 'lib2to3-converted reference, oracle/crosscheck_2to3.py'},
                      f, sort_keys=True)


if __name__ == '__main__':
    main()
