"""Drop-in command-line entry points.

* ``mapper_main`` — replaces ``mapper.py`` in ``runAnalysis.sh``/Hadoop
  streaming: same CWD files (``config.py``, the DB named by
  ``ACCESSLIST_DATABASE_FILENAME``), same ``mapred_input_dir`` host rule
  (``mapper.py:107-117``), same stdout bytes (``mapper.py:154-155,184-186``);
  the log text is parsed (``textparse``) and classified on the GPU.
* ``reducer_main`` — replaces ``connlist-reducer.py`` (and ``reducer.py``):
  sorted mapper stream on stdin, the reference report on stdout
  (``connlist-reducer.py:62-211``); aggregation runs on the GPU, one group per
  run of equal keys, so even unsorted input prints what the reference prints.
* ``run_main`` — the fused job (``mapper | sort | reducer`` in one GPU pass):
  ``rsa_run.py --db accesslists.db [--cap N] LOGFILE...``; the host of each
  file is its parent directory name, as Hadoop's ``mapred_input_dir`` gives it;
  the text is parsed on the GPU, order keys included (``textparse``).

Error behaviour follows the reference: the same exception classes at the same
validation points (``KeyError`` for a missing ``'in'`` binding or protocol
list, ``ValueError`` for malformed addresses or ports past a 64-bit int),
config/DB problems reported on stderr with exit status 1.  The mapper never
validates the month (``mapper.py:127-131``); the fused job dies where
``mapper | sort | reducer`` would under ``set -o pipefail``, after printing
what the reducer printed (``pipeline.finish_job``).
"""

import os
import sys

import numpy as np

from . import acldb
from .compile import CompiledRules
from .engine import Engine
from .pipeline import analyze_text
from .textparse import parse_text
from .report import mapper_output


def _write(text):
    sys.stdout.buffer.write(text.encode('latin-1'))


def load_config(path='config.py'):
    """``execfile(CONFIGFILE, config)`` as the reference does (mapper.py:16-24)."""
    config = {}
    try:
        with open(path) as f:
            code = compile(f.read(), path, 'exec')
        exec(code, config)  # noqa: S102 - the user's own config file, exactly like the reference's execfile
    except Exception:  # noqa: BLE001 - the reference catches everything here
        sys.stderr.write('Unable to load config file ({0})! Aborting.\n'.format(path))
        sys.exit(1)
    return config


def _open_db(name, role):
    try:
        return acldb.load(name)
    except Exception:  # noqa: BLE001 - mapper.py:80-100
        sys.stderr.write('Unable to open access-list database ("{0}"). Did you remember to run preprocessor? '
                         'Aborting {1}.\n'.format(name, role))
        sys.exit(1)


def mapper_main(argv=None):
    config = load_config()
    db = _open_db(config['ACCESSLIST_DATABASE_FILENAME'], 'mapper')
    try:
        hostname = os.environ['mapred_input_dir'].split('/')[-2]
    except KeyError as e:
        raise KeyError('Unable to determine hostname from mapred_input_dir! Environment variable not found: ' + str(e))
    if hostname not in db.firewalls or hostname not in db.accesslists:
        _write('Firewall {0} not present in data structure. Aborting.\n'.format(hostname))
        sys.exit(1)
    compiled = CompiledRules(db)
    compiled.ensure_lists()
    eng = Engine(0)
    eng.load_compiled(compiled)
    # stdin is streamed in chunks of whole lines (RSA_MAPPER_CHUNK bytes, cut
    # after the chunk's last '\n'; the final chunk keeps a last line without
    # one), so output starts before the input ends and memory stays bounded:
    # the mapper's lines are independent (mapper.py:119-189).  Each chunk's
    # text is parsed on the GPU (textparse); lines outside the device grammar
    # are decided by the host parser, in line order; an error line stops the
    # stream after the lines before it, as the reference dies there.
    chunk = max(int(os.environ.get('RSA_MAPPER_CHUNK', 256 << 20)), 1)
    src = sys.stdin.buffer
    carry = b''
    while True:
        block = src.read(chunk)
        data = carry + block
        if not data:
            break
        if block:
            cut = data.rfind(b'\n') + 1
            if cut == 0:          # no complete line yet: read on
                carry = data
                continue
            data, carry = data[:cut], data[cut:]
        else:
            carry = b''
        parsed = parse_text(eng, hostname, data, db, compiled, need_order=False)
        eng.refresh_compiled(compiled)     # lists derived for ports past 65535 (compile.list_id_oor)
        gids = eng.classify_only(parsed.batch()).cpu().numpy() if parsed.n else np.zeros(0, np.int32)
        _write(mapper_output(parsed, gids, compiled))
        sys.stdout.flush()
        if parsed.error is not None:
            raise parsed.error[1]
        if not block:
            break
    return 0


def reducer_main(argv=None):
    """connlist-reducer.py as a stdin -> stdout filter (reducer_stream: GPU
    parse and aggregation per chunk of RSA_REDUCER_CHUNK bytes, runs of equal
    keys decided once on the host, output as the runs complete)."""
    from .reducer_stream import ReducerStream
    config = load_config()
    db = _open_db(os.path.basename(config['ACCESSLIST_DATABASE_FILENAME']), 'reducer')
    cap = int(config['MAX_NUMBER_OF_CONNECTIONS_PER_RULE'])
    chunk = max(int(os.environ.get('RSA_REDUCER_CHUNK', 64 << 20)), 1)
    eng = Engine(0)

    def write(text):
        _write(text)
        sys.stdout.flush()

    job = ReducerStream(eng, db, cap, write, chunk=chunk)
    src = sys.stdin.buffer
    while True:
        block = src.read(min(chunk, 16 << 20))
        if not block:
            break
        job.feed(block)
    job.finish()
    return 0


def _host_of(path):
    parts = os.path.abspath(path).split('/')
    return parts[-2]


def run_main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description='Fused GPU ruleset analysis: logs -> reducer report')
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument('--db', help='accesslists.db (shelve) or .json')
    src.add_argument('--fortigate', help='a FortiGate config: the rule DB preprosess_fortigate_acl.py would store '
                                         '(restated, ruleset-analysis_amd/fortigate.py)')
    src.add_argument('--asa', help='a Cisco ASA/FWSM config: the rule DB preprosess_access_lists.py would store '
                                   '(restated, ruleset-analysis_amd/asa.py)')
    ap.add_argument('--cap', type=int, default=1000, help='MAX_NUMBER_OF_CONNECTIONS_PER_RULE')
    ap.add_argument('--host', help='firewall host for every input (default: parent directory name)')
    ap.add_argument('--hadoop-output', action='store_true',
                    help="print the report as Hadoop streaming stores it (every line + '\\t\\n', the form "
                         'postprocess_ruleset_analysis.py reads)')
    ap.add_argument('--postprocess', action='store_true',
                    help='print the postprocess_ruleset_analysis.py report (hit counts, zero-hit ACL lines, '
                         'connection lists) instead of the reducer report')
    ap.add_argument('--shadowed', action='store_true',
                    help='also log the rules shadowed by a more generic rule above them '
                         '(preprosess_access_lists.py:508-521) to stderr, computed on the GPU')
    ap.add_argument('logs', nargs='*')
    args = ap.parse_args(argv)
    if args.db:
        db = acldb.load(args.db)
    elif args.asa:
        from . import asa
        with open(args.asa, encoding='latin-1') as f:
            text = f.read()
        db = asa.build_db(text, timestamp=os.stat(args.asa).st_mtime, log=lambda m: sys.stderr.write(m))
    else:
        from . import fortigate
        with open(args.fortigate, encoding='latin-1') as f:
            text = f.read()
        db = fortigate.build_db(text, timestamp=os.stat(args.fortigate).st_mtime,
                                log=lambda m: sys.stderr.write(m))
    inputs = []
    for path in args.logs:
        with open(path, 'rb') as f:
            inputs.append((args.host or _host_of(path), f.read()))
    engine = None
    if args.shadowed:
        from .engine import Engine
        from .shadow import shadow_messages
        engine = Engine(0)
        for host in db.accesslists:
            for m in shadow_messages(engine, {a: e['rules'] for a, e in db.accesslists[host].items()}):
                sys.stderr.write('INFO - ' + m + '\n')
    if not inputs:
        return 0
    try:
        out, _res = analyze_text(inputs, db, cap=args.cap, engine=engine)
    except BaseException as exc:
        # the pipeline died (pipeline.finish_job): the reducer's stdout up to
        # there, then the exception; a failed Hadoop job stores no output
        part = getattr(exc, 'rsa_report', None)
        if part is not None and not (args.postprocess or args.hadoop_output):
            _write(''.join(l + '\n' for l in part))
            sys.stdout.flush()
        raise
    if args.postprocess or args.hadoop_output:
        from .postprocess import hadoop_output, postprocess
        k = out.index('') if '' in out else len(out)   # the noise records of the empty mapper records
        hadoop = hadoop_output(out[k:]) if args.postprocess else hadoop_output(out)
        if args.postprocess:
            _write(''.join(l + '\n' for l in postprocess(db.accesslists, hadoop)))
        else:
            _write(hadoop)
        return 0
    _write(''.join(l + '\n' for l in out))
    return 0
