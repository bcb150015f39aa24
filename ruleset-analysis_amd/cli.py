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
list, ``ValueError`` for malformed addresses), config/DB problems reported on
stderr with exit status 1.
"""

import os
import sys

import numpy as np

from . import acldb
from .compile import CompiledRules, TUPLE_DTYPE, F_HIT, F_BUILT
from .engine import DeviceBatch, Engine
from .logparse import reducer_fields, reducer_timestamp
from .py2text import PY2_WS, py2_int
from .pipeline import analyze_text
from .textparse import parse_text
from .report import mapper_output, reducer_report


def _stdin_lines():
    data = sys.stdin.buffer.read().decode('latin-1')
    out, start = [], 0
    while True:
        i = data.find('\n', start)
        if i < 0:
            if start < len(data):
                out.append(data[start:])
            return out
        out.append(data[start:i + 1])
        start = i + 1


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
        gids = eng.classify_only(parsed.batch()).cpu().numpy() if parsed.n else np.zeros(0, np.int32)
        _write(mapper_output(parsed, gids, compiled))
        sys.stdout.flush()
        if parsed.error is not None:
            raise parsed.error[1]
        if not block:
            break
    return 0


class _Interner(object):
    def __init__(self):
        self.ids = {}
        self.values = []

    def __call__(self, v):
        k = self.ids.get(v)
        if k is None:
            k = self.ids[v] = len(self.values)
            self.values.append(v)
        return k


def reducer_main(argv=None):
    import re  # noqa: F401 - BUILT lives in logparse
    config = load_config()
    db = _open_db(os.path.basename(config['ACCESSLIST_DATABASE_FILENAME']), 'reducer')
    cap = int(config['MAX_NUMBER_OF_CONNECTIONS_PER_RULE'])
    lines = _stdin_lines()
    runs = []            # (key, host, acl, rule)
    events = []          # ('noise', text) | ('run', run id)
    rows = []            # per line with a key: (run, flags, for, to, port, pspell, ts string)
    spell, ips, ports = _Interner(), _Interner(), _Interner()
    current = None
    error = None
    for raw in lines:
        line = raw.strip(PY2_WS)
        try:
            key, value = line.split('\t', 1)
            hostname, acl, ruleindex = key.split(';', 3)
            rule = db.accesslists[hostname][acl]['rules'][py2_int(ruleindex)]
            rule.hostname = hostname
            rule.accesslist = acl
        except ValueError:
            events.append(('noise', line))
            continue
        except (KeyError, IndexError) as exc:        # the reference dies here
            error = exc
            break
        if current is None or key != current:
            current = key
            runs.append((key, hostname, acl, rule))
            events.append(('run', len(runs) - 1))
        hit, res = reducer_fields(value)
        flags = F_HIT if hit else 0
        f = t = p = ps = 0
        ts = None
        if res is not None:
            flags |= F_BUILT
            ps, f, t, p = spell(res[5]), ips(res[6]), ips(res[8]), ports(res[9])
            if hit:
                ts = reducer_timestamp(res)
        rows.append((len(runs) - 1, flags, f, t, p, ps, ts))
    if len(ports.values) > 65536 or len(spell.values) > 256:
        raise NotImplementedError('more than 65536 distinct port strings or 256 protocol words')
    n = len(rows)
    tup = np.zeros(n, dtype=TUPLE_DTYPE)
    gids = np.zeros(n, dtype=np.int32)
    if n:
        arr = np.array([r[:6] for r in rows], dtype=np.int64)
        gids[:] = arr[:, 0]
        tup['flags'] = arr[:, 1]
        tup['src'] = arr[:, 2]
        tup['dst'] = arr[:, 3]
        tup['dport'] = arr[:, 4]
        tup['pspell'] = arr[:, 5]
    distinct_ts = sorted({r[6] for r in rows if r[6] is not None})
    code = {s: k for k, s in enumerate(distinct_ts)}
    ts = np.array([code.get(r[6], 0) for r in rows], dtype=np.uint32)
    order = np.arange(n, dtype=np.uint64)          # the input is already in reducer order
    eng = Engine(0)
    eng.set_rule_count(len(runs))
    b = DeviceBatch.from_numpy(tup, ts, order, eng.device, gids=gids)
    both = F_HIT | F_BUILT
    res = eng.run([b], cap, capacity=max(int(np.count_nonzero((tup['flags'] & both) == both)), 1))
    # decode interned fields back to text through the record fields
    out = _reduce_text(events, runs, res, cap, distinct_ts, spell.values, ips.values, ports.values,
                       finished=error is None)
    _write(''.join(l + '\n' for l in out))
    sys.stdout.flush()
    if error is not None:
        raise error
    return 0


def _reduce_text(events, runs, res, cap, ts_table, spells, ips, ports, finished=True):
    from .report import NOISE1, HEADER, table_order
    by_run = {}
    rec = res.records
    for k in np.argsort(rec['gid'], kind='stable'):
        by_run.setdefault(int(rec['gid'][k]), []).append(rec[k])
    out = []

    def block(r):
        key, host, acl, rule = runs[r]
        rws = by_run.get(r, [])
        if rws:
            rws = [rws[k] for k in table_order([spells[int(x['pspell'])] for x in rws],
                                               [ips[int(x['for_ip'])] for x in rws],
                                               [ips[int(x['to_ip'])] for x in rws],
                                               [ports[int(x['to_port'])] for x in rws],
                                               [int(x['min_order']) for x in rws])]
        lines = ['{0}: access-list {1}, rule {2}: {3}'.format(host, acl, rule.ruleindex, str(rule)),
                 '{0}'.format(rule.original), 'Total number of hits: {0}'.format(int(res.hits[r]))]
        if cap == 0 or int(res.thresh[r]) != 0xFFFFFFFFFFFFFFFF:
            lines.append('NOTE: Maximum number of connections ({0}) reached for this rule, additional connections '
                         'not displayed.'.format(cap))
        lines.append(HEADER)
        for x in rws:
            lines.append('%6d %4s %15s  %15s %-5s %19s  %19s' % (int(x['count']), spells[int(x['pspell'])],
                                                                 ips[int(x['for_ip'])], ips[int(x['to_ip'])],
                                                                 ports[int(x['to_port'])], ts_table[int(x['first'])],
                                                                 ts_table[int(x['last'])]))
        return lines

    prev = None
    for kind, v in events:
        if kind == 'noise':
            out.append(NOISE1)
            out.append('The line was: {0}'.format(v))
        else:
            if prev is not None:
                out.append('')
                out.extend(block(prev))
            prev = v
    if finished:
        out.append('')
        if prev is not None:
            out.extend(block(prev))
    return out


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
    out, _res = analyze_text(inputs, db, cap=args.cap, engine=engine)
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
