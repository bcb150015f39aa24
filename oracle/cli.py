"""ORACLE (test infrastructure only) — the oracle's mapper and reducer as Unix
filters, so the reference's no-Hadoop job can be timed as real processes:

    mapred_input_dir=/x/fw1/y python3 -m oracle.cli map DB.json < log \\
        | LC_ALL=C sort | python3 -m oracle.cli reduce DB.json [CAP] > report

(``mapper.py:107-189`` / ``connlist-reducer.py:62-211`` restated in
``oracle.mapper`` / ``oracle.reducer``; the host comes from
``$mapred_input_dir`` like ``mapper.py:107-112``).  Used by bench.py's CPU
baseline leg only.
"""

import io
import json
import os
import sys


def _db(path):
    from .crosscheck_2to3 import oracle_db
    with open(path) as f:
        return oracle_db(json.load(f))


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    mode, db_path = argv[0], argv[1]
    acls, fws = _db(db_path)
    stdin = io.TextIOWrapper(sys.stdin.buffer, encoding='latin-1', newline='\n')
    stdout = io.TextIOWrapper(sys.stdout.buffer, encoding='latin-1', newline='\n', write_through=False)
    # a Python 2 script that dies still flushes what it printed: the partial
    # output is written before the exception propagates (exit status 1)
    if mode == 'map':
        from .mapper import HostMissing, map_lines
        host = os.environ['mapred_input_dir'].split('/')[-2]
        out = []
        chunk = []
        try:
            for line in stdin:
                chunk.append(line)
                if len(chunk) >= 65536:
                    map_lines(chunk, host, acls, fws, out)
                    stdout.write(''.join(out))
                    out, chunk = [], []
            map_lines(chunk, host, acls, fws, out)
        except HostMissing:
            sys.exit(1)                                   # mapper.py:115-117 (the message is in out)
        finally:
            stdout.write(''.join(out))
            stdout.flush()
    elif mode == 'reduce':
        from .reducer import reduce_lines
        cap = int(argv[2]) if len(argv) > 2 else 1000
        lines = []
        try:
            reduce_lines(stdin, acls, cap, out=lines)
        finally:
            stdout.write(''.join(l + '\n' for l in lines))
            stdout.flush()
    else:
        raise SystemExit('usage: python -m oracle.cli map|reduce DB.json [CAP]')
    stdout.flush()


if __name__ == '__main__':
    main()
