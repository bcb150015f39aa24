"""ORACLE (test infrastructure only) — pin the death and edge cases of the
fused job to the reference itself.

Run in the build container only (``/root/reference`` does not exist on the GPU
box).  The cases are ``tests/death_cases.cases()``: one seeded synthetic log
with months ``months.index`` rejects (``connlist-reducer.py:151-164``), ports
past 65535 (``firewallrule.py:47-53``), a bad address and a firewall missing
from the DB (mapper deaths, ``mapper.py:115-117,138-142``), 200 protocol
spellings.  For each case the lib2to3-converted reference
(``crosscheck_2to3.prepare_reference`` / ``run_reference_job``) runs
``mapper | LC_ALL=C sort | connlist-reducer.py`` under ``set -o pipefail``;
the oracle's job (``death_cases.oracle_job``) must give the same stdout bytes
and die the same way, and the case is written to ``tests/golden_deaths/``:
its inputs (the base log once, each case's replaced lines) and the
reference's stdout sha256, byte count, exit status and exception.

One case cannot be reproduced under Python 3: ``port_python2_long`` (a port
past 2^63 - 1 is a Python 2 ``long``, which ``FirewallRule.__init__``
rejects at ``firewallrule.py:67-75``; Python 3 has one int type).  Its fixture
keeps the converted reference's output but is marked ``unpinned`` and the
tests compare that case with the oracle only.

Usage: ``python3 oracle/crosscheck_deaths.py``.
"""

import hashlib
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))

UNPINNED = {
    'port_python2_long': 'Python 3 has no long: the converted reference accepts the port that '
                         'firewallrule.py:67-75 rejects under Python 2',
}


def main():
    from oracle.crosscheck_2to3 import REF, prepare_reference, run_reference_job
    import death_cases as dc
    if not os.path.isdir(REF):
        sys.exit('reference not present; this script only runs in the build container')
    import rsa_pkg
    rsa_pkg.load()
    dbj, out = dc.cases()
    base = dc._base()[1]
    entries, bad = {}, []
    works = {}
    with tempfile.TemporaryDirectory(prefix='rsa_xdeath_') as tmp:
        for name in dc.NAMES:
            inputs, cap, _death = out[name]
            if cap not in works:
                works[cap] = os.path.join(tmp, 'cap%d' % cap)
                prepare_reference(works[cap], dbj, cap)
            ref = run_reference_job(works[cap], [(h, ''.join(ls)) for h, ls in inputs])
            status = 1 if (ref['map_rc'] or ref['reduce_rc']) else 0
            exc = ref['reduce_exc'] if ref['reduce_rc'] else ref['map_exc']
            red, err = dc.oracle_job(dbj, inputs, cap)
            o_text = ''.join(l + '\n' for l in red)
            agree = o_text == ref['reduce'] and dc.exc_name(err) == exc
            e = {'cap': cap, 'inputs': dc.encode_inputs(base, inputs),
                 'reference': {'stdout_sha256': hashlib.sha256(ref['reduce'].encode('latin-1')).hexdigest(),
                               'stdout_bytes': len(ref['reduce'].encode('latin-1')),
                               'stdout_lines': ref['reduce'].count('\n'), 'status': status, 'exception': exc,
                               'map_status': ref['map_rc'], 'reduce_status': ref['reduce_rc'],
                               'oracle_agrees': agree}}
            if name in UNPINNED:
                e['reference']['unpinned'] = UNPINNED[name]
            elif not agree:
                bad.append(name)
            assert dc.decode_inputs(base, e['inputs']) == [(h, list(ls)) for h, ls in inputs]
            entries[name] = e
            print('%-28s cap=%-5d status=%d exc=%-10s lines=%-5d oracle %s%s' % (
                name, cap, status, exc, e['reference']['stdout_lines'], 'OK' if agree else 'DIFF',
                ' (unpinned)' if name in UNPINNED else ''))
    if bad:
        sys.exit('oracle disagrees with the converted reference on: %s' % ', '.join(bad))
    entries['_source'] = 'lib2to3-converted reference, oracle/crosscheck_deaths.py'
    dc.save_fixture(dbj, base, entries)


if __name__ == '__main__':
    main()
