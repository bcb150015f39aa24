"""The C oracle (oracle/rsa_oracle.c, the checker of every large GPU test)
against the Python oracle (pinned byte for byte to the lib2to3-converted
reference, tests/golden) beyond the golden sizes: a synthetic 10k-rule ACL
with the cap engaged and shuffled input (sort order != input order), >= 50k
log lines rendered as text and run through oracle.pipeline (mapper | sort |
reducer) — per-rule hits and connection tables must agree."""
import numpy as np

from oracle import coracle
from oracle import pipeline as op
from oracle.crosscheck_2to3 import oracle_db
from ruleset_analysis_amd import synth


def _map_chunk(lines, dbj):
    from oracle.mapper import map_lines
    acls, fws = oracle_db(dbj)
    out = []
    map_lines(lines, 'fw1', acls, fws, out)
    return ''.join(out)


def test_c_oracle_equals_python_oracle_10k_rules_capped_shuffled():
    dbj, info = synth.make_db(77, 10000, broad=False)
    tr = synth.make_traffic((dbj, info), 60000, seed=78, zipf=1.3)
    perm = np.random.default_rng(79).permutation(60000)
    for k in ('src', 'dst', 'sport', 'dport', 'proto', 'ifc', 'form', 't', 'cid'):
        tr[k] = tr[k][perm]
    cap = 40
    lines = [l + '\n' for l in synth.render_lines(tr)]
    # mapper | LC_ALL=C sort | reducer, the mapper over 8 splits in parallel
    # processes (as Hadoop runs one mapper per split; it is pure Python)
    import multiprocessing as mproc
    chunks = [lines[k::8] for k in range(8)]
    with mproc.get_context('fork').Pool(8) as pool:
        mapped = ''.join(pool.starmap(_map_chunk, [(c, dbj) for c in chunks]))
    acls, _fws = oracle_db(dbj)
    from oracle.reducer import reduce_lines
    _red, blocks = reduce_lines(op._split_nl(op.c_sort(mapped)), acls, cap)
    R = coracle.OracleRules(dbj)
    cols, ts, order = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ts, order, cap)
    py = {}
    for b in blocks:
        gid = R.base[tuple(b['key'].split(';')[:2])] + int(b['key'].split(';')[2])
        py[gid] = b
    assert set(py) == set(int(g) for g in np.nonzero(ref['matches'])[0])
    rows = ref['rows']
    capped = 0
    for gid, b in py.items():
        assert int(ref['matches'][gid]) == b['matches']
        assert int(ref['hits'][gid]) == b['hits']
        assert (int(ref['n_conns'][gid]) >= cap) == b['capped']
        capped += b['capped']
        sel = np.nonzero(rows['gid'] == gid)[0]
        got = sorted((synth.PSPELL[int(rows['pspell'][k])], synth._dotted(rows['for_ip'][k]),
                      synth._dotted(rows['to_ip'][k]), str(int(rows['to_port'][k])), int(rows['count'][k]),
                      synth.ts_decode(int(rows['first'][k])), synth.ts_decode(int(rows['last'][k]))) for k in sel)
        want = sorted(tuple(c[0].split(';')) + (c[1], c[2], c[3]) for c in b['conns'])
        assert got == want, gid
    assert capped > 20
