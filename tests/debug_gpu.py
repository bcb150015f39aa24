import sys, os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import conftest
import numpy as np
from golden_io import load_case, split_lines
from oracle import coracle
from ruleset_analysis_amd import acldb
from ruleset_analysis_amd.compile import CompiledRules
from ruleset_analysis_amd.engine import Engine, DeviceBatch
from ruleset_analysis_amd.logparse import parse_logs
from ruleset_analysis_amd.pipeline import built_hit_count
case = sys.argv[1] if len(sys.argv) > 1 else 'cap1'
dbj, text, report, sha, params = load_case(case)
lines = split_lines(text)
db = acldb.load_json(dbj); comp = CompiledRules(db)
parsed = parse_logs([('fw1', lines)], db, comp)
eng = Engine(0)
ent, off = comp.packed(); eng.load_rules(ent, off, comp.n_rules)
b = DeviceBatch.from_numpy(parsed.tuples, parsed.ts, parsed.order, eng.device)
res = eng.run([b], params['cap'], capacity=built_hit_count(parsed.tuples))
g = eng.last_gids[0].cpu().numpy()
R = coracle.OracleRules(dbj)
cols, ts, order, tst, sp = coracle.inputs_from_text(R, 'fw1', lines)
ref = coracle.run(R, cols, ts, order, params['cap'])
print('gid equal', np.array_equal(g, ref['gid']), (g >= 0).sum(), (ref['gid'] >= 0).sum())
bad = np.nonzero(g != ref['gid'])[0]
print('n bad', len(bad))
for i in bad[:10]:
    t = parsed.tuples[i]
    print(i, g[i], ref['gid'][i], t, lines[i][:150])
print('matches eq', np.array_equal(res.matches, ref['matches']), res.matches.sum(), ref['matches'].sum())
print('hits eq', np.array_equal(res.hits, ref['hits']))
