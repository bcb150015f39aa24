"""Diagnosis of the natural-chain cfg4 case (tests/test_gpu_cfg4.py::
test_cfg4_natural_chain_over_65534_entries) stage by stage, each stage
synchronised and reported before the next starts."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import rsa_pkg  # noqa: E402

rsa_pkg.load()
from oracle import coracle  # noqa: E402
from ruleset_analysis_amd import fortigate, synth, synth_fg  # noqa: E402
from ruleset_analysis_amd.compile import CompiledRules  # noqa: E402
from ruleset_analysis_amd.engine import DeviceBatch, Engine  # noqa: E402
from ruleset_analysis_amd.pipeline import built_hit_count  # noqa: E402


def say(*a):
    print(*a, flush=True)


text, info = synth_fg.make_config(9, n_policies=300, n_wide=2)
comp = CompiledRules(fortigate.build_db(text))
comp.ensure_lists()
tr = synth_fg.make_traffic(info, 8000, seed=45)
tup, ts, order = synth.pack(tr, comp)
R = coracle.OracleRules.from_fortigate(text)
cols, ots, oorder = coracle.inputs_from_traffic(R, tr)
gref, _ = coracle.classify(R, cols['list'], cols['proto'], cols['src'], cols['dst'], cols['sport'], cols['dport'])
say('host ready: rules', comp.n_rules, 'hit+built', built_hit_count(tup))
import torch  # noqa: E402

eng = Engine(0)
b = DeviceBatch.from_numpy(tup, ts, order, eng.device)
stages = sys.argv[1].split(',') if len(sys.argv) > 1 else ['cls_pht', 'cls_bucket', 'job_pht', 'p1_bucket', 'job_bucket']
for st in stages:
    kind = st.split('_')[1]
    eng.load_compiled(comp, kind=kind)
    say('stage', st, 'index', eng.index_kind)
    if st.startswith('cls'):
        g = eng.classify_only(b)
        torch.cuda.synchronize()
        say('  classify_only equal to oracle:', bool(np.array_equal(g.cpu().numpy(), gref)))
    elif st.startswith('p1'):
        eng.reset(max(built_hit_count(tup), 1), 0)
        g = torch.empty(b.n, dtype=torch.int32, device=eng.device)
        eng.pass1(b, g)
        torch.cuda.synchronize()
        say('  pass 1 without table: gids equal:', bool(np.array_equal(g.cpu().numpy(), gref)))
    else:
        eng.reset(max(built_hit_count(tup), 1), 1000)
        g = torch.empty(b.n, dtype=torch.int32, device=eng.device)
        eng.pass1(b, g)
        torch.cuda.synchronize()
        say('  pass 1 done; gids equal:', bool(np.array_equal(g.cpu().numpy(), gref)))
        n = eng.resolve_cap()
        torch.cuda.synchronize()
        say('  cap resolved:', n)
        res = eng.results(1000)
        say('  records', len(res.records))
eng.close()
say('all stages done')
