"""bench.py's own multi-rank path on CPU: ``--gpus 2 --backend gloo
--cpu-model`` spawns two rank processes, each builds its contiguous shard of
the global synthetic log and runs dist.merge (all_reduce, all_to_all to owner
gid % world, threshold all_reduce, pass-2 exchange, gather) with the CPU model
of the HIP table (tests/cpu_model.py); rank 0's merged result must equal the C
oracle over the concatenated log (runAnalysis.sh:12,42-56 is what the merge
replaces)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import coracle
from ruleset_analysis_amd.compile import RECORD_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NO = 0xFFFFFFFFFFFFFFFF


def run_bench(tmp_path, extra, timeout=600):
    dump = str(tmp_path / 'merged.npz')
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', '1', '--warmup', '0', '--no-cpu-baseline',
           '--dump', dump] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0]), np.load(dump)


def check_dump_against_oracle(got, world, rules, lines, cap, seed=3):
    """rank 0's dumped result vs the C oracle over the ranks' shards in rank order."""
    import bench
    wl = bench.Workload('cfg3', rules=rules, cap=cap)
    assert wl.seed == seed
    dbj = wl.dbj
    trs = [c[1] for r in range(world) for c in bench.shard_chunks(wl, lines, r, world)]
    tr = {k: np.concatenate([t[k] for t in trs]) for k in ('src', 'dst', 'sport', 'dport', 'proto', 'ifc', 'form',
                                                          't', 'cid')}
    tr.update(interfaces=trs[0]['interfaces'], host=trs[0]['host'])
    R = coracle.OracleRules(dbj)
    cols, ts, order = coracle.inputs_from_traffic(R, tr)
    ref = coracle.run(R, cols, ts, order, cap)
    assert np.array_equal(got['matches'], ref['matches'])
    assert np.array_equal(got['hits'], ref['hits'])
    assert np.array_equal(got['thresh'] != NO, (ref['n_conns'] >= cap) & (cap > 0))
    recs = got['records'].view(RECORD_DTYPE)
    g = sorted((int(r['gid']), int(r['pspell']), int(r['for_ip']), int(r['to_ip']), int(r['to_port']),
                int(r['count']), int(r['first']), int(r['last'])) for r in recs)
    rows = ref['rows']
    want = sorted(zip(*(rows[k].astype(int).tolist() for k in ('gid', 'pspell', 'for_ip', 'to_ip', 'to_port',
                                                                'count', 'first', 'last'))))
    assert g == want
    assert (got['matches'] > 0).sum() > 10
    return ref


@pytest.mark.parametrize('world,cap', [(2, 15), (3, 100000), (8, 12)])
def test_bench_spawn_cpu_model_matches_oracle(tmp_path, world, cap):
    """World 8 is the driver's scaling run (one node): eight rank processes,
    the all_to_all routing to eight owners, the cap engaged."""
    rules, lines = 300, 12000
    line, got = run_bench(tmp_path, ['--backend', 'gloo', '--cpu-model', '--gpus', str(world), '--rules', str(rules),
                                     '--lines', str(lines), '--cap', str(cap)])
    assert line['n_gpus'] == world and line['cpu_model'] is True
    check_dump_against_oracle(got, world, rules, lines, cap)


def test_bench_refuses_mismatched_world(tmp_path):
    """Under torch.distributed.run, WORLD_SIZE must equal --gpus (no silent 1-GPU run)."""
    env = dict(os.environ, WORLD_SIZE='2', RANK='0', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT='1')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '8'], capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode == 2 and 'WORLD_SIZE=2' in p.stderr


def test_bench_refuses_more_gpus_than_visible():
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '64'], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 2 and 'GPU(s) visible' in p.stderr
