"""BASELINE config 3 at the bench's full per-GPU size (125M lines, 10,016
expanded rules, cap 1000) as a GPU test: too large for the C oracle, so the
size-independent properties `bench.py` checks after its timed steps must hold
-- index gids = a linear scan of the lists over every line, the line and hit
counters = the gid histograms, every uncapped rule's connection counts = its
hit+BUILT lines, and a rerun gives the bit-identical record set."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cfg3_full_size_properties():
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', '1', '--warmup', '1',
                        '--no-cpu-baseline'], capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line['config']['lines_per_gpu'] == 125_000_000 and line['config']['rules'] == 10016
    c = line['checks']
    for k in ('rerun_identical_records', 'matches_eq_gid_histogram', 'hits_eq_gid_histogram',
              'sum_matches_eq_classified_lines', 'uncapped_count_sum_eq_hit_built_lines', 'index_gids_eq_linear_scan'):
        assert c[k] is True, (k, c)
    assert c['uncapped_rules_checked'] > 5000 and c['ok']
