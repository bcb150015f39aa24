"""The oracle reproduces the golden outputs of the (lib2to3-converted) reference
byte for byte — the pin that makes it a trustworthy checker."""
import hashlib

import pytest

from conftest import golden_cases
from golden_io import load_case
from oracle import pipeline as op
from oracle.crosscheck_2to3 import oracle_db


@pytest.mark.parametrize('case', golden_cases())
def test_oracle_matches_reference_golden(case):
    dbj, text, report, mapper_sha, params = load_case(case)
    acls, fws = oracle_db(dbj)
    mapped, _srt, red, _blocks = op.run_pipeline(text, params['host'], acls, fws, cap=params['cap'])
    assert hashlib.sha256(mapped.encode('latin-1')).hexdigest() == mapper_sha
    assert ''.join(l + '\n' for l in red) == report


def test_c_sort_edge_cases():
    assert op.c_sort('') == ''
    assert op.c_sort('b\na') == 'a\nb\n'
    assert op.c_sort('x\n\ny\n') == '\nx\ny\n'
