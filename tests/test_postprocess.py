"""Downstream of the path: the Hadoop output form
of the reducer report and the zero-hit / connection-list report of
postprocess_ruleset_analysis.py, byte for byte against the lib2to3-converted
reference run on the golden cases (tests/golden/*/hadoop.txt ->
postprocess.txt, written by oracle/crosscheck_2to3.py)."""
import os

import pytest

from conftest import GOLDEN, golden_cases
from golden_io import load_case
from ruleset_analysis_amd import acldb
from ruleset_analysis_amd.postprocess import hadoop_output, postprocess

CASES = [c for c in golden_cases() if os.path.exists(os.path.join(GOLDEN, c, 'postprocess.txt'))]


def _read(case, name):
    with open(os.path.join(GOLDEN, case, name), encoding='latin-1', newline='') as f:
        return f.read()


@pytest.mark.parametrize('case', CASES)
def test_postprocess_matches_reference(case):
    dbj, _text, _report, _sha, _params = load_case(case)
    db = acldb.load_json(dbj)
    out = postprocess(db.accesslists, _read(case, 'hadoop.txt'))
    assert ''.join(l + '\n' for l in out) == _read(case, 'postprocess.txt')


@pytest.mark.parametrize('case', CASES)
def test_hadoop_output_form(case):
    report = _read(case, 'report.txt').split('\n')[:-1]
    k = report.index('')                    # the noise records a reduce partition may not receive
    assert hadoop_output(report[k:]) == _read(case, 'hadoop.txt')


def test_postprocess_needs_a_rule_header():
    """An entry without a rule header stops the reference at :96 (IndexError)."""
    dbj, _text, _report, _sha, _params = load_case(CASES[0])
    with pytest.raises(IndexError):
        postprocess(acldb.load_json(dbj).accesslists, 'Unable to unpack mapper input line, skipping it.\t\n')
