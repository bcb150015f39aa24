"""Helpers to read the committed golden cases (tests/golden/<case>/)."""
import json
import os

from conftest import GOLDEN


def load_case(name):
    d = os.path.join(GOLDEN, name)
    with open(os.path.join(d, 'db.json')) as f:
        dbj = json.load(f)
    with open(os.path.join(d, 'log.txt'), encoding='latin-1', newline='') as f:
        text = f.read()
    with open(os.path.join(d, 'report.txt'), encoding='latin-1', newline='') as f:
        report = f.read()
    with open(os.path.join(d, 'mapper.sha256')) as f:
        mapper_sha = f.read().strip()
    with open(os.path.join(d, 'params.json')) as f:
        params = json.load(f)
    return dbj, text, report, mapper_sha, params


def split_lines(text):
    out, start = [], 0
    while True:
        i = text.find('\n', start)
        if i < 0:
            if start < len(text):
                out.append(text[start:])
            return out
        out.append(text[start:i + 1])
        start = i + 1
