"""ORACLE (test infrastructure only) — the reference's no-Hadoop job
``mapred_input_dir=/x/<host>/y mapper.py < log | LC_ALL=C sort | reducer.py``
(Hadoop form ``runAnalysis.sh:42-56``).

Text is handled as latin-1 ``str`` so every byte maps to one code point and
Python's string order equals ``LC_ALL=C sort``'s byte order.
"""

from .mapper import map_lines
from .reducer import reduce_lines


def _split_nl(text):
    out, start = [], 0
    while True:
        i = text.find('\n', start)
        if i < 0:
            if start < len(text):
                out.append(text[start:])
            return out
        out.append(text[start:i + 1])
        start = i + 1


def c_sort(text):
    """``LC_ALL=C sort``: split on '\\n', byte-order sort, re-terminate."""
    if not text:
        return ''
    lines = text.split('\n')
    if text.endswith('\n'):
        lines.pop()
    lines.sort()
    return ''.join(l + '\n' for l in lines)


def run_pipeline(log_text, hostname, accesslists, firewalls, cap=1000):
    """Return (mapper_stdout, sorted_text, reducer_lines, reducer_blocks)."""
    out = []
    map_lines(_split_nl(log_text), hostname, accesslists, firewalls, out)
    mapped = ''.join(out)
    srt = c_sort(mapped)
    red, blocks = reduce_lines(_split_nl(srt), accesslists, cap)
    return mapped, srt, red, blocks


def run_multi(logs_by_host, accesslists, firewalls, cap=1000):
    """Several input directories (one host each) through one sort + reducer,
    as Hadoop feeds every mapper's output into the shuffle."""
    out = []
    for host, text in logs_by_host:
        map_lines(_split_nl(text), host, accesslists, firewalls, out)
    mapped = ''.join(out)
    srt = c_sort(mapped)
    red, blocks = reduce_lines(_split_nl(srt), accesslists, cap)
    return mapped, srt, red, blocks
