"""ORACLE (test infrastructure only) — restatement of the reducer,
``connlist-reducer.py:25-211`` (``reducer.py`` differs only at lines 34/37).

Python-2 semantics that matter and how they are kept:

* input lines are ``str`` decoded as latin-1 (byte-transparent); ``strip()`` is
  restricted to the ASCII whitespace Python 2's byte ``str.strip()`` removes;
* connection-table rows are ordered by the ``"TOIP TOPORT"`` string
  (``connlist-reducer.py:109-110``), a stable sort of ``conns.keys()``, so ties
  keep CPython 2.7 dict order, replayed by ``oracle.py2dict`` from the
  insertion order (SURVEY.md trap 8);
* the distinct-connection cap ``len(conns) < MAX`` guards every update
  (``:151``), so once the cap-th connection is inserted the table freezes.

``reduce_lines`` returns the printed lines (without ``'\\n'``) and a structured
per-block result list used by the parity tests.
"""

import re

from .py2dict import py2_keys

# connlist-reducer.py:25
BUILT = re.compile(r'[a-zA-Z]+ [0-9 ]?[0-9] ([0-9:]+) ([a-zA-Z]+) ([0-9]+) ([0-9]+) .* Built (out|in)bound '
                   r'([a-zA-Z]+) .* for [a-zA-Z0-9_-]+:([0-9.]+)/([0-9]+) .* to [a-zA-Z0-9_-]+:([0-9.]+)/([0-9]+)')
MONTHS = ['Jan', 'Feb', 'Mar', 'Apr', 'May', 'Jun', 'Jul', 'Aug', 'Sep', 'Oct', 'Nov', 'Dec']
PY2_WS = ' \t\n\r\x0b\x0c'
HEADER = '%6s %4s  %-15s %-14s %-5s %-19s  %-19s' % ('COUNT', 'PROTO', 'FROM IP', 'TO IP', 'PORT',
                                                     'FIRST SEEN', 'LAST SEEN')


def _block(out, rule, hits, conns, first, last, cap):
    # connlist-reducer.py:108-126 / 185-206
    order = sorted(py2_keys(list(conns)), key=lambda c: ' '.join(c.split(';')[2:4]))
    out.append('{0}: access-list {1}, rule {2}: {3}'.format(rule.hostname, rule.accesslist, rule.ruleindex, str(rule)))
    out.append('{0}'.format(rule.original))
    out.append('Total number of hits: {0}'.format(hits))
    if len(conns) >= cap:
        out.append('NOTE: Maximum number of connections ({0}) reached for this rule, additional connections '
                   'not displayed.'.format(cap))
    out.append(HEADER)
    rows = []
    for c in order:
        proto, from_ip, to_ip, to_port = c.split(';')
        out.append('%6d %4s %15s  %15s %-5s %19s  %19s' % (conns[c], proto, from_ip, to_ip, to_port,
                                                             first[c], last[c]))
        rows.append([c, conns[c], first[c], last[c]])
    return rows


def reduce_lines(lines, accesslists, cap=1000, out=None):
    """``out``: a list the printed lines are appended to (so a caller still
    has them when the reference's KeyError / IndexError / ValueError escapes)."""
    out = [] if out is None else out
    blocks = []
    conns, first, last = {}, {}, {}
    currentkey = ''
    currentrule = None
    hits = 0
    matches = 0
    for raw in lines:
        line = raw.strip(PY2_WS)
        try:                                                          # :63-79
            key, value = line.split('\t', 1)
            hostname, acl, ruleindex = key.split(';', 3)
            rule = accesslists[hostname][acl]['rules'][int(ruleindex)]
            rule.hostname = hostname
            rule.accesslist = acl
        except ValueError:
            out.append('Unable to unpack mapper input line, skipping it.')
            out.append('The line was: {0}'.format(line))
            continue
        if currentkey == '':
            currentkey = key
        if currentrule is None:
            currentrule = rule
        if key != currentkey:                                         # :91-136
            out.append('')
            rows = _block(out, currentrule, hits, conns, first, last, cap)
            blocks.append({'key': currentkey, 'matches': matches, 'hits': hits,
                           'capped': len(conns) >= cap, 'conns': rows})
            conns, first, last = {}, {}, {}
            currentkey, currentrule, hits, matches = key, rule, 0, 0
        matches += 1
        if value.find('-6-302013') != -1 or value.find('-6-302015') != -1:   # :146-148
            hits += 1
            if len(conns) < cap:                                      # :151
                m = BUILT.search(value)
                if m:
                    res = m.groups()
                    conn = ';'.join([res[5], res[6], res[8], res[9]])  # :162
                    month = str(MONTHS.index(res[1]) + 1).zfill(2)
                    ts = res[3] + '-' + month + '-' + res[2].zfill(2) + ' ' + res[0]
                    if conn in conns:
                        conns[conn] += 1
                        if ts < first[conn]:
                            first[conn] = ts
                        if ts > last[conn]:
                            last[conn] = ts
                    else:
                        conns[conn] = 1
                        first[conn] = ts
                        last[conn] = ts
    out.append('')                                                    # :185
    if currentrule is not None:
        rows = _block(out, currentrule, hits, conns, first, last, cap)
        blocks.append({'key': currentkey, 'matches': matches, 'hits': hits,
                       'capped': len(conns) >= cap, 'conns': rows})
    return out, blocks
