"""Text emitters with the reference's byte format.

* ``mapper_output`` — the mapper's stdout (``mapper.py:154-155,184-186``):
  ``host;acl;idx<TAB><line incl. its newline>`` followed by ``print``'s own
  newline (the blank record of SURVEY.md trap 4), or the two "missing ACL"
  messages.
* ``reducer_report`` — ``connlist-reducer.py``'s stdout for the sorted mapper
  stream, built from GPU ``Results``: every non-key record the sort places
  before a key group becomes the "Unable to unpack" noise pair
  (``:66-79``); every rule block is a blank line, the header, the original ACL
  line, the hit count, the cap NOTE (``:113-116``), the column header and the
  connection rows (``:119-126``) ordered by the ``"TOIP TOPORT"`` string, a
  stable sort of ``conns.keys()``: ties keep CPython 2.7 dict order, replayed
  from the first-seen order by ``py2dict`` (trap 8).
"""

import numpy as np

from .logparse import PY2_WS, D_CLASSIFY, D_MISSING
from .keytext import INTERNED, KeyText
from .py2dict import iteration_order

__all__ = ['mapper_output', 'reducer_report', 'block_lines', 'HEADER', 'dotted', 'KeyText', 'INTERNED']

HEADER = '%6s %4s  %-15s %-14s %-5s %-19s  %-19s' % ('COUNT', 'PROTO', 'FROM IP', 'TO IP', 'PORT', 'FIRST SEEN',
                                                     'LAST SEEN')
NOISE1 = 'Unable to unpack mapper input line, skipping it.'


def dotted(v):
    v = int(v)
    return '%d.%d.%d.%d' % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)


def _missing_msgs(acl, host, line):
    return ('Unable to process line because access-list {0} is missing from data structure for host {1}, '
            'skipping line.\n'.format(acl, host) + 'The skipped line is: {0}\n'.format(line))


def mapper_output(parsed, gids, compiled):
    """Mapper stdout text (str) for parsed lines and their first-match gids."""
    out = []
    disp = parsed.disposition
    for i in np.nonzero((disp == D_CLASSIFY) | (disp == D_MISSING))[0]:
        i = int(i)
        line = parsed.lines[i]
        if disp[i] == D_MISSING:
            out.append(_missing_msgs(parsed.acl_of[i], parsed.host_of[i], line))
            continue
        g = int(gids[i])
        if g < 0:
            continue
        out.append(compiled.key(g) + '\t' + line + '\n')
    return ''.join(out)


def _rows_by_gid(records):
    order = np.argsort(records['gid'], kind='stable')
    recs = records[order]
    gids, starts = np.unique(recs['gid'], return_index=True)
    ends = np.append(starts[1:], len(recs))
    return {int(g): recs[s:e] for g, s, e in zip(gids, starts, ends)}


def table_order(spell, from_ip, to_ip, to_port, first_seen):
    """Row order of one rule's connection table (connlist-reducer.py:109-110):
    ``conns.keys()`` of the Python 2 dict the rows were inserted into in
    first-seen order, stable-sorted by ``"TOIP TOPORT"``."""
    n = len(to_ip)
    sort_key = [to_ip[k] + ' ' + to_port[k] for k in range(n)]
    if len(set(sort_key)) == n:            # no ties: dict order cannot show
        return sorted(range(n), key=sort_key.__getitem__)
    fs = first_seen.tolist() if hasattr(first_seen, 'tolist') else list(first_seen)
    ins = sorted(range(n), key=fs.__getitem__)
    keys = [';'.join((spell[k], from_ip[k], to_ip[k], to_port[k])) for k in ins]
    py2 = [ins[j] for j in iteration_order(keys)]
    return sorted(py2, key=sort_key.__getitem__)


_OCTET = [str(k) for k in range(256)]


def dotted_list(values):
    """dotted() of a sequence of IPv4 values (one list pass)."""
    o = _OCTET
    return [o[v >> 24] + '.' + o[(v >> 16) & 255] + '.' + o[(v >> 8) & 255] + '.' + o[v & 255]
            for v in (values.tolist() if hasattr(values, 'tolist') else values)]


def key_strings(rows, spells, keytext=None):
    """(PROTO, FROMIP, TOIP, TOPORT) strings of one rule's records."""
    if keytext is None or not (rows['pspell'] & INTERNED).any():
        return ([spells[p] for p in rows['pspell'].tolist()], dotted_list(rows['for_ip']),
                dotted_list(rows['to_ip']), [str(p) for p in rows['to_port'].tolist()])
    return keytext.strings(rows, spells)


class MemoDecode(object):
    """A timestamp decoder with a memo: a report's rows share few distinct codes."""

    def __init__(self, decode):
        self.decode, self.memo = decode, {}

    def __call__(self, code):
        s = self.memo.get(code)
        if s is None:
            s = self.memo[code] = self.decode(code)
        return s


def table_rows(rows, spell, from_ip, to_ip, to_port, ts_decode):
    """The connection-table lines of one rule (connlist-reducer.py:119-126):
    ``rows`` its records, the key strings per record, ordered by table_order."""
    cnt = rows['count'].tolist()
    first = rows['first'].tolist()
    last = rows['last'].tolist()
    if not isinstance(ts_decode, MemoDecode):
        ts_decode = MemoDecode(ts_decode)
    return ['%6d %4s %15s  %15s %-5s %19s  %19s' % (cnt[k], spell[k], from_ip[k], to_ip[k], to_port[k],
                                                     ts_decode(first[k]), ts_decode(last[k]))
            for k in table_order(spell, from_ip, to_ip, to_port, rows['min_order'])]


def block_lines(host, acl, rule, hits, rows, capped, cap, ts_decode, pspell_table, keytext=None):
    """One rule block without the leading blank line (connlist-reducer.py:113-126)."""
    out = ['{0}: access-list {1}, rule {2}: {3}'.format(host, acl, rule.ruleindex, str(rule)),
           '{0}'.format(rule.original), 'Total number of hits: {0}'.format(int(hits))]
    if capped:
        out.append('NOTE: Maximum number of connections ({0}) reached for this rule, additional connections not '
                   'displayed.'.format(cap))
    out.append(HEADER)
    if rows is not None and len(rows):
        out.extend(table_rows(rows, *key_strings(rows, pspell_table, keytext), ts_decode))
    return out


def reducer_report(results, groups, noise, cap, ts_decode, pspell_table, n_blank=0, keytext=None, stop=None):
    """Reducer stdout lines.

    ``groups``: list of (sort_key, gid, host, acl, rule) for every aggregation
    group with at least one mapper line, in the order the reducer meets them.
    ``noise``: list of (position_key, raw_text) non-key records; a record is
    emitted before group g iff position_key < g's sort_key.  ``n_blank`` empty
    records (the mapper's doubled newlines) sort before everything else.
    ``keytext``: the KeyText of records with interned keys.  ``stop``: (gid,
    sorted line text) of the line the reducer dies at (``months.index``,
    ``connlist-reducer.py:164``): the lines end with what it printed before --
    every earlier group's block (the key test of the dying line already ran)
    and the noise sorted before that line -- and no final blank line.
    """
    rows = _rows_by_gid(results.records)
    ts_decode = MemoDecode(ts_decode)
    out = [NOISE1, 'The line was: '] * int(n_blank)
    ni = 0
    noise = sorted(noise, key=lambda t: t[0])
    prev = None
    for sk, gid, host, acl, rule in groups:
        while ni < len(noise) and noise[ni][0] < sk:
            out.append(NOISE1)
            out.append('The line was: {0}'.format(noise[ni][1].strip(PY2_WS)))
            ni += 1
        if prev is not None:
            out.append('')
            out.extend(_block(prev, results, rows, cap, ts_decode, pspell_table, keytext))
        if stop is not None and gid == stop[0]:
            while ni < len(noise) and noise[ni][0] < stop[1]:
                out.append(NOISE1)
                out.append('The line was: {0}'.format(noise[ni][1].strip(PY2_WS)))
                ni += 1
            return out
        prev = (gid, host, acl, rule)
    while ni < len(noise):
        out.append(NOISE1)
        out.append('The line was: {0}'.format(noise[ni][1].strip(PY2_WS)))
        ni += 1
    out.append('')
    if prev is not None:
        out.extend(_block(prev, results, rows, cap, ts_decode, pspell_table, keytext))
    return out


def _block(prev, results, rows, cap, ts_decode, pspell_table, keytext=None):
    gid, host, acl, rule = prev
    capped = cap == 0 or int(results.thresh[gid]) != 0xFFFFFFFFFFFFFFFF
    return block_lines(host, acl, rule, results.hits[gid], rows.get(gid), capped, cap, ts_decode, pspell_table,
                       keytext)
