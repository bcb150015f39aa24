"""Host-side parse of firewall log text into packed tuples.

This is the step *before* the hot path (SURVEY.md §8f row 1 — a GPU byte-scan
version is the next planned row); the drop-in CLIs need it to turn text into
what the HIP kernels consume.  It restates, per line:

* the mapper's parse — ``get_builtconn`` of the absent ``lib/fw-regex``
  submodule (``mapper.py:124-142``), by the definition documented in
  DESIGN.md §Parse (canonical Cisco "Built {in,out}bound {TCP,UDP}" messages);
  connection construction validates like ``FirewallRule.__init__``
  (``firewallrule.py:47-93``);
* the ACL lookup ``mapper.py:145-156`` and the candidate-list choice
  ``mapper.py:159-166`` (via ``CompiledRules.list_id``);
* the reducer's per-line facts for the same text (``connlist-reducer.py:146-165``):
  the hit test, the BUILT regex, the connection key and the timestamp string.

Outputs are numpy arrays: ``tuples`` (``TUPLE_DTYPE``), ``ts`` (uint32 codes,
the rank of the reducer timestamp string among all distinct ones — order
preserving, decoded through ``ts_table``) and ``order`` (uint64, the rank of
the line's bytes — the order ``LC_ALL=C sort`` gives the reducer within one key).
"""

import re

import numpy as np

from .compile import TUPLE_DTYPE, F_VALID, F_HIT, F_BUILT, F_SWAP
from .firewallrule import FirewallRule
from .ipaddr import IP
from .py2text import PY2_WS, py2_int, py2_is_int
from .keytext import INTERNED, MAX_SPELL_ID, KeyText

__all__ = ['ParsedLog', 'parse_logs', 'get_builtconn', 'BUILT', 'PY2_WS', 'reducer_fields',
           'D_IGNORE', 'D_NOACL', 'D_MISSING', 'D_CLASSIFY']

D_IGNORE, D_NOACL, D_MISSING, D_CLASSIFY = 0, 1, 2, 3

_GB = re.compile(r'^(?P<rmon>[A-Z][a-z]{2}) +(?P<rday>\d{1,2}) (?P<rtime>\d\d:\d\d:\d\d) '
                 r'(?:(?P<mon>[A-Z][a-z]{2}) +(?P<day>\d{1,2}) (?P<year>\d{4}) (?P<time>\d\d:\d\d:\d\d): )?'
                 r'.*?%(?:ASA|FWSM|PIX)-\d-\d{6}: Built (?P<dir>inbound|outbound) (?P<proto>TCP|UDP) connection \d+ '
                 r'for (?P<if1>[A-Za-z0-9_-]+):(?P<ip1>[0-9.]+)/(?P<p1>[0-9]+) \([^)]*\) '
                 r'to (?P<if2>[A-Za-z0-9_-]+):(?P<ip2>[0-9.]+)/(?P<p2>[0-9]+)', re.ASCII)

# connlist-reducer.py:25 (the reducer's own pattern, applied to the same line)
BUILT = re.compile(r'[a-zA-Z]+ [0-9 ]?[0-9] ([0-9:]+) ([a-zA-Z]+) ([0-9]+) ([0-9]+) .* Built (out|in)bound '
                   r'([a-zA-Z]+) .* for [a-zA-Z0-9_-]+:([0-9.]+)/([0-9]+) .* to [a-zA-Z0-9_-]+:([0-9.]+)/([0-9]+)')
_MONTHS = ['Jan', 'Feb', 'Mar', 'Apr', 'May', 'Jun', 'Jul', 'Aug', 'Sep', 'Oct', 'Nov', 'Dec']


def get_builtconn(line):
    """Mapper-side parse.  None for lines the mapper skips."""
    m = _GB.match(line)
    if not m:
        return None
    g = m.groupdict()
    if g['year']:
        when = (g['year'], g['mon'], g['day'], g['time'])
    else:
        when = (None, g['rmon'], g['rday'], g['rtime'])
    inbound = g['dir'] == 'inbound'
    near = (g['if1'], g['ip1'], g['p1'])
    far = (g['if2'], g['ip2'], g['p2'])
    a, b = (near, far) if inbound else (far, near)
    return {'year': when[0], 'month': when[1], 'day': when[2], 'time': when[3], 'protocol': g['proto'],
            'direction': g['dir'], 'interface_in': a[0], 'interface_out': b[0], 'src': a[1], 'dst': b[1],
            'sport': a[2], 'dport': b[2]}


def reducer_fields(stripped):
    """(hit, built_match_groups or None) for a stripped log line (connlist-reducer.py:146-153)."""
    hit = stripped.find('-6-302013') != -1 or stripped.find('-6-302015') != -1
    m = BUILT.search(stripped)
    return hit, (m.groups() if m else None)


def reducer_timestamp(res):
    """connlist-reducer.py:163-165 (ValueError for an unknown month, as the reducer)."""
    month = str(_MONTHS.index(res[1]) + 1).zfill(2)
    return res[3] + '-' + month + '-' + res[2].zfill(2) + ' ' + res[0]


def _canonical_v4(text):
    ip = IP(text)
    if ip._ipversion != 4 or ip._prefixlen != 32:
        return None
    v = ip.ip
    if '%d.%d.%d.%d' % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255) != text:
        return None
    return v


class ParseError(Exception):
    pass


class ParsedLog(object):
    """Packed form of one or more hosts' log lines."""

    def __init__(self):
        self.lines = []            # original lines (with terminator), all hosts
        self.host_of = []          # host per line
        self.disposition = None    # uint8 per line (D_*)
        self.acl_of = {}           # line index -> acl name for D_MISSING
        self.tuples = None
        self.ts = None
        self.order = None
        self.ts_table = []
        self.pspell_table = []
        self.error = None          # (line index, exception) — the mapper dies there
        self.n = 0
        self.keytext = None        # keytext.KeyText of the interned (non-canonical) reducer keys
        self.keyx = {}             # line index -> KeyText id of its interned reducer key
        self.bad_month = {}        # line index -> the ValueError months.index raises for its hit, BUILT line


def parse_logs(inputs, db, compiled, pspell_table=None, need_order=True, keytext=None):
    """inputs: iterable of (host, list_of_lines).  Lines keep their '\\n'.
    ``keytext``: a report.KeyText shared with other parses (a new one if None).

    Stops at the first line where the reference mapper would raise; the
    exception and line index are kept in ``.error`` and everything before it is
    parsed (the drop-in mapper prints that prefix and then re-raises).  A hit,
    BUILT line whose month ``months.index`` rejects is NOT an error here: the
    mapper never looks at the month (``mapper.py:127-131``) and the reducer
    only for a line it still inserts (``connlist-reducer.py:151-164``); such
    lines are kept in ``.bad_month`` (flag F_BUILT cleared: a hit, never a
    record) for the job to decide after aggregation."""
    P = ParsedLog()
    P.keytext = keytext if keytext is not None else KeyText()
    pspell = {} if pspell_table is None else {s: i for i, s in enumerate(pspell_table)}
    rows = []
    disp = []
    ts_str = []
    for host, lines in inputs:
        if host not in db.firewalls or host not in db.accesslists:
            P.error = (len(P.lines), SystemExit('Firewall {0} not present in data structure. Aborting.'.format(host)))
            break
        fw = db.firewalls[host]
        acls = db.accesslists[host]
        for line in lines:
            i = len(P.lines)
            try:
                row, d, ts = _parse_one(line, host, fw, acls, compiled, pspell, P, i)
            except (KeyError, ValueError) as exc:
                P.error = (i, exc)
                break
            P.lines.append(line)
            P.host_of.append(host)
            disp.append(d)
            rows.append(row)
            ts_str.append(ts)
        if P.error:
            break
    n = len(P.lines)
    P.n = n
    P.disposition = np.array(disp, dtype=np.uint8)
    P.tuples = np.zeros(n, dtype=TUPLE_DTYPE)
    if n:
        arr = np.array(rows, dtype=np.int64)
        for j, name in enumerate(TUPLE_DTYPE.names):
            P.tuples[name] = arr[:, j]
    # order-isomorphic timestamp codes
    distinct = sorted({s for s in ts_str if s is not None})
    code = {s: k for k, s in enumerate(distinct)}
    P.ts_table = distinct
    P.ts = np.array([code[s] if s is not None else 0 for s in ts_str], dtype=np.uint32)
    # order key = rank of the line bytes (sort's order within one key group)
    P.order = np.empty(n, dtype=np.uint64)
    if need_order:
        keys = [l[:-1] if l.endswith('\n') else l for l in P.lines]
        perm = sorted(range(n), key=keys.__getitem__)
        P.order[np.array(perm, dtype=np.int64)] = np.arange(n, dtype=np.uint64)
    else:
        P.order[:] = np.arange(n, dtype=np.uint64)
    P.pspell_table = [s for s, _ in sorted(pspell.items(), key=lambda kv: kv[1])]
    return P


def _parse_one(line, host, fw, acls, compiled, pspell, P, i):
    zero = (0, 0, 0, 0, 0, 0, 0)
    d = get_builtconn(line)
    if not d:
        return zero, D_IGNORE, None
    proto = d['protocol'].lower()
    # Connection(...) -> FirewallRule.__init__ validation (firewallrule.py:47-93)
    sport, dport = py2_int(d['sport']), py2_int(d['dport'])
    if not py2_is_int(sport) or not py2_is_int(dport):         # a Python 2 long (firewallrule.py:67-75)
        raise ValueError('Source port must be an integer or -1 for "No port"')
    src_ip = FirewallRule._address(d['src'], 'src')
    dst_ip = FirewallRule._address(d['dst'], 'dst')
    ifc = d['interface_in']
    if ifc not in fw:
        return zero, D_NOACL, None
    acl = fw[ifc]['in']
    if acl not in acls:
        P.acl_of[i] = acl
        return zero, D_MISSING, None
    lid = compiled.list_id(host, acl, proto)
    if src_ip._ipversion != 4 or dst_ip._ipversion != 4 or src_ip._prefixlen != 32 or dst_ip._prefixlen != 32:
        raise NotImplementedError('only IPv4 host addresses are supported in connection tuples: %r' % line)
    if sport > 65535 or dport > 65535:
        # int() of the log's digits is never range-checked: such a side matches
        # only rule sides that are NO_PORT or name the value (compile.list_id_oor)
        lid = compiled.list_id_oor(host, acl, proto, sport if sport > 65535 else None,
                                   dport if dport > 65535 else None)
        sport, dport = sport if sport <= 65535 else 0, dport if dport <= 65535 else 0
    flags = F_VALID
    stripped = line.strip(PY2_WS)
    hit, res = reducer_fields(stripped)
    ts = None
    ps = 0
    if hit:
        flags |= F_HIT
    if res is not None:
        flags |= F_BUILT
        for_ip, to_ip, to_port = res[6], res[8], res[9]
        if hit:
            try:
                ts = reducer_timestamp(res)
            except ValueError as exc:
                # months.index fails: decided after aggregation (parse_logs)
                P.bad_month[i] = exc
                return (src_ip.ip, dst_ip.ip, sport, dport, lid, flags & ~F_BUILT, 0), D_CLASSIFY, None
        word = res[5]
        if word not in pspell and len(pspell) < MAX_SPELL_ID:
            pspell[word] = len(pspell)
        ps = pspell.get(word)
        # the reducer keys its dict by the strings (connlist-reducer.py:167):
        # canonical text that names the tuple's own fields is carried as the
        # tuple's values, anything else as interned text
        if (for_ip, to_ip, to_port) == (d['src'], d['dst'], d['dport']):
            pass
        elif (for_ip, to_ip, to_port) == (d['dst'], d['src'], d['sport']):
            flags |= F_SWAP
        else:
            for_ip = None
        if ps is None or for_ip is None or not _canonical_key(for_ip, to_ip, to_port):
            P.keyx[i] = P.keytext((word, res[6], res[8], res[9]))
            ps = 0
    return (src_ip.ip, dst_ip.ip, sport, dport, lid, flags, ps), D_CLASSIFY, ts


def _canonical_key(for_ip, to_ip, to_port):
    try:
        return _canonical_v4(for_ip) is not None and _canonical_v4(to_ip) is not None and \
            str(int(to_port)) == to_port and int(to_port) <= 65535
    except ValueError:
        return False


def key_tuples(torch, tuples, keyx):
    """The aggregation tuples (int32 [n, 4] tensor) of classified lines: rows
    of lines with interned keys (``keyx``: line -> KeyText id) carry the id in
    place of the connection (src = id, dst = sport = dport = 0, pspell =
    INTERNED, no swap) -- what the device aggregates given the gids.  Returns
    ``tuples`` itself when there are none."""
    if not keyx:
        return tuples
    idx = np.fromiter(keyx.keys(), np.int64, len(keyx))
    rows = np.zeros(len(idx), TUPLE_DTYPE)
    old = tuples[torch.from_numpy(idx).to(tuples.device)].cpu().numpy().view(TUPLE_DTYPE).reshape(-1)
    rows['src'] = np.fromiter(keyx.values(), np.int64, len(keyx))
    rows['list'] = old['list']
    rows['flags'] = old['flags'] & np.uint8(0xFF ^ F_SWAP)
    rows['pspell'] = INTERNED
    out = tuples.clone()
    out[torch.from_numpy(idx).to(tuples.device)] = torch.from_numpy(rows.view(np.int32).reshape(-1, 4)).to(
        tuples.device)
    return out
