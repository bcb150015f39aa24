"""ORACLE (test infrastructure only) — Python harness around ``rsa_oracle.c``.

Builds the C oracle (``gcc`` into ``oracle/_build/``), lowers a rule DB (the
JSON form) with this oracle's own ``IP``/``FirewallRule`` restatements, builds
candidate lists the way ``mapper.py:159-166`` does, derives per-line inputs
either from log text (``oracle.fwregex`` + the reducer's BUILT regex) or from a
synthetic traffic dict, and runs classify + reduce.  Results are plain numpy
arrays keyed by gid, with gids assigned exactly as the product does (sorted
host, sorted acl, list position) so results compare index for index.
"""

import ctypes
import os
import re
import subprocess

import numpy as np

from .firewallrule import FirewallRule
from .fwregex import get_builtconn

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, '_build')
LIB = os.path.join(BUILD, 'librsa_oracle.so')
SRC = os.path.join(HERE, 'rsa_oracle.c')

_lib = None


def build():
    os.makedirs(BUILD, exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.run(['gcc', '-O2', '-fopenmp', '-shared', '-fPIC', '-o', LIB, SRC], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.rsa_oracle_reduce.restype = ctypes.c_int64
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


PROTO_ID = {'ip': 0, 'tcp': 1, 'udp': 2}


class OracleRules(object):
    def __init__(self, dbj):
        self.dbj = dbj
        self.groups = []
        self.base = {}
        rules = []
        for host in sorted(dbj['accesslists']):
            for acl in sorted(dbj['accesslists'][host]):
                self.base[(host, acl)] = len(rules)
                self.groups.append((host, acl))
                for r in dbj['accesslists'][host][acl]['rules']:
                    rules.append(FirewallRule(r['action'], r['protocol'], r['original'], r['src'], r['dst'],
                                              list(r['sport']), list(r['dport'])))
        self.rules = rules
        n = len(rules)
        self.n_rules = n
        self.action = np.array([1 if r.action == True else 0 for r in rules], np.uint8)  # noqa: E712
        self.proto_names = dict(PROTO_ID)
        self.proto = np.array([self._pid(r.protocol) for r in rules], np.uint8)
        self.v4src = np.array([1 if r.src._ipversion == 4 else 0 for r in rules], np.uint8)
        self.v4dst = np.array([1 if r.dst._ipversion == 4 else 0 for r in rules], np.uint8)
        self.src = np.array([r.src.ip if r.src._ipversion == 4 else 0 for r in rules], np.uint32)
        self.dst = np.array([r.dst.ip if r.dst._ipversion == 4 else 0 for r in rules], np.uint32)
        self.src_len = np.array([r.src.len() if r.src._ipversion == 4 else 0 for r in rules], np.uint64)
        self.dst_len = np.array([r.dst.len() if r.dst._ipversion == 4 else 0 for r in rules], np.uint64)
        self.src6 = np.array([_words6(r.src) for r in rules], np.uint64).reshape(-1)
        self.dst6 = np.array([_words6(r.dst) for r in rules], np.uint64).reshape(-1)
        ports, sp_off, sp_len, dp_off, dp_len = [], [], [], [], []
        for r in rules:
            sp_off.append(len(ports)); sp_len.append(len(r.sport)); ports.extend(r.sport)
            dp_off.append(len(ports)); dp_len.append(len(r.dport)); ports.extend(r.dport)
        self.ports = np.array(ports or [0], np.int32)
        self.sp_off = np.array(sp_off, np.uint32); self.sp_len = np.array(sp_len, np.uint32)
        self.dp_off = np.array(dp_off, np.uint32); self.dp_len = np.array(dp_len, np.uint32)
        self.lists = {}
        self.cand = []

    @classmethod
    def from_fortigate(cls, text):
        """Rules of a FortiGate config expanded by oracle.fortigate (the
        restated preprocessor), as the arrays the C oracle scans."""
        from . import fortigate
        host, firewalls, acls = fortigate.expand(text)
        self = cls.__new__(cls)
        self.groups, self.base = [], {}
        self.proto_names = dict(PROTO_ID)
        parts = []
        n = 0
        for acl in sorted(acls):
            self.base[(host, acl)] = n
            self.groups.append((host, acl))
            c = fortigate.as_columns(acls[acl])
            parts.append(c)
            n += len(c['action'])
        self.n_rules = n
        self.dbj = {'firewalls': firewalls,
                    'accesslists': {host: {acl: {'protocols': acls[acl].protocols} for acl in acls}}}
        cat = lambda k, dt: np.concatenate([p[k] for p in parts]).astype(dt) if parts else np.zeros(0, dt)
        self.action = cat('action', np.uint8)
        self.proto = np.array([self._pid(x) for p in parts for x in p['proto']], np.uint8)
        self.v4src = np.ones(n, np.uint8)
        self.v4dst = np.ones(n, np.uint8)
        self.src6 = self.dst6 = np.zeros(4 * n + 4, np.uint64)
        self.src, self.dst = cat('src', np.uint32), cat('dst', np.uint32)
        self.src_len, self.dst_len = cat('src_len', np.uint64), cat('dst_len', np.uint64)
        ports = np.empty(2 * n, np.int32)
        ports[0::2] = cat('sport', np.int32)
        ports[1::2] = cat('dport', np.int32)
        self.ports = ports if n else np.zeros(1, np.int32)
        self.sp_off = (2 * np.arange(n)).astype(np.uint32)
        self.dp_off = self.sp_off + 1
        self.sp_len = np.ones(n, np.uint32)
        self.dp_len = np.ones(n, np.uint32)
        self.rules = None
        self.lists = {}
        self.cand = []
        self.host = host
        return self

    def _pid(self, name):
        if name not in self.proto_names:
            self.proto_names[name] = len(self.proto_names)
        return self.proto_names[name]

    def list_id(self, host, acl, proto):
        """mapper.py:159-166 candidate list, as gids."""
        k = (host, acl, proto)
        if k not in self.lists:
            protos = self.dbj['accesslists'][host][acl]['protocols']
            if proto in ('tcp', 'udp'):
                idx = sorted(protos[proto] + protos['ip']) if proto in protos else protos['ip']
            else:
                idx = protos[proto]
            self.lists[k] = len(self.cand)
            self.cand.append([self.base[(host, acl)] + i for i in idx])
        return self.lists[k]

    def key(self, gid):
        for (host, acl) in reversed(self.groups):
            if gid >= self.base[(host, acl)]:
                return '%s;%s;%d' % (host, acl, gid - self.base[(host, acl)])
        raise KeyError(gid)


def classify(R, list_of, proto_of, src, dst, sport, dport):
    n = len(list_of)
    off = np.zeros(len(R.cand) + 1, np.uint32)
    for i, c in enumerate(R.cand):
        off[i + 1] = off[i] + len(c)
    cand = np.array([g for c in R.cand for g in c] or [0], np.uint32)
    gid = np.empty(n, np.int32)
    evals = ctypes.c_uint64(0)
    arrs = [np.ascontiguousarray(list_of, np.int32), np.ascontiguousarray(proto_of, np.uint32),
            np.ascontiguousarray(src, np.uint32), np.ascontiguousarray(dst, np.uint32),
            np.ascontiguousarray(sport, np.uint32), np.ascontiguousarray(dport, np.uint32)]
    lib().rsa_oracle_classify(ctypes.c_uint64(n), *[_p(a) for a in arrs], _p(off), _p(cand), _p(R.action),
                              _p(R.proto), _p(R.v4src), _p(R.v4dst), _p(R.src), _p(R.dst), _p(R.src_len),
                              _p(R.dst_len), _p(R.sp_off), _p(R.sp_len), _p(R.dp_off), _p(R.dp_len), _p(R.ports),
                              _p(gid), ctypes.byref(evals))
    return gid, int(evals.value)


def _words6(ip):
    """An IPv6 network as (ip hi, ip lo, last hi, last lo) uint64 words; zeros
    for an IPv4 one (the C oracle reads them only for IPv6 sides)."""
    if ip._ipversion == 4:
        return (0, 0, 0, 0)
    a, b = int(ip.ip), int(ip.ip) + ip.len() - 1
    m = (1 << 64) - 1
    return (a >> 64, a & m, b >> 64, b & m)


def shadow(R, host, acl):
    """preprosess_access_lists.py:508-521 for one ACL: per rule the first rule
    above it that contains it (list-local index) or -1."""
    beg = R.base[(host, acl)]
    ends = sorted(b for b in R.base.values() if b > beg)
    end = ends[0] if ends else R.n_rules
    cover = np.empty(end - beg, np.int32)
    lib().rsa_oracle_shadow(ctypes.c_uint32(beg), ctypes.c_uint32(end), _p(R.action), _p(R.proto), _p(R.v4src),
                            _p(R.v4dst), _p(R.src), _p(R.dst), _p(R.src_len), _p(R.dst_len), _p(R.sp_off),
                            _p(R.sp_len), _p(R.dp_off), _p(R.dp_len), _p(R.ports), _p(R.src6), _p(R.dst6),
                            _p(cover))
    return cover


def reduce(R, gid, flags, pspell, src, dst, sport, dport, ts, order, cap):
    n = len(gid)
    nr = R.n_rules
    matches = np.zeros(nr, np.uint64); hits = np.zeros(nr, np.uint64); nconn = np.zeros(nr, np.uint32)
    max_rows = int(min(n, nr * (cap + 1))) + 1
    cols = [np.zeros(max_rows, np.uint32) for _ in range(8)]
    arrs = [np.ascontiguousarray(gid, np.int32), np.ascontiguousarray(flags, np.uint8),
            np.ascontiguousarray(pspell, np.uint8), np.ascontiguousarray(src, np.uint32),
            np.ascontiguousarray(dst, np.uint32), np.ascontiguousarray(sport, np.uint32),
            np.ascontiguousarray(dport, np.uint32), np.ascontiguousarray(ts, np.uint32),
            np.ascontiguousarray(order, np.uint64)]
    rows = lib().rsa_oracle_reduce(ctypes.c_uint64(n), ctypes.c_uint32(nr), *[_p(a) for a in arrs],
                                   ctypes.c_uint32(cap), _p(matches), _p(hits), _p(nconn), *[_p(c) for c in cols],
                                   ctypes.c_uint64(max_rows))
    assert rows >= 0
    names = ['gid', 'for_ip', 'to_ip', 'to_port', 'pspell', 'count', 'first', 'last']
    table = {k: c[:rows].copy() for k, c in zip(names, cols)}
    return {'matches': matches, 'hits': hits, 'n_conns': nconn, 'rows': table}


# ---- inputs ---------------------------------------------------------------------
F_HIT, F_BUILT, F_SWAP = 2, 4, 8
_BUILT = re.compile(r'[a-zA-Z]+ [0-9 ]?[0-9] ([0-9:]+) ([a-zA-Z]+) ([0-9]+) ([0-9]+) .* Built (out|in)bound '
                    r'([a-zA-Z]+) .* for [a-zA-Z0-9_-]+:([0-9.]+)/([0-9]+) .* to [a-zA-Z0-9_-]+:([0-9.]+)/([0-9]+)')
_MON = ['Jan', 'Feb', 'Mar', 'Apr', 'May', 'Jun', 'Jul', 'Aug', 'Sep', 'Oct', 'Nov', 'Dec']


def _v4(s):
    a = [int(x) for x in s.split('.')]
    return (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]


def inputs_from_text(R, host, lines):
    """Per-line oracle inputs from log text (lines keep their '\\n').

    Spellings and timestamps are returned as strings (pspell id = index into
    ``spell``; ts = index into sorted distinct strings, order-preserving)."""
    fw = R.dbj['firewalls'][host]
    acls = R.dbj['accesslists'][host]
    n = len(lines)
    cols = {k: np.zeros(n, np.int64) for k in ('list', 'proto', 'src', 'dst', 'sport', 'dport', 'flags', 'pspell')}
    cols['list'][:] = -1
    ts_s = [None] * n
    spell = []
    for i, line in enumerate(lines):
        d = get_builtconn(line)
        if not d or d['interface_in'] not in fw:
            continue
        acl = fw[d['interface_in']]['in']
        if acl not in acls:
            continue
        p = d['protocol'].lower()
        cols['list'][i] = R.list_id(host, acl, p)
        cols['proto'][i] = R._pid(p)
        cols['src'][i], cols['dst'][i] = _v4(d['src']), _v4(d['dst'])
        cols['sport'][i], cols['dport'][i] = int(d['sport']), int(d['dport'])
        v = line.strip(' \t\n\r\x0b\x0c')
        f = F_HIT if (v.find('-6-302013') != -1 or v.find('-6-302015') != -1) else 0
        m = _BUILT.search(v)
        if m:
            res = m.groups()
            f |= F_BUILT
            if (res[6], res[8], res[9]) != (d['src'], d['dst'], d['dport']):
                f |= F_SWAP
            if res[5] not in spell:
                spell.append(res[5])
            cols['pspell'][i] = spell.index(res[5])
            ts_s[i] = res[3] + '-' + str(_MON.index(res[1]) + 1).zfill(2) + '-' + res[2].zfill(2) + ' ' + res[0]
        cols['flags'][i] = f
    distinct = sorted({s for s in ts_s if s is not None})
    code = {s: k for k, s in enumerate(distinct)}
    ts = np.array([code.get(s, 0) for s in ts_s], np.uint32)
    keys = [l[:-1] if l.endswith('\n') else l for l in lines]
    order = np.empty(n, np.uint64)
    order[np.array(sorted(range(n), key=keys.__getitem__), dtype=np.int64)] = np.arange(n, dtype=np.uint64)
    return cols, ts, order, distinct, spell


def inputs_from_traffic(R, tr):
    """Per-line oracle inputs straight from a synth traffic dict (the meaning of
    each synthetic message form, DESIGN.md §Synthetic workload)."""
    F_BUILT_FORM, F_NONHIT, F_NOYEAR, F_TEARDOWN, F_NOACL, F_OUTBOUND = range(6)
    form = tr['form']
    n = len(form)
    host = tr['host']
    names = ('tcp', 'udp')
    lst = np.full(n, -1, np.int64)
    acl_of = tr.get('acl_of') or ['%s_access_in' % ifc for ifc in tr['interfaces']]
    for p in (0, 1):
        for k, ifc in enumerate(tr['interfaces']):
            w = np.isin(form, [F_BUILT_FORM, F_NONHIT, F_NOYEAR]) & (tr['ifc'] == k) & (tr['proto'] == p)
            if w.any():
                lst[w] = R.list_id(host, acl_of[k], names[p])
        w = (form == F_OUTBOUND) & (tr['proto'] == p)
        if w.any():
            lst[w] = R.list_id(host, tr.get('inside_acl', 'inside_access_in'), names[p])
    proto = np.where(tr['proto'] == 0, PROTO_ID['tcp'], PROTO_ID['udp'])
    flags = (np.where(np.isin(form, [F_BUILT_FORM, F_NOYEAR, F_OUTBOUND]), F_HIT, 0)
             | np.where(np.isin(form, [F_BUILT_FORM, F_NONHIT, F_OUTBOUND]), F_BUILT, 0)
             | np.where(form == F_OUTBOUND, F_SWAP, 0))
    t = tr['t'].astype(np.uint64)
    order = ((t << np.uint64(36)) | (tr['proto'].astype(np.uint64) << np.uint64(35))
             | ((form == F_OUTBOUND).astype(np.uint64) << np.uint64(34)) | tr['cid'].astype(np.uint64))
    cols = {'list': lst, 'proto': proto, 'src': tr['src'], 'dst': tr['dst'], 'sport': tr['sport'],
            'dport': tr['dport'], 'flags': flags, 'pspell': tr['proto']}
    return cols, tr['t'].astype(np.uint32), order


def run(R, cols, ts, order, cap):
    gid, evals = classify(R, cols['list'], cols['proto'], cols['src'], cols['dst'], cols['sport'], cols['dport'])
    res = reduce(R, gid, cols['flags'], cols['pspell'], cols['src'], cols['dst'], cols['sport'], cols['dport'], ts,
                 order, cap)
    res['gid'] = gid
    res['evals'] = evals
    return res
