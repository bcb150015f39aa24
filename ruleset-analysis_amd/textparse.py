"""Log text -> packed inputs on the GPU.

The host side of ``rsa_text_count_lines`` / ``rsa_text_line_offsets`` /
``rsa_parse_text`` / ``rsa_order_keys`` (``csrc/textparse.hip``): one
firewall's log bytes go to HBM once; the device splits lines, parses each one
(the mapper's ``get_builtconn`` + ACL resolution, ``mapper.py:123-166``, and the
reducer's hit test / BUILT regex / key / timestamp, ``connlist-reducer.py:146-165``)
and ranks the lines' bytes for the order keys (the ``LC_ALL=C sort`` between
the phases, ``runAnalysis.sh:42-56``).  The result is what ``logparse.parse_logs``
produces, without a Python loop over the lines.

Lines outside the device grammar come back as ``LINE_HOST`` and are decided
by the host parser (``logparse._parse_one``) in line order — so a line the
reference would die on raises the same exception here, at the same line.
Timestamps are fixed-width codes (``ts_pack``; years 2000-2127).
"""

import ctypes
import warnings

import numpy as np

from . import logparse
from .compile import F_BUILT, F_HIT, TUPLE_DTYPE
from .keytext import KeyText

__all__ = ['IFC_DTYPE', 'SPELL_DTYPE', 'LINE_IGNORE', 'LINE_NOACL', 'LINE_MISSING', 'LINE_CLASSIFY', 'LINE_HOST',
           'DEFAULT_SPELLS', 'ts_pack', 'ts_unpack', 'interface_table', 'spell_table', 'ParsedText', 'parse_text',
           'concat']

LINE_IGNORE, LINE_NOACL, LINE_MISSING, LINE_CLASSIFY, LINE_HOST = 0, 1, 2, 3, 4
assert (LINE_IGNORE, LINE_NOACL, LINE_MISSING, LINE_CLASSIFY) == (logparse.D_IGNORE, logparse.D_NOACL,
                                                                   logparse.D_MISSING, logparse.D_CLASSIFY)
LIST_HOST = 0xFFFF
IFC_NAME_MAX = 47
TS_YEAR0 = 2000
DEFAULT_SPELLS = ('TCP', 'UDP')

IFC_DTYPE = np.dtype([('name', 'S48'), ('len', '<u4'), ('kind', '<u4'), ('list_tcp', '<u2'), ('list_udp', '<u2'),
                      ('reserved', '<u4')])
SPELL_DTYPE = np.dtype([('word', 'S15'), ('len', 'u1')])
assert IFC_DTYPE.itemsize == 64 and SPELL_DTYPE.itemsize == 16

_MONTH = {m: k for k, m in enumerate(logparse._MONTHS)}


def ts_pack(s):
    """Code of a reducer timestamp string 'YYYY-MM-DD HH:MM:SS' (the order of
    the strings), or None outside the code range (include/ruleset_hip.h)."""
    if len(s) != 19 or s[4] != '-' or s[7] != '-' or s[10] != ' ' or s[13] != ':' or s[16] != ':':
        return None
    parts = (s[0:4], s[5:7], s[8:10], s[11:13], s[14:16], s[17:19])
    if not all(p.isascii() and p.isdigit() for p in parts):
        return None
    y, mo, d, h, mi, se = (int(p) for p in parts)
    if not (TS_YEAR0 <= y < TS_YEAR0 + 128 and 1 <= mo <= 12 and d <= 31 and h <= 23 and mi <= 59 and se <= 59):
        return None
    return ((((y - TS_YEAR0) * 12 + mo - 1) * 32 + d) * 86400) + h * 3600 + mi * 60 + se


def ts_unpack(code):
    code = int(code)
    day_code, sec = divmod(code, 86400)
    ym, d = divmod(day_code, 32)
    y, mo = divmod(ym, 12)
    return '%04d-%02d-%02d %02d:%02d:%02d' % (y + TS_YEAR0, mo + 1, d, sec // 3600, (sec // 60) % 60, sec % 60)


def interface_table(db, compiled, host):
    """rsa_parse_ifc rows for one firewall and the ACL name of each row.
    Creates the (acl, tcp/udp) candidate lists the lines can need."""
    fw = db.firewalls[host]
    acls = db.accesslists[host]
    rows, names = [], []
    for ifc in fw:
        raw = ifc.encode('latin-1') if isinstance(ifc, str) else None
        if raw is None or not 0 < len(raw) <= IFC_NAME_MAX:
            continue            # such a line is decided by the host parser
        row = np.zeros((), IFC_DTYPE)
        row['name'] = raw
        row['len'] = len(raw)
        row['list_tcp'] = row['list_udp'] = LIST_HOST
        acl = None
        try:
            acl = fw[ifc]['in']
        except (KeyError, TypeError, IndexError):
            row['kind'] = LINE_HOST
        if acl is not None:
            if acl not in acls:
                row['kind'] = LINE_MISSING
            else:
                row['kind'] = LINE_CLASSIFY
                for field, proto in (('list_tcp', 'tcp'), ('list_udp', 'udp')):
                    try:
                        lid = compiled.list_id(host, acl, proto)
                    except KeyError:
                        continue
                    if lid < LIST_HOST:
                        row[field] = lid
        rows.append(row)
        names.append(acl)
    return np.array(rows, IFC_DTYPE), names


def spell_table(spells):
    """rsa_parse_spell rows, row k = spelling id k (at most 64; a spelling
    longer than 15 bytes gets an empty row the device never matches)."""
    out = np.zeros(min(len(spells), 64), SPELL_DTYPE)
    for k, w in enumerate(spells[:64]):
        raw = w.encode('latin-1')
        if 0 < len(raw) <= 15:
            out[k]['word'] = raw
            out[k]['len'] = len(raw)
    return out


class _Lines(object):
    """Lazy view of the lines (str, latin-1, with their '\\n')."""

    def __init__(self, data, off):
        self.data, self.off = data, off

    def __len__(self):
        return len(self.off) - 1

    def __getitem__(self, i):
        return self.data[int(self.off[i]):int(self.off[i + 1])].decode('latin-1')


class _HostOf(object):
    def __init__(self, starts, hosts):
        self.starts, self.hosts = np.asarray(starts, np.int64), hosts

    def __getitem__(self, i):
        return self.hosts[int(np.searchsorted(self.starts, i, side='right')) - 1]


def _hb_mask(torch, tuples, kind):
    """Lines with a reducer timestamp: CLASSIFY, hit and BUILT (numpy bool)."""
    if not len(kind):
        return np.zeros(0, bool)
    fl = ((tuples[:, 3] >> 16) & 0xFF).cpu().numpy()
    both = F_HIT | F_BUILT
    return (kind == LINE_CLASSIFY) & ((fl & both) == both)


def _retable(parts, P):
    """Switch timestamps to dense ranks of the distinct strings (what
    logparse does) when a string falls outside the code range: parts =
    [(ts tensor, hb mask, decode, {line: string} overrides)], rewritten in place;
    P.ts_decode / ts_table follow."""
    strs = set()
    per = []
    for ts, hb, decode, extra in parts:
        h = ts.cpu().numpy().view(np.uint32)
        use = hb.copy()
        for i in extra:
            use[i] = False
        u, inv = np.unique(h[use], return_inverse=True)
        us = [decode(c) for c in u]
        strs.update(us)
        strs.update(extra.values())
        per.append((ts, h, use, us, inv, extra))
    table = sorted(strs)
    rank = {t: k for k, t in enumerate(table)}
    for ts, h, use, us, inv, extra in per:
        out = h.copy()
        if len(us):
            out[use] = np.array([rank[t] for t in us], np.uint32)[inv]
        for i, t in extra.items():
            out[i] = rank[t]
        ts.copy_(ts.new_tensor(out.view(np.int32)))
    P.ts_table = table
    P.ts_decode = table.__getitem__


class ParsedText(object):
    """What logparse.ParsedLog holds, with the packed arrays left in HBM:
    ``tuples`` (int32 [n, 4]), ``ts`` (int32), ``order`` (int64) torch tensors."""

    def __init__(self):
        self.n = 0
        self.disposition = np.zeros(0, np.uint8)
        self.acl_of = {}
        self.nl = np.zeros(0, bool)
        self.lines = _Lines(b'', np.zeros(1, np.uint64))
        self.host_of = _HostOf([0], [None])
        self.tuples = self.ts = self.order = None
        self.pspell_table = list(DEFAULT_SPELLS)
        self.ts_decode = ts_unpack   # packed codes (ts_table None), or dense ranks of ts_table
        self.ts_table = None
        self.error = None
        self.n_host = 0               # lines the host parser decided
        self.keytext = None           # keytext.KeyText of interned reducer keys (host-parsed lines)
        self.keyx = {}                # line -> KeyText id of its interned key (logparse._parse_one)
        self.bad_month = {}           # line -> ValueError of months.index (logparse.parse_logs)
        self._d_text = self._d_off = None   # device text / line offsets (parse_text keep_text=True)

    def batch(self):
        from .engine import DeviceBatch
        return DeviceBatch(self.tuples, self.ts, self.order)


def split_lines_device(ctx, torch, text, n_bytes, hint=None):
    """Line start offsets of device text in one pass (``rsa_text_split``):
    (off tensor of n + 1 int64, n).  The offset buffer is sized from ``hint``
    (an expected line count) or one line per 48 bytes; when the text holds more
    lines, the library reports the count and the split runs again into a buffer
    of that size."""
    from .native import NativeError, RSA_ERR_CAPACITY
    v = lambda t: ctypes.c_void_p(t.data_ptr())
    cap = int(hint) if hint is not None else n_bytes // 48 + 16
    nl = ctypes.c_uint64(0)
    for _ in range(2):
        off = torch.empty(cap + 1, dtype=torch.int64, device=text.device)
        try:
            ctx.call('rsa_text_split', v(text), ctypes.c_uint64(n_bytes), v(off), ctypes.c_uint64(cap), ctypes.byref(nl))
            n = int(nl.value)
            return off[:n + 1], n
        except NativeError as e:
            if e.code != RSA_ERR_CAPACITY or int(nl.value) <= cap:
                raise
            cap = int(nl.value)
    raise RuntimeError('rsa_text_split: line count changed between passes')


def _device_bytes(torch, data, device):
    t = torch.empty(len(data), dtype=torch.uint8, device=device)
    if len(data):
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')          # read-only source buffer: copied, never written
            t.copy_(torch.frombuffer(memoryview(data), dtype=torch.uint8))
    return t


def parse_text(engine, host, data, db, compiled, pspell=None, order_base=0, need_order=True, keep_text=False,
               keytext=None):
    """Parse one firewall's log bytes on the GPU.  ``pspell``: the spelling ->
    id dict shared across calls (ids of new spellings are appended);
    ``keytext``: the KeyText of non-canonical reducer keys, likewise shared.
    ``keep_text``: keep the device text and line offsets on the result
    (``_d_text``/``_d_off``) for ``order_keys_global`` over several inputs."""
    torch = engine.torch
    ctx = engine.ctx
    P = ParsedText()
    P.keytext = keytext if keytext is not None else KeyText()
    if pspell is None:
        pspell = {}
    for w in DEFAULT_SPELLS:
        pspell.setdefault(w, len(pspell))
    spells = [w for w, _ in sorted(pspell.items(), key=lambda kv: kv[1])]
    if host not in db.firewalls or host not in db.accesslists:
        P.error = (0, SystemExit('Firewall {0} not present in data structure. Aborting.'.format(host)))
        P.pspell_table = spells
        return P
    dev = engine.device
    text = _device_bytes(torch, data, dev)
    v = lambda t: ctypes.c_void_p(t.data_ptr())
    off, n = split_lines_device(ctx, torch, text, len(data))
    n_all = n       # (n may end at a line the mapper dies on, below)
    ifcs, acl_names = interface_table(db, compiled, host)
    sp = spell_table(spells)
    tuples = torch.zeros((max(n, 1), 4), dtype=torch.int32, device=dev)[:n]
    ts = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)[:n]
    disp = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)[:n]
    order = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
    if n:
        ctx.call('rsa_parse_text', v(text), v(off), ctypes.c_uint64(n), ifcs.ctypes.data_as(ctypes.c_void_p),
                 ctypes.c_uint32(len(ifcs)), sp.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(sp)),
                 v(tuples), v(ts), v(disp))
        if need_order:
            ctx.call('rsa_order_keys', v(text), v(off), ctypes.c_uint64(n), ctypes.c_uint64(order_base), v(order))
        else:
            order.copy_(torch.arange(order_base, order_base + n, dtype=torch.int64, device=dev))
    h_off = off.cpu().numpy().view(np.uint64)
    h_disp = disp.cpu().numpy().view(np.uint32)
    kind = (h_disp & 0xFF).astype(np.uint8)
    P.lines = _Lines(data, h_off)
    P.host_of = _HostOf([0], [host])
    for i in np.nonzero(kind == LINE_MISSING)[0]:
        P.acl_of[int(i)] = acl_names[int(h_disp[i] >> 8)]
    # lines outside the device grammar: the host parser, in line order
    hosts_idx = np.nonzero(kind == LINE_HOST)[0]
    P.n_host = len(hosts_idx)
    if len(hosts_idx):
        fw, acls = db.firewalls[host], db.accesslists[host]
        rows = np.zeros(len(hosts_idx), TUPLE_DTYPE)
        tcodes = np.zeros(len(hosts_idx), np.uint32)
        odd_ts = {}                   # line -> reducer timestamp string outside the code range
        keep = len(hosts_idx)
        for j, i in enumerate(hosts_idx):
            i = int(i)
            line = P.lines[i]
            try:
                row, d, ts_str = logparse._parse_one(line, host, fw, acls, compiled, pspell, P, i)
            except (KeyError, ValueError) as exc:
                P.error = (i, exc)
                keep = j
                n = i
                break
            kind[i] = d
            if d == LINE_CLASSIFY:
                rows[j] = row
                if ts_str is not None:
                    code = ts_pack(ts_str)
                    if code is None:
                        odd_ts[i] = ts_str
                    else:
                        tcodes[j] = code
        if keep:
            idx = torch.from_numpy(hosts_idx[:keep].astype(np.int64)).to(dev)
            tuples[idx] = torch.from_numpy(rows[:keep].view(np.int32).reshape(-1, 4)).to(dev)
            ts[idx] = torch.from_numpy(tcodes[:keep].view(np.int32)).to(dev)
        if odd_ts:
            _retable([(ts[:n], _hb_mask(torch, tuples[:n], kind[:n]), ts_unpack, {i: t for i, t in odd_ts.items()
                                                                              if i < n})], P)
    P.n = n
    P.disposition = kind[:n]
    P.acl_of = {i: a for i, a in P.acl_of.items() if i < n}
    P.keyx = {i: k for i, k in P.keyx.items() if i < n}
    P.bad_month = {i: e for i, e in P.bad_month.items() if i < n}
    P.nl = np.zeros(n, bool)
    if n:
        P.nl[:] = True
        if not data.endswith(b'\n') and n == n_all:
            P.nl[-1] = False
    P.tuples, P.ts, P.order = tuples[:n], ts[:n], order[:n]
    if keep_text:
        P._d_text, P._d_off = text, off
    P.pspell_table = [w for w, _ in sorted(pspell.items(), key=lambda kv: kv[1])]
    return P


def order_keys_global(engine, parts, group=None):
    """Order keys of all lines of several inputs ranked together: the
    reference's ``cat f1 f2 ... | mapper | LC_ALL=C sort`` (or Hadoop's shuffle
    sort over every split, ``runAnalysis.sh:42-56``) orders a key group's lines
    by their bytes across all inputs, and the cap freeze follows that order
    (``connlist-reducer.py:151``).  ``parts``: ParsedText from ``parse_text(...,
    keep_text=True)``; each part's ``order`` is replaced by its lines' global
    ranks (lines past a part's error are left out), the device text released.
    ``group`` (int32 tensor over the parts' lines, in order): rank within
    groups (``rsa_order_keys_grouped``) -- with each line's rule as its group
    (-1: a line the reducer never orders) the keys are what the reducer
    compares, and lines of different rules are never compared."""
    torch = engine.torch
    live = [p for p in parts if p.n and p._d_text is not None]
    if live:
        dev = engine.device
        texts, offs, shift = [], [], 0
        for p in live:
            texts.append(p._d_text)
            offs.append(p._d_off[:p.n] + shift)
            shift += p._d_text.numel()
        offs.append(torch.tensor([shift], dtype=torch.int64, device=dev))
        text = torch.cat(texts) if len(texts) > 1 else texts[0]
        off = torch.cat(offs)
        total = int(off.numel()) - 1
        order = torch.empty(total, dtype=torch.int64, device=dev)
        v = lambda t: ctypes.c_void_p(t.data_ptr())
        if group is None:
            engine.ctx.call('rsa_order_keys', v(text), v(off), ctypes.c_uint64(total), ctypes.c_uint64(0), v(order))
        else:
            g = group.to(torch.int32).contiguous()
            assert g.numel() == total
            engine.ctx.call('rsa_order_keys_grouped', v(text), v(off), ctypes.c_uint64(total), v(g),
                            ctypes.c_uint64(0), v(order))
        a = 0
        for p in live:
            p.order = order[a:a + p.n]
            a += p.n
        del text, off
    for p in parts:
        p._d_text = p._d_off = None


def concat(parts, torch):
    """One ParsedText over several hosts' ParsedText (line indices shifted);
    like parse_logs, nothing after the first error is kept."""
    if len(parts) == 1:
        return parts[0]
    P = ParsedText()
    starts, hosts, acl_of, keyx, bad = [], [], {}, {}, {}
    base = 0
    kept = []
    for p in parts:
        kept.append(p)
        starts.append(base)
        hosts.append(p.host_of.hosts[0])
        for i, a in p.acl_of.items():
            acl_of[base + i] = a
        for i, k in p.keyx.items():
            keyx[base + i] = k
        for i, e in p.bad_month.items():
            bad[base + i] = e
        if p.error is not None:
            P.error = (base + p.error[0], p.error[1])
            base += p.n
            break
        base += p.n
    datas = [p.lines.data for p in kept]
    off = [np.zeros(1, np.uint64)]
    shift = 0
    for p, d in zip(kept, datas):
        off.append(p.lines.off[1:p.n + 1] + np.uint64(shift))
        shift += len(d)
    P.lines = _Lines(b''.join(datas), np.concatenate(off))
    P.host_of = _HostOf(starts, hosts)
    P.acl_of = acl_of
    P.keyx = keyx
    P.bad_month = bad
    P.keytext = kept[0].keytext
    assert all(p.keytext is P.keytext for p in kept), 'parts parsed with different KeyText'
    P.n = base
    P.disposition = np.concatenate([p.disposition for p in kept])
    P.nl = np.concatenate([p.nl for p in kept])
    with_rows = [p for p in kept if p.tuples is not None]
    if with_rows:
        P.tuples = torch.cat([p.tuples for p in with_rows])
        P.ts = torch.cat([p.ts for p in with_rows])
        P.order = torch.cat([p.order for p in with_rows])
    P.pspell_table = kept[-1].pspell_table
    P.n_host = sum(p.n_host for p in kept)
    if any(p.ts_table is not None for p in with_rows):
        _retable([(p.ts, _hb_mask(torch, p.tuples, p.disposition), p.ts_decode, {}) for p in with_rows], P)
        P.ts = torch.cat([p.ts for p in with_rows])
    return P
