"""The reducer drop-in on the GPU, streaming (``connlist-reducer.py:62-211``).

Input: the sorted mapper stream (``host;acl;idx<TAB><log line>`` per line) on
stdin; output: the reference report, byte for byte.  Per chunk of whole lines
(``RSA_REDUCER_CHUNK`` bytes):

1. the bytes go to HBM once; the device splits the lines and parses each one
   (``rsa_parse_reduce``: strip, ``split('\\t', 1)``, the hit test and the
   BUILT regex on the value, key fields, timestamp code, and whether the key
   bytes equal the previous line's);
2. the host decides each *run* of equal keys once (``key.split(';', 3)``,
   ``int(ruleindex)``, the rule lookup, with the reference's ValueError noise
   and KeyError/IndexError death) and the lines the device left to it (text
   outside the device grammar, decided by ``logparse.reducer_fields`` exactly
   as the reference's regex does) -- no Python loop over the other lines;
3. the runs are aggregated on the GPU (``rsa_aggregate_gids``: run id as the
   rule, line order as the sort order, the cap freeze exact) and their blocks
   emitted.

The run still open at the end of a chunk is carried into the next one (its
block prints when the next key arrives, as in the reference), so memory stays
bounded by the chunk plus the longest run.  A line whose month the reducer's
``months.index`` rejects kills the reference only if it reaches that code
(hit, BUILT, the rule's dict not yet full): the line is checked against the
rule's cap threshold after aggregation, and the job is redone up to it.

Keys are the reducer's strings (``PROTO;FROMIP;TOIP;TOPORT``): canonical
dotted quads and ports are carried as values (one to one with their text);
a line whose address or port text is not canonical is parsed on the host and
its whole key text is interned (``pspell == 0x80`` marks such keys), so two
spellings of one address stay two connections, as in the reference.
"""

import ctypes

import numpy as np

from . import textparse
from .compile import F_BUILT, F_HIT, TUPLE_DTYPE
from .logparse import reducer_fields, reducer_timestamp, _canonical_v4
from .py2text import PY2_WS, py2_int
from .keytext import MAX_SPELL_ID
from .report import HEADER, INTERNED, NOISE1, KeyText, MemoDecode, _rows_by_gid, key_strings, table_rows

__all__ = ['ReducerStream']

RED_KEYED, RED_NOISE, RED_SAME = 0, 1, 0x100


class ReducerStream(object):
    """One reducer job over a byte stream: ``feed(bytes)`` as input arrives,
    ``finish()`` at EOF; report text goes to ``write`` as runs complete."""

    def __init__(self, engine, db, cap, write, chunk=64 << 20):
        self.eng, self.db, self.cap, self.write = engine, db, int(cap), write
        self.chunk = max(int(chunk), 1)
        self.pending = b''
        self.spells = list(textparse.DEFAULT_SPELLS)      # spelling ids (the device table holds the first 64)
        self.spell_ids = {w: k for k, w in enumerate(self.spells)}
        self.istr = KeyText()                             # interned text of non-canonical keys
        self.need = self.chunk                            # bytes to gather before the next chunk is processed
        self.lines_done = 0

    # ---- streaming ------------------------------------------------------------------------------------
    def feed(self, data):
        self.pending += data
        if len(self.pending) >= self.need:
            cut = self.pending.rfind(b'\n') + 1
            if cut:
                carry = self._process(self.pending[:cut], final=False)
                # one open run filled the whole chunk: gather twice as much first
                self.need = 2 * cut if len(carry) == cut else self.chunk
                self.pending = carry + self.pending[cut:]

    def finish(self):
        data, self.pending = self.pending, b''
        self._process(data, final=True)

    # ---- one chunk ------------------------------------------------------------------------------------
    def _process(self, data, final):
        """Parse and aggregate ``data`` (whole lines unless final); emit every
        completed run and return the bytes of the run still open (not final)."""
        eng, torch = self.eng, self.eng.torch
        ctx = eng.ctx
        v = lambda t: ctypes.c_void_p(t.data_ptr())
        text = textparse._device_bytes(torch, data, eng.device)
        dev = eng.device
        off, n = textparse.split_lines_device(ctx, torch, text, len(data))
        tuples = torch.zeros((max(n, 1), 4), dtype=torch.int32, device=dev)[:n]
        ts = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)[:n]
        disp = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)[:n]
        sp = textparse.spell_table(self.spells)
        if n:
            ctx.call('rsa_parse_reduce', v(text), v(off), ctypes.c_uint64(n), sp.ctypes.data_as(ctypes.c_void_p),
                     ctypes.c_uint32(len(sp)), v(tuples), v(ts), v(disp))
        h_off = off.cpu().numpy().view(np.uint64)
        d = disp.cpu().numpy().view(np.uint32)
        kind, same = d & 0xFF, (d & RED_SAME) != 0
        line = lambda i: data[int(h_off[i]):int(h_off[i + 1])].decode('latin-1')
        # empty lines (the mapper's blank records, all sorted to the front) are
        # "Unable to unpack" noise with nothing to parse: handled as runs
        blank = (kind == RED_NOISE) & (np.diff(h_off.astype(np.int64)) <= 1) if n else np.zeros(0, bool)

        # runs: the host decides each line that does not repeat its predecessor's key
        status = np.full(n, -1, np.int64)       # run id of the line, -1 noise
        runs = []                               # (key, host, acl, rule, first line)
        events = []                             # (line, 'noise', text) | (line, 'run', id)
        current = None
        stop, error = n, None
        decide = np.nonzero(~same & ~blank)[0]
        for i in decide:
            i = int(i)
            if kind[i] == RED_NOISE:
                events.append((i, 'noise', line(i).strip(PY2_WS)))
                continue
            ln = line(i).strip(PY2_WS)
            try:
                key, _value = ln.split('\t', 1)
                hostname, acl, ruleindex = key.split(';', 3)
                rule = self.db.accesslists[hostname][acl]['rules'][py2_int(ruleindex)]
                rule.hostname = hostname
                rule.accesslist = acl
            except ValueError:
                events.append((i, 'noise', ln))
                continue
            except (KeyError, IndexError) as exc:        # the reference dies here
                stop, error = i, exc
                break
            if current is None or key != current:
                current = key
                runs.append((key, hostname, acl, rule, i))
                events.append((i, 'run', len(runs) - 1))
            status[i] = len(runs) - 1
        # lines repeating their predecessor's key take its decision
        if n:
            src = np.where(same, -1, np.arange(n))
            src = np.maximum.accumulate(src)
            status = status[np.maximum(src, 0)]
            rep = np.nonzero(same[:stop] & (status[:stop] < 0))[0]     # repeats of a noise key
            for i in rep:
                events.append((int(i), 'noise', line(int(i)).strip(PY2_WS)))
        status[stop:] = -1
        events = [e for e in events if e[0] < stop]
        events.sort(key=lambda e: e[0])

        # carry the open run (not final): everything from its first line on
        carry_from = n
        if not final and error is None and runs:
            carry_from = runs[-1][4]
            runs = runs[:-1]
            events = [e for e in events if e[0] < carry_from]
            status[carry_from:] = -1
            stop = carry_from
        carry = data[int(h_off[carry_from]):] if carry_from < n else b''
        if not final and error is None and carry_from == 0 and n:
            # one run fills the chunk: read on before aggregating it
            return data

        # lines the device left to the host, and timestamps the reducer would reject
        h_tup = None
        odd_ts = {}
        bad_month = []
        host_lines = np.nonzero((kind[:stop] == textparse.LINE_HOST) & (status[:stop] >= 0))[0]
        if len(host_lines):
            h_tup = np.zeros(len(host_lines), TUPLE_DTYPE)
            h_ts = np.zeros(len(host_lines), np.uint32)
            for j, i in enumerate(host_lines):
                i = int(i)
                ln = line(i).strip(PY2_WS)
                value = ln.split('\t', 1)[1]
                hit, res = reducer_fields(value)
                flags = F_HIT if hit else 0
                if res is not None:
                    flags |= F_BUILT
                    h_tup[j]['pspell'], h_tup[j]['src'], h_tup[j]['dst'], h_tup[j]['dport'] = self._conn(res)
                    if hit:
                        try:
                            tstr = reducer_timestamp(res)
                        except ValueError as exc:
                            bad_month.append((i, exc))
                            flags &= ~F_BUILT          # counted as a hit; no record unless it kills the job
                            tstr = None
                        if tstr is not None:
                            code = textparse.ts_pack(tstr)
                            if code is None:
                                odd_ts[i] = tstr
                            else:
                                h_ts[j] = code
                h_tup[j]['flags'] = flags
            idx = torch.from_numpy(host_lines.astype(np.int64)).to(dev)
            tuples[idx] = torch.from_numpy(h_tup.view(np.int32).reshape(-1, 4)).to(dev)
            ts[idx] = torch.from_numpy(h_ts.view(np.int32)).to(dev)
        res, ts_decode = self._aggregate(tuples[:stop], ts[:stop], status[:stop], kind[:stop], odd_ts, len(runs))
        if bad_month:
            thresh = res.thresh
            for i, exc in bad_month:
                r = int(status[i])
                if self.cap > 0 and (int(thresh[r]) == 0xFFFFFFFFFFFFFFFF or i < int(thresh[r])):
                    # the reference reaches months.index at this line: redo the job up to it
                    # (the key test of this line already ran: a run starting here
                    # printed the block before it, as the reference does)
                    stop, error = i, exc
                    status[stop:] = -1
                    runs = [x for x in runs if x[4] <= stop]
                    events = [e for e in events if e[0] < stop or (e[0] == stop and e[1] == 'run')]
                    odd_ts = {k: t for k, t in odd_ts.items() if k < stop}
                    res, ts_decode = self._aggregate(tuples[:stop], ts[:stop], status[:stop], kind[:stop], odd_ts,
                                                     len(runs))
                    break
        if blank[:stop].any():   # runs of empty lines: one event per run
            b = np.concatenate([[False], blank[:stop], [False]]).astype(np.int8)
            edges = np.diff(b)
            for a, e in zip(np.nonzero(edges == 1)[0].tolist(), np.nonzero(edges == -1)[0].tolist()):
                events.append((a, 'blanks', e - a))
            events.sort(key=lambda e: e[0])
        mode = 'error' if error is not None else 'final' if final else 'carry'
        self.write(self._report(events, runs, res, ts_decode, mode))
        self.lines_done += stop
        if error is not None:
            raise error
        return carry

    def _conn(self, res):
        """(pspell, from, to, port) fields of a host-parsed BUILT match: the
        values of a canonical key, else (INTERNED, id of the key text, 0, 0)."""
        word, f, t, p = res[5], res[6], res[8], res[9]
        try:
            vf, vt = _canonical_v4(f), _canonical_v4(t)
        except ValueError:
            vf = vt = None
        canon = vf is not None and vt is not None and p.isdigit() and (len(p) == 1 or p[0] != '0') and int(p) < 65536
        sid = self.spell_ids.get(word)
        if sid is None and len(self.spells) < MAX_SPELL_ID:
            sid = self.spell_ids[word] = len(self.spells)
            self.spells.append(word)
        if canon and sid is not None:
            return sid, vf, vt, int(p)
        return INTERNED, self.istr((word, f, t, p)), 0, 0

    def _aggregate(self, tuples, ts, status, kind, odd_ts, n_runs):
        eng, torch = self.eng, self.eng.torch
        from .engine import DeviceBatch
        n = len(status)
        gids = torch.from_numpy(status.astype(np.int32)).to(eng.device)
        both = F_HIT | F_BUILT
        fl = ((tuples[:, 3] >> 16) & 0xFF).cpu().numpy() if n else np.zeros(0, np.int64)
        hb = ((fl & both) == both) & (status >= 0)
        ts_decode = textparse.ts_unpack
        if odd_ts:
            class _P(object):
                pass
            P = _P()
            textparse._retable([(ts, hb, textparse.ts_unpack, dict(odd_ts))], P)
            ts_decode = P.ts_decode
        order = torch.arange(n, dtype=torch.int64, device=eng.device)
        eng.set_rule_count(max(n_runs, 1))
        b = DeviceBatch(tuples, ts, order, gids)
        res = eng.run([b], self.cap, capacity=max(int(hb.sum()), 1))
        return res, ts_decode

    def _report(self, events, runs, res, ts_decode, mode):
        """connlist-reducer.py's stdout for these events: noise pairs at their
        lines, a block per run when the next one starts; mode 'final' (input
        ended): the blank line and the last block; 'carry': the last block too
        (the carried run's key follows); 'error': the reference died at the
        next line, before printing the last block."""
        by_run = _rows_by_gid(res.records)
        out = []
        cap = self.cap
        parts = []      # text already joined (runs of blank-line noise pairs)
        ts_decode = MemoDecode(ts_decode)

        def block(r):
            _key, host, acl, rule, _first = runs[r]
            lines = ['{0}: access-list {1}, rule {2}: {3}'.format(host, acl, rule.ruleindex, str(rule)),
                     '{0}'.format(rule.original), 'Total number of hits: {0}'.format(int(res.hits[r]))]
            if cap == 0 or int(res.thresh[r]) != 0xFFFFFFFFFFFFFFFF:
                lines.append('NOTE: Maximum number of connections ({0}) reached for this rule, additional '
                             'connections not displayed.'.format(cap))
            lines.append(HEADER)
            rows = by_run.get(r)
            if rows is not None and len(rows):
                lines.extend(table_rows(rows, *key_strings(rows, self.spells, self.istr), ts_decode))
            return lines

        prev = None
        for _i, what, val in events:
            if what == 'blanks':
                if out:
                    parts.append(''.join(l + '\n' for l in out))
                    out = []
                parts.append((NOISE1 + '\nThe line was: \n') * val)
            elif what == 'noise':
                out.append(NOISE1)
                out.append('The line was: {0}'.format(val))
            else:
                if prev is not None:
                    out.append('')
                    out.extend(block(prev))
                prev = val
        if mode == 'final':
            out.append('')
            if prev is not None:
                out.extend(block(prev))
        elif mode == 'carry' and prev is not None:
            # the chunk's last complete run: its block prints when the carried
            # run's key arrives (always the next chunk's first run)
            out.append('')
            out.extend(block(prev))
        parts.append(''.join(l + '\n' for l in out))
        return ''.join(parts)
