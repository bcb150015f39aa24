"""The fused job on one GPU: log text -> reducer report, without the
intermediate mapper text or the sort (the reference's
``mapper.py | LC_ALL=C sort | connlist-reducer.py``, ``runAnalysis.sh:42-56``).

The output is byte-identical to what the reference pipeline prints for the
same input (blocks in key byte order, the mapper's blank records turned into
the reducer's "Unable to unpack" noise pairs first), with connection-table
ties in CPython 2.7 dict order (SURVEY.md trap 8, ``py2dict.py``).

Deaths follow the pipeline too (``set -o pipefail``): when the mapper dies at
a line (``KeyError``/``ValueError`` of ``mapper.py:138-166``, or the missing
firewall of ``:115-117``, whose message the reducer then reads as noise), the
report is the reducer's over the lines before it and the mapper's exception
is raised after it; when the reducer dies in ``months.index``
(``connlist-reducer.py:164``: a matched hit BUILT line with a month outside
``Jan..Dec`` while its rule's dict is not full), the report stops where the
reducer stopped printing and that ``ValueError`` is raised.  Either way the
exception carries the printed lines as ``rsa_report``.
"""

import numpy as np

from .compile import CompiledRules, F_HIT, F_BUILT
from .engine import Engine, DeviceBatch
from .keytext import KeyText
from .logparse import parse_logs, key_tuples, D_CLASSIFY, D_MISSING
from .report import reducer_report

__all__ = ['analyze', 'analyze_text', 'assemble_report', 'built_hit_count', 'reducer_death', 'finish_job']

NO_THRESHOLD = 0xFFFFFFFFFFFFFFFF


def built_hit_count(tuples):
    both = F_HIT | F_BUILT
    return int(np.count_nonzero((tuples['flags'] & both) == both))


def reducer_death(parsed, gids, results, compiled, cap):
    """(gid, line index) of the line the reference reducer dies at, or None.

    Candidates are the hit BUILT lines whose month ``months.index`` rejects
    (``parsed.bad_month``; aggregated as hits without a record).  The reducer
    reaches the call for such a line only if the mapper emitted it (gid >= 0)
    and ``len(conns) < cap`` still holds (``connlist-reducer.py:151``): cap > 0
    and the rule either never fills its dict or fills it at a later line --
    order < P, the order key of the line inserting the cap-th connection
    (``Results.thresh``).  The reducer meets them in key order (the key bytes
    then the tab, as ``LC_ALL=C sort`` orders the mapper lines), then by line
    order within a key."""
    bad = getattr(parsed, 'bad_month', None)
    if not bad or cap <= 0:
        return None
    idx = np.fromiter(bad.keys(), np.int64, len(bad))
    g = np.asarray(gids)[idx].astype(np.int64)
    idx, g = idx[g >= 0], g[g >= 0]
    if not len(idx):
        return None
    order = parsed.order
    if hasattr(order, 'cpu'):
        o = order[order.new_tensor(idx)].cpu().numpy().view(np.uint64)
    else:
        o = np.asarray(order, np.uint64)[idx]
    th = results.thresh[g]
    reach = (th == np.uint64(NO_THRESHOLD)) | (o < th)
    if not reach.any():
        return None
    best = min(zip(idx[reach].tolist(), g[reach].tolist(), o[reach].tolist()),
               key=lambda t: (compiled.key(t[1]) + '\t', t[2]))
    return best[1], best[0]


def finish_job(parsed, gids, results, compiled, cap):
    """The report of a finished job; raises the pipeline's death (module
    docstring) with the printed lines attached as ``rsa_report``."""
    death = reducer_death(parsed, gids, results, compiled, cap)
    out = assemble_report(parsed, gids, results, compiled, cap, stop=death)
    exc = None
    if death is not None:
        exc = parsed.bad_month[death[1]]
    elif parsed.error is not None:
        exc = parsed.error[1]
    if exc is not None:
        exc.rsa_report = out
        raise exc
    return out


def assemble_report(parsed, gids, results, compiled, cap, ts_decode=None, pspell_table=None, stop=None):
    """Reducer stdout lines for parsed lines, their gids and the GPU results
    (``stop``: (gid, line index) of the reducer's dying line, reducer_death)."""
    db = compiled.db
    groups = []
    for gid in np.nonzero(results.matches > 0)[0]:
        gid = int(gid)
        host, acl, i = compiled.locate(gid)
        key = '%s;%s;%d' % (host, acl, i)
        groups.append((key + '\t', gid, host, acl, db.accesslists[host][acl]['rules'][i]))
    groups.sort(key=lambda g: g[0])
    disp = parsed.disposition
    nl = getattr(parsed, 'nl', None)
    if nl is None:
        nl = np.array([l.endswith('\n') for l in parsed.lines], dtype=bool) if parsed.n else np.zeros(0, bool)
    matched = (disp == D_CLASSIFY) & (gids >= 0)
    n_blank = int(np.count_nonzero(matched & nl))
    noise = []
    for i in np.nonzero(disp == D_MISSING)[0]:
        i = int(i)
        line = parsed.lines[i]
        msg = ('Unable to process line because access-list {0} is missing from data structure for host {1}, '
               'skipping line.'.format(parsed.acl_of[i], parsed.host_of[i]))
        skipped = 'The skipped line is: ' + (line[:-1] if nl[i] else line)
        noise.append((msg, msg))
        noise.append((skipped, skipped))
        if nl[i]:
            n_blank += 1
    err = getattr(parsed, 'error', None)
    if err is not None and isinstance(err[1], SystemExit):
        msg = str(err[1])       # mapper.py:116: printed on stdout, read by the reducer as a record
        noise.append((msg, msg))
    stop_at = None
    if stop is not None:
        line = parsed.lines[stop[1]]
        stop_at = (stop[0], compiled.key(stop[0]) + '\t' + (line[:-1] if nl[stop[1]] else line))
    if ts_decode is None:
        ts_decode = getattr(parsed, 'ts_decode', None) or parsed.ts_table.__getitem__
    if pspell_table is None:
        pspell_table = parsed.pspell_table
    return reducer_report(results, groups, noise, cap, ts_decode, pspell_table, n_blank=n_blank,
                          keytext=getattr(parsed, 'keytext', None), stop=stop_at)


def analyze(inputs, db, cap=1000, device=0, engine=None):
    """inputs: iterable of (host, lines-with-newlines).  Returns (report lines, results)."""
    compiled = CompiledRules(db)
    parsed = parse_logs(inputs, db, compiled)
    eng = engine if engine is not None else Engine(device)
    eng.load_compiled(compiled)
    batch = DeviceBatch.from_numpy(parsed.tuples, parsed.ts, parsed.order, eng.device)
    cap_n = max(built_hit_count(parsed.tuples), 1)
    if parsed.keyx:
        # lines with interned reducer keys: classified on their tuples,
        # aggregated under their key ids (logparse.key_tuples)
        g = eng.classify_only(batch)
        agg = DeviceBatch(key_tuples(eng.torch, batch.tuples, parsed.keyx), batch.ts, batch.order, g)
        results = eng.run([agg], cap, capacity=cap_n)
        gids = g.cpu().numpy()
    else:
        results = eng.run([batch], cap, capacity=cap_n)
        gids = eng.last_gids[0].cpu().numpy() if parsed.n else np.zeros(0, np.int32)
    return finish_job(parsed, gids, results, compiled, cap), results


def analyze_text(inputs, db, cap=1000, device=0, engine=None):
    """The fused job from raw log bytes: inputs = iterable of (host, bytes).
    The text is parsed on the GPU (textparse), the lines classified, then
    ranked for the reducer's order: by their bytes within each rule (grouped
    order keys over all inputs together, as ``cat f1 f2 | mapper | sort`` orders
    a key's lines across files -- the reducer only ever compares one rule's
    lines), and aggregated with their gids; returns (report lines, results)."""
    from . import textparse
    compiled = CompiledRules(db)
    compiled.ensure_lists()
    eng = engine if engine is not None else Engine(device)
    torch = eng.torch
    parts, pspell, keytext = [], {}, KeyText()
    for host, data in inputs:
        p = textparse.parse_text(eng, host, data, db, compiled, pspell=pspell, need_order=False, keep_text=True,
                                 keytext=keytext)
        parts.append(p)
        if p.error is not None:       # the mapper dies here: the lines before it still reach the reducer
            break
    eng.load_compiled(compiled)
    n = sum(p.n for p in parts)
    if n == 0:
        for p in parts:
            p._d_text = p._d_off = None
        parsed = textparse.concat(parts, torch)
        results = eng.run([], cap, capacity=1)
        return finish_job(parsed, np.zeros(0, np.int32), results, compiled, cap), results
    tuples = torch.cat([p.tuples for p in parts if p.n])
    gids = eng.classify_only(DeviceBatch(tuples, None, None))
    flags = (tuples[:, 3] >> 16) & 0xFF
    both = F_HIT | F_BUILT
    ranked = (flags & both) == both
    hb_n = int(ranked.sum().item())
    base, bad = 0, []
    for p in parts:
        bad.extend(base + i for i in p.bad_month)
        base += p.n
    if bad:
        # lines months.index rejects are ranked with their rule's lines: the
        # reducer dies at one only if it comes before the cap freeze
        ranked[torch.tensor(bad, dtype=torch.int64, device=gids.device)] = True
    textparse.order_keys_global(eng, parts, group=torch.where(ranked & (gids >= 0), gids, torch.full_like(gids, -1)))
    parsed = textparse.concat(parts, torch)
    batch = DeviceBatch(key_tuples(torch, parsed.tuples, parsed.keyx), parsed.ts, parsed.order, gids)
    results = eng.run([batch], cap, capacity=max(hb_n, 1))
    return finish_job(parsed, gids.cpu().numpy(), results, compiled, cap), results
