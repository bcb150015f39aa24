"""The fused job on one GPU: log text -> reducer report, without the
intermediate mapper text or the sort (the reference's
``mapper.py | LC_ALL=C sort | connlist-reducer.py``, ``runAnalysis.sh:42-56``).

The output is byte-identical to what the reference pipeline prints for the
same input (blocks in key byte order, the mapper's blank records turned into
the reducer's "Unable to unpack" noise pairs first), with connection-table
ties in CPython 2.7 dict order (SURVEY.md trap 8, ``py2dict.py``).
"""

import numpy as np

from .compile import CompiledRules, F_HIT, F_BUILT
from .engine import Engine, DeviceBatch
from .keytext import KeyText
from .logparse import parse_logs, key_tuples, D_CLASSIFY, D_MISSING
from .report import reducer_report

__all__ = ['analyze', 'analyze_text', 'assemble_report', 'built_hit_count']


def built_hit_count(tuples):
    both = F_HIT | F_BUILT
    return int(np.count_nonzero((tuples['flags'] & both) == both))


def assemble_report(parsed, gids, results, compiled, cap, ts_decode=None, pspell_table=None):
    """Reducer stdout lines for parsed lines, their gids and the GPU results."""
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
    if ts_decode is None:
        ts_decode = getattr(parsed, 'ts_decode', None) or parsed.ts_table.__getitem__
    if pspell_table is None:
        pspell_table = parsed.pspell_table
    return reducer_report(results, groups, noise, cap, ts_decode, pspell_table, n_blank=n_blank,
                          keytext=getattr(parsed, 'keytext', None))


def analyze(inputs, db, cap=1000, device=0, engine=None):
    """inputs: iterable of (host, lines-with-newlines).  Returns (report lines, results)."""
    compiled = CompiledRules(db)
    parsed = parse_logs(inputs, db, compiled)
    if parsed.error is not None:
        raise parsed.error[1]
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
    return assemble_report(parsed, gids, results, compiled, cap), results


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
        if p.error is not None:
            break
    if any(p.error is not None for p in parts):
        for p in parts:
            p._d_text = p._d_off = None
        parsed = textparse.concat(parts, torch)
        raise parsed.error[1]
    eng.load_compiled(compiled)
    n = sum(p.n for p in parts)
    if n == 0:
        for p in parts:
            p._d_text = p._d_off = None
        parsed = textparse.concat(parts, torch)
        results = eng.run([], cap, capacity=1)
        return assemble_report(parsed, np.zeros(0, np.int32), results, compiled, cap), results
    tuples = torch.cat([p.tuples for p in parts if p.n])
    gids = eng.classify_only(DeviceBatch(tuples, None, None))
    flags = (tuples[:, 3] >> 16) & 0xFF
    both = F_HIT | F_BUILT
    hb = (flags & both) == both
    textparse.order_keys_global(eng, parts, group=torch.where(hb & (gids >= 0), gids, torch.full_like(gids, -1)))
    parsed = textparse.concat(parts, torch)
    batch = DeviceBatch(key_tuples(torch, parsed.tuples, parsed.keyx), parsed.ts, parsed.order, gids)
    results = eng.run([batch], cap, capacity=max(int(hb.sum().item()), 1))
    return assemble_report(parsed, gids.cpu().numpy(), results, compiled, cap), results
