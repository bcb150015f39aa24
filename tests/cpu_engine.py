"""TEST INFRASTRUCTURE ONLY — a CPU stand-in for ``engine.Engine`` so the
host logic around the hot path (``pipeline.analyze``: the parse, the
reducer-death decision, report assembly) runs in the ``-m "not gpu"`` suite.
Classification and aggregation come from ``cpu_model`` (brute-force first
match over the compiled lists, the numpy model of the connection table); the
GPU tests run the same host logic over the real library.

Nothing in the product imports this module.
"""
import numpy as np
import torch

from cpu_model import NumpyBackend, classify_entries
from ruleset_analysis_amd.compile import TUPLE_DTYPE
from ruleset_analysis_amd.engine import Results


class CpuEngine(object):
    def __init__(self):
        self.torch = torch
        self.device = torch.device('cpu')
        self.last_gids = []
        self.compiled = None

    def load_compiled(self, compiled, *a, **k):
        self.compiled = compiled
        self.n_rules = compiled.n_rules

    def refresh_compiled(self, compiled):
        self.compiled = compiled

    def _tuples(self, b):
        return b.tuples.numpy().astype(np.int32).reshape(-1).view(TUPLE_DTYPE)

    def classify_only(self, b, out=None):
        ent, off = self.compiled.packed()
        g = classify_entries(ent, off, self._tuples(b))
        return torch.from_numpy(g.astype(np.int32))

    def run(self, batches, cap, capacity, keep_gids=True):
        gids, tups, tss, orders = [], [], [], []
        self.last_gids = []
        for b in batches:
            g = b.gids if b.gids is not None else self.classify_only(b)
            self.last_gids.append(g)
            gids.append(g.numpy())
            tups.append(self._tuples(b))
            tss.append(b.ts.numpy().view(np.uint32))
            orders.append(b.order.numpy().view(np.uint64))
        cat = lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt)
        tup = cat(tups, TUPLE_DTYPE)
        be = NumpyBackend.from_packed(self.n_rules, cap, cat(gids, np.int32), tup, cat(tss, np.uint32),
                                      cat(orders, np.uint64))
        if be.resolve_cap():
            be.recount()
        c = be.counters()
        if cap == 0:            # len(conns) < 0 never holds: no table rows (connlist-reducer.py:151)
            be.local.t.clear()
        recs = be.emit_final().numpy().view(np.dtype([('min_order', '<u8'), ('gid', '<u4'), ('for_ip', '<u4'),
                                                       ('to_ip', '<u4'), ('to_port', '<u2'), ('pspell', 'u1'),
                                                       ('pad', 'u1'), ('count', '<u4'), ('first', '<u4'),
                                                       ('last', '<u4'), ('pad2', '<u4')]))
        return Results(c['matches'].numpy().astype(np.uint64), c['hits'].numpy().astype(np.uint64),
                       c['distinct'].numpy().astype(np.uint32), c['thresh'].numpy().view(np.uint64).copy(),
                       recs.copy(), cap)
