"""Device orchestration of the hot path on one MI355X.

PyTorch is plumbing here: it owns HBM buffers (tuples, counters, outputs) and
the HIP stream; every computation happens in ``libruleset_hip.so`` through the
C ABI (``native.Ctx``).  There is no CPU path: without a GPU or without the
library, constructing an ``Engine`` raises.

One job = pass 1 (classify + aggregate) over every batch, cap resolution,
pass 2 over every batch if any rule is capped, then emission of the connection
tables.  ``Results`` holds the per-rule counters and the connection records.
"""

import ctypes

import numpy as np

from . import native
from .native import RSA_ERR_CAPACITY, NativeError
from .compile import RECORD_DTYPE, RULE_DTYPE, TUPLE_DTYPE

__all__ = ['Engine', 'Results', 'DeviceBatch']


def _torch():
    import torch
    return torch


class Results(object):
    def __init__(self, matches, hits, distinct, thresh, records, cap):
        self.matches = matches      # uint64 [R]
        self.hits = hits            # uint64 [R]
        self.distinct = distinct    # uint32 [R]
        self.thresh = thresh        # uint64 [R] (0xFFFF.. = not capped)
        self.records = records      # RECORD_DTYPE [M]
        self.cap = cap

    def capped(self, gid):
        return int(self.thresh[gid]) != 0xFFFFFFFFFFFFFFFF or (self.cap == 0 and self.matches[gid] > 0)


class DeviceBatch(object):
    """Tuples/timestamps/order keys resident in HBM (torch tensors)."""

    def __init__(self, tuples, ts, order, gids=None):
        self.tuples = tuples    # uint8 [n*16] or int32 [n,4]
        self.ts = ts            # int32 [n]  (uint32 codes)
        self.order = order      # int64 [n]  (uint64 keys)
        self.gids = gids        # int32 [n] or None
        self.n = int(ts.numel()) if ts is not None else int(tuples.shape[0])

    @classmethod
    def from_numpy(cls, tuples, ts, order, device, gids=None):
        torch = _torch()
        assert tuples.dtype == TUPLE_DTYPE
        t = torch.from_numpy(np.ascontiguousarray(tuples).view(np.int32).reshape(-1, 4)).to(device)
        s = torch.from_numpy(np.ascontiguousarray(ts, dtype=np.uint32).view(np.int32)).to(device)
        o = torch.from_numpy(np.ascontiguousarray(order, dtype=np.uint64).view(np.int64)).to(device)
        g = None
        if gids is not None:
            g = torch.from_numpy(np.ascontiguousarray(gids, dtype=np.int32)).to(device)
        return cls(t, s, o, g)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class Engine(object):
    def __init__(self, device=0):
        torch = _torch()
        if not torch.cuda.is_available():
            raise native.NativeUnavailable('no HIP device visible: the hot path has no CPU fallback')
        self.torch = torch
        self.device = torch.device('cuda', device)
        torch.cuda.set_device(self.device)
        self.ctx = native.Ctx(device)
        self._emit_buf, self._emit_cap = None, 0   # emission buffer kept between calls (emit_device)
        self._route_buf, self._route_cap, self._route_counts = None, 0, None   # export_routed's buffers
        self.stream = torch.cuda.current_stream(self.device)
        self.ctx.call('rsa_set_stream', ctypes.c_void_p(self.stream.cuda_stream))
        self.n_rules = 0
        self.counters = None
        self.last_gids = []

    # ---- setup -------------------------------------------------------------------
    def load_rules(self, entries, offsets, n_rules):
        entries = np.ascontiguousarray(entries)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        self.ctx.call('rsa_load_rules', entries.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(entries)),
                      offsets.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(offsets) - 1),
                      ctypes.c_uint32(n_rules))
        self._bind(n_rules)

    def load_index(self, index):
        """Upload an index (image, residual entries): compile.build_index() or
        bucketindex.build_bucket_index()."""
        image, resid = (np.ascontiguousarray(a) for a in index)
        self._index_hold = (image, resid)
        # which index is loaded (reporting): RSA4 'pht', RSA5 'bucket' / 'bucket-filtered'
        self.index_kind = 'pht' if int(image[1]) == 0x34415352 else (
            'bucket-filtered' if int(image[5]) & 1 else 'bucket')
        v = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        self.ctx.call('rsa_load_index', v(image), ctypes.c_uint32(len(image)), v(resid), ctypes.c_uint32(len(resid)))

    def set_option(self, option, value):
        self.ctx.call('rsa_set_option', ctypes.c_int(option), ctypes.c_int64(int(value)))

    def use_index(self, on):
        self.set_option(native.RSA_OPT_USE_INDEX, 1 if on else 0)

    def auto_filter(self, on):
        self.set_option(native.RSA_OPT_AUTO_FILTER, 1 if on else 0)

    def last_pass1_times(self):
        """(classification ms, aggregation ms) of the last pass-1 call (HIP events on the ctx stream)."""
        a, b = ctypes.c_float(0), ctypes.c_float(0)
        self.ctx.call('rsa_last_pass1_times', ctypes.byref(a), ctypes.byref(b))
        return float(a.value), float(b.value)

    def last_pass1_launches(self):
        """Classification launches (filter slices) of the last pass-1 call."""
        n = ctypes.c_uint32(0)
        self.ctx.call('rsa_last_pass1_launches', ctypes.byref(n))
        return int(n.value)

    def last_pass1_ms(self):
        ms = ctypes.c_float(0)
        self.ctx.call('rsa_last_pass1_ms', ctypes.byref(ms))
        return float(ms.value)

    def load_compiled(self, compiled, index=True, prefix=0, chunk=None, kind=None):
        """Upload a CompiledRules' lists and its index (``kind``: 'auto', the
        default (CompiledRules.index), 'pht', 'bucket' or 'bucket-filtered' --
        the RSA_INDEX environment variable overrides the default; the first ``prefix`` entries per list
        are scanned linearly, records hold at most ``chunk`` entries each,
        chained)."""
        import os
        packed = compiled.packed()
        ent, off = packed
        self.load_rules(ent, off, compiled.n_rules)
        if index:
            kind = kind or os.environ.get('RSA_INDEX', 'auto')
            self.load_index(compiled.index(prefix=prefix, chunk=chunk, kind=kind))
        self._loaded = (compiled, packed, index, prefix, chunk, kind)

    def refresh_compiled(self, compiled):
        """Re-upload ``compiled`` if lists were added since load_compiled (the
        host parse derives lists for lines with ports past 65535,
        CompiledRules.list_id_oor); a no-op otherwise."""
        held = getattr(self, '_loaded', None)
        if held is None or held[0] is not compiled:
            self.load_compiled(compiled)
        elif held[1] is not compiled.packed():
            self.load_compiled(compiled, *held[2:])

    def set_rule_count(self, n_rules):
        """Rule count of jobs over given gids (rsa_aggregate_gids: the reducer
        drop-in's runs, the merge owners): any loaded candidate lists are
        replaced by none, so the count may change between jobs."""
        self.load_rules(np.zeros(0, RULE_DTYPE), np.zeros(1, np.uint32), n_rules)
        self._loaded = None

    def _bind(self, n_rules):
        torch = self.torch
        n = max(int(n_rules), 1)
        self.n_rules = int(n_rules)
        self.counters = {
            'matches': torch.zeros(n, dtype=torch.int64, device=self.device),
            'hits': torch.zeros(n, dtype=torch.int64, device=self.device),
            'distinct': torch.zeros(n, dtype=torch.int32, device=self.device),
            'thresh': torch.full((n,), -1, dtype=torch.int64, device=self.device),
        }
        c = self.counters
        self.ctx.call('rsa_bind_counters', _ptr(c['matches']), _ptr(c['hits']), _ptr(c['distinct']), _ptr(c['thresh']))

    # ---- the job -----------------------------------------------------------------
    def reset(self, capacity, cap):
        self.ctx.call('rsa_reset', ctypes.c_uint64(int(capacity)), ctypes.c_uint32(int(cap)))

    def pass1(self, b, gid_out=None):
        if b.gids is not None:
            self.ctx.call('rsa_aggregate_gids', _ptr(b.tuples), _ptr(b.ts), _ptr(b.order), _ptr(b.gids),
                          ctypes.c_uint64(b.n))
        else:
            self.ctx.call('rsa_classify', _ptr(b.tuples), _ptr(b.ts), _ptr(b.order), ctypes.c_uint64(b.n),
                          _ptr(gid_out))

    def resolve_cap(self, sync=True):
        """The cap resolution; returns the number of capped rules.  With
        sync=False the count stays on the device (None is returned): a
        following pass2 then runs unconditionally and its kernels skip their
        work on the device when no rule is capped -- one host round trip less."""
        if not sync:
            self.ctx.call('rsa_resolve_cap', None)
            return None
        n = ctypes.c_uint32(0)
        self.ctx.call('rsa_resolve_cap', ctypes.byref(n))
        return int(n.value)

    def pass2(self, b, gids=None):
        g = b.gids if b.gids is not None else gids
        self.ctx.call('rsa_recount', _ptr(b.tuples), _ptr(b.ts), _ptr(b.order), _ptr(g), ctypes.c_uint64(b.n))

    def stats(self, reset=True):
        """Profiling counters (RSA_OPT_STATS): table lines, extra probes, atomic-path probes, slot atomics."""
        out = (ctypes.c_uint64 * 4)()
        self.ctx.call('rsa_stats', out, ctypes.c_int(1 if reset else 0))
        return [int(v) for v in out]

    def table_size(self):
        n = ctypes.c_uint64(0)
        self.ctx.call('rsa_table_size', ctypes.byref(n))
        return int(n.value)

    def emit_device(self, mode='final'):
        """Records as a torch uint8 tensor [M*40] on device (a view of a buffer
        the engine keeps between calls).  The buffer is sized from the last
        table size seen; only when the records do not fit (the library reports
        the count it needed) is the table size read and the emission repeated,
        so a steady job pays one host round trip here, not two."""
        n = ctypes.c_uint64(0)
        size = self._emit_cap
        if size == 0:
            size = self.table_size()
        for _ in range(2):
            buf = self._emit_buffer(size)
            try:
                if mode == 'final':
                    self.ctx.call('rsa_emit', _ptr(buf), ctypes.c_uint64(size), ctypes.byref(n))
                else:
                    which = {'pass1': 0, 'pass2': 1, 'pass1_kept': 2}[mode]
                    self.ctx.call('rsa_export', ctypes.c_int(which), _ptr(buf), ctypes.c_uint64(size),
                                  ctypes.byref(n))
                break
            except NativeError as e:
                if e.code != RSA_ERR_CAPACITY or int(n.value) <= size:
                    raise
                size = self.table_size()
        # the buffer is reused by the next emission: callers that keep records
        # across calls clone them
        return buf[: int(n.value) * RECORD_DTYPE.itemsize]

    def export_routed(self, mode, world, capacity=None):
        """rsa_export_routed: the exported records grouped by owner rank (gid %
        world) into a device buffer the engine keeps, and their per-owner
        counts as a device int64 tensor [world]; no host round trip.  Returns
        (buf, counts, capacity in records): records past the capacity are
        dropped, so a caller whose counts sum past it exports again with
        capacity=that sum."""
        torch = self.torch
        which = {'pass1': 0, 'pass2': 1, 'pass1_kept': 2}[mode]
        size = int(capacity or self._emit_cap or self.table_size())
        size = max(size, 1)
        if self._route_buf is None or self._route_cap < size:
            self._route_buf = torch.empty(size * RECORD_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
            self._route_cap = size
        if self._route_counts is None or self._route_counts.numel() != world:
            self._route_counts = torch.zeros(world, dtype=torch.int64, device=self.device)
        self.ctx.call('rsa_export_routed', ctypes.c_int(which), ctypes.c_uint32(world), _ptr(self._route_buf),
                      ctypes.c_uint64(self._route_cap), _ptr(self._route_counts))
        return self._route_buf, self._route_counts, self._route_cap

    def _emit_buffer(self, size):
        size = max(int(size), 1)
        if self._emit_buf is None or self._emit_cap < size:
            self._emit_buf = self.torch.empty(size * RECORD_DTYPE.itemsize, dtype=self.torch.uint8,
                                              device=self.device)
            self._emit_cap = size
        return self._emit_buf

    def import_records(self, buf, which):
        n = buf.numel() // RECORD_DTYPE.itemsize
        self.ctx.call('rsa_import', ctypes.c_int(which), _ptr(buf), ctypes.c_uint64(n))

    def results(self, cap):
        c = self.counters
        recs = self.emit_device('final')
        self.torch.cuda.synchronize(self.device)
        host = recs.cpu().numpy().view(RECORD_DTYPE)
        R = self.n_rules
        return Results(c['matches'][:R].cpu().numpy().view(np.uint64), c['hits'][:R].cpu().numpy().view(np.uint64),
                       c['distinct'][:R].cpu().numpy().view(np.uint32), c['thresh'][:R].cpu().numpy().view(np.uint64),
                       host.copy(), cap)

    def run(self, batches, cap, capacity, keep_gids=True, sync_cap=True):
        """Full single-GPU job over device batches; returns Results.  With
        sync_cap=False the capped-rule count is not read back (resolve_cap
        sync=False) and the recount always runs."""
        torch = self.torch
        self.reset(capacity, cap)
        gid_bufs = []
        for b in batches:
            g = None
            if b.gids is None and keep_gids:
                g = torch.empty(b.n, dtype=torch.int32, device=self.device)
            self.pass1(b, g)
            gid_bufs.append(g)
        n_capped = self.resolve_cap(sync=sync_cap)
        if n_capped is None or n_capped > 0:
            for b, g in zip(batches, gid_bufs):
                self.pass2(b, g)
        self.last_gids = gid_bufs
        return self.results(cap)

    def classify_only(self, b, out=None):
        """First-match gid per tuple (mapper drop-in); no aggregation."""
        torch = self.torch
        g = out if out is not None else torch.empty(b.n, dtype=torch.int32, device=self.device)
        self.ctx.call('rsa_classify_only', _ptr(b.tuples), ctypes.c_uint64(b.n), _ptr(g))
        return g

    def close(self):
        if self.ctx is not None:
            self.ctx.close()
            self.ctx = None
