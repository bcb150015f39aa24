"""Multi-GPU merge — the MI355X replacement of the Hadoop shuffle
(``runAnalysis.sh:42-56``: map output partitioned by key hash to 4 reducers).

One process per GPU (``torch.distributed``; backend ``nccl`` = RCCL over xGMI
on the GPU box, ``gloo`` in the CPU tests).  Every rank classifies and
aggregates its own contiguous shard of the log (pass 1, rule tables
replicated).  Rank r owns the rules with ``gid % world == r`` (the reducer
partitioning), and its pass-1 table doubles as the merged table of those
rules: their entries stay where pass 1 put them.  Exports come out of the
library already grouped by owner, with their per-owner counts on the device
(``rsa_export_routed``), so each exchange is one all_to_all of the counts,
one host read of the send and receive sizes, and one all_to_all of the rows.
Then:

1. ``all_reduce(SUM)`` of the per-rule line and hit counters;
2. each rank resolves its shard's own cap thresholds and sends the entries of
   rules owned elsewhere that can still reach the report (no threshold, or
   min_order <= the shard's P, which bounds the global P from above) to their
   owners (``all_to_all``); owners merge them into their table (count sum,
   first-seen min, last-seen max, min order key);
3. owners resolve the cap of their rules; ``all_reduce(MAX)`` of the threshold
   vector (other ranks' rules at "none") gives every rank every rule's P;
4. if any rule is capped: every rank recounts its shard's occurrences with
   order <= P (pass 2 from its kept pass-1 records), sends the pass-2 sums of
   rules owned elsewhere to their owners, which add them;
5. the owners' final rows are gathered to rank 0.

At world 1 nothing moves: the merge is the single-GPU job.  The order keys
are global, so the cap logic is shard-agnostic.  Records are 40-byte
``rsa_conn_record`` rows moved as uint8 tensors.

On the GPU (``EngineBackend``) the whole sequence runs inside the library,
behind one C-ABI call (``rsa_merge`` in ``csrc/merge.hip``): over RCCL
(``rsa_merge_rccl``, the library's own communicator on the ctx's device) when
the group's backend is ``nccl``, else over this group through host-buffer
callbacks (``rsa_transport.host_buffers``; gloo, several ranks sharing one
GPU).  Python only creates the communicator and copies the resulting rows into
a torch tensor.  The Python protocol below (``merge(..., impl='python')``) is
the same sequence step for step: the model the CPU tests run over numpy
backends (tests/cpu_model.py), and a GPU cross-check of the library's.
"""

import ctypes

import numpy as np

from .compile import RECORD_DTYPE

__all__ = ['merge', 'gather_rows', 'OwnerRows', 'merged_to_host', 'EngineBackend', 'Exported', 'route_records',
           'ShardOverflow']

REC = RECORD_DTYPE.itemsize
NO_THRESHOLD = -1   # 0xFFFF_FFFF_FFFF_FFFF viewed as int64


def _host_staged(dist, group):
    """gloo cannot move device tensors: stage them through host memory (tests /
    several ranks sharing one GPU).  RCCL moves HBM to HBM directly."""
    try:
        return dist.get_backend(group) == 'gloo'
    except Exception:  # noqa: BLE001
        return False


def _all_reduce(t, dist, group, op=None):
    kw = {} if op is None else {'op': op}
    if t.is_cuda and _host_staged(dist, group):
        h = t.cpu()
        dist.all_reduce(h, group=group, **kw)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group, **kw)


def _all_to_all(out, inp, dist, group, out_splits=None, in_splits=None):
    if inp.is_cuda and _host_staged(dist, group):
        h = torch_empty_like_cpu(out)
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(h)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def _all_gather(parts, t, dist, group):
    if t.is_cuda and _host_staged(dist, group):
        hp = [p.cpu() for p in parts]
        dist.all_gather(hp, t.cpu(), group=group)
        for p, h in zip(parts, hp):
            p.copy_(h)
    else:
        dist.all_gather(parts, t, group=group)


def _gather0(t, sizes, rank, world, dist, group):
    """Rows of every rank to rank 0 only (the emission rank): dist.gather of
    equal-size padded buffers (RCCL point-to-point sends over xGMI; the other
    ranks receive nothing).  Returns the list of parts on rank 0, else None."""
    import torch
    pad = max(max(sizes), 1)
    padded = torch.zeros(pad, dtype=torch.uint8, device=t.device)
    padded[:t.numel()] = t
    staged = t.is_cuda and _host_staged(dist, group)
    src = padded.cpu() if staged else padded
    parts = None
    if rank == 0:
        parts = [torch.empty(pad, dtype=torch.uint8, device=src.device) for _ in range(world)]
    dist.gather(src, gather_list=parts, dst=0, group=group)
    if rank != 0:
        return None
    return [(p.to(t.device) if staged else p)[:s] for p, s in zip(parts, sizes)]


class _Trace(object):
    """RSA_MERGE_TRACE=1: per-phase wall time of the merge on stderr (with a
    device synchronise per phase, so only for diagnosis)."""

    def __init__(self, rank):
        import os
        import time
        self.on = os.environ.get('RSA_MERGE_TRACE') == '1'
        self.rank, self.time, self.t, self.parts = rank, time, None, []

    def __call__(self, what, dev=None):
        if not self.on:
            return
        import sys
        import torch
        if dev is not None and dev.type == 'cuda':
            torch.cuda.synchronize(dev)
        now = self.time.perf_counter()
        if self.t is not None:
            self.parts.append('%s %.2f' % (what, (now - self.t) * 1e3))
        self.t = now
        if what == 'end':
            sys.stderr.write('[merge rank %d] ms: %s\n' % (self.rank, ', '.join(self.parts)))


def torch_empty_like_cpu(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype)


class ShardOverflow(RuntimeError):
    """Some rank's pass-1 table overflowed (RSA_ERR_CAPACITY): raised on every
    rank together, so all of them can rerun the job with a larger table instead
    of the healthy ranks waiting in the next collective.  ``needed``: the
    entries the largest failing table must hold (its own entries plus the
    records it received for the rules it owns; 0 if unknown)."""
    code = -4    # native.RSA_ERR_CAPACITY

    def __init__(self, msg, needed=0):
        RuntimeError.__init__(self, msg)
        self.needed = int(needed)


class Exported(object):
    """One rank's export of a merge phase, already grouped by owner rank (gid %
    world): ``buf`` uint8 rows (40 B each) with owner r's records forming
    segment r, ``counts`` int64 [world] (device) the segment sizes, ``capacity``
    the rows ``buf`` holds; ``again(n)`` exports once more into n rows (the
    library drops rows past the capacity and reports the true counts) and
    returns (buf, counts, capacity)."""

    def __init__(self, buf, counts, capacity, again=None):
        self.buf, self.counts, self.capacity, self.again = buf, counts, int(capacity), again

    @classmethod
    def empty(cls, world, device):
        import torch
        return cls(torch.zeros(0, dtype=torch.uint8, device=device), torch.zeros(world, dtype=torch.int64,
                                                                                  device=device), 0)


def route_records(exp, world, dist, group=None, flag=0, stats=None, phase='route'):
    """all_to_all of an owner-grouped export (``Exported``) to the owners;
    returns the received bytes.  The per-owner counts go first, with ``flag``
    (this rank's error flag) riding along, and the phase's ONE host read takes
    the send and receive sizes together; if any rank sent a non-zero flag,
    every rank returns None instead.  ``stats`` (a dict): the rows this rank
    sent to other ranks, kept to itself and received, under ``phase``."""
    import torch
    counts = exp.counts.to(torch.int64)
    send_c = torch.stack([counts, torch.full_like(counts, int(flag))], 1).reshape(-1)
    recv_c = torch.empty_like(send_c)
    _all_to_all(recv_c, send_c, dist, group)
    h = [int(x) for x in torch.cat([counts, recv_c]).cpu().tolist()]
    if any(h[world + 2 * r + 1] for r in range(world)):
        return None
    total = sum(h[:world])
    buf = exp.buf
    if total > exp.capacity:      # the export dropped rows past its buffer: again at the exact size
        buf, _counts, _cap = exp.again(total)
        if stats is not None:
            stats['reexports'] = stats.get('reexports', 0) + 1
    sc = [c * REC for c in h[:world]]
    rc = [h[world + 2 * r] * REC for r in range(world)]
    if stats is not None:
        rank = dist.get_rank(group)
        stats[phase + '_sent_rows'] = total - h[rank]
        stats[phase + '_self_rows'] = h[rank]
        stats[phase + '_recv_rows'] = sum(rc) // REC - h[world + 2 * rank]
    out = torch.empty(sum(rc), dtype=torch.uint8, device=buf.device)
    _all_to_all(out, buf[:total * REC], dist, group, rc, sc)
    return out


def _overflow(e):
    return getattr(e, 'code', None) == ShardOverflow.code


class _HostTransport(object):
    """rsa_transport over a torch.distributed group with host buffers: the
    library stages device data through pinned host memory and these callbacks
    run the group's collectives on CPU tensors viewing that memory (gloo)."""

    def __init__(self, dist, group, world, rank):
        from . import native
        self.dist, self.group, self.world = dist, group, world
        self.error = None
        self._ar = native.ALL_REDUCE_FN(self._all_reduce)
        self._a2a = native.ALL_TO_ALLV_FN(self._all_to_allv)
        self.t = native.Transport(None, world, rank, 1, self._ar, self._a2a)

    def _all_reduce(self, _self, buf, n, op, _stream):
        try:
            import torch
            t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(n,))) if n else torch.zeros(0, dtype=torch.int64)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op else self.dist.ReduceOp.SUM, group=self.group)
            return 0
        except BaseException as e:  # noqa: BLE001 - reported by merge() after the call returns
            self.error = e
            return 1

    def _all_to_allv(self, _self, send, sb, recv, rb, _stream):
        try:
            import torch
            sbl = [int(sb[r]) for r in range(self.world)]
            rbl = [int(rb[r]) for r in range(self.world)]

            def view(addr, n):
                if not n:
                    return torch.zeros(0, dtype=torch.uint8)
                return torch.from_numpy(np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(addr)))
            self.dist.all_to_all_single(view(recv, sum(rbl)), view(send, sum(sbl)), rbl, sbl, group=self.group)
            return 0
        except BaseException as e:  # noqa: BLE001
            self.error = e
            return 1


class _LoopbackTransport(object):
    """World 1 without a process group (merge(..., dist=None,
    force_exchange=True)): every collective over the library's pinned host
    buffers is an identity -- the all_reduce leaves the vector, the
    all_to_allv copies this rank's one segment to itself."""

    def __init__(self):
        from . import native
        self.error = None
        self._ar = native.ALL_REDUCE_FN(lambda _s, _buf, _n, _op, _st: 0)
        self._a2a = native.ALL_TO_ALLV_FN(self._copy)
        self.t = native.Transport(None, 1, 0, 1, self._ar, self._a2a)

    def _copy(self, _self, send, sb, recv, rb, _stream):
        n = int(sb[0])
        if n != int(rb[0]):
            return 1
        if n:
            ctypes.memmove(recv, send, n)
        return 0


def rccl_comm(eng, dist, group, world, rank):
    """The library's RCCL communicator for this engine and group (created once,
    collectively: rank 0's unique id is broadcast over the group)."""
    import torch
    from . import native
    key = (id(group), world, rank)
    have = getattr(eng, '_rccl_comm', None)
    if have is not None and have[0] == key:
        return have[1]
    lib = native.load()
    uid = (ctypes.c_uint8 * 128)()
    if rank == 0:
        rc = lib.rsa_rccl_unique_id(uid)
        if rc:
            raise native.NativeError(rc, 'rsa_rccl_unique_id failed (RCCL not found?)')
    t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=eng.device)
    dist.broadcast(t, 0, group=group)
    uid = (ctypes.c_uint8 * 128)(*t.cpu().tolist())
    comm = ctypes.c_void_p()
    eng.ctx.call('rsa_rccl_comm_create', ctypes.c_int32(world), ctypes.c_int32(rank), uid, ctypes.byref(comm))
    eng._rccl_comm = (key, comm)
    return comm


class _LibMerge(object):
    """One rank's side of rsa_merge / rsa_gather (the library's protocol)."""

    def __init__(self, eng, dist, group, world, rank, force_exchange=False):
        from . import native
        self.native, self.eng, self.world, self.rank = native, eng, world, rank
        self.flags = native.RSA_MERGE_ALWAYS_EXCHANGE if force_exchange else 0
        self.rccl = None
        self.host = None
        if dist is not None and world >= 1 and (world > 1 or force_exchange):
            if not _host_staged(dist, group):
                self.rccl = rccl_comm(eng, dist, group, world, rank)
            else:
                self.host = _HostTransport(dist, group, world, rank)
        elif dist is None and world == 1 and force_exchange:
            self.host = _LoopbackTransport()
        if self.host is None:
            # world 1 without a group, or RCCL: the struct is only read for world/rank
            self.t = native.Transport(None, world, rank, 1, native.ALL_REDUCE_FN(), native.ALL_TO_ALLV_FN())
        else:
            self.t = self.host.t

    def _check(self, rc, what, info=None):
        err = self.host.error if self.host is not None else None
        if self.host is not None:
            self.host.error = None
        if err is not None:
            raise err
        if rc == self.native.RSA_ERR_CAPACITY:
            msg = self.eng.ctx.lib.rsa_last_error(self.eng.ctx.h)
            raise ShardOverflow('%s: %s' % (what, msg.decode() if msg else ''),
                                needed=int(info.needed) if info is not None else 0)
        self.eng.ctx.check(rc, what)

    def merge(self, batches, gather, stats=None):
        from .engine import _ptr
        n = self.native
        arr = (n.ShardBatch * max(len(batches), 1))()
        for i, (b, g) in enumerate(batches):
            gid = b.gids if b.gids is not None else g
            arr[i] = n.ShardBatch(_ptr(b.tuples).value, _ptr(b.ts).value, _ptr(b.order).value, _ptr(gid).value, b.n)
        info = n.MergeInfo()
        flags = self.flags | (n.RSA_MERGE_GATHER if gather else 0)
        lib, h = self.eng.ctx.lib, self.eng.ctx.h
        if self.rccl is not None:
            rc = lib.rsa_merge_rccl(h, self.rccl, arr, len(batches), flags, ctypes.byref(info))
        else:
            rc = lib.rsa_merge(h, ctypes.byref(self.t), arr, len(batches), flags, ctypes.byref(info))
        self._check(rc, 'rsa_merge', info)
        if stats is not None:
            for ph in ('route1', 'route2'):
                if ph == 'route1' or info.pass2:
                    for k in ('sent', 'self', 'recv'):
                        stats['%s_%s_rows' % (ph, k)] = int(getattr(info, '%s_%s' % (ph, k)))
            stats['reexports'] = int(info.reexports)
            if self.world > 1 or self.flags:
                stats['allreduce_bytes'] = int(info.allreduce_bytes)
                stats['pass2'] = bool(info.pass2)
                stats['owner_rows'] = int(info.owner_rows)
                stats['gather_rows_to_rank0'] = int(info.gather_rows)
        return info

    def gather(self):
        info = self.native.MergeInfo()
        lib, h = self.eng.ctx.lib, self.eng.ctx.h
        if self.rccl is not None:
            rc = lib.rsa_gather_rccl(h, self.rccl, ctypes.byref(info))
        else:
            rc = lib.rsa_gather(h, ctypes.byref(self.t), ctypes.byref(info))
        self._check(rc, 'rsa_gather')
        return info

    def rows(self, which):
        """The last merge's own rows (0) or gathered rows (1) as a uint8 tensor."""
        import torch
        from .engine import _ptr
        nr = ctypes.c_uint64(0)
        lib, h = self.eng.ctx.lib, self.eng.ctx.h
        rc = lib.rsa_merge_rows(h, which, None, 0, ctypes.byref(nr))
        if rc not in (self.native.RSA_OK, self.native.RSA_ERR_CAPACITY):
            self.eng.ctx.check(rc, 'rsa_merge_rows')
        out = torch.empty(int(nr.value) * REC, dtype=torch.uint8, device=self.eng.device)
        if nr.value:
            self.eng.ctx.call('rsa_merge_rows', which, _ptr(out), nr, ctypes.byref(nr))
        return out


class OwnerRows(object):
    """merge(..., gather=False): this rank's own rules' final rows -- the
    counterpart of one Hadoop reducer's part file (runAnalysis.sh:42-56 runs
    NUM_REDUCERS reducers whose outputs stay separate files of the job's
    -output directory) -- with the merged counters and every rank's row bytes.
    gather_rows() collects them on rank 0 as merge() would have."""

    def __init__(self, final, sizes, matches, hits, distinct, thresh, lib=None):
        self.final, self.sizes = final, sizes
        self.matches, self.hits, self.distinct, self.thresh = matches, hits, distinct, thresh
        self.lib = lib     # _LibMerge of the library's protocol: it gathers (rsa_gather)


def gather_rows(part, dist, world, rank, group=None, to_host=True):
    """The owners' rows of merge(..., gather=False) on rank 0: merge()'s result
    there, None elsewhere."""
    import torch
    if part.lib is not None:
        part.lib.gather()
        if rank != 0:
            return None
        recs = part.lib.rows(1)
        out = (recs, part.matches, part.hits, part.distinct, part.thresh)
        return merged_to_host(out) if to_host else out
    parts = _gather0(part.final, part.sizes, rank, world, dist, group) if world > 1 else [part.final]
    if rank != 0:
        return None
    recs = parts[0] if world == 1 else torch.cat(parts)
    out = (recs, part.matches, part.hits, part.distinct, part.thresh)
    return merged_to_host(out) if to_host else out


def merge(backend, dist, world, rank, group=None, to_host=True, gather=True, stats=None, impl=None,
          force_exchange=False):
    """Run the protocol; returns (records, matches, hits, distinct, thresh) on
    rank 0 and None elsewhere: numpy arrays (records as RECORD_DTYPE rows), or
    with to_host=False the device tensors as they stand in rank 0's HBM
    (records as uint8 rows; see merged_to_host), which is where the
    single-GPU job leaves its result too.  gather=False: every rank returns
    its OwnerRows instead (the rows stay with their owners, as the
    reference's reducer outputs do; gather_rows collects them).

    One host read per phase: the route counts (with the overflow flag), the
    thresholds (with the import overflow need), the pass-2 route counts, and
    the gather sizes (riding on the distinct-count all_reduce).  At world 1
    there is no collective and no extra read: the shard's own cap resolution
    says whether pass 2 runs, as in the single-GPU job.  ``stats`` (a dict)
    receives the rows each exchange moved (route_records) and the collective
    bytes of the counter, threshold and size vectors.

    impl: 'lib' (the default for an EngineBackend) runs the protocol inside
    the library (rsa_merge); 'python' runs it here (the default for the CPU
    model backends).  force_exchange (lib): every collective runs even at
    world 1 (RSA_MERGE_ALWAYS_EXCHANGE, a one-GPU check of the transport)."""
    if impl is None:
        impl = 'lib' if isinstance(backend, EngineBackend) else 'python'
    if impl == 'lib':
        return _merge_lib(backend, dist, world, rank, group, to_host, gather, stats, force_exchange)
    import torch
    tr = _Trace(rank)
    c = backend.counters()
    dev = c['matches'].device
    tr('start', dev)
    n_rules = c['thresh'].numel()
    multi = world > 1
    if multi:
        # line and hit counters in one all_reduce
        mh = torch.cat([c['matches'], c['hits']])
        _all_reduce(mh, dist, group)
        c['matches'].copy_(mh[:n_rules])
        c['hits'].copy_(mh[n_rules:])
        others = (torch.arange(n_rules, device=dev) % world) != rank    # rules owned elsewhere
    tr('counters', dev)
    backend.set_owner(world, rank)
    try:
        failed = 0
        try:
            exported = backend.export(0)
        except Exception as e:  # noqa: BLE001 - a table overflow must not strand the other ranks
            if not _overflow(e):
                raise
            exported = Exported.empty(world, dev)
            failed = 1
        tr('export1', dev)
        if multi:
            recv = route_records(exported, world, dist, group, flag=failed, stats=stats, phase='route1')
            if recv is None:
                raise ShardOverflow('distinct-connection table overflow on at least one rank')
            tr('route1', dev)
            failed = 0
            if recv.numel():
                # the received entries join the owned ones: the thresholds of the
                # owned rules are resolved again over the merged entries (with
                # nothing received, the shard's own resolution already is that)
                try:
                    backend.import_records(recv, 0)
                    backend.resolve_cap()
                except Exception as e:  # noqa: BLE001
                    if not _overflow(e):
                        raise
                    # the table must hold the shard's entries and every received one
                    failed = max(backend.table_need(recv.numel() // REC), 1)
            tr('import1', dev)
            # thresholds of the owned rules (MAX: the others say "none" = -1),
            # with the overflow flag (the entries a failed table needs) riding along
            thresh = torch.cat([c['thresh'].masked_fill(others, NO_THRESHOLD),
                                torch.tensor([failed], dtype=torch.int64, device=dev)])
            _all_reduce(thresh, dist, group, op=dist.ReduceOp.MAX)
            capped_any, need = (int(x) for x in torch.stack([(thresh[:-1] != NO_THRESHOLD).any().to(torch.int64),
                                                             thresh[-1]]).cpu().tolist())
            if need:
                raise ShardOverflow('distinct-connection table overflow on at least one rank (merge import)',
                                    needed=need)
            thresh = thresh[:-1]
        else:
            if failed:
                raise ShardOverflow('distinct-connection table overflow')
            capped_any, thresh = backend.capped, c['thresh']
        tr('cap', dev)
        if capped_any:
            if multi:
                backend.set_thresh(thresh)
            backend.recount()
            if multi:
                recv2 = route_records(backend.export(1), world, dist, group, stats=stats, phase='route2')
                if recv2.numel():
                    backend.import_records(recv2, 1)
            tr('pass2', dev)
        final = backend.emit_final()
        if multi:
            # the distinct counts of the owned rules and every rank's row
            # bytes (for the gather) in one all_reduce, one host read
            dsz = torch.zeros(n_rules + world, dtype=torch.int64, device=dev)
            dsz[:n_rules] = c['distinct'].masked_fill(others, 0).to(torch.int64)
            dsz[n_rules + rank] = final.numel()
            _all_reduce(dsz, dist, group)
            distinct = dsz[:n_rules].to(c['distinct'].dtype)
        else:
            distinct = c['distinct']
        tr('emit', dev)
    finally:
        backend.set_owner(0, 0)
    sizes = [int(s) for s in dsz[n_rules:].cpu().tolist()] if multi else [final.numel()]
    if stats is not None and multi:
        # all_reduce payloads: line+hit counters, thresholds (+ flag), distinct counts + row sizes
        stats['allreduce_bytes'] = 8 * (2 * n_rules + (n_rules + 1) + (n_rules + world))
        stats['pass2'] = bool(capped_any)
        stats['owner_rows'] = final.numel() // REC
        stats['gather_rows_to_rank0'] = sum(sizes[1:]) // REC
    if not gather:
        tr('end', dev)
        return OwnerRows(final, sizes, c['matches'], c['hits'], distinct, thresh)
    # the owners' rows to rank 0
    if multi:
        parts = _gather0(final, sizes, rank, world, dist, group)
    else:
        parts = [final]
    tr('gather', dev)
    if rank != 0:
        tr('end')
        return None
    recs = parts[0] if world == 1 else torch.cat(parts)
    out = (recs, c['matches'], c['hits'], distinct, thresh)
    if to_host:
        out = merged_to_host(out)
    tr('end', dev)
    return out


def _merge_lib(backend, dist, world, rank, group, to_host, gather, stats, force_exchange):
    """merge() through rsa_merge: the library runs the whole sequence; the
    counters it merged stay in the engine's bound tensors."""
    eng = backend.eng
    lm = _LibMerge(eng, dist, group, world, rank, force_exchange=force_exchange)
    tr = _Trace(rank)
    tr('start', eng.device)
    lm.merge(list(zip(backend.batches, backend.gid_bufs)), gather=False, stats=stats)
    tr('merge', eng.device)
    c = eng.counters
    part = OwnerRows(lm.rows(0), None, c['matches'], c['hits'], c['distinct'], c['thresh'], lib=lm)
    if not gather:
        tr('end', eng.device)
        return part
    out = gather_rows(part, dist, world, rank, group, to_host=to_host)
    tr('end', eng.device)
    return out


def merged_to_host(out):
    """merge(..., to_host=False)'s device tensors as merge()'s numpy result."""
    if out is None or isinstance(out[0], np.ndarray):
        return out
    recs, matches, hits, distinct, thresh = out
    return (recs.cpu().numpy().view(RECORD_DTYPE).copy(), matches.cpu().numpy().view(np.uint64).copy(),
            hits.cpu().numpy().view(np.uint64).copy(), distinct.cpu().numpy().view(np.uint32).copy(),
            thresh.cpu().numpy().view(np.uint64).copy())


class EngineBackend(object):
    """Binds the protocol to this rank's HIP context: ``eng`` holds the
    shard's pass-1 table (and, during the merge, the merged entries of the
    rules this rank owns)."""

    def __init__(self, eng, batches, gid_bufs, cap):
        self.eng = eng
        self.world = 0
        self.batches = batches
        self.gid_bufs = gid_bufs
        self.cap = cap
        self.capped = 0     # rules the shard's own cap resolution (export(0)) found capped

    def counters(self):
        return self.eng.counters

    def set_owner(self, world, rank):
        from . import native
        self.world = world
        self.eng.set_option(native.RSA_OPT_OWNER_WORLD, world)
        self.eng.set_option(native.RSA_OPT_OWNER_RANK, rank)

    def export(self, which):
        """Entries of rules owned elsewhere, grouped by owner (``Exported``):
        which 0 = the pass-1 aggregates that can still reach the report (after
        the shard's own cap resolution), 1 = the pass-2 sums.  A single rank
        owns every rule: nothing to scan for."""
        if which == 0:
            self.capped = self.eng.resolve_cap()
        dev = self.eng.device
        if self.world == 1:
            return Exported.empty(1, dev)
        mode = 'pass1_kept' if which == 0 else 'pass2'
        buf, counts, cap = self.eng.export_routed(mode, self.world)
        return Exported(buf, counts, cap, lambda n: self.eng.export_routed(mode, self.world, capacity=n))

    def import_records(self, buf, which):
        self.eng.import_records(buf, which)

    def table_need(self, n_received):
        """Entries the table needs to hold this shard's pass-1 entries and
        n_received imported records (each possibly new)."""
        return self.eng.table_size() + int(n_received)

    def resolve_cap(self):
        return self.eng.resolve_cap()

    def set_thresh(self, thresh):
        self.eng.counters['thresh'].copy_(thresh)

    def recount(self):
        for b, g in zip(self.batches, self.gid_bufs):
            self.eng.pass2(b, g)

    def emit_final(self):
        return self.eng.emit_device('final')
