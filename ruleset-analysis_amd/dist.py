"""Multi-GPU merge — the MI355X replacement of the Hadoop shuffle
(``runAnalysis.sh:42-56``: map output partitioned by key hash to 4 reducers).

One process per GPU (``torch.distributed``; backend ``nccl`` = RCCL over xGMI
on the GPU box, ``gloo`` in the CPU tests).  Every rank classifies and
aggregates its own contiguous shard of the log (pass 1, rule tables
replicated).  Then:

1. ``all_reduce(SUM)`` of the per-rule line and hit counters;
2. ``all_to_all`` of the compacted (rule, connection) pass-1 records to the
   owner rank ``gid % world`` (the reducer partitioning), where they are merged
   (count sum, first-seen min, last-seen max, min order key);
3. each owner resolves the cap for its rules; ``all_reduce(MAX)`` of the
   threshold vector gives every rank every rule's threshold P;
4. if any rule is capped: every rank recounts its shard's occurrences with
   order <= P (pass 2), the pass-2 records go to the owners by ``all_to_all``
   and are summed there;
5. the owners' final records are gathered to rank 0 for emission.

The order keys are global, so the cap logic is shard-agnostic.  Records are
40-byte ``rsa_conn_record`` rows moved as uint8 tensors; routing uses torch
index ops only.
"""

import numpy as np

from .compile import RECORD_DTYPE

__all__ = ['merge', 'EngineBackend', 'route_records']

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


def torch_empty_like_cpu(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype)


def route_records(buf, world, dist, group=None):
    """all_to_all of record bytes to owner rank gid % world; returns received bytes."""
    import torch
    n = buf.numel() // REC
    rows = buf.view(-1, REC)
    gid = rows[:, 8:12].contiguous().view(torch.int32).view(-1).to(torch.int64) if n else \
        torch.zeros(0, dtype=torch.int64, device=buf.device)
    owner = gid % world
    perm = torch.argsort(owner, stable=True)
    send = rows[perm].contiguous().view(-1)
    counts = torch.bincount(owner, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(counts)
    _all_to_all(recv_counts, counts, dist, group)
    sc = [int(c) * REC for c in counts.cpu().tolist()]
    rc = [int(c) * REC for c in recv_counts.cpu().tolist()]
    out = torch.empty(sum(rc), dtype=torch.uint8, device=buf.device)
    _all_to_all(out, send, dist, group, rc, sc)
    return out


def merge(backend, dist, world, rank, group=None):
    """Run the protocol; returns (records ndarray, matches, hits, distinct, thresh) on
    rank 0 and None elsewhere."""
    import torch
    c = backend.local_counters()
    _all_reduce(c['matches'], dist, group)
    _all_reduce(c['hits'], dist, group)
    recv = route_records(backend.export(0), world, dist, group)
    backend.owner_reset(max(recv.numel() // REC, 1))
    backend.owner_import(recv, 0)
    backend.owner_resolve_cap()
    oc = backend.owner_counters()
    thresh = oc['thresh'].clone()
    _all_reduce(thresh, dist, group, op=dist.ReduceOp.MAX)
    capped_any = bool((thresh != NO_THRESHOLD).any().item())
    if capped_any:
        backend.set_local_thresh(thresh)
        backend.local_recount()
        recv2 = route_records(backend.export(1), world, dist, group)
        backend.owner_import(recv2, 1)
        backend.set_owner_thresh(thresh)
    final = backend.owner_emit()
    distinct = oc['distinct'].clone()
    _all_reduce(distinct, dist, group)
    # gather the owners' rows to rank 0 (padded all_gather: sizes first)
    size = torch.tensor([final.numel()], dtype=torch.int64, device=final.device)
    sizes = [torch.zeros_like(size) for _ in range(world)]
    _all_gather(sizes, size, dist, group)
    sizes = [int(s.item()) for s in sizes]
    pad = max(max(sizes), 1)
    padded = torch.zeros(pad, dtype=torch.uint8, device=final.device)
    padded[:final.numel()] = final
    parts = [torch.empty(pad, dtype=torch.uint8, device=final.device) for _ in range(world)]
    _all_gather(parts, padded, dist, group)
    if rank != 0:
        return None
    recs = np.concatenate([p[:s].cpu().numpy() for p, s in zip(parts, sizes)]).view(RECORD_DTYPE)
    return (recs.copy(), c['matches'].cpu().numpy().view(np.uint64).copy(),
            c['hits'].cpu().numpy().view(np.uint64).copy(), distinct.cpu().numpy().view(np.uint32).copy(),
            thresh.cpu().numpy().view(np.uint64).copy())


class EngineBackend(object):
    """Binds the protocol to two HIP contexts on this rank's GPU: ``local`` holds
    the shard's pass-1 table, ``owner`` the merged table of the rules this rank
    owns."""

    def __init__(self, local, owner, batches, gid_bufs, cap):
        self.local = local
        self.owner = owner
        self.batches = batches
        self.gid_bufs = gid_bufs
        self.cap = cap

    def local_counters(self):
        return self.local.counters

    def export(self, which):
        return self.local.emit_device('pass1' if which == 0 else 'pass2')

    def owner_reset(self, capacity):
        self.owner.reset(capacity, self.cap)

    def owner_import(self, buf, which):
        self.owner.import_records(buf, which)

    def owner_resolve_cap(self):
        return self.owner.resolve_cap()

    def owner_counters(self):
        return self.owner.counters

    def set_local_thresh(self, thresh):
        self.local.counters['thresh'].copy_(thresh)

    def set_owner_thresh(self, thresh):
        self.owner.counters['thresh'].copy_(thresh)

    def local_recount(self):
        for b, g in zip(self.batches, self.gid_bufs):
            self.local.pass2(b, g)

    def owner_emit(self):
        return self.owner.emit_device('final')
