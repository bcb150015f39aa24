"""The host-buffer rsa_transport of dist.py (the callbacks rsa_merge calls for
a gloo group): two gloo ranks on the CPU call the struct's function pointers
the way csrc/merge.hip does -- pinned-host-like ctypes buffers, per-rank byte
counts -- and get the collectives' results in those buffers."""
import ctypes
import os

import numpy as np
import torch.multiprocessing as mp

from test_dist_merge import _free_port


def _worker(rank, world, port, out_q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from ruleset_analysis_amd.dist import _HostTransport
    ht = _HostTransport(dist, None, world, rank)
    t = ht.t
    res = {}
    # all_reduce SUM and MAX over int64 in place
    a = (ctypes.c_int64 * 5)(*[rank * 10 + i for i in range(5)])
    assert t.all_reduce_i64(None, a, 5, 0, None) == 0
    res['sum'] = list(a)
    b = (ctypes.c_int64 * 3)(-1, rank, -1 if rank else 7)
    assert t.all_reduce_i64(None, b, 3, 1, None) == 0
    res['max'] = list(b)
    # all_to_allv: rank r sends (r + 1) * (p + 1) bytes of value 16 r + p to rank p
    sb = [(rank + 1) * (p + 1) for p in range(world)]
    rb = [(p + 1) * (rank + 1) for p in range(world)]
    send = (ctypes.c_uint8 * sum(sb))(*[16 * rank + p for p in range(world) for _ in range(sb[p])])
    recv = (ctypes.c_uint8 * sum(rb))()
    SB, RB = (ctypes.c_uint64 * world)(*sb), (ctypes.c_uint64 * world)(*rb)
    assert t.all_to_allv(None, ctypes.addressof(send), SB, ctypes.addressof(recv), RB, None) == 0
    res['recv'] = list(recv)
    # a gather-shaped exchange: only rank 0 receives; empty segments elsewhere
    gs = [3] + [0] * (world - 1)
    gr = [3] * world if rank == 0 else [0] * world
    gsend = (ctypes.c_uint8 * 3)(rank, rank, rank)
    grecv = (ctypes.c_uint8 * max(sum(gr), 1))()
    assert t.all_to_allv(None, ctypes.addressof(gsend), (ctypes.c_uint64 * world)(*gs),
                         ctypes.addressof(grecv), (ctypes.c_uint64 * world)(*gr), None) == 0
    res['gather'] = list(grecv)[:sum(gr)]
    # a failing collective reports 1 and keeps the exception for merge()
    assert t.all_reduce_i64(None, ctypes.POINTER(ctypes.c_int64)(), 4, 0, None) == 1 and ht.error is not None
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_host_transport_two_ranks():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r]['sum'] == [sum(k * 10 + i for k in range(world)) for i in range(5)]
        assert got[r]['max'] == [-1, world - 1, 7]
        want = [16 * p + r for p in range(world) for _ in range((p + 1) * (r + 1))]
        assert got[r]['recv'] == want
    assert got[0]['gather'] == [0, 0, 0, 1, 1, 1]
    assert got[1]['gather'] == []
    assert np.all(np.array(got[0]['sum']) == np.array(got[1]['sum']))
