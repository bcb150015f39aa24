"""The partial-key bucket index (ruleset-analysis_amd/bucketindex.py, image
RSA5): its host model of the device lookup gives the brute-force first match
(min gid over the compiled candidate lists, the reference's mapper.py:168-189
scan) on ASA-shaped and FortiGate-shaped (run-compressed, chained) lists."""
import numpy as np
import pytest

from cpu_model import classify_entries
from ruleset_analysis_amd import acldb, bucketindex as bi, fortigate, synth, synth_fg
from ruleset_analysis_amd.compile import CompiledRules, PHT_LIST_WORDS, _records


def _check(index, ent, off, tup, every=1):
    want = classify_entries(ent, off, tup)
    n = 0
    for i in range(0, len(tup), every):
        t = tup[i]
        if not t['flags'] & 1:
            continue
        g = bi.bucket_lookup(index, ent, off, int(t['list']), int(t['src']), int(t['dst']),
                             int(t['sport']) | (int(t['dport']) << 16))
        assert g == want[i], i
        n += 1
    return n


@pytest.mark.parametrize('kind', ['bucket', 'bucket-filtered'])
@pytest.mark.parametrize('broad,prefix', [(False, 0), (True, 0), (False, 16)])
def test_lookup_equals_scan_asa(broad, prefix, kind):
    dbj, info = synth.make_db(71, 3000, interfaces=('outside', 'partner'), broad=broad)
    comp = CompiledRules(acldb.load_json(dbj))
    comp.ensure_lists()
    ent, off = comp.packed()
    index = comp.index(prefix=prefix, kind=kind)
    assert int(index[0][1]) == bi.BKT_MAGIC
    st = bi.bucket_stats(index)
    assert sum(s[1] for s in st) >= 4 and sum(s[3] for s in st) > 0.9 * len(ent) - sum(s[2] for s in st) - 64
    tr = synth.make_traffic((dbj, info), 12000, seed=72, p_unmatched=0.3)
    tup, _ts, _o = synth.pack(tr, comp)
    assert _check(index, ent, off, tup) > 8000


@pytest.mark.parametrize('kind', ['bucket', 'bucket-filtered'])
def test_lookup_equals_scan_fortigate_chained(kind):
    """Run-compressed stepped entries (gid depends on the port) and lists
    chained over records of 700 entries."""
    text, info = synth_fg.make_config(7, n_policies=30, n_wide=1, n_mid=1, n_syslog=2, wide_members=(2, 3))
    comp = CompiledRules(fortigate.build_db(text))
    comp.ensure_lists()
    ent, off = comp.packed()
    assert (ent['step'] != 0).sum() > 5
    index = comp.index(chunk=700, kind=kind)
    recs = _records(index[0])
    assert len(recs) > len(off) - 1                       # chained records exist
    tr = synth_fg.make_traffic(info, 4000, seed=8)
    tup, _ts, _o = synth.pack(tr, comp)
    assert _check(index, ent, off, tup) > 2000


def test_image_invariants():
    """What rsa_load_index validates: tables in ascending min gid, buckets
    inside the image, every slot's rows inside the residual array and
    first-gid ascending, record entry ranges covering each list."""
    dbj, info = synth.make_db(73, 2000, broad=False)
    comp = CompiledRules(acldb.load_json(dbj))
    comp.ensure_lists()
    ent, off = comp.packed()
    image, resid = comp.index(kind='bucket-filtered')
    assert int(image[5]) == 1
    words = len(image)
    for r in _records(image):
        prev = 0
        for j in range(r[1]):
            t = [int(v) for v in image[r[0] + bi.BKT_TABLE_WORDS * j: r[0] + bi.BKT_TABLE_WORDS * (j + 1)]]
            sm, dm, pm, boff, nb, foff, mg, base = t
            assert mg >= prev and 1 <= nb <= 0x10000 and boff % 2 == 0 and boff + 2 * nb <= words
            prev = mg
            for s in range(2 * nb):
                w = int(image[boff + s])
                ln = (w >> 16) & 0x1F
                if ln:
                    rows = resid[base + (w & 0xFFFF): base + (w & 0xFFFF) + ln]
                    assert len(rows) == ln and (np.diff(rows['gid'].astype(np.int64)) >= 0).all()
                    # every row of the bucket has the bucket's key under the template
                    keys = {(int(x['src_lo']) & sm, int(x['dst_lo']) & dm, int(x['port_lo']) & pm) for x in rows}
                    assert len(keys) == 1
                    h = bi.bkt_hash(*[np.uint32(k) for k in keys.pop()], bi.SEED_KEY)
                    assert foff + (w & 0xFFFF) + ln <= words
                    f = image[foff + (w & 0xFFFF): foff + (w & 0xFFFF) + ln]
                    assert np.array_equal(f, bi.row_filters(rows))
                    b1, b2, tag = (int(x) for x in bi.bkt_buckets(h, nb))
                    assert s // 2 in (b1, b2) and (w >> 21) == tag
    assert PHT_LIST_WORDS == 20


def test_hash_matches_device_constants():
    """bkt_hash / bkt_buckets as include/ruleset_hip.h states them."""
    from ruleset_analysis_amd.compile import fmix32
    ks, kd, kp, seed = 0x0B000000, 0x0A000100, 0x00500000, bi.SEED_KEY
    x = (ks ^ ((kd * 0x9E3779B1) & 0xFFFFFFFF) ^ ((kp * 0x85EBCA77) & 0xFFFFFFFF) ^ seed) & 0xFFFFFFFF
    h = int(fmix32(np.uint32(x)))
    assert h == int(bi.bkt_hash(np.uint32(ks), np.uint32(kd), np.uint32(kp), seed))
    b1, b2, tag = (int(v) for v in bi.bkt_buckets(np.uint32(h), 1000))
    assert (b1, b2, tag) == (((h & 0xFFFF) * 1000) >> 16, ((h >> 16) * 1000) >> 16, ((h >> 16) ^ h) & 0x7FF)


def test_row_filter_passes_every_contained_connection():
    """A row's filter never rejects a connection the row contains (it only
    checks bits the row is exact on), and rejects most others."""
    dbj, info = synth.make_db(74, 1500, broad=True)
    comp = CompiledRules(acldb.load_json(dbj))
    comp.ensure_lists()
    ent, off = comp.packed()
    f = bi.row_filters(ent)
    tr = synth.make_traffic((dbj, info), 3000, seed=75)
    tup, _ts, _o = synth.pack(tr, comp)
    from ruleset_analysis_amd.compile import _match
    rng = np.random.default_rng(76)
    passed = rejected = 0
    for i in rng.choice(len(tup), 400, replace=False):
        t = tup[i]
        ports = int(t['sport']) | (int(t['dport']) << 16)
        L = int(t['list'])
        for k in range(int(off[L]), int(off[L + 1])):
            ok = bi.row_passes(int(f[k]), int(t['src']), int(t['dst']), ports)
            if _match(ent[k], int(t['src']), int(t['dst']), ports):
                assert ok
                passed += 1
            elif not ok:
                rejected += 1
    assert passed > 100 and rejected > 0
