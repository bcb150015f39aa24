"""Seeded synthetic rule databases and ASA connection logs.

Nothing here comes from the reference: it ships no logs, configs or fixtures
(``.gitignore:48-51``).  The generators follow the reference's data shapes:

* ``make_db`` writes what ``preprosess_access_lists.py`` would store for
  ASA ``access-list NAME extended ...`` lines: each line is expanded to
  ``|dport| x |dst| x |sport| x |src|`` ``FirewallRule`` records with dport
  outermost (``preprosess_access_lists.py:256-276``), ``rulenum`` = line number,
  ``ruleindex`` = list position (``:466-487``), and ``protocols`` maps each
  protocol to its rule indices (``:489-494``).  Every ACL ends with
  ``deny ip any any`` so the ``'ip'`` list the mapper indexes unconditionally
  for tcp/udp (``mapper.py:161,164``) exists.
* ``make_traffic`` draws connection tuples, mostly inside some permit rule
  (so the first match is spread over the ACL) plus unmatched noise, and a mix
  of message forms that exercise the reducer's edge cases: non-hit message ids
  (``connlist-reducer.py:146``), lines the BUILT regex rejects (``:152``),
  lines the mapper ignores, interfaces without an ACL (``mapper.py:145-149``)
  and outbound connections (reducer key swapped relative to the tuple).
* ``render_lines`` produces the log text; ``pack`` produces the packed tuples
  directly (what the host parser would produce from that text) for sizes where
  text is pointless — ``tests/test_synth_pack.py`` pins the two against each
  other.

All arrays are numpy; generation is vectorised so 10^8-line workloads build in
seconds.
"""

import numpy as np

__all__ = ['make_db', 'make_traffic', 'make_traffic_population', 'render_lines', 'pack', 'order_keys', 'ts_decode',
           'PSPELL', 'FORM_NAMES', 'COMMON_PORTS']

COMMON_PORTS = np.array([80, 443, 22, 25, 53, 123, 389, 445, 636, 993, 1433, 3306, 3389, 5432, 8080, 8443],
                        dtype=np.int64)
PREFIX_MASKS = {8: '255.0.0.0', 16: '255.255.0.0', 20: '255.255.240.0', 24: '255.255.255.0',
                28: '255.255.255.240', 30: '255.255.255.252'}

# message forms (per line)
F_BUILT, F_NONHIT, F_NOYEAR, F_TEARDOWN, F_NOACL, F_OUTBOUND = range(6)
FORM_NAMES = ['built', 'nonhit', 'noyear', 'teardown', 'noacl', 'outbound']


def _dotted(v):
    v = int(v)
    return '%d.%d.%d.%d' % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)


class _AddrSpace(object):
    """Address pools: internal servers live in 10/8, clients in 'public' space."""

    def __init__(self, rng, n_clients=4096, n_servers=2048):
        self.clients = np.unique(rng.integers(0x0B000000, 0xDF000000, size=n_clients * 2, dtype=np.int64))
        rng.shuffle(self.clients)
        self.clients = self.clients[:n_clients]
        self.servers = np.unique(rng.integers(0x0A000000, 0x0AFFFFFF, size=n_servers * 2, dtype=np.int64))
        rng.shuffle(self.servers)
        self.servers = self.servers[:n_servers]


def _addr_item(rng, pool, plens):
    """One address spec item -> (preprocessor text, net int, prefixlen)."""
    base = int(pool[rng.integers(len(pool))])
    plen = int(rng.choice(plens))
    if plen == 32:
        return _dotted(base), base, 32
    net = base & ~((1 << (32 - plen)) - 1) & 0xFFFFFFFF
    return '%s/%s' % (_dotted(net), PREFIX_MASKS[plen]), net, plen


def _addr_spec(rng, pool, p_any, p_host, p_net, p_group, net_plens):
    """Returns (acl text fragment, [(text, net, plen), ...])."""
    u = rng.random()
    if u < p_any:
        return 'any', [('any', 0, 0)]
    u -= p_any
    if u < p_host:
        t, n, l = _addr_item(rng, pool, [32])
        return 'host ' + t, [(t, n, l)]
    u -= p_host
    if u < p_net:
        t, n, l = _addr_item(rng, pool, net_plens)
        return t.replace('/', ' '), [(t, n, l)]
    k = int(rng.integers(2, 5))
    items, seen = [], set()
    for _ in range(k):
        it = _addr_item(rng, pool, [32] + list(net_plens))
        if it[0] not in seen:
            seen.add(it[0])
            items.append(it)
    return 'object-group GRP%d' % int(rng.integers(1 << 30)), items


def _acl_lines(rng, space, acl, n_rules, kind, broad=True):
    """Generate ACL lines until ~n_rules expanded rules; returns rule dicts and meta.

    ``broad=False`` redraws the destination of any permit whose source and
    destination are both ``any`` (so no early catch-all permit shadows the rest
    of the list and traffic drawn from a rule first-matches at or near it)."""
    rules, meta = [], []
    lineno = 0
    target = max(2, int(n_rules))
    while len(rules) < target - 1:
        lineno += 1
        action = bool(rng.random() < 0.85)
        proto = str(rng.choice(['tcp', 'udp', 'ip'], p=[0.6, 0.25, 0.15]))
        if kind == 'inside':
            s_txt, srcs = _addr_spec(rng, space.servers, 0.1, 0.3, 0.6, 0.0, [16, 24])
            d_txt, dsts = _addr_spec(rng, space.clients, 0.6, 0.2, 0.2, 0.0, [16, 24])
        else:
            s_txt, srcs = _addr_spec(rng, space.clients, 0.40, 0.25, 0.25, 0.10, [8, 16, 24])
            d_txt, dsts = _addr_spec(rng, space.servers, 0.12, 0.55, 0.23, 0.10, [24, 28])
            while not broad and action and s_txt == 'any' and d_txt == 'any':
                d_txt, dsts = _addr_spec(rng, space.servers, 0.12, 0.55, 0.23, 0.10, [24, 28])
        sports, dports, sp_txt, dp_txt = [], [], '', ''
        if proto in ('tcp', 'udp'):
            if rng.random() < 0.04:
                p = int(rng.choice(COMMON_PORTS))
                sports, sp_txt = [p], ' eq %d' % p
            u = rng.random()
            if u < 0.70:
                p = int(rng.choice(COMMON_PORTS)) if rng.random() < 0.7 else int(rng.integers(1, 65536))
                dports, dp_txt = [p], ' eq %d' % p
            elif u < 0.82:
                lo = int(rng.integers(1024, 60000))
                hi = lo + int(rng.integers(1, 6))
                dports, dp_txt = list(range(lo, hi + 1)), ' range %d %d' % (lo, hi)
        size = max(1, len(dports)) * len(dsts) * max(1, len(sports)) * len(srcs)
        if len(rules) + size > target - 1:
            if size > 1:
                continue
        text = 'access-list %s extended %s %s %s%s %s%s' % (acl, 'permit' if action else 'deny', proto, s_txt,
                                                            sp_txt, d_txt, dp_txt)
        for dp in (dports or [-1]):
            for d in dsts:
                for sp in (sports or [-1]):
                    for s in srcs:
                        rules.append({'action': action, 'protocol': proto, 'original': text, 'src': s[0],
                                      'dst': d[0], 'sport': [sp], 'dport': [dp], 'comments': [],
                                      'rulenum': lineno, 'ruleindex': len(rules)})
                        meta.append((action, proto, s[1], s[2], d[1], d[2], sp, dp))
    lineno += 1
    text = 'access-list %s extended deny ip any any' % acl
    rules.append({'action': False, 'protocol': 'ip', 'original': text, 'src': 'any', 'dst': 'any',
                  'sport': [-1], 'dport': [-1], 'comments': [], 'rulenum': lineno, 'ruleindex': len(rules)})
    meta.append((False, 'ip', 0, 0, 0, 0, -1, -1))
    protocols = {}
    for r in rules:
        protocols.setdefault(r['protocol'], []).append(r['ruleindex'])
    return rules, protocols, meta


def make_db(seed, n_rules, host='fw1', interfaces=('outside',), inside_rules=16, with_inside=True, broad=True):
    """Seeded rule DB (JSON-able dict) plus per-ACL numeric rule metadata.

    ``broad``: allow ``permit ... any ... any`` lines anywhere in the outside
    ACLs (they shadow everything after them: short scans).  The bench
    workloads use ``broad=False`` — first matches spread over the whole list.

    ``interfaces``: each gets its own ``<ifc>_access_in`` ACL of ``n_rules``
    expanded rules bound ``in``.  ``with_inside`` adds a small
    ``inside_access_in`` for outbound connections.
    """
    rng = np.random.default_rng(seed)
    space = _AddrSpace(rng)
    firewalls = {host: {}}
    acls, meta = {}, {}
    for ifc in interfaces:
        acl = '%s_access_in' % ifc
        rules, protos, m = _acl_lines(rng, space, acl, n_rules, 'outside', broad=broad)
        acls[acl] = {'rules': rules, 'protocols': protos, 'timestamp': 1373846400.0}
        meta[acl] = m
        firewalls[host][ifc] = {'in': acl}
    if with_inside:
        acl = 'inside_access_in'
        rules, protos, m = _acl_lines(rng, space, acl, inside_rules, 'inside')
        acls[acl] = {'rules': rules, 'protocols': protos, 'timestamp': 1373846400.0}
        meta[acl] = m
        firewalls[host]['inside'] = {'in': acl}
    db = {'firewalls': firewalls, 'accesslists': {host: acls}}
    return db, {'space': space, 'meta': meta, 'host': host, 'interfaces': list(interfaces),
                'with_inside': with_inside}


def _sample_in(rng, net, plen, n, pool, cap=256):
    """n addresses inside net/plen (plen 0 -> from pool); at most `cap` distinct."""
    if plen == 0:
        return pool[rng.integers(0, len(pool), size=n)]
    size = 1 << (32 - plen)
    return net + rng.integers(0, min(size, cap), size=n)


def make_traffic(db_and_info, n, seed, form_probs=(0.86, 0.04, 0.04, 0.03, 0.02, 0.01), p_unmatched=0.10,
                 t0=15 * 86400, span=3 * 3600, zipf=None, cid0=1000000):
    """Connection tuples + message forms, as numpy arrays (one entry per line).

    Returns dict with int64 arrays src, dst, sport, dport, proto (0 tcp 1 udp),
    ifc (index into info['interfaces'] for inbound forms), form, t (seconds
    from Jul 1 00:00:00), cid.
    """
    db, info = db_and_info
    rng = np.random.default_rng(seed)
    space = info['space']
    ifcs = info['interfaces']
    form = rng.choice(len(form_probs), size=n, p=np.asarray(form_probs) / np.sum(form_probs))
    if not info['with_inside']:
        form[form == F_OUTBOUND] = F_BUILT
    ifc = rng.integers(0, len(ifcs), size=n)
    src = np.zeros(n, np.int64)
    dst = np.zeros(n, np.int64)
    sport = rng.integers(1024, 65536, size=n)
    dport = COMMON_PORTS[rng.integers(0, len(COMMON_PORTS), size=n)]
    proto = (rng.random(n) < 0.3).astype(np.int64)
    # inbound lines: draw from a permit rule of the ACL on the chosen interface
    for k, name in enumerate(ifcs):
        meta = info['meta']['%s_access_in' % name]
        permits = np.array([i for i, m in enumerate(meta) if m[0]], dtype=np.int64)
        sel = np.nonzero((ifc == k) & (form != F_OUTBOUND))[0]
        if len(sel) == 0 or len(permits) == 0:
            continue
        if zipf:
            ranks = np.minimum(rng.zipf(zipf, size=len(sel)) - 1, len(permits) - 1)
            perm = rng.permutation(len(permits))
            pick = permits[perm[ranks]]
        else:
            pick = permits[rng.integers(0, len(permits), size=len(sel))]
        m = np.array(meta, dtype=object)
        sn = np.array([int(x) for x in m[:, 2]], np.int64)
        sl = np.array([int(x) for x in m[:, 3]], np.int64)
        dn = np.array([int(x) for x in m[:, 4]], np.int64)
        dl = np.array([int(x) for x in m[:, 5]], np.int64)
        sp = np.array([int(x) for x in m[:, 6]], np.int64)
        dp = np.array([int(x) for x in m[:, 7]], np.int64)
        pr = np.array([{'tcp': 0, 'udp': 1}.get(x, -1) for x in m[:, 1]], np.int64)
        r = pick
        for plen in np.unique(sl[r]):
            w = sl[r] == plen
            src[sel[w]] = _sample_in(rng, sn[r][w], plen, int(w.sum()), space.clients)
        for plen in np.unique(dl[r]):
            w = dl[r] == plen
            dst[sel[w]] = _sample_in(rng, dn[r][w], plen, int(w.sum()), space.servers)
        has_sp = sp[r] >= 0
        sport[sel[has_sp]] = sp[r][has_sp]
        has_dp = dp[r] >= 0
        dport[sel[has_dp]] = dp[r][has_dp]
        fixed = pr[r] >= 0
        proto[sel[fixed]] = pr[r][fixed]
        # unmatched noise: random everything
        un = sel[rng.random(len(sel)) < p_unmatched]
        src[un] = space.clients[rng.integers(0, len(space.clients), size=len(un))]
        dst[un] = rng.integers(0x0A000000, 0x0B000000, size=len(un))
        dport[un] = rng.integers(1, 65536, size=len(un))
    ob = np.nonzero(form == F_OUTBOUND)[0]
    src[ob] = space.servers[rng.integers(0, len(space.servers), size=len(ob))]
    dst[ob] = space.clients[rng.integers(0, len(space.clients), size=len(ob))]
    t = t0 + (np.arange(n, dtype=np.int64) * span) // max(n, 1)
    cid = cid0 + np.arange(n, dtype=np.int64)
    return {'src': src, 'dst': dst, 'sport': sport, 'dport': dport, 'proto': proto, 'ifc': ifc, 'form': form,
            't': t, 'cid': cid, 'interfaces': list(ifcs), 'host': info['host']}


def _mix64(x, salt):
    """splitmix64 finaliser of (x + salt) over uint64 arrays (per-rank streams)."""
    with np.errstate(over='ignore'):
        z = np.asarray(x, np.uint64) + np.uint64(salt) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def zipf_ranks(rng, n, s, population):
    """n ranks in [0, population) with P(rank = k) ~ (k + 1)^-s: numpy's
    unbounded Zipf draws, those beyond the population drawn again."""
    out = rng.zipf(s, size=n).astype(np.int64) - 1
    bad = np.nonzero(out >= population)[0]
    while len(bad):
        out[bad] = rng.zipf(s, size=len(bad)).astype(np.int64) - 1
        bad = bad[out[bad] >= population]
    return out


def make_traffic_population(db_and_info, n, seed, s=1.1, population=10 ** 8,
                            form_probs=(0.86, 0.04, 0.04, 0.03, 0.02, 0.01), p_unmatched=0.10,
                            t0=15 * 86400, span=3 * 3600, cid0=1000000, pop_seed=None):
    """BASELINE config 5's traffic: every line's connection --
    interface, protocol, (src, dst, dport) -- is connection number r of a
    fixed population of ``population`` connections, r drawn Zipf(s) per line,
    so hot connections repeat (the many-occurrences-of-one-key path of the
    reducer dict, ``connlist-reducer.py:167-172``) while rules with a large
    share of the population go far past the cap.  Connection r is a pure
    function of r (splitmix64 streams): it lies inside a permit rule of the
    ACL of its interface (one of ``p_unmatched`` of them is random noise);
    the source port, message form and time stay per line.  Same dict layout
    as ``make_traffic``.  ``pop_seed`` (default ``seed``) fixes the
    population: chunks of one log drawn with different ``seed`` and the same
    ``pop_seed`` share it."""
    db, info = db_and_info
    rng = np.random.default_rng(seed)
    space = info['space']
    ifcs = info['interfaces']
    r = zipf_ranks(rng, n, s, population).astype(np.uint64)
    seed = seed if pop_seed is None else pop_seed
    u = lambda k: _mix64(r, seed * 64 + k)
    form = rng.choice(len(form_probs), size=n, p=np.asarray(form_probs) / np.sum(form_probs))
    if not info['with_inside']:
        form[form == F_OUTBOUND] = F_BUILT
    ifc = (u(0) % np.uint64(len(ifcs))).astype(np.int64)
    src = np.zeros(n, np.int64)
    dst = np.zeros(n, np.int64)
    sport = rng.integers(1024, 65536, size=n)
    dport = COMMON_PORTS[(u(1) % np.uint64(len(COMMON_PORTS))).astype(np.int64)]
    proto = ((u(2) % np.uint64(10)) < np.uint64(3)).astype(np.int64)
    unmatched = (u(3) % np.uint64(1000)) < np.uint64(int(p_unmatched * 1000))
    for k, name in enumerate(ifcs):
        meta = info['meta']['%s_access_in' % name]
        permits = np.array([i for i, m in enumerate(meta) if m[0]], dtype=np.int64)
        sel = np.nonzero((ifc == k) & (form != F_OUTBOUND))[0]
        if len(sel) == 0 or len(permits) == 0:
            continue
        m = np.array(meta, dtype=object)
        sn = np.array([int(x) for x in m[:, 2]], np.int64)
        sl = np.array([int(x) for x in m[:, 3]], np.int64)
        dn = np.array([int(x) for x in m[:, 4]], np.int64)
        dl = np.array([int(x) for x in m[:, 5]], np.int64)
        sp = np.array([int(x) for x in m[:, 6]], np.int64)
        dp = np.array([int(x) for x in m[:, 7]], np.int64)
        pr = np.array([{'tcp': 0, 'udp': 1}.get(x, -1) for x in m[:, 1]], np.int64)
        rs = r[sel]
        # the rule of a connection: skewed to the head of the ACL (a power law
        # over the permit rules), so some rules collect far more distinct
        # connections than the cap while others stay below it
        q = (_mix64(rs, seed * 64 + 4) >> np.uint64(11)).astype(np.float64) / float(1 << 53)
        rule = permits[np.minimum((len(permits) * q ** 3).astype(np.int64), len(permits) - 1)]
        hs = _mix64(rs, seed * 64 + 5)
        hd = _mix64(rs, seed * 64 + 6)
        ssize = np.int64(1) << (32 - sl[rule])
        s_off = (hs % np.minimum(ssize, 1 << 16).astype(np.uint64)).astype(np.int64)
        src[sel] = np.where(sl[rule] == 0, 0x0B000000 + (hs % np.uint64(0xD4000000)).astype(np.int64), sn[rule] + s_off)
        dsize = np.where(dl[rule] == 0, np.int64(1) << 24, np.int64(1) << (32 - dl[rule]))
        d_off = (hd % np.minimum(dsize, 1 << 16).astype(np.uint64)).astype(np.int64)
        dst[sel] = np.where(dl[rule] == 0, 0x0A000000 + d_off, dn[rule] + d_off)
        has_sp = sp[rule] >= 0
        sport[sel[has_sp]] = sp[rule][has_sp]
        has_dp = dp[rule] >= 0
        dport[sel[has_dp]] = dp[rule][has_dp]
        fixed = pr[rule] >= 0
        proto[sel[fixed]] = pr[rule][fixed]
        un = sel[unmatched[sel]]
        hu = _mix64(r[un], seed * 64 + 7)
        src[un] = 0x0B000000 + (hu % np.uint64(0xD4000000)).astype(np.int64)
        dst[un] = 0x0A000000 + ((hu >> np.uint64(32)) % np.uint64(1 << 24)).astype(np.int64)
        dport[un] = 1 + ((hu >> np.uint64(8)) % np.uint64(65535)).astype(np.int64)
    ob = np.nonzero(form == F_OUTBOUND)[0]
    ho = _mix64(r[ob], seed * 64 + 8)
    src[ob] = space.servers[(ho % np.uint64(len(space.servers))).astype(np.int64)]
    dst[ob] = space.clients[((ho >> np.uint64(20)) % np.uint64(len(space.clients))).astype(np.int64)]
    t = t0 + (np.arange(n, dtype=np.int64) * span) // max(n, 1)
    cid = cid0 + np.arange(n, dtype=np.int64)
    return {'src': src, 'dst': dst, 'sport': sport, 'dport': dport, 'proto': proto, 'ifc': ifc, 'form': form,
            't': t, 'cid': cid, 'interfaces': list(ifcs), 'host': info['host'], 'rank': r.astype(np.int64)}


def _clock(t):
    day = t // 86400
    s = t % 86400
    return int(day), '%02d:%02d:%02d' % (s // 3600, (s // 60) % 60, s % 60)


def render_lines(tr):
    """Log text lines (without newline) for the traffic dict."""
    out = []
    P = ('TCP', 'UDP')
    MID = ('302013', '302015')
    inside = tr.get('inside_ifc', 'inside')
    for i in range(len(tr['form'])):
        f = int(tr['form'][i])
        day, hms = _clock(int(tr['t'][i]))
        pr = int(tr['proto'][i])
        s, d = _dotted(tr['src'][i]), _dotted(tr['dst'][i])
        sp, dp = int(tr['sport'][i]), int(tr['dport'][i])
        cid = '%010d' % int(tr['cid'][i])
        ifc = tr['interfaces'][int(tr['ifc'][i])]
        head = 'Jul %02d %s Jul %02d 2013 %s: ' % (day, hms, day, hms)
        if f == F_BUILT or f == F_NOACL:
            if f == F_NOACL:
                ifc = 'dmz'
            out.append('%s%%ASA-6-%s: Built inbound %s connection %s for %s:%s/%d (%s/%d) to inside:%s/%d (%s/%d)'
                       % (head, MID[pr], P[pr], cid, ifc, s, sp, s, sp, d, dp, d, dp))
        elif f == F_NONHIT:
            out.append('%s%%ASA-5-%s: Built inbound %s connection %s for %s:%s/%d (%s/%d) to inside:%s/%d (%s/%d)'
                       % (head, MID[pr], P[pr], cid, ifc, s, sp, s, sp, d, dp, d, dp))
        elif f == F_NOYEAR:
            out.append('Jul %02d %s fw1 : %%ASA-6-%s: Built inbound %s connection %s for %s:%s/%d (%s/%d) '
                       'to inside:%s/%d (%s/%d)' % (day, hms, MID[pr], P[pr], cid, ifc, s, sp, s, sp, d, dp, d, dp))
        elif f == F_TEARDOWN:
            out.append('%s%%ASA-6-302014: Teardown %s connection %s for %s:%s/%d to inside:%s/%d duration 0:00:01 '
                       'bytes 1024 TCP FINs' % (head, P[pr], cid, ifc, s, sp, d, dp))
        else:  # outbound: initiator (src) is inside, 'for' side is the outside peer
            out.append('%s%%ASA-6-%s: Built outbound %s connection %s for outside:%s/%d (%s/%d) to %s:%s/%d '
                       '(%s/%d)' % (head, MID[pr], P[pr], cid, d, dp, d, dp, inside, s, sp, s, sp))
    return out


PSPELL = ['TCP', 'UDP']


def order_keys(tr):
    """uint64 keys order-isomorphic to the byte order of the rendered lines among
    the lines that can enter a connection table (hit + BUILT forms): time,
    then message id digit (302013 < 302015 <=> TCP < UDP), then direction
    ('inbound' < 'outbound'), then the zero-padded connection id."""
    t = tr['t'].astype(np.uint64)
    x = tr['proto'].astype(np.uint64)
    d = (tr['form'] == F_OUTBOUND).astype(np.uint64)
    return (t << np.uint64(36)) | (x << np.uint64(35)) | (d << np.uint64(34)) | tr['cid'].astype(np.uint64)


def ts_decode(code):
    """Timestamp code (seconds from Jul 1 2013 00:00:00) -> reducer string."""
    day, hms = _clock(int(code))
    return '2013-07-%02d %s' % (day, hms)


def pack(tr, compiled):
    """Packed tuples/ts/order for the traffic, equal to what logparse produces
    from ``render_lines(tr)`` (pinned by tests/test_synth_pack.py)."""
    from .compile import TUPLE_DTYPE, F_VALID as FL_VALID, F_HIT as FL_HIT, F_BUILT as FL_BUILT, F_SWAP as FL_SWAP
    n = len(tr['form'])
    form = tr['form']
    host = tr['host']
    ifcs = tr['interfaces']
    out = np.zeros(n, dtype=TUPLE_DTYPE)
    out['src'] = tr['src'].astype(np.uint32)
    out['dst'] = tr['dst'].astype(np.uint32)
    out['sport'] = tr['sport'].astype(np.uint16)
    out['dport'] = tr['dport'].astype(np.uint16)
    out['pspell'] = tr['proto'].astype(np.uint8)
    valid = np.isin(form, [F_BUILT, F_NONHIT, F_NOYEAR, F_OUTBOUND])
    lists = np.zeros(n, dtype=np.int64)
    names = ('tcp', 'udp')
    acl_of = tr.get('acl_of') or ['%s_access_in' % ifc for ifc in ifcs]
    for p in (0, 1):
        for k, ifc in enumerate(ifcs):
            w = valid & (form != F_OUTBOUND) & (tr['ifc'] == k) & (tr['proto'] == p)
            if w.any():
                lists[w] = compiled.list_id(host, acl_of[k], names[p])
        w = (form == F_OUTBOUND) & (tr['proto'] == p)
        if w.any():
            lists[w] = compiled.list_id(host, tr.get('inside_acl', 'inside_access_in'), names[p])
    out['list'] = lists.astype(np.uint16)
    flags = np.where(valid, FL_VALID, 0)
    flags = flags | np.where(np.isin(form, [F_BUILT, F_NOYEAR, F_OUTBOUND]), FL_HIT, 0)
    flags = flags | np.where(np.isin(form, [F_BUILT, F_NONHIT, F_OUTBOUND]), FL_BUILT, 0)
    flags = flags | np.where(form == F_OUTBOUND, FL_SWAP, 0)
    out['flags'] = flags.astype(np.uint8)
    out['pspell'][(flags & FL_BUILT) == 0] = 0
    ts = tr['t'].astype(np.uint32)
    return out, ts, order_keys(tr)
