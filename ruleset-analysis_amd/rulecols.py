"""Columnar store of one access list's expanded rules.

The preprocessors expand every ACL line or FortiGate policy into one
``FirewallRule`` per (address, address, port) combination
(``preprosess_access_lists.py:256-276``, ``preprosess_fortigate_acl.py:184-215``);
a policy with a wide port range becomes tens of thousands of rules, and a
policy set with expanded address groups and ranges (BASELINE config 4) millions.
``RuleColumns`` keeps those rules as numpy columns instead of Python objects:
it is a drop-in for the ``'rules'`` list of ``accesslists.db``
(``len``, ``rules[i]`` materialises the ``FirewallRule`` the reference would
have stored, with ``ruleindex = i``), and ``CompiledRules`` lowers it to
candidate-list entries without touching Python objects (``lower``).

Every stored rule has one port (or ``NO_PORT``) per side -- the shape both
preprocessors produce for tcp/udp/ip rules (SURVEY.md trap 3) -- and an IPv4
or IPv6 network per address side.  IPv6 sides are rare and are kept aside:
``fam`` has bit 0 (source) / bit 1 (destination) set, the side's ``src``/
``dst`` column holds an index into ``nets6`` (the address text the rule was
built from) and its ``*_len`` the prefix length.  Such a rule keeps its list
position (its ``ruleindex``) but never matches the IPv4 connections of a log:
IPy answers False for an address of another version
(``firewallrule.py:82,91,154,158``).
"""

import numpy as np

from .firewallrule import FirewallRule

__all__ = ['RuleColumns', 'FAM_SRC6', 'FAM_DST6', 'Nets6']

FAM_SRC6, FAM_DST6 = 1, 2


def _dotted(v):
    v = int(v)
    return '%d.%d.%d.%d' % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)


class Nets6(object):
    """Interned IPv6 address texts of one rule store (``RuleColumns.nets6``)."""

    def __init__(self):
        self.texts, self.ids = [], {}

    def __call__(self, text):
        k = self.ids.get(text)
        if k is None:
            k = self.ids[text] = len(self.texts)
            self.texts.append(text)
        return k


class RuleColumns(object):
    """Columns (one entry per expanded rule, in ruleindex order):

    action bool; proto uint8 (index into ``proto_names``); src/dst uint32 network
    address and uint8 prefix length; sport/dport int32 (-1 = NO_PORT); orig,
    comment, rulenum int32 indices into ``originals``, ``comments``,
    ``rulenums``; fam uint8 (FAM_SRC6 / FAM_DST6: that side is the IPv6
    network ``nets6[src or dst]`` of prefix length ``*_len``)."""

    def __init__(self, action, proto, proto_names, src, src_len, dst, dst_len, sport, dport, orig, originals,
                 comment=None, comments=None, rulenum=None, rulenums=None, fam=None, nets6=None):
        n = len(action)
        self.action = np.asarray(action, bool)
        self.proto = np.asarray(proto, np.uint8)
        self.proto_names = list(proto_names)
        self.src = np.asarray(src, np.uint32)
        self.src_len = np.asarray(src_len, np.uint8)
        self.dst = np.asarray(dst, np.uint32)
        self.dst_len = np.asarray(dst_len, np.uint8)
        self.sport = np.asarray(sport, np.int32)
        self.dport = np.asarray(dport, np.int32)
        self.orig = np.asarray(orig, np.int32)
        self.originals = list(originals)
        self.comment = np.zeros(n, np.int32) if comment is None else np.asarray(comment, np.int32)
        self.comments = [[]] if comments is None else list(comments)
        self.rulenum = np.zeros(n, np.int32) if rulenum is None else np.asarray(rulenum, np.int32)
        self.rulenums = [-1] if rulenums is None else list(rulenums)
        self.fam = np.zeros(n, np.uint8) if fam is None else np.asarray(fam, np.uint8)
        self.nets6 = [] if nets6 is None else list(nets6)
        for a in (self.proto, self.src, self.src_len, self.dst, self.dst_len, self.sport, self.dport, self.orig,
                  self.comment, self.rulenum, self.fam):
            if len(a) != n:
                raise ValueError('rule columns differ in length')
        self._cache = {}

    def __len__(self):
        return len(self.action)

    def _addr(self, ip, plen):
        return '%s/%d' % (_dotted(ip), plen) if plen != 32 else _dotted(ip)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        i = int(i)
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError('rule index out of range')
        r = self._cache.get(i)
        if r is None:
            sp, dp = int(self.sport[i]), int(self.dport[i])
            f = int(self.fam[i])
            if f & FAM_SRC6:
                src = self.nets6[int(self.src[i])]
            else:
                src = 'any' if self.src_len[i] == 0 and self.src[i] == 0 else self._addr(self.src[i], self.src_len[i])
            if f & FAM_DST6:
                dst = self.nets6[int(self.dst[i])]
            else:
                dst = 'any' if self.dst_len[i] == 0 and self.dst[i] == 0 else self._addr(self.dst[i], self.dst_len[i])
            r = FirewallRule(bool(self.action[i]), self.proto_names[self.proto[i]], self.originals[self.orig[i]], src,
                             dst, [sp], [dp], comments=self.comments[self.comment[i]],
                             rulenum=self.rulenums[self.rulenum[i]], ruleindex=i)
            self._cache[i] = r
        return r

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]

    def protocols(self):
        """proto name -> int64 array of rule indices (the ``proto2rule`` map)."""
        return {name: np.flatnonzero(self.proto == k).astype(np.int64) for k, name in enumerate(self.proto_names)
                if (self.proto == k).any()}

    def lower(self, idxs, proto, base, oor=(None, None)):
        """Candidate-list entries (compile.RULE_DTYPE) of the rules ``idxs`` for a
        connection of protocol ``proto``: the connection-independent part of
        ``FirewallRule.__contains__`` (firewallrule.py:146-150: permit, protocol
        'ip' or equal) filters, the rest lowers to integer ranges.  ``oor``:
        (sport, dport) of a connection whose port on that side is past 65535
        (None: in range); such a side matches only a NO_PORT rule side or one
        naming that port (``:162-171``) and is lowered to "any port" (the
        tuple carries 0 there, ``CompiledRules.list_id_oor``)."""
        from .compile import RULE_DTYPE
        idx = np.unique(np.asarray(idxs, np.int64))
        if len(idx) and (idx[0] < 0 or idx[-1] >= len(self)):
            raise IndexError('candidate index out of range')
        names = self.proto_names
        ok_proto = np.array([nm == 'ip' or nm == proto for nm in names], bool)
        # an IPv6 side never contains the connection's IPv4 address
        keep = self.action[idx] & ok_proto[self.proto[idx]] & (self.fam[idx] == 0)
        sp = self.sport[idx].astype(np.int64)
        dp = self.dport[idx].astype(np.int64)
        for col, v in ((sp, oor[0]), (dp, oor[1])):
            if v is None:
                keep &= (col == -1) | ((col >= 0) & (col <= 65535))
            else:
                keep &= (col == -1) | (col == v)
                col[:] = -1
        idx, sp, dp = idx[keep], sp[keep], dp[keep]
        out = np.zeros(len(idx), RULE_DTYPE)
        slen = self.src_len[idx].astype(np.int64)
        dlen = self.dst_len[idx].astype(np.int64)
        out['src_lo'] = self.src[idx]
        out['src_span'] = ((np.int64(1) << (32 - slen)) - 1).astype(np.uint32)
        out['dst_lo'] = self.dst[idx]
        out['dst_span'] = ((np.int64(1) << (32 - dlen)) - 1).astype(np.uint32)
        slo = np.where(sp < 0, 0, sp)
        sspan = np.where(sp < 0, 0xFFFF, 0)
        dlo = np.where(dp < 0, 0, dp)
        dspan = np.where(dp < 0, 0xFFFF, 0)
        out['port_lo'] = (slo | (dlo << 16)).astype(np.uint32)
        out['port_span'] = (sspan | (dspan << 16)).astype(np.uint32)
        out['gid'] = (base + idx).astype(np.uint32)
        return out
