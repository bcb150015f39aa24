"""ORACLE (test infrastructure only) — restatement of the parts of third-party
``IPy.IP`` that the reference's hot path relies on.

IPy is imported by ``firewallrule.py:5`` and used at ``firewallrule.py:31,82,91``
(construction), ``:154,158`` (``other.src not in self.src``) and ``:116-124``
(``str``).  IPy is NOT vendored in ``/root/reference`` and not installed here;
no version is pinned anywhere in the reference (``README.md:23-24`` only names
it).  This restates IPy's published behaviour:

* parse ``a.b.c.d``, ``a.b.c.d/len``, ``a.b.c.d/m.m.m.m`` (contiguous netmask),
  ``a.b.c.d-e.f.g.h`` (exact prefix range), short dotted forms padded with
  zeros (``10.1`` -> ``10.1.0.0``), decimal integers, and IPv6 text;
* reject a network with host bits set (``ValueError``) — IPy's default
  ``make_net=0``;
* ``len()`` = number of addresses; ``item in net`` is
  ``item.ip >= net.ip and item.ip < net.ip + net.len() - item.len() + 1``
  with a version mismatch answering False (IPy >= 0.81 behaviour — older IPy
  compared raw integers; documented in DESIGN.md as an unpinned choice);
* ``str()`` = ``strCompressed()``: dotted quad plus ``/len`` unless the prefix
  is a single host (``NoPrefixForSingleIp``).
"""

import ipaddress


def _parse_v4_dotted(s):
    parts = s.split('.')
    if len(parts) > 4:
        raise ValueError("IPv4 Address with more than 4 bytes")
    parts += ['0'] * (4 - len(parts))
    val = 0
    for p in parts:
        if not p.isdigit():
            raise ValueError("%r: single byte must be 0 <= byte < 256" % (s,))
        b = int(p)
        if b > 255:
            raise ValueError("%r: single byte must be 0 <= byte < 256" % (s,))
        val = (val << 8) | b
    return val


def _parse_addr(s):
    """Return (int, version) for an address string without prefix."""
    if ':' in s:
        return int(ipaddress.IPv6Address(s)), 6
    if s.isdigit():
        v = int(s)
        if v <= 0xFFFFFFFF:
            return v, 4
        if v <= (1 << 128) - 1:
            return v, 6
        raise ValueError("IP Address can't be larger than 2**128")
    return _parse_v4_dotted(s), 4


def _netmask_to_prefixlen(m, bits):
    # IPy._netmaskToPrefixlen: mask must be contiguous ones followed by zeros
    plen = 0
    while plen < bits and (m >> (bits - 1 - plen)) & 1:
        plen += 1
    if (m & ((1 << (bits - plen)) - 1)) != 0:
        raise ValueError("Netmask 0x%x can't be expressed as an prefix." % m)
    return plen


class IP(object):
    """IPy.IP-compatible value: ``ip`` (int), ``_prefixlen``, ``_ipversion``."""

    def __init__(self, data, ipversion=0, make_net=0):
        if isinstance(data, IP):
            self.ip = data.ip
            self._prefixlen = data._prefixlen
            self._ipversion = data._ipversion
            return
        if isinstance(data, int):
            if data < 0:
                raise ValueError("IP Address can't be negative")
            self.ip = data
            self._ipversion = ipversion or (4 if data <= 0xFFFFFFFF else 6)
            self._prefixlen = 32 if self._ipversion == 4 else 128
            return
        if not isinstance(data, str):
            raise TypeError("Unsupported data type: %r" % (type(data),))
        s = data.strip()
        if '-' in s:
            lo_s, hi_s = s.split('-', 1)
            lo, v = _parse_addr(lo_s)
            hi, v2 = _parse_addr(hi_s)
            if v != v2:
                raise ValueError("first-last notation only allowed for same IP version")
            bits = 32 if v == 4 else 128
            size = hi - lo + 1
            if size <= 0 or size & (size - 1):
                raise ValueError("the range %s is not on a network boundary." % s)
            plen = bits - (size.bit_length() - 1)
            ip = lo
        elif '/' in s:
            addr_s, pl_s = s.split('/', 1)
            ip, v = _parse_addr(addr_s)
            bits = 32 if v == 4 else 128
            if '.' in pl_s or ':' in pl_s:
                m, _mv = _parse_addr(pl_s)
                plen = _netmask_to_prefixlen(m, bits)
            else:
                plen = int(pl_s)
        else:
            ip, v = _parse_addr(s)
            bits = 32 if v == 4 else 128
            plen = bits
        if ipversion and ipversion != v:
            raise ValueError("%r: wrong IP version" % (data,))
        if plen < 0 or plen > bits:
            raise ValueError("%r: invalid prefix length" % (data,))
        hostmask = (1 << (bits - plen)) - 1
        if ip & hostmask:
            if make_net:
                ip &= ~hostmask
            else:
                raise ValueError("IP('%s') has invalid prefix length (%s)" % (s, plen))
        self.ip = ip
        self._prefixlen = plen
        self._ipversion = v

    # -- IPy API used by the path -------------------------------------------------
    def version(self):
        return self._ipversion

    def prefixlen(self):
        return self._prefixlen

    def len(self):
        bits = 32 if self._ipversion == 4 else 128
        return 1 << (bits - self._prefixlen)

    def __contains__(self, item):
        if isinstance(item, IP):
            if item._ipversion != self._ipversion:
                return False
        else:
            item = IP(item)
        return item.ip >= self.ip and item.ip < self.ip + self.len() - item.len() + 1

    def __str__(self):
        if self._ipversion == 4:
            a = self.ip
            s = '%d.%d.%d.%d' % ((a >> 24) & 255, (a >> 16) & 255, (a >> 8) & 255, a & 255)
            return s if self._prefixlen == 32 else s + '/%d' % self._prefixlen
        s = str(ipaddress.IPv6Address(self.ip))
        return s if self._prefixlen == 128 else s + '/%d' % self._prefixlen

    def __repr__(self):
        return "IP('%s')" % str(self)

    def __eq__(self, other):
        if not isinstance(other, IP):
            return False
        return (self.ip, self._prefixlen, self._ipversion) == (other.ip, other._prefixlen, other._ipversion)

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return hash((self.ip, self._prefixlen, self._ipversion))
