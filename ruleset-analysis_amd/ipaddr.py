"""IPy-compatible address value used by the drop-in ``FirewallRule``.

The reference stores ``IPy.IP`` objects inside every rule (``firewallrule.py:5,
31, 82, 91``) and pickles them into ``accesslists.db``.  IPy is not available
here, so this class offers the same state (``ip``, ``_prefixlen``,
``_ipversion`` — the attribute names an unpickled ``IPy.IP`` carries) and the
behaviour the path needs: parsing of the textual forms the preprocessors write
(``preprosess_access_lists.py:139-154``: ``any`` is handled by the rule, a bare
host, ``addr/netmask``, object-group members), containment, length and
``str()``.  The compiled GPU tables only ever see ``(ip, prefixlen, version)``.
"""

import ipaddress

from .py2text import py2_int, py2_isdigit, py2_strip

__all__ = ['IP']

_V4_BITS = 32
_V6_BITS = 128


def _bits(version):
    return _V4_BITS if version == 4 else _V6_BITS


def _addr_value(text):
    """Address text without prefix -> (int value, version)."""
    if ':' in text:
        return int(ipaddress.IPv6Address(text)), 6
    if py2_isdigit(text):
        v = int(text)
        return v, (4 if v < (1 << 32) else 6)
    octets = text.split('.')
    if len(octets) > 4 or not all(py2_isdigit(o) and int(o) < 256 for o in octets):
        raise ValueError('invalid IPv4 address %r' % (text,))
    octets = octets + ['0'] * (4 - len(octets))
    value = 0
    for o in octets:
        value = value * 256 + int(o)
    return value, 4


def _mask_to_len(mask, bits):
    inv = ((1 << bits) - 1) ^ mask
    if inv & (inv + 1):
        raise ValueError('netmask %#x is not contiguous' % mask)
    return bits - inv.bit_length()


class IP(object):
    """Network or host address with IPy's observable behaviour."""

    def __init__(self, data, ipversion=0, make_net=0):
        if isinstance(data, IP):
            self.ip, self._prefixlen, self._ipversion = data.ip, data._prefixlen, data._ipversion
            return
        if isinstance(data, int):
            version = ipversion or (4 if 0 <= data < (1 << 32) else 6)
            self.ip, self._prefixlen, self._ipversion = data, _bits(version), version
            return
        text = py2_strip(str(data))
        if '-' in text:
            first, last = text.split('-', 1)
            lo, version = _addr_value(first)
            hi, v2 = _addr_value(last)
            span = hi - lo + 1
            if v2 != version or span <= 0 or span & (span - 1):
                raise ValueError('range %r is not a single network' % (text,))
            prefixlen = _bits(version) - (span.bit_length() - 1)
            value = lo
        elif '/' in text:
            addr, pfx = text.split('/', 1)
            value, version = _addr_value(addr)
            if '.' in pfx or ':' in pfx:
                prefixlen = _mask_to_len(_addr_value(pfx)[0], _bits(version))
            else:
                prefixlen = py2_int(pfx)
        else:
            value, version = _addr_value(text)
            prefixlen = _bits(version)
        if ipversion and ipversion != version:
            raise ValueError('%r is not IPv%d' % (text, ipversion))
        if not 0 <= prefixlen <= _bits(version):
            raise ValueError('invalid prefix length in %r' % (text,))
        host = (1 << (_bits(version) - prefixlen)) - 1
        if value & host:
            if not make_net:
                raise ValueError("IP('%s') has invalid prefix length (%s)" % (text, prefixlen))
            value &= ~host
        self.ip, self._prefixlen, self._ipversion = value, prefixlen, version

    # IPy accessors
    def version(self):
        return self._ipversion

    def prefixlen(self):
        return self._prefixlen

    def int(self):
        return self.ip

    def len(self):
        return 1 << (_bits(self._ipversion) - self._prefixlen)

    def netmask_int(self):
        bits = _bits(self._ipversion)
        return ((1 << bits) - 1) ^ ((1 << (bits - self._prefixlen)) - 1)

    def __contains__(self, item):
        other = item if isinstance(item, IP) else IP(item)
        if other._ipversion != self._ipversion:
            return False
        return self.ip <= other.ip and other.ip + other.len() <= self.ip + self.len()

    def __str__(self):
        if self._ipversion == 4:
            text = str(ipaddress.IPv4Address(self.ip))
        else:
            text = str(ipaddress.IPv6Address(self.ip))
        if self._prefixlen == _bits(self._ipversion):
            return text
        return '%s/%d' % (text, self._prefixlen)

    def __repr__(self):
        return "IP('%s')" % self

    def _key(self):
        return (self.ip, self._prefixlen, self._ipversion)

    def __eq__(self, other):
        return isinstance(other, IP) and self._key() == other._key()

    def __ne__(self, other):
        return not self == other

    def __hash__(self):
        return hash(self._key())

    # pickles written by Python 2 IPy carry extra attributes; keep only the state
    def __setstate__(self, state):
        if isinstance(state, tuple):          # (dict, slots) form
            state = state[0] or {}
        self.ip = int(state.get('ip', 0))
        self._prefixlen = int(state.get('_prefixlen', 32))
        self._ipversion = int(state.get('_ipversion', 4))
