"""ORACLE (test infrastructure only) — restatement of ``firewallrule.py:8-174``.

Semantics kept exactly, Python-2 idioms mapped to Python 3:

* constructor normalisation ``firewallrule.py:33-103``: a string action goes
  through ``bool()`` (so ``'False'`` is True — reference behaviour kept), string
  ports become ``[int]``, scalars become one-element lists, empty lists become
  ``[NO_PORT]``, non-int items raise ``ValueError``; ``'any'`` maps to the shared
  ``ANY = IP('0.0.0.0/0')``, anything else goes through ``IP()``;
* ``__eq__`` compares ``__dict__`` (``:106-111``);
* ``__str__`` (``:113-118``) / ``__repr__`` (``:121-125``);
* ``__contains__`` (``:128-174``): action equal, protocol ``'ip'`` or equal,
  src/dst prefix containment, port-list containment unless ``[NO_PORT]``.
"""

from .ipy import IP


class FirewallRule(object):
    NO_PORT = -1
    ANY = IP('0.0.0.0/0')

    def __init__(self, action, protocol, original, src, dst, sport=NO_PORT, dport=NO_PORT,
                 comments=[], rulenum=-1, ruleindex=-1):
        if isinstance(action, str):
            action = bool(action)
        if not isinstance(action, bool):
            raise ValueError('action must be True/False where True=Permit and False=Deny')
        try:
            if isinstance(sport, str):
                sport = [int(sport)]
            if isinstance(dport, str):
                dport = [int(dport)]
        except ValueError:
            raise ValueError('unable to convert either source or destination port to Integer')
        sport = sport if isinstance(sport, list) else [sport]
        dport = dport if isinstance(dport, list) else [dport]
        if not sport:
            sport = [self.NO_PORT]
        if not dport:
            dport = [self.NO_PORT]
        # Python 2: int() of a literal past sys.maxint (2^63 - 1) is a long, which
        # isinstance(p, int) rejects (firewallrule.py:67-75)
        py2int = lambda p: isinstance(p, int) and -(1 << 63) <= p < (1 << 63)
        if any(not py2int(p) for p in sport) or any(not py2int(p) for p in dport):
            raise ValueError('Source port must be an integer or -1 for "No port"')
        self.src = self._addr(src, 'src')
        self.dst = self._addr(dst, 'dst')
        self.action = action
        self.protocol = str(protocol)
        self.original = original
        self.sport = sport
        self.dport = dport
        self.comments = comments
        self.rulenum = rulenum
        self.ruleindex = ruleindex

    def _addr(self, value, name):
        if value == 'any':
            return self.ANY
        try:
            return IP(value)
        except ValueError as e:
            raise ValueError('argument "%s" must be a valid IP address or network. Error: %s' % (name, e))

    def __eq__(self, other):
        return isinstance(other, FirewallRule) and self.__dict__ == other.__dict__

    __hash__ = None

    def __str__(self):
        verb = 'permit' if self.action else 'deny'
        s = str(self.src)
        if self.sport != [self.NO_PORT]:
            s += ':' + str(self.sport)
        d = str(self.dst)
        if self.dport != [self.NO_PORT]:
            d += ':' + str(self.dport)
        return '%s %s %s -> %s' % (verb, self.protocol, s, d)

    def __repr__(self):
        return ("FirewallRule(%r, %r, '%s', '%s', '%s', sport=%r, dport=%r, comments=%r, rulenum=%s, ruleindex=%s)"
                % (self.action, self.protocol, self.original, self.src, self.dst, self.sport, self.dport,
                   self.comments, self.rulenum, self.ruleindex))

    def __contains__(self, other):
        if not isinstance(other, FirewallRule):
            raise ValueError('both objects must be FirewallRule objects')
        if self.action != other.action:
            return False
        if self.protocol != 'ip' and self.protocol != other.protocol:
            return False
        if other.src not in self.src or other.dst not in self.dst:
            return False
        if self.sport != [self.NO_PORT] and any(p not in self.sport for p in other.sport):
            return False
        if self.dport != [self.NO_PORT] and any(p not in self.dport for p in other.dport):
            return False
        return True
