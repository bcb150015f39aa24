"""Drop-in ``FirewallRule`` (reference: ``firewallrule.py:8-174``).

Same constructor signature, attributes (``action, protocol, original, src, dst,
sport, dport, comments, rulenum, ruleindex``), ``NO_PORT``/``ANY`` class
attributes, ``__eq__``/``__str__``/``__repr__`` and the ``__contains__``
predicate, so code written against the reference (and rule objects unpickled
from its ``accesslists.db``) keeps working.  The per-line evaluation of
``__contains__`` is what the HIP kernels replace; ``compile.py`` lowers each
rule to the integer predicate they evaluate.
"""

from .ipaddr import IP
from .py2text import py2_int, py2_is_int

__all__ = ['FirewallRule']


def _as_port_list(value, what):
    if isinstance(value, str):
        try:
            value = [py2_int(value)]
        except ValueError:
            raise ValueError('unable to convert either source or destination port to Integer')
    if not isinstance(value, list):
        value = [value]
    if not value:
        value = [FirewallRule.NO_PORT]
    for p in value:
        if not py2_is_int(p):              # a Python 2 long (|p| > sys.maxint) is not an int either
            raise ValueError('%s port must be an integer or -1 for "No port"' % what)
    return value


class FirewallRule(object):
    NO_PORT = -1
    ANY = IP('0.0.0.0/0')

    def __init__(self, action, protocol, original, src, dst, sport=NO_PORT, dport=NO_PORT,
                 comments=[], rulenum=-1, ruleindex=-1):
        if isinstance(action, str):
            action = bool(action)   # reference quirk kept: bool('False') is True
        if not isinstance(action, bool):
            raise ValueError('action must be True/False where True=Permit and False=Deny')
        sport = _as_port_list(sport, 'Source')
        dport = _as_port_list(dport, 'Source')   # the reference's message says "Source" for both
        self.src = self._address(src, 'src')
        self.dst = self._address(dst, 'dst')
        self.action = action
        self.protocol = str(protocol)
        self.original = original
        self.sport = sport
        self.dport = dport
        self.comments = comments
        self.rulenum = rulenum
        self.ruleindex = ruleindex

    @classmethod
    def _address(cls, value, name):
        if value == 'any':
            return cls.ANY
        try:
            return IP(value)
        except ValueError as exc:
            raise ValueError('argument "%s" must be a valid IP address or network. Error: %s' % (name, exc))

    def __eq__(self, other):
        if not isinstance(other, FirewallRule):
            return False
        return self.__dict__ == other.__dict__

    __hash__ = None

    def __str__(self):
        src = str(self.src) if self.sport == [self.NO_PORT] else '%s:%s' % (self.src, self.sport)
        dst = str(self.dst) if self.dport == [self.NO_PORT] else '%s:%s' % (self.dst, self.dport)
        return ' '.join(['permit' if self.action else 'deny', self.protocol, src, '->', dst])

    def __repr__(self):
        return ("FirewallRule({!r}, {!r}, '{}', '{}', '{}', sport={!r}, dport={!r}, comments={!r}, "
                "rulenum={}, ruleindex={})").format(self.action, self.protocol, self.original, self.src, self.dst,
                                                    self.sport, self.dport, self.comments, self.rulenum,
                                                    self.ruleindex)

    def __contains__(self, other):
        if not isinstance(other, FirewallRule):
            raise ValueError('both objects must be FirewallRule objects')
        return (self.action == other.action
                and (self.protocol == 'ip' or self.protocol == other.protocol)
                and other.src in self.src
                and other.dst in self.dst
                and (self.sport == [self.NO_PORT] or all(p in self.sport for p in other.sport))
                and (self.dport == [self.NO_PORT] or all(p in self.dport for p in other.dport)))

    # rule objects unpickled from a Python 2 shelve arrive without __init__
    def __setstate__(self, state):
        self.__dict__.update(state)
