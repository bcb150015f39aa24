"""The rule database the path consumes: ``accesslists.db``.

Schema (written by ``preprosess_access_lists.py:525-550`` and
``preprosess_fortigate_acl.py:406-431``; read by ``mapper.py:79-100`` and
``connlist-reducer.py:32-49``)::

    {'firewalls':   {host: {interface: {'in'|'out': acl}}},
     'accesslists': {host: {acl: {'rules': [FirewallRule, ...],
                                  'protocols': {proto: [ruleindex, ...]},
                                  'timestamp': mtime}}}}

Two on-disk forms are accepted:

* the reference's Python-2 ``shelve`` (a dbm file of protocol-0 pickles holding
  old-style ``firewallrule.FirewallRule`` instances and ``IPy.IP`` objects).  It
  is read with a restricted unpickler that maps exactly those classes onto this
  package's ``FirewallRule`` / ``IP`` and refuses every other global;
* a JSON form (``save_json``/``load_json``) that this repo uses for fixtures and
  for moving a compiled DB to machines without the dbm flavour that wrote it.
"""

import io
import json
import os
import pickle

from .firewallrule import FirewallRule
from .ipaddr import IP

__all__ = ['AclDB', 'load', 'load_shelve', 'load_json', 'save_json', 'DBError']


class DBError(Exception):
    """Raised where the reference prints 'Unable to open/load ... database' and exits 1."""


class AclDB(object):
    def __init__(self, firewalls, accesslists):
        self.firewalls = firewalls
        self.accesslists = accesslists

    def rule_count(self):
        return sum(len(a['rules']) for h in self.accesslists.values() for a in h.values())


_ALLOWED = {
    ('firewallrule', 'FirewallRule'): FirewallRule,
    ('mapper', 'Connection'): FirewallRule,
    ('IPy', 'IP'): IP,
    ('IPy', 'IPint'): IP,
}


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return _ALLOWED[(module, name)]
        if (module, name) in (('copy_reg', '_reconstructor'), ('copyreg', '_reconstructor')):
            import copyreg
            return copyreg._reconstructor
        if (module, name) in (('__builtin__', 'object'), ('builtins', 'object')):
            return object
        if (module, name) in (('__builtin__', 'set'), ('builtins', 'set')):
            return set
        raise pickle.UnpicklingError('global %s.%s is not allowed in accesslists.db' % (module, name))


def _unpickle(blob):
    return _RestrictedUnpickler(io.BytesIO(blob), encoding='latin1').load()


def _open_dbm(path):
    import dbm
    errors = []
    candidates = [path]
    if path.endswith('.db'):
        candidates.append(path[:-3])
    for cand in candidates:
        try:
            import dbm.ndbm
            return dbm.ndbm.open(cand, 'r')
        except Exception as exc:  # noqa: BLE001 - try the next flavour
            errors.append(exc)
        try:
            return dbm.open(cand, 'r')
        except Exception as exc:  # noqa: BLE001
            errors.append(exc)
    raise DBError('Unable to open access-list database ("{0}"): {1}'.format(path, errors[-1] if errors else ''))


def load_shelve(path):
    db = _open_dbm(path)
    try:
        try:
            accesslists = _unpickle(db[b'accesslists'])
            firewalls = _unpickle(db[b'firewalls'])
        except KeyError as exc:
            raise DBError('Unable to load key {0} from access-list database.'.format(exc))
    finally:
        db.close()
    return AclDB(firewalls, accesslists)


def _rule_from_json(r):
    rule = FirewallRule(bool(r['action']), r['protocol'], r['original'], r['src'], r['dst'],
                        list(r['sport']), list(r['dport']), comments=list(r.get('comments', [])),
                        rulenum=r.get('rulenum', -1), ruleindex=r.get('ruleindex', -1))
    return rule


def load_json(path_or_obj):
    obj = path_or_obj
    if isinstance(path_or_obj, (str, os.PathLike)):
        with open(path_or_obj) as f:
            obj = json.load(f)
    accesslists = {}
    for host, acls in obj['accesslists'].items():
        accesslists[host] = {}
        for acl, entry in acls.items():
            accesslists[host][acl] = {
                'rules': [_rule_from_json(r) for r in entry['rules']],
                'protocols': {p: list(v) for p, v in entry['protocols'].items()},
                'timestamp': entry.get('timestamp', 0),
            }
    return AclDB(obj['firewalls'], accesslists)


def _rule_to_json(rule):
    return {'action': rule.action, 'protocol': rule.protocol, 'original': rule.original,
            'src': 'any' if rule.src is FirewallRule.ANY else str(rule.src),
            'dst': 'any' if rule.dst is FirewallRule.ANY else str(rule.dst),
            'sport': list(rule.sport), 'dport': list(rule.dport), 'comments': list(rule.comments),
            'rulenum': rule.rulenum, 'ruleindex': rule.ruleindex}


def to_json_obj(db):
    return {'firewalls': db.firewalls,
            'accesslists': {h: {a: {'rules': [_rule_to_json(r) for r in e['rules']],
                                    'protocols': e['protocols'], 'timestamp': e.get('timestamp', 0)}
                                for a, e in acls.items()}
                            for h, acls in db.accesslists.items()}}


def save_json(db, path):
    with open(path, 'w') as f:
        json.dump(to_json_obj(db), f, indent=0, sort_keys=True)


def load(path):
    """Load ``accesslists.db`` (shelve) or a ``.json`` DB."""
    if str(path).endswith('.json'):
        return load_json(path)
    return load_shelve(path)
