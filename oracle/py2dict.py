"""ORACLE (test infrastructure only) — CPython 2.7 ``dict`` iteration order for
``str`` keys, restated structure-for-structure from CPython 2.7
``Objects/dictobject.c`` (``PyDict_SetItem`` -> ``insertdict`` ->
``lookdict_string``; ``dictresize`` -> ``insertdict_clean``) and
``Objects/stringobject.c`` (``string_hash``), 64-bit ``long``/``size_t``, hash
randomisation off (the 2.7 default).

The reference reducer prints a rule's connection table in ``conns.keys()``
order after a stable sort on ``"TOIP TOPORT"`` (``connlist-reducer.py:109-110``),
so ties keep this order (SURVEY.md trap 8).  Pinned by published CPython 2.7
values: ``hash('a') == 12416037344`` (64-bit) / ``-468864544`` (32-bit), and
``{'a': 1, 'b': 2, 'c': 3}`` printing as ``{'a': 1, 'c': 3, 'b': 2}``
(tests/test_py2dict.py).  The product has its own implementation
(``ruleset-analysis_amd/py2dict.py``); this one is the checker.
"""

ULONG = (1 << 64) - 1
PyDict_MINSIZE = 8
PERTURB_SHIFT = 5


def string_hash(s):
    """stringobject.c string_hash: C long arithmetic, returned as a signed int."""
    p = s.encode('latin-1')
    n = len(p)
    if n == 0:
        return 0
    x = p[0] << 7
    for c in p:
        x = ((1000003 * x) & ULONG) ^ c
    x ^= n
    if x & (1 << 63):
        x -= 1 << 64
    if x == -1:
        x = -2
    return x


class Py2Dict(object):
    """Slot table of a PyDictObject (keys only; values live elsewhere)."""

    def __init__(self):
        self.ma_fill = 0
        self.ma_used = 0
        self.ma_mask = PyDict_MINSIZE - 1
        self.ma_table = [None] * PyDict_MINSIZE      # None = NULL key, else (hash, key)

    def _lookdict_string(self, key, hash_):
        mask = self.ma_mask
        ep0 = self.ma_table
        i = hash_ & ULONG & mask               # i = hash & mask (size_t)
        ep = ep0[i]
        if ep is None or ep[1] == key:
            return i
        perturb = hash_ & ULONG                # for (perturb = hash; ; perturb >>= PERTURB_SHIFT)
        while True:
            i = ((i << 2) + i + perturb + 1) & ULONG
            ep = ep0[i & mask]
            if ep is None or (ep[0] == hash_ and ep[1] == key):
                return i & mask
            perturb >>= PERTURB_SHIFT

    def _insertdict_clean(self, key, hash_):
        mask = self.ma_mask
        ep0 = self.ma_table
        i = hash_ & ULONG & mask
        perturb = hash_ & ULONG
        while ep0[i & mask] is not None:
            i = ((i << 2) + i + perturb + 1) & ULONG
            perturb >>= PERTURB_SHIFT
        ep0[i & mask] = (hash_, key)
        self.ma_fill += 1
        self.ma_used += 1

    def _dictresize(self, minused):
        newsize = PyDict_MINSIZE
        while newsize <= minused and newsize > 0:
            newsize <<= 1
        oldtable = self.ma_table
        self.ma_table = [None] * newsize
        self.ma_mask = newsize - 1
        self.ma_used = 0
        self.ma_fill = 0
        for ep in oldtable:                     # old slots in order
            if ep is not None:
                self._insertdict_clean(ep[1], ep[0])

    def setitem(self, key):
        """PyDict_SetItem(mp, key, value) for a str key."""
        hash_ = string_hash(key)
        n_used = self.ma_used
        slot = self._lookdict_string(key, hash_)
        if self.ma_table[slot] is None:         # insertdict: a new key
            self.ma_fill += 1
            self.ma_table[slot] = (hash_, key)
            self.ma_used += 1
        if not (self.ma_used > n_used and self.ma_fill * 3 >= (self.ma_mask + 1) * 2):
            return
        self._dictresize((2 if self.ma_used > 50000 else 4) * self.ma_used)

    def keys(self):
        return [ep[1] for ep in self.ma_table if ep is not None]


def py2_keys(keys_in_insertion_order):
    """``d.keys()`` of a Python 2.7 dict built by inserting these keys in order."""
    d = Py2Dict()
    for k in keys_in_insertion_order:
        d.setitem(k)
    return d.keys()
