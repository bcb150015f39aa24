"""Interned text of reducer connection keys outside the canonical form."""

__all__ = ['INTERNED', 'MAX_SPELL_ID', 'KeyText']


def _dotted(v):
    return '%d.%d.%d.%d' % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)


INTERNED = 0x80     # record pspell value of an interned key: for_ip is a KeyText id of the whole key
MAX_SPELL_ID = INTERNED - 1     # protocol spelling ids 0..126 ride in canonical rows


class KeyText(object):
    """Interned text of whole connection keys ``PROTO;FROMIP;TOIP;TOPORT``
    (``connlist-reducer.py:162``) that the packed form cannot carry: addresses
    or ports that are not canonical dotted quads and ports (``10.0.0.01``,
    ``080``, ``70000``), BUILT fields that differ from the mapper's tuple, or a
    protocol spelling past the first ``MAX_SPELL_ID`` distinct ones.  The
    reducer keys its dict by the strings (``:167``), so such a line is
    aggregated under the 32-bit id of its key text (record ``pspell =
    INTERNED``, ``for_ip`` = id, ``to_ip = to_port = 0``) and printed back from
    here; ids run to 2^32, so no input is refused."""

    def __init__(self):
        self.ids, self.values = {}, []

    def __call__(self, key):
        """Id of a key (a (proto, from, to, port) tuple of strings)."""
        k = self.ids.get(key)
        if k is None:
            k = len(self.values)
            if k > 0xFFFFFFFF:   # checked before the key is stored: no dangling id
                raise OverflowError('more than 2^32 distinct interned connection keys')
            self.ids[key] = k
            self.values.append(key)
        return k

    def strings(self, rows, spells):
        """(PROTO, FROMIP, TOIP, TOPORT) strings of one rule's records, some
        of them interned."""
        ps = rows['pspell'].tolist()
        s = self.values
        out = ([], [], [], [])
        for p, f, t, q in zip(ps, rows['for_ip'].tolist(), rows['to_ip'].tolist(), rows['to_port'].tolist()):
            vals = s[f] if p == INTERNED else (spells[p], _dotted(f), _dotted(t), str(q))
            for col, x in zip(out, vals):
                col.append(x)
        return out
