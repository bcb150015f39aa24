"""Interned text of reducer connection keys outside the canonical form."""

__all__ = ['INTERNED', 'KeyText']


def _dotted(v):
    return '%d.%d.%d.%d' % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)


INTERNED = 0x80     # record pspell bit: the key's address / port fields are KeyText ids


class KeyText(object):
    """Interned text of connection keys that are not canonical dotted quads and
    ports (``10.0.0.01``, ``080``, or BUILT fields that differ from the mapper's
    tuple): the reducer keys its dict by the strings (connlist-reducer.py:167),
    so such a key is aggregated under ids of its own text (``pspell |
    INTERNED``) and printed back from here."""

    def __init__(self):
        self.ids, self.values = {}, []

    def __call__(self, text):
        k = self.ids.get(text)
        if k is None:
            k = self.ids[text] = len(self.values)
            self.values.append(text)
        return k

    def strings(self, rows, spells):
        """(PROTO, FROMIP, TOIP, TOPORT) strings of one rule's records, some
        of them interned."""
        ps = rows['pspell'].tolist()
        s = self.values
        out = ([], [], [], [])
        for p, f, t, q in zip(ps, rows['for_ip'].tolist(), rows['to_ip'].tolist(), rows['to_port'].tolist()):
            if p & INTERNED:
                vals = (spells[p & ~INTERNED], s[f], s[t], s[q])
            else:
                vals = (spells[p], _dotted(f), _dotted(t), str(q))
            for col, x in zip(out, vals):
                col.append(x)
        return out
