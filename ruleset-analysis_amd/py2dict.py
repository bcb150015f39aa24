"""Iteration order of a Python 2.7 ``dict`` of ``str`` keys (64-bit CPython).

The reference reducer is Python 2: each rule block's connection table is
printed in ``conns.keys()`` order after a *stable* sort on the
``"TOIP TOPORT"`` string (``connlist-reducer.py:109-110,190-191``), so rows
that tie on that string come out in CPython 2.7 dict slot order — SURVEY.md
trap 8.  ``conns`` is a fresh ``{}`` per block and insert-only
(``:129,167-176``), with keys ``'PROTO;FROMIP;TOIP;TOPORT'`` (``:162``), so its
final slot layout is a pure function of the keys in first-insertion order.
This module replays it (CPython 2.7 ``Objects/dictobject.c`` and
``Objects/stringobject.c``, hash randomisation off, the 2.7 default):

* ``string_hash``: ``x = s[0] << 7; x = (1000003 * x) ^ c`` for every byte;
  ``x ^= len``; ``-1 -> -2`` — C ``long`` (64-bit) arithmetic;
* insertion: slot ``i = hash & mask``; while occupied,
  ``i = 5 * i + perturb + 1`` (unsigned, ``i`` not reduced), slot ``i & mask``,
  ``perturb >>= 5`` (``perturb`` starts as ``hash`` as unsigned);
* after inserting a NEW key: if ``fill * 3 >= (mask + 1) * 2`` resize to the
  smallest power of two ``> 4 * used`` (``> 2 * used`` above 50000 keys),
  minimum 8, re-inserting the old table's entries in slot order.

Host-side emitter logic only; nothing here runs on the GPU.
"""

import numpy as np

__all__ = ['string_hash', 'string_hashes', 'insert_order_to_iter_order', 'iteration_order']

M64 = (1 << 64) - 1
PERTURB_SHIFT = 5
MINSIZE = 8


def string_hash(s):
    """CPython 2.7 hash of a byte string (``bytes`` or latin-1 ``str``), as an
    unsigned 64-bit value (the bit pattern of the C ``long``)."""
    b = s.encode('latin-1') if isinstance(s, str) else bytes(s)
    if not b:
        return 0
    x = (b[0] << 7) & M64
    for c in b:
        x = ((1000003 * x) & M64) ^ c
    x ^= len(b)
    if x == M64:              # -1 is reserved for errors
        x = M64 - 1           # -2
    return x


def string_hashes(keys):
    """Vectorised ``string_hash`` over a list of str keys -> uint64 array."""
    n = len(keys)
    if n == 0:
        return np.zeros(0, np.uint64)
    enc = [k.encode('latin-1') for k in keys]
    lens = np.array([len(e) for e in enc], np.int64)
    L = int(lens.max())
    buf = np.zeros((n, max(L, 1)), np.uint64)
    flat = np.frombuffer(b''.join(e.ljust(L, b'\0') for e in enc), dtype=np.uint8).reshape(n, L) if L else None
    if L:
        buf[:, :] = flat
    with np.errstate(over='ignore'):
        x = buf[:, 0] << np.uint64(7)
        mul = np.uint64(1000003)
        for j in range(L):
            live = lens > j
            x = np.where(live, (mul * x) ^ buf[:, j], x)
        x ^= lens.astype(np.uint64)
    x[x == np.uint64(M64)] = np.uint64(M64 - 1)
    x[lens == 0] = 0
    return x


def insert_order_to_iter_order(hashes):
    """Slot order of an insert-only dict whose distinct keys (given by their
    hashes, in insertion order) were inserted one by one: returns the
    insertion indices in ``keys()`` order."""
    hashes = [int(h) for h in hashes]
    mask = MINSIZE - 1
    table = [-1] * MINSIZE
    fill = 0

    def place(tab, msk, h, k):
        i = h & msk
        if tab[i] >= 0:
            perturb = h
            while True:
                i = (5 * i + perturb + 1) & M64
                if tab[i & msk] < 0:
                    i &= msk
                    break
                perturb >>= PERTURB_SHIFT
        tab[i] = k

    for k, h in enumerate(hashes):
        place(table, mask, h, k)
        fill += 1
        if fill * 3 >= (mask + 1) * 2:
            minused = (2 if fill > 50000 else 4) * fill
            size = MINSIZE
            while size <= minused:
                size <<= 1
            new = [-1] * size
            for q in table:
                if q >= 0:
                    place(new, size - 1, hashes[q], q)
            table, mask = new, size - 1
    return [q for q in table if q >= 0]


def iteration_order(keys):
    """``keys()`` order of a fresh Python 2.7 dict after inserting the distinct
    str ``keys`` in this order: a permutation of ``range(len(keys))``."""
    return insert_order_to_iter_order(string_hashes(list(keys)))
