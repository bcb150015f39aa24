"""Python 2 byte-string text semantics on latin-1 ``str``.

The reference runs under Python 2 on byte strings: ``strip()``
and ``split()`` only know the six ASCII whitespace bytes, ``lower()`` only
changes ``A-Z``, ``int()`` only takes ASCII digits, and ``re``'s ``\\d``/``\\s``/
``\\w`` are ASCII classes.  This package decodes config and log text as
latin-1 (one code point per byte), where Python 3's ``str`` methods also treat
``\\x1c-\\x1f``, ``\\x85`` and ``\\xa0`` as whitespace, lowercase ``\\xc0-\\xde``,
and accept ``_`` digit separators in ``int()`` — so every place that restates
reference text handling goes through these helpers instead.
"""

import re

__all__ = ['PY2_WS', 'PY2_MAXINT', 'py2_strip', 'py2_split', 'py2_lower', 'py2_int', 'py2_isdigit', 'py2_is_int']

PY2_WS = ' \t\n\r\x0b\x0c'          # what Python 2's byte-string strip()/split() treat as whitespace
PY2_MAXINT = (1 << 63) - 1          # sys.maxint of a 64-bit Python 2: int() of a larger literal is a long
_SPLIT = re.compile('[' + re.escape(PY2_WS) + ']+')
_LOWER = str.maketrans('ABCDEFGHIJKLMNOPQRSTUVWXYZ', 'abcdefghijklmnopqrstuvwxyz')
_INT = re.compile(r'[ \t\n\r\x0b\x0c]*[+-]?[0-9]+[ \t\n\r\x0b\x0c]*\Z')


def py2_strip(s):
    """``s.strip()`` of a Python 2 byte string."""
    return s.strip(PY2_WS)


def py2_split(s):
    """``s.split()`` (no argument) of a Python 2 byte string."""
    s = s.strip(PY2_WS)
    return _SPLIT.split(s) if s else []


def py2_lower(s):
    """``s.lower()`` of a Python 2 byte string (ASCII letters only)."""
    return s.translate(_LOWER)


def py2_isdigit(s):
    """``s.isdigit()`` of a Python 2 byte string (non-empty, ASCII digits only)."""
    return bool(s) and all('0' <= c <= '9' for c in s)


def py2_int(s):
    """``int(s)`` of a Python 2 byte string (ValueError as Python 2 raises it);
    ints pass through."""
    if isinstance(s, int):
        return s
    if not _INT.match(s):
        raise ValueError('invalid literal for int() with base 10: %r' % (s,))
    return int(s.strip(PY2_WS))


def py2_is_int(v):
    """``isinstance(v, int)`` under Python 2 for a number ``int()`` produced:
    values outside a 64-bit machine word are ``long``, not ``int``
    (``firewallrule.py:67-75`` rejects them as ports)."""
    return isinstance(v, int) and -PY2_MAXINT - 1 <= v <= PY2_MAXINT
