"""ORACLE — test infrastructure only. NOT part of the product path.

This package is a CPU restatement of the reference's hot path
(arnesund/ruleset-analysis: ``mapper.py | LC_ALL=C sort | connlist-reducer.py``)
used purely as a checker.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import, call, link or execute anything
under ``oracle/``; the product (``ruleset-analysis_amd/``) never does.

Modules (each function cites the reference file:line it restates):

* ``ipy``          — the subset of third-party ``IPy.IP`` the path uses
                     (IPy is not vendored; version unpinned).
* ``firewallrule`` — ``firewallrule.py:8-174`` (rule record + ``__contains__``).
* ``fwregex``      — ``get_builtconn`` of the absent ``lib/fw-regex`` submodule
                     (contract restated from ``mapper.py:124-145``; parity
                     unpinned for forms other than ``Built inbound TCP|UDP``).
* ``mapper``       — ``mapper.py:107-189``.
* ``reducer``      — ``connlist-reducer.py:25-211`` (``reducer.py`` is identical
                     except for the DB path, lines 34/37).
* ``pipeline``     — the no-Hadoop job ``mapper | LC_ALL=C sort | reducer``.
* ``rsa_oracle.c`` — the same classify + aggregate semantics over packed
                     arrays, in C, for parity at sizes pure Python cannot reach.

Pinning: ``firewallrule.py:177-220`` known-answer tests (tests/test_oracle_kat.py)
and golden report fixtures produced by a transient 2to3 conversion of the
reference scripts run in the build container (``oracle/crosscheck_2to3.py``,
fixtures under ``tests/golden/``).
"""
