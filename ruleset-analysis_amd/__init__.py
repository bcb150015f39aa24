"""ruleset-analysis on MI355X: first-match ACL classification of firewall
connection logs fused with per-rule hit/connection aggregation, in HIP for
gfx950 behind a C ABI (``include/ruleset_hip.h``).

Host-side modules mirror the reference's surface (``FirewallRule``,
``accesslists.db``, the mapper/reducer stdin/stdout contracts); the work runs
in ``libruleset_hip.so`` via ``native``/``engine``.  Import this package via
``rsa_pkg.load()`` (the directory name is not a Python identifier).
"""

__version__ = '0.1.0'
