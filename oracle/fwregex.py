"""ORACLE (test infrastructure only) — restatement of ``get_builtconn``.

The reference imports it from the git submodule ``lib/fw-regex``
(``mapper.py:6,11``; ``.gitmodules:1-3``), which is ABSENT from
``/root/reference`` and unreachable offline, so its contract is restated from
its call site (``mapper.py:124-145``: a dict with ``year, month, day, time,
protocol, direction, interface_in, interface_out, src, dst, sport, dport`` or a
falsy value).  Parity is therefore UNPINNED for anything but the canonical
Cisco ASA/FWSM/PIX "Built {inbound|outbound} {TCP|UDP} connection" message
(%-6-302013 / 302015), which is the only form the synthetic logs use.

Definition used by this build (and by the product's host parser — the two are
written independently against this same definition):

* header: relay ``Mon d HH:MM:SS`` then optionally the device date
  ``Mon d YYYY HH:MM:SS:``; ``year`` is the device year or None;
* body: ``%(ASA|FWSM|PIX)-<sev>-<6 digits>: Built (inbound|outbound) (TCP|UDP)
  connection <id> for IFC:IP/PORT (...) to IFC:IP/PORT``;
* inbound: the ``for`` side is the source / ingress interface; outbound: the
  ``to`` side is (the initiator sits behind the ``to`` interface) — an
  assumption about fw-regex, documented in DESIGN.md.
"""

import re

_HEAD = re.compile(r'^([A-Z][a-z]{2}) +(\d{1,2}) (\d\d:\d\d:\d\d) '
                   r'(?:([A-Z][a-z]{2}) +(\d{1,2}) (\d{4}) (\d\d:\d\d:\d\d): )?')
_BODY = re.compile(r'%(?:ASA|FWSM|PIX)-\d-\d{6}: Built (inbound|outbound) (TCP|UDP) connection \d+ '
                   r'for ([A-Za-z0-9_-]+):([0-9.]+)/([0-9]+) \([^)]*\) '
                   r'to ([A-Za-z0-9_-]+):([0-9.]+)/([0-9]+)')


def get_builtconn(line):
    h = _HEAD.match(line)
    if not h:
        return None
    b = _BODY.search(line, h.end())
    if not b:
        return None
    if h.group(6):
        month, day, year, time = h.group(4), h.group(5), h.group(6), h.group(7)
    else:
        month, day, year, time = h.group(1), h.group(2), None, h.group(3)
    direction, proto, ifc1, ip1, p1, ifc2, ip2, p2 = b.groups()
    if direction == 'inbound':
        ifc_in, src, sport, ifc_out, dst, dport = ifc1, ip1, p1, ifc2, ip2, p2
    else:
        ifc_in, src, sport, ifc_out, dst, dport = ifc2, ip2, p2, ifc1, ip1, p1
    return {'year': year, 'month': month, 'day': day, 'time': time,
            'protocol': proto, 'direction': direction,
            'interface_in': ifc_in, 'interface_out': ifc_out,
            'src': src, 'dst': dst, 'sport': sport, 'dport': dport}
