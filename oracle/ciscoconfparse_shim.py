"""ORACLE (test infrastructure only) — stand-in for the absent third-party
``ciscoconfparse`` package, as ``oracle/crosscheck_asa.py`` installs it next to
the lib2to3-converted ``preprosess_access_lists.py`` (which uses only
``CiscoConfParse(path).find_all_children(regex)``, ``:342,393,405``).

Restated from ciscoconfparse's published behaviour (version unpinned: the
reference ships no requirements file): a configuration line's children are the
following lines indented deeper than it; ``find_all_children`` returns every
line matching the regex and all its descendants, in file order, each once,
without the trailing newline."""

import re


class CiscoConfParse(object):
    def __init__(self, config):
        with open(config) as f:
            self.lines = [l.rstrip('\r\n') for l in f]

    def find_all_children(self, linespec):
        rx = re.compile(linespec)
        take = set()
        for i, l in enumerate(self.lines):
            if not rx.search(l):
                continue
            take.add(i)
            ind = len(l) - len(l.lstrip(' '))
            j = i + 1
            while j < len(self.lines):
                c = self.lines[j]
                if c.strip() == '' or len(c) - len(c.lstrip(' ')) <= ind:
                    break
                take.add(j)
                j += 1
        return [self.lines[i] for i in sorted(take)]
