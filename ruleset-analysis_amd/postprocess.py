"""Downstream of the path: the Hadoop output form of the reducer report and
the zero-hit / connection-list report of ``postprocess_ruleset_analysis.py``.

* ``hadoop_output``: Hadoop streaming writes every reducer stdout line as a
  (key, empty value) pair through ``TextOutputFormat``: ``line + '\\t\\n'``; a
  ``hadoop dfs -getmerge`` of the job output is what the postprocessor reads
  and splits on ``'\\t\\n\\t\\n'`` (``postprocess_ruleset_analysis.py:86``; the
  blank line before each rule block, ``connlist-reducer.py:113``).
* ``postprocess``: restates ``postprocess_ruleset_analysis.py:77-177`` — every
  entry is attached to its rule (``:94-105``), then three sections: the whole
  rule set with hit counts (``:107-123``), the ACL lines none of whose expanded
  rules had a hit (``:125-160``), and each supported rule's connection list
  (``:163-177``).  Hosts iterate in Python 2 dict order of first appearance
  (``seenhosts``, ``py2dict``); ACLs in order of first appearance.

Host-side text work (the report is per rule, not per log line).
"""

import re

from .py2dict import iteration_order
from .py2text import py2_strip

__all__ = ['hadoop_output', 'postprocess', 'SUPPORTED_PROTOCOLS']

SUPPORTED_PROTOCOLS = ['ip', 'tcp', 'udp']
SUPPORTED_ACTIONS = [True]
_ENTRY = re.compile(r'([a-zA-Z0-9_-]+): access-list ([a-zA-Z0-9_-]+), rule ([0-9]+):', re.DOTALL)
_HITS = re.compile(r'Total number of hits: ([0-9]+)', re.DOTALL)


def hadoop_output(lines):
    """Reducer stdout lines as Hadoop streaming stores them (TextOutputFormat,
    key = the line, empty value)."""
    return ''.join(l + '\t\n' for l in lines)


def postprocess(accesslists, text):
    """Lines printed by postprocess_ruleset_analysis.py for the merged Hadoop
    output ``text`` and the rule DB's ``accesslists``."""
    entries = text.split('\t\n\t\n')
    results = {}                     # (host, acl) -> {ruleindex: entry}
    seen_order, seen = [], {}
    for entry in entries:
        firewall, acl, ruleindex = _ENTRY.findall(entry)[0]      # IndexError as the reference
        accesslists[firewall][acl]['rules'][int(ruleindex)]      # IndexError / KeyError as the reference
        results.setdefault((firewall, acl), {})[int(ruleindex)] = entry
        if firewall not in seen:
            seen[firewall] = []
            seen_order.append(firewall)
        if acl not in seen[firewall]:
            seen[firewall].append(acl)
    hosts = [seen_order[k] for k in iteration_order(seen_order)]
    out = ['ENTIRE RULESET WITH HITCOUNTS', '']
    hitcount = {}
    for fw in hosts:
        for acl in seen[fw]:
            res = results.get((fw, acl), {})
            rules = accesslists[fw][acl]['rules']
            hc = []
            for i in range(len(rules)):
                entry = res.get(i)
                h = int(_HITS.findall(entry)[0]) if entry is not None else 0
                hc.append(h)
                rule = rules[i]
                if rule.protocol in SUPPORTED_PROTOCOLS and rule.action in SUPPORTED_ACTIONS:
                    out.append(' {0:15}  {1}  ({2})'.format(h, rule.original, str(rule)))
            hitcount[(fw, acl)] = hc
    out.append('')
    out.extend(['DISTINCT RULES WITH NO HITS', ''])
    for fw in hosts:
        for acl in seen[fw]:
            rules = accesslists[fw][acl]['rules']
            hc = hitcount[(fw, acl)]
            current = None
            nonehits = True
            for i in range(len(rules)):
                rule = rules[i]
                if current is None:
                    current = rule
                if rule.rulenum == current.rulenum:
                    if hc[i] > 0:
                        nonehits = False
                else:
                    if nonehits and current.protocol in SUPPORTED_PROTOCOLS and current.action in SUPPORTED_ACTIONS:
                        out.extend(py2_strip(line) for line in current.comments)
                        out.append('{0}'.format(current.original))
                    current = rule
                    nonehits = False if hc[i] > 0 else True
    out.append('')
    out.extend(['CONNLIST FOR EACH RULE', ''])
    for fw in hosts:
        for acl in seen[fw]:
            res = results.get((fw, acl), {})
            rules = accesslists[fw][acl]['rules']
            for i in range(len(rules)):
                rule = rules[i]
                if rule.protocol in SUPPORTED_PROTOCOLS and rule.action in SUPPORTED_ACTIONS:
                    if i in res:
                        out.append(res[i])
                        out.append('')
                    else:
                        out.append('{0}: access-list {1}, rule {2}: {3}'.format(fw, acl, str(rule.ruleindex), str(rule)))
                        out.append('{0}'.format(rule.original))
                        out.append('')
    return out
