"""Config-5 candidate funnel per SCAN group and pattern kind (tablesim over a random sample of the
config-5 bank): D events, candidate pairs, FIRST matches, pairs per match.
usage: python tools/c5_pairs.py [N_ROWS]"""
import collections
import importlib
import os
import random
import re
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
compiler = importlib.import_module("context-based-pii_amd.compiler")
rulegen = importlib.import_module("context-based-pii_amd.rulegen")
from tablesim import TableSim  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
c5 = rulegen.Config5()
path = os.path.join(tempfile.gettempdir(), "c5_pairs.json")
c5.save(path)
comp = compiler.compile_rules(compiler.Rules.load(path))
sim = TableSim(comp)
bank = c5.build_bank()
r = random.Random(1)
idx = [r.randrange(len(bank.texts)) for _ in range(N)]
pats = comp.rules.patterns
group_of = {}
for g, gp in enumerate(comp.scan_groups):
    for p in gp:
        group_of[p] = g


def kind(p):
    t = pats[p].type_name
    if not t.startswith("CUSTOM_"):
        return "builtin"
    m = re.match(r"CUSTOM_ID_(\d+)", t)
    if m:
        return f"regex{int(m.group(1)) % 5}"
    return "dict"


ev = collections.Counter()
pairs = collections.Counter()
matched = collections.Counter()
pk = collections.Counter()
mk = collections.Counter()
pp = collections.Counter()
mp = collections.Counter()
for i in idx:
    t = bank.texts[i]
    agent = bank.roles[i] == 1
    for pos, sd, sk in sim.scan(t, agent):
        a = sim.d_accept(t, pos, sd) if sd >= 0 else 0
        g = sd >> 20
        if a:
            ev[g] += 1
        for k in range(int(sim.d_off[a]), int(sim.d_off[a + 1])):
            p = int(sim.d_ids[k])
            pairs[group_of[p]] += 1
            pk[kind(p)] += 1
            pp[p] += 1
            if sim.first_run(p, t, pos) >= 0:
                matched[group_of[p]] += 1
                mk[kind(p)] += 1
                mp[p] += 1
print(f"{N} rows; groups {len(comp.scan_groups)}")
for g in sorted(set(ev) | set(pairs)):
    gp = comp.scan_groups[g]
    print(f"group {g}: {len(gp):3d} patterns  events/row "
          f"{ev[g] / N:6.3f} pairs/row {pairs[g] / N:6.3f} matched/row {matched[g] / N:6.3f} "
          f"pairs/match {pairs[g] / max(1, matched[g]):6.2f}  kinds {dict(collections.Counter(kind(p) for p in gp))}")
print("per kind: pairs/row, matched/row, pairs/match")
for k in sorted(pk):
    print(f"  {k:8s} {pk[k] / N:7.3f} {mk[k] / N:7.3f} {pk[k] / max(1, mk[k]):6.2f}")
print(f"total pairs/row {sum(pairs.values()) / N:.3f}  matched/row {sum(matched.values()) / N:.3f}")
print("top patterns by unmatched pairs/row: pattern, type, prefix, pairs/row, matched/row")
for p, c in sorted(pp.items(), key=lambda x: -(x[1] - mp[x[0]]))[:15]:
    print(f"  {p:4d} {pats[p].type_name:34s} {str(pats[p].scan_prefix):5s} {c / N:7.3f} {mp[p] / N:7.3f}  {pats[p].pattern[:60]}")
