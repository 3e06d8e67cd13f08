"""Sparse-stage statistics of the bench corpus (events, pairs, FIRST matches per pattern) via tablesim."""
import collections
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
synth = importlib.import_module("context-based-pii_amd.synth")
compiler = importlib.import_module("context-based-pii_amd.compiler")
from tablesim import TableSim

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
comp = compiler.compile_default()
sim = TableSim(comp)
bank = synth.build_bank(16384, 16384, seed=synth.SEED)
meta = synth.corpus_meta(N // 100, 100, bank, seed=synth.SEED)
data = synth.gather_bytes(meta, bank)
o = meta.offsets
pairs = collections.Counter()
matched = collections.Counter()
ev_n = 0
steps = 0
for i in range(meta.n):
    t = data[o[i]:o[i + 1]].tobytes()
    ev = sim.scan(t, meta.role[i] == 1)
    for pos, sd, sk in ev:
        cd, _ = sim._classes(t, pos)
        a = int(sim.dacc[sd, cd])
        if a:
            ev_n += 1
        for k in range(int(sim.d_off[a]), int(sim.d_off[a + 1])):
            p = int(sim.d_ids[k])
            pairs[p] += 1
            e = sim.first_run(p, t, pos)
            if e >= 0:
                matched[p] += 1
names = [comp.rules.patterns[p].type_name for p in range(sim.P)]
print(f"utterances {meta.n}  D events/utt {ev_n / meta.n:.3f}  pairs/utt {sum(pairs.values()) / meta.n:.3f}  "
      f"matched/utt {sum(matched.values()) / meta.n:.3f}")
for p in sorted(pairs, key=lambda p: -pairs[p]):
    print(f"  {p:3d} {names[p]:28s} pairs/utt {pairs[p] / meta.n:.3f} matched/utt {matched[p] / meta.n:.3f}")
