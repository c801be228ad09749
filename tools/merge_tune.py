"""Merge newly tuned TunableOp entries (gpurun_out/tune0.csv) into a shipped table."""
import sys

new, table = sys.argv[1], sys.argv[2]
try:
    old = open(table).read().splitlines()
except FileNotFoundError:
    old = []
val = [l for l in old if l.startswith("Validator")]
ent = {",".join(l.split(",")[:2]): l for l in old if l and not l.startswith("Validator")}
for l in open(new).read().splitlines():
    if l.startswith("Validator"):
        if not val:
            val.append(l)
        continue
    if l:
        ent[",".join(l.split(",")[:2])] = l
if not val:
    val = [l for l in open(new).read().splitlines() if l.startswith("Validator")]
open(table, "w").write("\n".join(val + list(ent.values())) + "\n")
print(f"{table}: {len(ent)} entries")
