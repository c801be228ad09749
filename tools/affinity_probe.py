import os, sys
sys.path.insert(0, ".")
from paddle_operator_amd.utils import topology
t = topology._from_sysfs()
print("allowed", len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:40])
if t:
    for i, g in enumerate(t.gpus[:8]):
        print("gpu", i, len(g.cpus), g.cpus[:8], "...")
print("nproc", os.cpu_count())
