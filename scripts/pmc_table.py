"""Per-kernel mean of every counter in gpurun_out/gemm_pmc_<tag>/pmc*/ (one line per kernel)."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/pmc*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-60:]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[k]["VGPR"] = [float(r.get("VGPR_Count") or 0)]
        acc[k]["AGPR"] = [float(r.get("Accum_VGPR_Count") or 0)]
for k, cs in acc.items():
    print(k)
    print("   " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
