import json,sys
for line in open(sys.argv[1]):
    if not line.startswith('{'): continue
    d=json.loads(line)
    print(d["config"]["workload"], round(d["ms_per_step"],3), [(k["kernel"][5:],round(k["avg_us"],1),round(k["frac"],3)) for k in d["edge_kernels"]])
    if "bf16" in d: print(" bf16", round(d["bf16"]["ms_per_step"],3), [(k["kernel"][5:],round(k["avg_us"],1),round(k["frac"],3)) for k in d["bf16"]["edge_kernels"]])
