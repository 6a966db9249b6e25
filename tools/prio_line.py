import json, sys
d = json.load(open("gpurun_out/prio.json"))
s = d["stages_ms_per_step"]
print(sys.argv[1], d["value"], s["ba:wall"], s["sg:gnn x18"], s["sg:sinkhorn"])
