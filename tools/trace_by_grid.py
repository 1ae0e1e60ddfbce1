"""Per (kernel, grid) average durations from a rocprofv3 kernel trace, beside the bench
line's per-shape averages (the contract's check that the trace agrees with the HIP-event
timers of the timed region).
Usage: python3 tools/trace_by_grid.py TRACE_DIR [bench.json] > out.json"""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
g = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "blind_rotate" not in k and "k_ks" not in k:
        continue
    g[(k, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {"launches": [{"kernel": k, "workgroups": wg, "calls": len(v), "avg_ms": sum(v) / len(v)}
                    for (k, wg), v in sorted(g.items())]}
match = [e for e in out["launches"] if "blind_rotate" in e["kernel"] and e["workgroups"] <= 256]
if match:
    out["match_br_avg_ms"] = sum(e["avg_ms"] for e in match) / len(match)
if len(sys.argv) > 2:
    b = json.load(open(sys.argv[2]))["roofline"]
    out["bench_br_avg_ms"] = b["br_avg_ms"]
    out["bench_per_shape_avg_ms"] = {s: v["avg_ms"] for s, v in b["per_shape"].items() if v}
print(json.dumps(out, indent=1))
