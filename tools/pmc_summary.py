"""Summarise rocprofv3 PMC passes (tools/profile.sh output) for the BR kernel.

HBM bytes per launch = (FETCH_SIZE x 2 + WRITE_SIZE) KiB x 1024, with the gfx950
FETCH_SIZE correction (x2 for 16-B-per-lane streaming reads,
MI355X_MICROARCH.md HBM section).  Launches are grouped by grid size; the
per-match average over the blind-rotation launches of one has_match is what
bench.py reports as roofline.traffic.
The compute side: VALU wave-instructions (SQ_INSTS_VALU) per active-CU clock,
active CUs = min(workgroups, 256), clocks = GRBM_GUI_ACTIVE / 8 (the sum over the
8 XCDs; MI355X_MICROARCH.md "DVFS give-back"), summed over the match's launches.
The kernel source hash lets bench.py flag a summary of an older kernel as stale.
Usage: python3 tools/pmc_summary.py PROFDIR OUT.json [k]
"""
import collections
import csv
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d, name):
    p = os.path.join(d, name, "run_counter_collection.csv")
    rows = list(csv.DictReader(open(p)))
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = (k, int(r["Grid_Size"]))
        out[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        out[key]["_wg"] = [float(r["Workgroup_Size"])]
    return out


def main():
    d, out_path = sys.argv[1], sys.argv[2]
    fetch, write = load(d, "pmc_fetch"), load(d, "pmc_write")
    sq, lds = load(d, "pmc_sq"), load(d, "pmc_lds")
    launches = []
    for key in sorted(fetch):
        k, grid = key
        if "blind_rotate" not in k:
            continue
        f = fetch[key]["FETCH_SIZE"]
        w = write.get(key, {}).get("WRITE_SIZE", [0.0])
        wg = fetch[key]["_wg"][0]
        # k_blind_rotate_fft<N, K, E, LAT, B>: B bootstraps per workgroup (the pair shape: 2)
        targs = k.split("<")[1].rstrip(">").split(",") if "<" in k else []
        per_wg = int(targs[4]) if "blind_rotate_fft" in k and len(targs) >= 5 else 1
        ent = {"kernel": k, "grid": grid, "workgroups": int(grid // wg), "bootstraps": int(grid // wg) * per_wg,
               "calls": len(f),
               "fetch_bytes": 2 * 1024 * sum(f) / len(f), "write_bytes": 1024 * sum(w) / len(w)}
        ent["hbm_bytes"] = ent["fetch_bytes"] + ent["write_bytes"]
        s = sq.get(key, {})
        if s:
            avg = {c: sum(v) / len(v) for c, v in s.items()}
            wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
            ent["wave_cycle_split"] = {"active": avg.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                       "issue_stall": avg.get("SQ_WAIT_INST_ANY", 0) / wc,
                                       "parked": avg.get("SQ_WAIT_ANY", 0) / wc}
            ent["valu_insts"] = avg.get("SQ_INSTS_VALU")
        l = lds.get(key, {})
        if l:
            avg = {c: sum(v) / len(v) for c, v in l.items()}
            ent["lds_bank_conflict_cycles"] = avg.get("SQ_LDS_BANK_CONFLICT")
            ent["lds_insts"] = avg.get("SQ_INSTS_LDS")
            ent["grbm_gui_active_per_xcd"] = avg.get("GRBM_GUI_ACTIVE", 0) / 8
        launches.append(ent)
    # one has_match = the launches of the four levels; the saturated probe is the biggest grid
    sat = max(launches, key=lambda e: e["grid"]) if launches else None
    match = [e for e in launches if e is not sat]
    per_launch = sum(e["hbm_bytes"] * e["calls"] for e in match) / max(1, sum(e["calls"] for e in match))
    ring = "fft" if any("blind_rotate_fft" in e.get("kernel", "") for e in launches) else "rns"
    valu = sum(e.get("valu_insts") or 0 for e in match)
    cu_clk = sum(min(e["workgroups"], 256) * e.get("grbm_gui_active_per_xcd", 0) for e in match)
    h = hashlib.sha256()  # as bench.kernel_source_sha
    for rel in ("csrc/fft_br.hip", "csrc/fft_br_pair.hip", "Makefile"):
        h.update(open(os.path.join(REPO, "fhe-regex_amd", rel), "rb").read())
    res = {"hbm_bytes_per_launch": per_launch, "ring": ring, "k": int(sys.argv[3]) if len(sys.argv) > 3 else 1,
           "valu_per_cu_clk": valu / cu_clk if valu and cu_clk else None,
           "kernel_sha": h.hexdigest()[:16],
           "note": "FETCH_SIZE x2 (gfx950) + WRITE_SIZE, blind-rotation launches of the match, averaged per "
                   "launch; valu_per_cu_clk = sum SQ_INSTS_VALU / sum min(workgroups, 256) GRBM_GUI_ACTIVE/8",
           "launches": launches}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "valu_per_cu_clk", "kernel_sha")}, indent=1))


if __name__ == "__main__":
    main()
