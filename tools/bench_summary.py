"""One-screen summary of a bench.py JSON line (tools/gpu_run.sh)."""
import json
import sys


def main(path):
    d = json.load(open(path))
    c = d["config"]
    r = d.get("roofline") or {}
    print(f"{path}: n_gpus={d['n_gpus']} {c['workload']} [{c['params']}, {c['shard']}, {d['scaling']}] "
          f"ms_per_step={d['ms_per_step']:.3f} value={d['value']:.0f} levels={d['levels']} "
          f"ok={d['result_decrypted'] == d['result_expected']} steps_ok={d.get('results_ok_steps')}")
    if r:
        ns = r.get("north_star_hbm") or {}
        print(f"  roofline frac={r['frac']:.3f} br_avg_ms={r['br_avg_ms']:.3f} pmc_stale={r.get('pmc_stale')} "
              f"north_star_hbm={ns.get('shape')}:{ns.get('physical_frac')} met={ns.get('met')}")
        for k, v in (r.get("per_shape") or {}).items():
            if v:
                print(f"  {k}: launches={v['launches']} per_launch={v['bootstraps_per_launch']:.0f} "
                      f"avg_ms={v['avg_ms']:.3f} frac={v['frac']:.3f}")
    for key in ("latency_probe", "kernel_saturated", "power", "fresh_content", "faithful", "faithful_tree", "inflight", "inflight_1ctx",
                "strong_starts", "weak_matches", "step_latency"):
        v = d.get(key)
        if v:
            if isinstance(v, dict):
                v = {k: (round(x, 4) if isinstance(x, float) else x) for k, x in v.items() if k not in ("per_rank", "note")}
            print(f"  {key}: {v}")
    if d.get("per_rank"):
        print(f"  per_rank: {d['per_rank']}")
    cb = d.get("cpu_baseline")
    if cb:
        print(f"  cpu: {cb['value']:.0f}/s on {cb['cores']} cores, 1t {cb['value_1t']:.1f}/s, match "
              f"{cb['match_ms']:.0f} ms, bit_identical={cb['cpu_gpu_bit_identical']}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
