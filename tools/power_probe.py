"""Power, clock and throttle state of the GPU across the blind-rotation launch shapes.

Question: the saturated launches issue 0.58 VALU per CU-clock
against a measured 0.84 peak, and the chip clocks down from 2.43 GHz (1-16 bootstraps) to
~1.93 GHz (>= 254).  Is that clock-down the package power limit (PPT)?  If so, a higher issue
rate at the same energy per instruction turns into a lower clock, not into more bootstraps/s,
and the lever for saturated throughput is energy per bootstrap.

    python tools/power_probe.py OUT_DIR [--counts 1,16,254,512,2048] [--no-match] [--reps-scale X]
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_V.so python tools/power_probe.py ...   (a variant)
    python tools/power_probe.py --report OUT_DIR                                   (re-analyse)

A sampler child (started before anything touches the GPU; amdsmi reads the driver's
metrics table, no HIP) records every visible GPU's gpu_metrics every few ms; the workload
process runs phases of repeated launches (keyswitch + blind rotation, `fr_dev_bench_pbs`) and
one of back-to-back `/abc/` x 256 matches, and writes each phase's monotonic interval.
The report (OUT_DIR/power.json) gives per phase, for the GPU whose power rose: mean socket
power, gfx clock, the energy per bootstrap from the energy accumulator, and the fraction of
the phase the firmware spent power-limited (ppt_residency_acc) or thermally limited.
"""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

FIELDS = ("current_socket_power", "average_socket_power", "current_gfxclk", "current_gfxclks",
          "average_gfxclk_frequency", "energy_accumulator", "accumulation_counter", "ppt_residency_acc",
          "socket_thm_residency_acc", "vr_thm_residency_acc", "hbm_thm_residency_acc", "prochot_residency_acc",
          "throttle_status", "indep_throttle_status", "temperature_hotspot", "temperature_mem",
          "average_gfx_activity", "voltage_gfx", "firmware_timestamp")


def sampler(out_path, stop_path, period_s=0.004):
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    meta = []
    for h in hs:
        m = {"bdf": amdsmi.amdsmi_get_gpu_device_bdf(h)}
        for name, fn in (("power_cap", amdsmi.amdsmi_get_power_cap_info), ("energy", amdsmi.amdsmi_get_energy_count)):
            try:
                m[name] = fn(h)
            except Exception as e:  # noqa: BLE001 -- record what the driver refuses
                m[name] = repr(e)
        meta.append(m)
    with open(out_path, "w") as f:
        f.write(json.dumps({"meta": meta}) + "\n")
        while not os.path.exists(stop_path):
            t = time.monotonic()
            rows = []
            for h in hs:
                try:
                    g = amdsmi.amdsmi_get_gpu_metrics_info(h)
                    rows.append({k: g.get(k) for k in FIELDS})
                except Exception as e:  # noqa: BLE001
                    rows.append({"err": repr(e)})
            f.write(json.dumps({"t": t, "g": rows}, default=str) + "\n")
            dt = period_s - (time.monotonic() - t)
            if dt > 0:
                time.sleep(dt)
    amdsmi.amdsmi_shut_down()


def _num(v):
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, str):
        try:
            return float(v.split()[0])
        except ValueError:
            return None
    return None


def _clk(row):
    v = row.get("current_gfxclks")
    if isinstance(v, list):
        xs = [_num(x) for x in v]
        xs = [x for x in xs if x is not None and 0 < x < 10000]
        if xs:
            return sum(xs) / len(xs)
    return _num(row.get("current_gfxclk"))


def analyse(samples_path, phases):
    lines = open(samples_path).read().splitlines()
    meta = json.loads(lines[0])["meta"]
    samples = [json.loads(x) for x in lines[1:] if x]
    ng = len(meta)
    # the GPU of this run: the largest power spread over the run
    spread = []
    for i in range(ng):
        p = [_num(s["g"][i].get("current_socket_power")) for s in samples if i < len(s["g"])]
        p = [x for x in p if x is not None]
        spread.append((max(p) - min(p)) if p else -1)
    gi = max(range(ng), key=lambda i: spread[i])
    res = _num((meta[gi].get("energy") or {}).get("counter_resolution")) if isinstance(meta[gi].get("energy"), dict) else None
    out = {"gpu": meta[gi], "n_samples": len(samples), "phases": []}
    for ph in phases:
        inside = [s for s in samples if ph["t0"] <= s["t"] <= ph["t1"]]
        rows = [s["g"][gi] for s in inside]
        rec = {k: ph[k] for k in ph if k not in ("t0", "t1")}
        rec["seconds"] = ph["t1"] - ph["t0"]
        rec["samples"] = len(rows)
        if rows:
            pw = [x for x in (_num(r.get("current_socket_power")) for r in rows) if x is not None]
            ck = [x for x in (_clk(r) for r in rows) if x is not None]
            rec["power_w_mean"] = sum(pw) / len(pw) if pw else None
            rec["power_w_max"] = max(pw) if pw else None
            rec["gfxclk_mhz_mean"] = sum(ck) / len(ck) if ck else None
            rec["gfxclk_mhz_min"] = min(ck) if ck else None
            rec["hotspot_c_max"] = max((_num(r.get("temperature_hotspot")) or 0) for r in rows)
            rec["throttle_status"] = sorted({str(r.get("throttle_status")) for r in rows})
            rec["indep_throttle_status"] = sorted({str(r.get("indep_throttle_status")) for r in rows})
            first, last = rows[0], rows[-1]
            acc = (_num(last.get("accumulation_counter")) or 0) - (_num(first.get("accumulation_counter")) or 0)
            for key in ("ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc",
                        "hbm_thm_residency_acc", "prochot_residency_acc"):
                d = (_num(last.get(key)) or 0) - (_num(first.get(key)) or 0)
                rec[key.replace("_acc", "_frac")] = d / acc if acc > 0 else None
            e = (_num(last.get("energy_accumulator")) or 0) - (_num(first.get("energy_accumulator")) or 0)
            dt = inside[-1]["t"] - inside[0]["t"]
            if res and e > 0 and dt > 0:
                joules = e * res * 1e-6  # counter_resolution is in microjoules
                rec["energy_j"] = joules
                rec["power_w_from_energy"] = joules / dt
                if ph.get("bootstraps"):
                    rec["mj_per_bootstrap"] = 1e3 * joules / dt * (ph["t1"] - ph["t0"]) / ph["bootstraps"]
        out["phases"].append(rec)
    return out


def workload(out_dir, phases, counts, reps_scale=1.0, match=True, idle_s=1.0):
    sys.path.insert(0, os.path.join(ROOT, "fhe-regex_amd"))
    import numpy as np
    import fheregex as F
    blob = open(os.path.join(ROOT, "tests", "golden", "client_key"), "rb").read()
    ck, sk = F.gen_keys(blob, seed=1, device=0)
    ctx = ck.ctx
    rng = np.random.default_rng(5)
    s = "".join(chr(c) for c in rng.integers(0x20, 0x7F, 256))
    s = s[:200] + "abc" + s[203:]
    hs = ctx.encrypt_upload_str(s, seed=3)

    def mark(name, fn, bootstraps):
        fn()  # warm
        t0 = time.monotonic()
        n = fn()
        t1 = time.monotonic()
        phases.append({"phase": name, "t0": t0, "t1": t1, "bootstraps": (n or 0) * bootstraps})
        print(f"{name}: {t1 - t0:.2f} s", flush=True)

    def idle():
        time.sleep(idle_s)
        return 0

    # about 1.2 s of launches per phase
    reps_of = {1: 900, 16: 900, 254: 800, 512: 500, 2048: 130}
    mark("idle", idle, 0)
    for cnt in counts:
        reps = max(2, int(reps_scale * reps_of.get(cnt, max(2, int(1.2e3 / (1.3 + 4.8e-3 * cnt))))))
        sel = [hs[i % len(hs)] for i in range(cnt)]

        def run(sel=sel, reps=reps):
            ctx.dev_bench_pbs(sel, reps)
            return reps
        mark(f"launch_{cnt}", run, cnt)

    if not match:
        return
    out, st = ctx.has_match(hs, "/abc/")
    per = int(st.blind_rotations)

    def matches(reps=250):
        for i in range(reps):
            o, _ = ctx.has_match(hs, "/abc/")
            if i + 1 < reps:
                ctx.release(o)
        assert ctx.decrypt_radix(ctx.download_radix(o)) == 1  # waits for the last match
        ctx.release(o)
        return reps
    mark("metric_match", matches, per)
    mark("idle_after", idle, 0)


def main():
    if len(sys.argv) >= 2 and sys.argv[1] == "--sample":
        sampler(sys.argv[2], sys.argv[3])
        return 0
    if len(sys.argv) >= 2 and sys.argv[1] == "--report":
        return report(sys.argv[2])
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--counts", default="1,16,254,512,2048", help="bootstraps per launch, one phase each")
    ap.add_argument("--reps-scale", type=float, default=1.0, help="scale every phase's launch count")
    ap.add_argument("--no-match", action="store_true", help="skip the /abc/ x 256 match phase")
    ap.add_argument("--idle", type=float, default=1.0, help="seconds of the idle phases")
    args = ap.parse_args()
    out_dir = args.out_dir
    os.makedirs(out_dir, exist_ok=True)
    samples = os.path.join(out_dir, "samples.jsonl")
    stop = os.path.join(out_dir, ".stop")
    if os.path.exists(stop):
        os.remove(stop)
    # the sampler starts before this process touches the GPU
    child = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--sample", samples, stop])
    time.sleep(2.0)
    phases = []
    rc = 0
    try:
        workload(out_dir, phases, [int(c) for c in args.counts.split(",") if c], args.reps_scale,
                 not args.no_match, args.idle)
    except Exception as e:  # noqa: BLE001 -- still stop the sampler and report what ran
        print("workload failed:", repr(e), flush=True)
        rc = 1
    finally:
        open(stop, "w").close()
        child.wait(timeout=30)
        with open(os.path.join(out_dir, "phases.json"), "w") as f:
            json.dump(phases, f)
    return report(out_dir) or rc


def report(out_dir):
    samples = os.path.join(out_dir, "samples.jsonl")
    phases = json.load(open(os.path.join(out_dir, "phases.json")))
    rep = analyse(samples, phases)
    with open(os.path.join(out_dir, "power.json"), "w") as f:
        json.dump(rep, f, indent=1, default=str)
    for p in rep["phases"]:
        print(json.dumps({k: p.get(k) for k in ("phase", "seconds", "samples", "power_w_mean", "gfxclk_mhz_mean",
                                                  "ppt_residency_frac", "socket_thm_residency_frac", "mj_per_bootstrap",
                                                  "throttle_status")}, default=str), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
