"""tools/power_probe.py's analysis on fabricated metric samples (the sampler itself needs a GPU).

Pins: the GPU of the run is the one whose power moved; a phase's mean power, mean gfx clock over
the XCDs, energy per bootstrap from the accumulator (counter_resolution in microjoules) and the
PPT residency as a fraction of the accumulation counter.
"""
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import power_probe as pp  # noqa: E402


def _row(power, clk, energy, acc, ppt):
    return {"current_socket_power": power, "current_gfxclks": [clk] * 8, "energy_accumulator": energy,
            "accumulation_counter": acc, "ppt_residency_acc": ppt, "socket_thm_residency_acc": 0,
            "temperature_hotspot": 50, "throttle_status": "N/A", "indep_throttle_status": "N/A"}


def test_analyse_phases(tmp_path):
    res_uj = 15.3
    meta = [{"bdf": "0000:11:00.0", "energy": {"counter_resolution": res_uj}},
            {"bdf": "0000:72:00.0", "energy": {"counter_resolution": res_uj}}]
    lines = [json.dumps({"meta": meta})]
    # 1 s idle at 280 W, then 1 s of load at 1,300 W with PPT active 10% of the time; the other GPU flat
    e, acc, ppt = 0.0, 0, 0
    for i in range(201):
        t = i * 0.01
        load = t > 1.0
        w = 1300.0 if load else 280.0
        if i:
            e += w * 0.01 / (res_uj * 1e-6)
            acc += 10
            ppt += 1 if load else 0
        lines.append(json.dumps({"t": t, "g": [_row(200, 2400, 0, acc, 0),
                                              _row(w, 2300 if load else 2400, int(e), acc, ppt)]}))
    path = tmp_path / "samples.jsonl"
    path.write_text("\n".join(lines) + "\n")
    phases = [{"phase": "idle", "t0": 0.0, "t1": 0.995, "bootstraps": 0},
              {"phase": "load", "t0": 1.005, "t1": 2.0, "bootstraps": 1000}]
    rep = pp.analyse(str(path), phases)
    assert rep["gpu"]["bdf"] == "0000:72:00.0"
    idle, load = rep["phases"]
    assert idle["power_w_mean"] == pytest.approx(280.0)
    assert idle["gfxclk_mhz_mean"] == pytest.approx(2400.0)
    assert idle["ppt_residency_frac"] == 0
    assert load["power_w_mean"] == pytest.approx(1300.0)
    assert load["power_w_from_energy"] == pytest.approx(1300.0, rel=0.02)
    assert load["gfxclk_mhz_mean"] == pytest.approx(2300.0)
    assert load["ppt_residency_frac"] == pytest.approx(0.1)
    # 1,300 W over the phase's ~1 s and 1,000 bootstraps: ~1.3 J each
    assert load["mj_per_bootstrap"] == pytest.approx(1300.0 * (2.0 - 1.005), rel=0.02)
