"""The committed measurement records hang together (CPU only): bench.py attaches
a traffic record only to a line of the same build, workload, window and
launch structure, and every committed final bench line carries the record of
its own build, with roofline arithmetic that follows from its fields."""
import json
import os
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CONFIGS = ["2", "3", "4", "4_fz0", "5"]


def _record(name):
    return json.load(open(os.path.join(ROOT, "profiles", f"traffic_config{name}.json")))


def _args(t):
    return types.SimpleNamespace(config=t["config"], clusters=t["clusters_per_gpu"], sim_steps=t["sim_steps_per_step"],
                                 window=t["window"], warmup=t["warmup"], steps=t["steps"], fz=t.get("fz", 1))


@pytest.mark.parametrize("name", CONFIGS)
def test_traffic_record_attaches_only_to_its_own_run(name):
    t = _record(name)
    a = _args(t)
    got = bench.measured_traffic(a, t["kernel"], t["mbox_cap"], t["build_id"], t["alg_bytes_per_launch"])
    assert got is not None and got["bytes_per_launch"] == t["bytes_per_launch"]
    # another build, another launch structure, another window: not attached
    assert bench.measured_traffic(a, t["kernel"], t["mbox_cap"], "0" * 16, t["alg_bytes_per_launch"]) is None
    assert bench.measured_traffic(a, t["kernel"], t["mbox_cap"], t["build_id"], 1.5 * t["alg_bytes_per_launch"]) is None
    a2 = types.SimpleNamespace(**vars(a))
    a2.steps += 1
    assert bench.measured_traffic(a2, t["kernel"], t["mbox_cap"], t["build_id"], t["alg_bytes_per_launch"]) is None


@pytest.mark.parametrize("name", CONFIGS)
def test_final_bench_lines_carry_their_builds_traffic(name):
    line = json.loads(open(os.path.join(ROOT, "profiles", "r6final", f"bench_config{name}.json")).read())
    r, t = line["roofline"], _record(name)
    assert line["build_id"] == t["build_id"] and line["build_matches_sources"]
    assert r["traffic"] == pytest.approx(t["bytes_per_launch"]) and r["kernel"] == t["kernel"]
    assert r["alg_bytes_per_launch"] == pytest.approx(t["alg_bytes_per_launch"], rel=1e-9)
    achieved = r["alg_bytes_per_launch"] / (r["avg_launch_ms"] / 1e3) / 1e9
    assert r["achieved"] == pytest.approx(achieved, rel=1e-9)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-9)
    ok, n = (int(x) for x in line["parity_sampled"].split("/"))
    assert ok == n > 0
