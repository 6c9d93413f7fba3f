"""G1-G14 (SURVEY.md §8 semantic gotchas) as hand-derived scripted traces,
checked on the CPU oracle here and on the HIP kernels under -m gpu.

Every expected value in tests/golden/kats.json["gtraces"] was derived from
the Go source (paxos/paxos.go, socket.go, ballot.go, quorum.go, node.go,
http.go; the derivation is stored next to each trace), not produced by either
backend, so these pin both implementations to the reference independently of
each other."""
import pytest

import gtrace_lib as gt
import oracle_lib as ol

IDS = [t["name"] for t in gt.GTRACES]
CASES = [(t, s) for t in gt.GTRACES for s in gt.seeds_for(t)]
CASE_IDS = [f"{t['name']}-s{s}" for t, s in CASES]


def test_every_gotcha_has_a_trace():
    covered = {g for t in gt.GTRACES for g in t["gotchas"]}
    assert covered == {f"G{i}" for i in range(1, 15)}


@pytest.mark.parametrize("tr,seed", CASES, ids=CASE_IDS)
def test_gtrace_oracle(tr, seed):
    cfg, wl, faults = gt.build(tr, seed)
    sim = ol.OracleSim(cfg, wl, faults=faults)
    errs = gt.run(sim, tr, exec_log=lambda s, r: s.exec_log(0, r))
    assert not errs, "\n".join(errs)


@pytest.mark.gpu
@pytest.mark.parametrize("tr,seed", CASES, ids=CASE_IDS)
def test_gtrace_gpu(tr, seed):
    from paxi_amd.sim import Simulation
    cfg, wl, faults = gt.build(tr, seed)
    cfg.steps_per_launch = 1
    sim = Simulation(cfg, wl, faults=faults)
    # the device keeps an executed-history digest, not the log: compare it to
    # the oracle's digest of the hand-derived executed sequence
    errs = gt.run(sim, tr)
    ref = ol.OracleSim(*gt.build(tr, seed)[:2], faults=gt.build(tr, seed)[2])
    gt.run(ref, tr)
    for r, (a, b) in enumerate(zip(sim.read_state(), ref.read_state())):
        if a.digest != b.digest:
            errs.append(f"replica {r} executed digest differs from the oracle's")
    assert not errs, "\n".join(errs)
