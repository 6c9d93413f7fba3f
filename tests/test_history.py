"""paxi_amd.history: History.WriteFile / ReadFile formats (history.go:74-178)
on histories recorded by the CPU oracle (the device's history records have the
same layout; tests/test_parity_abd_gpu.py pins them to the oracle)."""
from paxi_amd import abi
from paxi_amd.history import History, Operation
import oracle_lib as ol


class _OracleAsSim:
    """Adapter: History.from_simulation over the oracle (test side only)."""
    def __init__(self, o, cfg):
        self.o, self.cfg = o, cfg

    def history(self, c):
        return self.o.history(c)


def _hist():
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=3, seed=3, keys=4, history=128)
    wl = abi.make_workload(outstanding=3, target=[0, 1, 2], write_ppm=500_000)
    o = ol.OracleSim(cfg, wl)
    o.step(1500)
    return History.from_simulation(_OracleAsSim(o, cfg), step_ns=1_000_000)


def test_from_simulation_maps_reads_and_writes():
    hs = _hist()
    assert len(hs) == 3 and all(len(h.operations) > 50 for h in hs)
    for h in hs:
        for key, ops in h.shard.items():
            assert 0 <= key < 4
            for op in ops:
                assert (op.input is None) != (op.output is None)
                assert op.start <= op.end and op.start % 1_000_000 == 0


def test_write_file_format(tmp_path):
    h = History()
    h.add(1, 7, None, 100_000_000, 600_000_000)
    h.add(2, None, 7, 0, 1_500_000_000)
    h.add(1, 9, None, 1_600_000_000, 2_400_000_000)
    h.write_file(str(tmp_path / "history"))
    lines = (tmp_path / "history.csv").read_text().splitlines()
    # sorted by start; a PerSecond line each time an op ends past the next second
    assert lines == ["<nil>,7,0.000000,1.500000",
                     "PerSecond 1500.000000 1",
                     "7,<nil>,0.100000,0.600000",
                     "9,<nil>,1.600000,2.400000",
                     "PerSecond 650.000000 2"]


def test_log_round_trip(tmp_path):
    for h in _hist():
        p = str(tmp_path / "log.csv")
        h.write_log(p)
        r = History.read_file(p)
        assert sorted(r.shard) == sorted(h.shard)
        for k in h.shard:
            want = [Operation(None if o.input is None else str(o.input), None if o.output is None else str(o.output),
                              o.start, o.end) for o in h.shard[k]]
            assert r.shard[k] == want


def test_read_file_rejects_short_records(tmp_path):
    p = tmp_path / "bad.csv"
    p.write_text("1,2,3\n")
    try:
        History.read_file(str(p))
    except ValueError as e:
        assert "format error" in str(e)
    else:
        raise AssertionError("expected a format error")
