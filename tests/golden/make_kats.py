"""Writes tests/golden/kats.json: known-answer vectors for the oracle.

Sources (data only — inputs and expected outputs, no reference code):
  * ballot_test.go:7-22            NewBallot(0, "2.1"), Next twice -> N()==2, ID()=="2.1"
  * checker_test.go:6-136          linearizability histories + expected anomaly counts
                                   ("== 0", "> 0", "== 2") of TestLinerizabilityChecker
                                   and TestNonUniqueValue
  * hand-derived from the Go source (BASELINE.md anchors):
      - NewBallot(1,"1.1") = 4295032833, (1,"1.2") = 4295032834, (2,"2.3") = 8590065667
      - Majority thresholds 2/3/5 at N=3/5/9 (quorum.go:60-62: size > n/2)
      - FGrid 3x3 minimum quorum sizes (quorum.go:100-119)
      - config 1 (N=3, one client, 1000 sequential writes to 1.1, no faults):
        P1a 2, P1b 2, P2a/P2b/P3 2000 each = 6004 socket messages; leader
        1.1 ends active with ballot 4295032833, slot 999, execute 1000.
Run: python tests/golden/make_kats.py
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")

kats = {
    "ballot_test": {"start_n": 0, "zone": 2, "node": 1, "nexts": 2, "expect_n": 2, "expect_id": [2, 1]},
    "ballot_values": [[1, 1, 1, 4295032833], [1, 1, 2, 4295032834], [2, 2, 3, 8590065667]],
    "majority_min": {"3": 2, "5": 3, "9": 5},
    # [fz, q1_min, q2_min] for a 3x3 grid; fz=0 is the Grid (GridRow / GridColumn) variant
    "fgrid_3x3_min": [[0, 3, 3], [1, 4, 4], [2, 2, 6]],
    # checker_test.go: (input, output, start, end); null = nil.  expect: "zero" | "nonzero" | int
    "checker": [
        {"name": "single", "ops": [[42, None, 0, 24]], "expect": "zero"},
        {"name": "concurrent_wr", "ops": [[42, None, 0, 5], [None, 42, 3, 10]], "expect": "zero"},
        {"name": "no_dependency", "ops": [[1, None, 0, 5], [None, 2, 6, 10], [3, None, 11, 15], [None, 4, 16, 20]],
         "expect": "zero"},
        {"name": "concurrent_reads", "ops": [[0, None, 0, 0], [100, None, 0, 100], [None, 100, 5, 35], [None, 0, 30, 60]],
         "expect": "zero"},
        {"name": "nonconcurrent_reads", "ops": [[0, None, 0, 0], [100, None, 0, 100], [None, 100, 5, 25], [None, 0, 30, 60]],
         "expect": "nonzero"},
        {"name": "read_misses_write", "ops": [[1, None, 0, 5], [2, None, 6, 10], [None, 1, 11, 15]], "expect": "nonzero"},
        {"name": "cross_reads", "ops": [[1, None, 0, 5], [2, None, 0, 5], [None, 1, 6, 10], [None, 2, 6, 10]],
         "expect": "nonzero"},
        {"name": "two_anomalies", "ops": [[1, None, 0, 5], [2, None, 6, 10], [None, 1, 11, 15], [None, 1, 12, 16]],
         "expect": 2},
        {"name": "link_between_writes", "ops": [[1, None, 0, 5], [None, 1, 6, 10], [2, None, 7, 10], [None, 1, 11, 15]],
         "expect": "nonzero"},
        {"name": "non_unique_value", "ops": [[1, None, 0, 5], [1, None, 0, 5], [None, 1, 6, 10], [None, 1, 6, 10]],
         "expect": 0},
    ],
    "config1": {
        "npz": [3], "writes": 1000, "target": 0,
        "delivered": {"P1a": 2, "P1b": 2, "P2a": 2000, "P2b": 2000, "P3": 2000},
        "delivered_total": 6004,
        "leader_ballot": 4295032833, "leader_slot": 999, "leader_execute": 1000,
        "steps_per_request": 3,
    },
}

if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote", OUT)
