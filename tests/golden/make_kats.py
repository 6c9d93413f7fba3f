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
    # Tie order: Go's sort.Sort(byTime) is not stable, so ops
    # with equal start have no defined order in the reference; here they keep
    # the canonical order.  Five ops: W2 = write 2 [1,1], W1 = write 1 [2,2],
    # Ra = read 0 [3,3], Rb = read 0 [4,4], R2 = read 2 [4,5]; orders a and b
    # differ only in Rb / R2, which both start at 4.  Derived by hand from
    # checker.go:69-104 with vertices in insertion order:
    #   both: R2 merges into W2 (match), inheriting W1->W2 and Ra->W2; the DFS
    #     from W2 finds W2->W1->W2 (gray {W2, W1}): anomaly 1; the cut removes
    #     W1->W2 (start 2 > end 1), leaving the cycle W2->Ra->W2.
    #   a: Rb was handled before R2 (no match, acyclic then) and no read
    #     follows: 1 anomaly.
    #   b: Rb comes after R2; Cycle() runs again and finds W2->W1->Ra->W2
    #     (gray {W2, W1, Ra}): anomaly 2, cut Ra->W2 (3 > 1): 2 anomalies.
    "lin_tie_order": {"a": [[2, None, 1, 1], [1, None, 2, 2], [None, 0, 3, 3], [None, 0, 4, 4], [None, 2, 4, 5]],
                      "b": [[2, None, 1, 1], [1, None, 2, 2], [None, 0, 3, 3], [None, 2, 4, 5], [None, 0, 4, 4]],
                      "expect_a": 1, "expect_b": 2},
    "config1": {
        "npz": [3], "writes": 1000, "target": 0,
        "delivered": {"P1a": 2, "P1b": 2, "P2a": 2000, "P2b": 2000, "P3": 2000},
        "delivered_total": 6004,
        "leader_ballot": 4295032833, "leader_slot": 999, "leader_execute": 1000,
        "steps_per_request": 3,
    },
}



# ---------------------------------------------------------------------------
# G-traces: the semantic gotchas of SURVEY.md §8 (G1-G14) as scripted
# one-cluster traces.  Every expected value below was derived by hand from the
# Go source, step by step, under the delivery schedule of DESIGN.md §3 (a
# message sent at step t with delay d is handled at step t+1+d; a replica
# handles its inbox in a merge of per-source FIFO queues).  Scripted Slow /
# Drop windows serialise the arrivals, so each trace's outcome does not depend
# on the merge order (the tests rerun them under several seeds).  The
# derivation of each trace is kept next to it; A, B, C, D, E are replicas
# 0..4 = IDs 1.1..1.5.
# ---------------------------------------------------------------------------
def ballot(n, zone, node):          # ballot.go:15-17 NewBallot
    return (n << 32) | (zone << 16) | node


NEVER = 0xFFFFFFFF
DROP, SLOW, FLAKY, CRASH = 0, 1, 2, 3
ALL = 0xFF
CLIENT = 31


def rep(ballot_=0, slot=-1, execute=0, active=0, p1_acks=0, npending=0, delivered=None, client_requests=0,
        sent=0, dropped=0, discarded=0, commits=0, replies=0, flags=0, executed=()):
    return {"ballot": ballot_, "slot": slot, "execute": execute, "active": active, "p1_acks": p1_acks,
            "npending": npending, "delivered": delivered or {}, "client_requests": client_requests, "sent": sent,
            "dropped": dropped, "discarded": discarded, "commits": commits, "replies": replies, "flags": flags,
            "executed": list(executed)}


B1 = ballot(1, 1, 1)   # (1, 1.1) = 4295032833
B1B = ballot(1, 1, 2)  # (1, 1.2)
B1C = ballot(1, 1, 3)  # (1, 1.3)
B2B = ballot(2, 1, 2)  # (2, 1.2)
B2C = ballot(2, 1, 3)  # (2, 1.3)

gtraces = [
    {
        "name": "single_write_staggered_p1b",
        "gotchas": ["G1", "G4", "G7", "G9"],
        "config": {"npz": [3], "max_delay": 2},
        "workload": {"outstanding": 1, "max_requests": 1, "target": [0]},
        "faults": [[SLOW, 2, 0, 2, 0, NEVER]],
        "inject": [],
        "steps": 10,
        "derivation": [
            "t0 A: client cid1; ballot 0 -> Ballot.ID()=='0.0' != 1.1 (ballot.go:43-47, G9) -> HandleRequest pends it and runs P1a: b=(1,1.1), quorum={A} (paxos.go:104-106), Broadcast to B,C only (G1). A.sent=2",
            "t1 B,C: HandleP1a adopt b; P1b{b,{}} -> A. B's arrives t2, C's is slowed 2 -> t4",
            "t2 A: HandleP1b(B): ACK(B) -> {A,B} is a majority of 3 only because of the self-ACK (G1) -> active; P2a slot 0 -> B,C. A.sent=4",
            "t3 B,C: HandleP2a -> entry, P2b -> A (B's at t4, C's slowed -> t6)",
            "t4 A: P1b(C) ignored: p.active (paxos.go:185, G4); P2b(B) -> {A,B} commit, P3 -> B,C, exec replies the client. A.sent=6",
            "t5 B,C: HandleP3 -> exec slot 0",
            "t6 A: P2b(C): exec deleted the entry (paxos.go:366) -> !exist -> ignored (paxos.go:273, G7)",
        ],
        "checkpoints": [{"after": 3, "replicas": {"0": {"active": 1, "p1_acks": 3, "ballot": B1, "slot": 0,
                                                        "delivered": {"P1b": 1}}}}],
        "expect": [
            rep(B1, 0, 1, 1, 3, 0, {"P1b": 2, "P2b": 2}, 1, 6, commits=1, replies=1, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[1]),
        ],
    },
    {
        "name": "crashed_replica_takes_client_requests",
        "gotchas": ["G10", "G11"],
        "config": {"npz": [3], "max_delay": 0},
        "workload": {"outstanding": 2, "max_requests": 1, "target": [0, 1]},
        "faults": [[CRASH, 0, ALL, 0, 0, NEVER]],
        "inject": [],
        "steps": 40,
        "derivation": [
            "Crash(t<=0) is forever (socket.go:192, G11): A stays crashed for all 40 steps",
            "t0 A: the HTTP request reaches MessageChan directly (http.go:99), so a crashed node still handles it (G10): pend, P1a (1,1.1); both sends dropped by s.crash (socket.go:69). sent=2 dropped=2",
            "t0 B: client cid2 -> P1a (1,1.2) -> A, C",
            "t1 A: Recv discards while crashed (socket.go:111-118): discarded=1. C adopts (1,1.2), P1b -> B",
            "t2 B: ACK(C) -> {B,C} active, P2a slot 0 cmd 2 -> A, C",
            "t3 A discards the P2a (2). C: P2b -> B.  t4 B: commit, P3 -> A, C, exec replies worker 1",
            "t5 A discards the P3 (3); C executes.  Worker 0's request stays pending at A forever",
        ],
        "checkpoints": [],
        "expect": [
            rep(B1, -1, 0, 0, 1, 1, {}, 1, 2, 2, 3),
            rep(B1B, 0, 1, 1, 6, 0, {"P1b": 1, "P2b": 1}, 1, 6, commits=1, replies=1, executed=[2]),
            rep(B1B, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[2]),
        ],
    },
    {
        "name": "crash_window_ends_p2a_strands_pending",
        "gotchas": ["G10", "G11"],
        "config": {"npz": [3], "max_delay": 0},
        "workload": {"outstanding": 2, "max_requests": 1, "target": [0, 1]},
        "faults": [[CRASH, 0, ALL, 0, 0, 3]],
        "inject": [],
        "steps": 40,
        "derivation": [
            "Crash(t>0) ends (socket.go:192-198): A is crashed at steps 0-2 only",
            "t0 as in the permanent crash: A pends cid1 and its P1a (1,1.1) is dropped twice; B runs P1a (1,1.2)",
            "t1 A discards B's P1a (discarded=1); C adopts (1,1.2) -> P1b -> B.  t2 B active, P2a slot 0 cmd 2 -> A, C",
            "t3 A is up: HandleP2a (1,1.2) >= (1,1.1) -> adopt, slot 0, entry, P2b -> B.  HandleP2a does not forward p.requests (paxos.go:236-260): cid1 stays pending forever",
            "t4 B: first P2b commits slot 0 (P3 -> A, C), exec replies worker 1; the second P2b finds the entry deleted (G7)",
            "t5 A, C execute slot 0",
        ],
        "checkpoints": [],
        "expect": [
            rep(B1B, 0, 1, 0, 1, 1, {"P2a": 1, "P3": 1}, 1, 3, 2, 1, executed=[2]),
            rep(B1B, 0, 1, 1, 6, 0, {"P1b": 1, "P2b": 2}, 1, 6, commits=1, replies=1, executed=[2]),
            rep(B1B, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[2]),
        ],
    },
    {
        "name": "dueling_proposers_forward_via_p1a",
        "gotchas": ["G3", "G4", "G7", "G13", "G14"],
        "config": {"npz": [3], "max_delay": 1},
        "workload": {"outstanding": 2, "max_requests": 1, "target": [0, 2]},
        "faults": [[SLOW, 0, 1, 1, 0, NEVER], [SLOW, 1, 2, 1, 0, NEVER]],
        "inject": [],
        "steps": 12,
        "derivation": [
            "t0 A: cid1 -> P1a bA=(1,1.1) -> C (t1), B (slowed, t2).  C: cid2 -> P1a bC=(1,1.3) -> A, B (t1)",
            "t1 A: HandleP1a(bC) > bA -> adopt, active=false, forward() (paxos.go:143, G14): node.Forward(C, cid1) records forwards[cid1] and sends the Request; then P1b{bC} -> C",
            "t1 C: HandleP1a(bA) < bC: no change, but the P1b is still sent, carrying p.ballot = bC (paxos.go:157, G3) -> A.  B: adopt bC, P1b -> C (slowed, t3)",
            "t2 A: P1b{bC} from C: not lower, not active; bC.ID() != A -> no ACK: a rejection is not a NACK (quorum.go:12-19, G13); A's phase-1 quorum stays {A}",
            "t2 B: HandleP1a(bA) < bC -> P1b{bC} -> A (G3).  C: the Request (cid1) from A pends (IsLeader via ballot.ID()); P1b(A) -> {C,A} active -> P2a slot 0 = cid2, slot 1 = cid1 -> A, B",
            "t3 A: P1b{bC} from B: no effect; P2a 0, 1 -> entries, P2b -> C.  B: same, P2bs slowed to t5.  C: B's P1b is ignored, C is active (G4)",
            "t4 C: commit 0 (reply worker 1), commit 1: its request came from A, so exec's reply goes back over the socket to A (node.go:83-87)",
            "t5 A: P3 0, P3 1, then the Reply: forwards[cid1] answers worker 0.  C: B's P2bs hit deleted entries (G7)",
            "Duel settles with no retry or backoff: 22 socket messages, every replica executes cid2 then cid1",
        ],
        "checkpoints": [{"after": 2, "replicas": {"0": {"ballot": B1C, "npending": 0, "p1_acks": 1},
                                                  "2": {"ballot": B1C, "active": 0, "npending": 1}}},
                        {"after": 3, "replicas": {"2": {"active": 1, "p1_acks": 5, "slot": 1}}}],
        "expect": [
            rep(B1C, 1, 2, 0, 1, 0, {"P1a": 1, "P1b": 2, "P2a": 2, "P3": 2, "Reply": 1}, 1, 6, replies=1,
                executed=[2, 1]),
            rep(B1C, 1, 2, 0, 0, 0, {"P1a": 2, "P2a": 2, "P3": 2}, sent=4, executed=[2, 1]),
            rep(B1C, 1, 2, 1, 5, 0, {"P1a": 1, "Request": 1, "P1b": 2, "P2b": 4}, 1, 12, commits=2, replies=1,
                executed=[2, 1]),
        ],
        "totals": {"delivered_total": 22, "sent": 22, "dropped": 0, "commits": 2, "replies": 2},
    },
    {
        "name": "dueling_proposers_forward_via_p1b",
        "gotchas": ["G3", "G4", "G7", "G14"],
        "config": {"npz": [3], "max_delay": 2},
        "workload": {"outstanding": 2, "max_requests": 1, "target": [0, 2]},
        "faults": [[SLOW, 0, 1, 1, 0, NEVER], [SLOW, 1, 2, 1, 0, NEVER], [SLOW, 2, 0, 2, 0, 1]],
        "inject": [],
        "steps": 12,
        "derivation": [
            "As the P1a-path duel, but C's P1a to A (sent t0) is slowed to t3, so A learns of bC from C's rejecting P1b first",
            "t1 C: HandleP1a(bA) -> P1b{bC} -> A (t2, G3).  B: adopt bC, P1b -> C (slowed, t3)",
            "t2 A: HandleP1b{bC}: not lower, not active; update(); bC > bA -> adopt, active=false, forward() (paxos.go:195-199, G14): Request cid1 -> C.  B: rejects A's P1a with P1b{bC} -> A",
            "t3 A: C's P1a(bC) (no change) -> P1b{bC} -> C; B's P1b: no effect.  C: B's P1b ACKs -> {C,B} active; with A's Request (either order) slot 0 = cid2, slot 1 = cid1",
            "t4 A, B: P2bs (B's slowed).  C: A's P1b ignored (G4).  t5 C commits both, Reply -> A.  t6 A replies worker 0; C ignores B's late P2bs (G7)",
        ],
        "checkpoints": [{"after": 3, "replicas": {"0": {"ballot": B1C, "npending": 0, "delivered": {"P1b": 1}}}}],
        "expect": [
            rep(B1C, 1, 2, 0, 1, 0, {"P1a": 1, "P1b": 2, "P2a": 2, "P3": 2, "Reply": 1}, 1, 6, replies=1,
                executed=[2, 1]),
            rep(B1C, 1, 2, 0, 0, 0, {"P1a": 2, "P2a": 2, "P3": 2}, sent=4, executed=[2, 1]),
            rep(B1C, 1, 2, 1, 6, 0, {"P1a": 1, "Request": 1, "P1b": 2, "P2b": 4}, 1, 12, commits=2, replies=1,
                executed=[2, 1]),
        ],
        "totals": {"delivered_total": 22, "sent": 22, "dropped": 0, "commits": 2, "replies": 2},
    },
    {
        "name": "stale_leader_p2b_reject_and_replace",
        "gotchas": ["G3", "G4", "G7", "G14"],
        "config": {"npz": [3], "max_delay": 3, "ephemeral_leader": 1},
        "workload": {"outstanding": 1, "max_requests": 1, "target": [0]},
        "faults": [[SLOW, 2, 0, 1, 0, 2], [SLOW, 0, 1, 1, 10, 11], [SLOW, 2, 0, 3, 10, 11]],
        "inject": [[10, 0, 100], [10, 2, 200]],
        "steps": 30,
        "derivation": [
            "t0-t5: A is elected with b1=(1,1.1) (C's P1b slowed to t3 and ignored, G4) and commits cid1 at slot 0 everywhere",
            "t10 (injected): A, active, P2a(b1, slot 1, cid100) -> C (t11), B (slowed, t12).  C (-ephemeral_leader: paxos/replica.go:61) pends cid200 and runs P1a: b2=(2,1.3) -> B (t11), A (slowed 3, t14)",
            "t11 B: adopt b2 -> P1b{b2,{}} -> C.  C: HandleP2a(b1) < b2 -> P2b{b2, slot 1} -> A anyway (paxos.go:262, G3)",
            "t12 A: HandleP2b{b2}: entry 1 exists, uncommitted, b2 >= e.ballot, b2 > p.ballot -> adopt, active=false (paxos.go:281-284).  B: rejects A's P2a -> P2b{b2} -> A.  C: ACK(B) -> active, P2a(b2, slot 1, cid200) -> A, B",
            "t13 A: HandleP2a(b2, 1, cid200) replaces entry 1 (b2 > b1): its command differs and it holds cid100's request -> Forward(C, cid100) (paxos.go:245-249); P2b -> C.  B's P2b{b2}: no effect in either order",
            "t14 A: C's P1a arrives late: P1b{b2, Log{1:(cid200,b2)}} -> C.  C: first P2b commits slot 1 (cid200), the second finds it deleted (G7); the forwarded Request cid100 -> P2a slot 2",
            "t15 C ignores A's P1b (active, G4); A, B commit slot 1 and accept slot 2.  t16 C commits slot 2 and replies to A (Reply).  t17 A, B execute slot 2",
        ],
        "checkpoints": [{"after": 13, "replicas": {"0": {"ballot": B2C, "active": 0}, "2": {"active": 1, "p1_acks": 6}}}],
        "expect": [
            rep(B2C, 2, 3, 0, 3, 0, {"P1a": 1, "P1b": 2, "P2a": 2, "P2b": 4, "P3": 2, "Reply": 1}, 2, 12, commits=1,
                replies=1, executed=[1, 200, 100]),
            rep(B2C, 2, 3, 0, 0, 0, {"P1a": 2, "P2a": 4, "P3": 3}, sent=6, executed=[1, 200, 100]),
            rep(B2C, 2, 3, 1, 6, 0, {"P1a": 1, "P2a": 2, "P3": 1, "P1b": 2, "P2b": 4, "Request": 1}, 1, 14, commits=2,
                executed=[1, 200, 100]),
        ],
        "totals": {"delivered_total": 32, "sent": 32, "dropped": 0, "commits": 3, "replies": 1},
    },
    {
        "name": "nil_gap_blocks_exec_p3_ballot_zero",
        "gotchas": ["G5", "G6"],
        "config": {"npz": [3], "max_delay": 1, "ephemeral_leader": 1},
        "workload": {"outstanding": 1, "max_requests": 3, "target": [0]},
        "faults": [[SLOW, 2, 0, 1, 0, 2], [DROP, 0, 1, 0, 2, 6], [SLOW, 2, 1, 1, 16, 17], [SLOW, 2, 1, 1, 18, 19]],
        "inject": [[15, 1, 500]],
        "steps": 30,
        "derivation": [
            "A is elected with b1 at t2 (P1b of B; C's is slowed and ignored).  Drop A->B during t2-5 loses P2a(slot 0), P3(slot 0) and P2a(slot 1) to B (dropped=3); C's acks commit slots 0, 1",
            "t8 B: HandleP3(slot 1) with no entry: &entry{} keeps ballot 0, command cid2, commit (paxos.go:326-331, G6); exec stops at the missing slot 0 (paxos.go:347-349, G5)",
            "t9-t11: slot 2 (cid3) is accepted and committed everywhere; B still executes nothing",
            "t15 (injected cid500 at B, -ephemeral_leader): B runs P1a b=(2,1.2).  t16 A, C adopt; their P1b logs are empty (all their entries executed)",
            "t17 B: ACK(A) -> active; the re-proposal loop over [execute=0, slot=2] skips the nil slot 0 (paxos.go:211, G5) and the committed 1, 2; cid500 -> slot 3",
            "t19 B commits slot 3 (A's P2b; C's is slowed to t20 and finds it committed) but exec is still blocked at slot 0: cid500 is never answered",
        ],
        "checkpoints": [],
        "expect": [
            rep(B2B, 3, 4, 0, 3, 0, {"P1a": 1, "P1b": 2, "P2a": 1, "P2b": 4, "P3": 1}, 3, 16, 3, commits=3, replies=3,
                executed=[1, 2, 3, 500]),
            rep(B2B, 3, 0, 1, 3, 0, {"P1a": 1, "P2a": 1, "P3": 2, "P1b": 2, "P2b": 2}, 1, 8, commits=1, executed=[]),
            rep(B2B, 3, 4, 0, 0, 0, {"P1a": 2, "P2a": 4, "P3": 4}, sent=6, executed=[1, 2, 3, 500]),
        ],
        "log": {"replica": 1, "slot_lo": 0, "entries": [
            {"slot": 0, "flags": 0x10, "ballot": 0, "cmd": 0, "acks": 0, "request": 0},
            {"slot": 1, "flags": 0x13, "ballot": 0, "cmd": 2, "acks": 0, "request": 0},
            {"slot": 2, "flags": 0x13, "ballot": B1, "cmd": 3, "acks": 0, "request": 0},
            {"slot": 3, "flags": 0x1F, "ballot": B2B, "cmd": 500, "acks": 3, "request": 500 | (CLIENT << 27)},
            {"slot": 4, "flags": 0x10, "ballot": 0, "cmd": 0, "acks": 0, "request": 0}]},
        "totals": {"delivered_total": 27, "sent": 30, "dropped": 3, "commits": 4, "replies": 3},
    },
    {
        "name": "thrifty_multicast_quorum",
        "gotchas": ["G6", "G8"],
        "config": {"npz": [5], "max_delay": 3, "thrifty": 1},
        "workload": {"outstanding": 1, "max_requests": 1, "target": [0]},
        "faults": [[SLOW, 2, 0, 1, 0, NEVER], [SLOW, 3, 0, 2, 0, NEVER], [SLOW, 4, 0, 3, 0, NEVER]],
        "inject": [],
        "steps": 12,
        "derivation": [
            "t0 A: P1a (1,1.1) broadcast to B..E (Broadcast is never thrifty).  t1: P1bs to A arrive at t2 (B), t3 (C), t4 (D), t5 (E)",
            "t2 A: {A,B} is not a majority of 5.  t3: {A,B,C} -> active; P2a is sent with MulticastQuorum(N/2+1 = 3) (paxos.go:126-127; socket.go:132-145) to the 3 peers after A in ring order: B, C, D; E gets none (G8)",
            "t5 A: P2b(B) -> {A,B}; E's late P1b ignored.  t6 P2b(C) -> {A,B,C} commit, P3 broadcast to all 4 peers.  t7 D's P2b hits the deleted entry (G7)",
            "t7 E: HandleP3 with no entry creates &entry{} (G6), commits and executes slot 0",
        ],
        "checkpoints": [],
        "expect": [
            rep(B1, 0, 1, 1, 7, 0, {"P1b": 4, "P2b": 3}, 1, 11, commits=1, replies=1, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P3": 1}, sent=1, executed=[1]),
        ],
        "totals": {"delivered_total": 18, "sent": 18, "dropped": 0, "commits": 1, "replies": 1},
    },
    {
        "name": "fault_filter_order",
        "gotchas": ["G6", "G10", "G12"],
        "config": {"npz": [3], "max_delay": 2},
        "workload": {"outstanding": 1, "max_requests": 2, "target": [0]},
        "faults": [[DROP, 0, 1, 0, 0, 1], [SLOW, 0, 1, 2, 0, NEVER], [FLAKY, 0, 2, 1000000, 3, 4],
                   [SLOW, 0, 2, 1, 0, NEVER], [CRASH, 0, ALL, 0, 15, NEVER]],
        "inject": [[16, 0, 300]],
        "steps": 25,
        "derivation": [
            "socket.Send checks crash, then drop, then flaky, then slow (socket.go:69-106, G12): a message both dropped and slowed is dropped, never delivered late",
            "t0 A: P1a (1,1.1): to B dropped (drop wins over the slow link), to C slowed 1 -> t2",
            "t2 C: adopt, P1b -> A.  t3 A: active; P2a slot 0: to B slowed 2 (t6), to C flaky p=1 (rand.Float64() < 1.0 always) -> dropped before any delay",
            "t6 B: first contact is the P2a: adopt (1,1.1), entry, P2b.  t7 A: commit slot 0; P3 -> B (t10), C (t9); reply -> cid2 arrives t8",
            "t8 A: P2a slot 1 -> B (t11), C (t10).  t9 C: P3 for a slot it never accepted: &entry{} (G6), executes slot 0",
            "t10 B executes slot 0; C accepts slot 1.  t11 A commits slot 1 with C's P2b, replies cid2 (last request); B accepts.  t12 B's P2b hits the deleted entry",
            "t15 A crashes for good; t16 an injected request still reaches it (G10): P2a slot 2, both sends dropped by the crash before the slow links apply",
        ],
        "checkpoints": [{"after": 3, "replicas": {"1": {"ballot": 0, "delivered": {}}, "0": {"dropped": 1}}}],
        "expect": [
            rep(B1, 2, 2, 1, 5, 0, {"P1b": 1, "P2b": 3}, 3, 12, 4, commits=2, replies=2, executed=[1, 2]),
            rep(B1, 1, 2, 0, 0, 0, {"P2a": 2, "P3": 2}, sent=2, executed=[1, 2]),
            rep(B1, 1, 2, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 2}, sent=2, executed=[1, 2]),
        ],
        "totals": {"delivered_total": 12, "sent": 16, "dropped": 4, "commits": 2, "replies": 2},
    },
    {
        "name": "broadcast_sorted_order_flaky_sequence",
        "gotchas": ["G2"],
        "config": {"npz": [5], "max_delay": 0, "seed": 1},
        "workload": {"outstanding": 1, "max_requests": 1, "target": [0]},
        "faults": [[FLAKY, 0, ALL, 500000, 0, 1]],
        "inject": [],
        "steps": 10,
        "seed_dependent": True,
        "derivation": [
            "Go ranges over a map in Broadcast (socket.go:149); the build fixes sorted IDs.Less order (G2), and Flaky's draw for the k-th send of a step is fmix32(step_key ^ tag(FLAKY, sender, k)) (DESIGN.md §3.4)",
            "seed 1, cluster 0, step 0: the draws for sends 0..3 hit p=0.5 as [keep, drop, keep, drop] (computed below), so in sorted order B and D get the P1a and C, E do not; reversed order would reach E and C instead",
            "t2 A: P1b(B), P1b(D) -> {A,B,D} majority -> P2a to all four (flaky window over).  t3 C, E first hear of b1 through the P2a.  t4 A commits on the second P2b; the third and fourth find the entry deleted (G7)",
        ],
        "checkpoints": [{"after": 2, "replicas": {"1": {"delivered": {"P1a": 1}}, "2": {"delivered": {}},
                                                  "3": {"delivered": {"P1a": 1}}, "4": {"delivered": {}}}}],
        "expect": [
            rep(B1, 0, 1, 1, 11, 0, {"P1b": 2, "P2b": 4}, 1, 12, 2, commits=1, replies=1, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P2a": 1, "P3": 1}, sent=1, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P1a": 1, "P2a": 1, "P3": 1}, sent=2, executed=[1]),
            rep(B1, 0, 1, 0, 0, 0, {"P2a": 1, "P3": 1}, sent=1, executed=[1]),
        ],
        "totals": {"delivered_total": 16, "sent": 18, "dropped": 2, "commits": 1, "replies": 1},
    },
]


def _flaky_pattern(seed, p_ppm, nsend):
    """Drop decisions of sends 0..nsend-1 of replica 0 at step 0, cluster 0 (DESIGN.md §3.4 PRNG)."""
    m64 = (1 << 64) - 1

    def mix64(z):
        z ^= z >> 30; z = (z * 0xbf58476d1ce4e5b9) & m64
        z ^= z >> 27; z = (z * 0x94d049bb133111eb) & m64
        return z ^ (z >> 31)

    def fmix32(h):
        h ^= h >> 16; h = (h * 0x85ebca6b) & 0xFFFFFFFF
        h ^= h >> 13; h = (h * 0xc2b2ae35) & 0xFFFFFFFF
        return h ^ (h >> 16)

    kc = mix64(seed ^ mix64(0x9E3779B97F4A7C15)) & 0xFFFFFFFF
    hs = fmix32(kc ^ 0)
    return [((fmix32(hs ^ ((4 << 28) | k)) * 1000000) >> 32) < p_ppm for k in range(nsend)]


assert _flaky_pattern(1, 500000, 4) == [False, True, False, True]   # the G2 trace's premise
kats["gtraces"] = gtraces

if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote", OUT)
