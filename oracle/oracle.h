/*
 * oracle.h — CPU restatement of the reference's simulation-mode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (paxi_amd/csrc).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * Pinning: the reference is Go and no Go toolchain exists in this image
 * (SURVEY.md §8c), so it cannot be built or run here.  The oracle is pinned by
 * the reference's own known-answer tests (ballot_test.go:7-22,
 * checker_test.go:6-136) and by hand-derived KATs computed from the Go source
 * (BASELINE.md "Correctness anchors": config 1 = 6004 messages, leader ballot
 * 4295032833, 1000 identical executed commands), committed under tests/golden.
 */
#ifndef PAXISIM_ORACLE_H
#define PAXISIM_ORACLE_H
#include "../include/paxisim.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_sim oracle_sim;

int  oracle_create(const paxisim_config* cfg, const paxisim_workload* wl,
                   const paxisim_fault_process* fp, oracle_sim** out);
int  oracle_destroy(oracle_sim* h);
int  oracle_fault_add(oracle_sim* h, const paxisim_fault* f);
/* nthreads > 1 shards clusters over POSIX threads (CPU baseline only). */
int  oracle_step(oracle_sim* h, uint32_t nsteps, int nthreads);
/* test hook: 0 runs a step's replicas in index order, 1 reversed, 2 shuffled per (cluster, step) */
int  oracle_set_replica_order(oracle_sim* h, uint32_t mode);
int  oracle_stats_get(oracle_sim* h, paxisim_stats* out);
int  oracle_read_state(oracle_sim* h, uint64_t cluster_lo, uint64_t n,
                       paxisim_replica_state* out);
int  oracle_read_instances(oracle_sim* h, uint64_t cluster_lo, uint64_t n,
                           paxisim_instance_state* out);
int  oracle_check(oracle_sim* h, uint64_t* violations);
int  oracle_inject(oracle_sim* h, uint64_t cluster, uint32_t replica, uint32_t cid);
int  oracle_read_inbox(oracle_sim* h, uint64_t cluster, uint32_t replica, paxisim_inbox_record* out,
                       uint32_t cap, uint32_t* n_out);
int  oracle_deliver(oracle_sim* h, uint64_t cluster, uint32_t replica, uint32_t src,
                    const paxisim_inbox_record* recs, uint32_t n);
int  oracle_read_log(oracle_sim* h, uint64_t cluster, uint32_t replica, uint32_t key, int32_t slot_lo,
                     uint32_t n, paxisim_log_entry* out);
/* Executed command ids of (cluster, replica | key << 16), in slot order (KAT support). */
int  oracle_exec_log(oracle_sim* h, uint64_t cluster, uint32_t replica,
                     uint32_t* buf, uint32_t cap, uint32_t* n_out);
/* History.Linearizable over every (cluster, key) of the ABD op history. */
int  oracle_lin_check(oracle_sim* h, uint64_t* anomalies, uint64_t* ops);
int  oracle_history(oracle_sim* h, uint64_t cluster, uint32_t* buf, uint32_t cap_ops, uint32_t* n_out);
int  oracle_read_kv(oracle_sim* h, uint64_t cluster, uint32_t replica, uint32_t* values, uint32_t n);
int  oracle_read_client(oracle_sim* h, uint64_t cluster, paxisim_worker_state* out, uint32_t cap, uint32_t* n_out);
int  oracle_command(oracle_sim* h, uint64_t cluster, uint32_t cid, uint32_t* key, uint32_t* write);
int  oracle_history_load(oracle_sim* h, uint64_t cluster, uint32_t replica, const uint32_t* ops, uint32_t n);
const char* oracle_last_error(void);

/* Reference KAT helpers (ballot.go / quorum.go / checker.go restated). */
uint64_t oracle_new_ballot(uint32_t n, uint32_t zone, uint32_t node);
uint64_t oracle_ballot_next(uint64_t b, uint32_t zone, uint32_t node);
int      oracle_quorum(uint32_t kind, uint32_t fz, uint32_t n_zones,
                       const uint32_t* npz, uint32_t ack_mask);
/* Linearizability checker (checker.go:69-104, lib/graph.go:180-232):
 * ops[6*i ..] = {has_input, input, has_output, output, start, end}
 * (a write has an input, a read an output; value 0 is a real value, distinct
 * from nil as in Go's interface{}).  Returns the anomaly count, or -1. */
int      oracle_linearizable(const int64_t* ops, int n_ops);

#ifdef __cplusplus
}
#endif
#endif
