// jsp_multi.h — the device-set engine behind jsp_engine_create_multi
// (SURVEY.md §8b "one per device set", §8e): one process (the Go manager,
// main.go:161-190, builds one engine) drives several GPUs. The node rows are
// sharded by whole level-0 domains over one shard engine per listed device;
// the shards of one device tally straight into their own (disjoint) leaf
// columns of that device's zero-initialised [C+1][L] buffer -- and, for leaf
// classes, fold their leaves' feasibility bits into the feasibility words --
// the devices' buffers are SUM-combined by one RCCL all-reduce group over
// xGMI (ncclCommInitAll in this process; the words' bits are disjoint, so a
// sum is their OR), and the first shard runs the deterministic assignment.
// Integer sums make the result bit-exact for any device set
// (tests/test_multi_gpu.py).
#pragma once
#include <stdint.h>

#include "../../include/jsplace_bench.h"

namespace jspm {

struct Multi;

int create(const int* device_ids, int n_devices, Multi** out);
void destroy(Multi* m);
int device_of(const Multi* m);  // the first device of the set (the assignment runs there)

int topology_upload(Multi* m, const jsp_topology* t);
int snapshot_upload(Multi* m, const jsp_nodes* nodes);
int snapshot_patch(Multi* m, const uint32_t* rows, uint32_t n, const uint64_t* labels, const uint32_t* taints,
                   const uint32_t* free_res, const int32_t* excl_owner);
int classes_upload(Multi* m, const jsp_job_class* classes, uint32_t C);
int place(Multi* m, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs, int32_t* assign_out,
          uint32_t* tally_out, uint32_t* occ_out, jsp_stats* stats);
int resolve(Multi* m, const int32_t* leader_rows, const uint32_t* levels, uint32_t n, int32_t* domain_out);
int audit(Multi* m, const int32_t* leader_rows, const uint32_t* levels, const uint32_t* follower_off,
          const int32_t* follower_domains, uint32_t n_jobs, uint32_t* bad_out);
// forwards a setting to every shard: 0 set_fused, 1 set_service, 2 set_timing
int forward(Multi* m, int what, int value);
int sync(Multi* m);
int check(Multi* m);
int get_timing(Multi* m, jsp_timing* out, int reset);
void* stream(Multi* m);
int shard_count(const Multi* m);
int n_devices(const Multi* m);  // distinct devices (RCCL ranks)

}  // namespace jspm

// error reporting of the engine (jsp_last_error), for the device-set module
int jsp_internal_set_err(int code, const char* fmt, ...);

// Internal entry points of a shard engine (jsp_engine.cc), on its own stream:
// whether it can fold its leaf classes' feasibility into its tally; its
// feasibility words (and their count); a tally that folds into `fold_feas`
// (null: none); the assignment on given tallies (folded: the feasibility
// words are already in the engine's own buffer); a non-blocking check of its
// launches' error word.
bool jspi_fold_ok(jsp_engine* e);
uint64_t* jspi_feas(jsp_engine* e, uint32_t* words);
int jspi_tally(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, uint64_t* fold_feas);
int jspi_assign(jsp_engine* e, const uint32_t* d_cap, const uint32_t* d_occ, uint32_t ld, const uint32_t* run_class,
                const uint32_t* run_len, uint32_t n_runs, uint32_t J, int32_t* assign, bool folded);
int jspi_check(jsp_engine* e);
