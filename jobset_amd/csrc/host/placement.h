// placement.h — the host side of the engine boundary that the reference's
// controller would own: the Go
// `pkg/placement` package restated in C++ over Kubernetes objects as JSON.
//
//   Planner::sync     informer-cache Nodes and bound Pods -> the engine's SoA
//                     snapshot (deterministic sorted dictionaries), uploaded
//                     whole when its structure changed, else as a row patch
//                     (jsp_snapshot_patch) of the rows whose columns changed
//   Planner::plan     a JobSet's child Jobs (replicated-job runs in
//                     globalJobIndex order, one requirement class per pod
//                     template) -> jsp_place -> a domain per job
//   label_nodes       the node-selector strategy's node patches from a plan
//                     (deterministic replacement for hack/label_nodes/
//                     label_nodes.py:36-120)
#pragma once
#include <map>
#include <string>
#include <vector>

#include "../../../include/jsplace.h"
#include "json.h"

namespace jsk {

// One node-label predicate of the dictionary: a node's bit is set when the
// predicate holds on its labels. Selector terms map onto them:
//   nodeSelector {k: v} / In [v..]  -> required  (k In {v..})
//   NotIn [v..]                       -> forbidden (k In {v..})
//   Exists / DoesNotExist             -> required / forbidden (k Exists)
//   Gt / Lt v                         -> required  (k Gt v) / (k Lt v)
struct LabelPred {
    std::string key;
    std::string op;                  // "In", "Exists", "Gt", "Lt"
    std::vector<std::string> values; // sorted (In), one value (Gt/Lt)
    bool operator<(const LabelPred& o) const;
    bool operator==(const LabelPred& o) const;
    bool holds(const Json& labels) const;
};

// A NoSchedule / NoExecute taint of the dictionary (PreferNoSchedule is a
// preference, not a predicate).
struct TaintKey {
    std::string key, value, effect;
    bool operator<(const TaintKey& o) const;
    bool operator==(const TaintKey& o) const;
};

// One pod template's requirements, as the engine sees them.
struct ClassSpec {
    std::vector<LabelPred> req, forbid;
    Json tolerations;                 // the template's tolerations (array)
    std::vector<uint64_t> res;        // per configured resource, in its unit
    uint32_t pods = 1;                // parallelism
    int level = -1;                   // index of the exclusive-topology key
};

struct Err2 {  // error text ("" = ok) and an error class for the JSON layer
    std::string msg;
    bool ok() const { return msg.empty(); }
};

// Kubernetes quantity ("500m", "1536000Mi", "2", "1.5Gi", "1e3") in the
// unit of a resource: cpu -> millicores, memory / ephemeral-storage -> MiB,
// anything else -> whole units. round_up: requests round up, allocatable down.
bool parse_quantity(const std::string& q, const std::string& resource, bool round_up, uint64_t* out);

// Effective pod request of one resource: max(sum over containers, max over
// init containers), in the resource's unit.
uint64_t pod_request(const Json& podSpec, const std::string& resource);

class Planner {
public:
    Planner(jsp_engine* e, std::vector<std::string> level_keys, std::vector<std::string> resources);

    // Rebuild the snapshot from the cache objects and bring the engine up to
    // date. Returns {"rows","leaves","domains","labelWords","taintBits",
    // "skippedNodes","upload": "full"|"patch"|"none","patchedRows",
    // "exclusiveJobs"}.
    Err2 sync(const std::map<std::string, Json>& nodes, const std::map<std::string, Json>& pods, Json* stats);

    // The requirement class of a pod template (job template spec.template);
    // registers its label predicates in the dictionary (a new predicate makes
    // the next sync a full upload). `topology_key` = the exclusive-topology key.
    Err2 class_of(const Json& podTemplateSpec, int64_t parallelism, const std::string& topology_key, ClassSpec* out);

    // The engine's form of classes (label/taint bits of the current dictionaries).
    Err2 encode(const std::vector<ClassSpec>& classes, std::vector<jsp_job_class>* out) const;

    // Place runs (class index, job count) in global order. Classes are
    // uploaded to the engine first. assign: domain id per job, -1 unplaceable.
    Err2 place(const std::vector<ClassSpec>& classes, const std::vector<uint32_t>& run_class,
               const std::vector<uint32_t>& run_len, std::vector<int32_t>* assign, jsp_stats* st);

    // snapshot lookups
    int level_of(const std::string& key) const;
    bool row_of(const std::string& node, int32_t* row) const;
    const std::vector<std::string>& domain_values(int level) const { return domain_values_[level]; }
    int32_t domain_id(int level, const std::string& value) const;
    // rows [first, end) of domain d at `level`
    void domain_rows(int level, int32_t d, uint32_t* first, uint32_t* end) const;
    // domain id at `level` of snapshot row `row` (host lookup, no engine call)
    int32_t row_domain(uint32_t row, int level) const;
    const std::string& row_node(uint32_t row) const { return row_node_[row]; }
    jsp_engine* engine() const { return eng_; }
    bool synced() const { return synced_; }
    // A Node was added, modified or removed in the cache since the last sync:
    // the snapshot's row -> domain answers may be stale, so the webhook and
    // reconciler lookups take the reference's Node Get path until the next
    // sync (serving() false). Pod events do not change a row's domain.
    void note_node_event() { nodes_dirty_ = true; }
    bool serving() const { return synced_ && !nodes_dirty_; }
    // the host copy of the columns (tests compare a patched engine with a re-ingest)
    Json columns() const;

private:
    Err2 rebuild(const std::map<std::string, Json>& nodes, const std::map<std::string, Json>& pods);
    Err2 upload_full();
    int pred_bit(const LabelPred& p) const;

    jsp_engine* eng_;
    std::vector<std::string> level_keys_, res_;
    std::vector<LabelPred> preds_;    // sorted dictionary
    bool preds_dirty_ = true;
    std::vector<TaintKey> taints_;    // sorted dictionary
    bool synced_ = false;
    bool nodes_dirty_ = false;
    // structure
    std::vector<std::string> row_node_;
    std::map<std::string, int32_t> node_row_;
    std::vector<std::vector<std::string>> domain_values_;
    std::vector<std::map<std::string, int32_t>> domain_ids_;
    std::vector<std::vector<uint32_t>> first_leaf_;  // per level, [D_k + 1]
    std::vector<uint32_t> leaf_start_;               // [L + 1]
    // columns
    uint32_t W_ = 1;
    std::vector<uint64_t> labels_;  // [W][N]
    std::vector<uint32_t> taint_bits_;
    std::vector<uint32_t> free_;    // [R][N]
    std::vector<int32_t> excl_;
    std::vector<std::string> skipped_;
    uint32_t exclusive_jobs_ = 0;
};

// Node patches of the node-selector strategy for the jobs of a plan: every
// node of job j's domain gets the namespaced-job label and the no-schedule
// taint, as label_nodes.py's patch body (hack/label_nodes/label_nodes.py:65-80).
Json label_nodes(const Planner& pl, int level, const std::vector<std::string>& namespaced_jobs,
                 const std::vector<int32_t>& assign);

}  // namespace jsk
