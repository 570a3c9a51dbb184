// placement.cc — see placement.h. Snapshot ingestion from informer-cache
// objects, requirement classes from pod templates, and the plan call.
//
// Reference reads this replaces: the per-pod Node Gets of topologyFromPod
// (pkg/webhooks/pod_mutating_webhook.go:181-189) and leaderPodTopology
// (pkg/controllers/pod_controller.go:250-258), over the nodes the manager may
// list and watch (config/components/rbac/role.yaml:16-23). The predicate
// semantics restate kube-scheduler's NodeAffinity / TaintToleration /
// NodeResourcesFit filters, which are not in the reference:
// parity unpinned, see DESIGN.md §2.
#include "placement.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>

namespace jsk {

namespace {

const char* const kExclusiveKey = "alpha.jobset.sigs.k8s.io/exclusive-topology";  // jobset_types.go:41
const char* const kJobKey = "jobset.sigs.k8s.io/job-key";                         // jobset_types.go:35
const char* const kNamespacedJobKey = "alpha.jobset.sigs.k8s.io/namespaced-job";  // jobset_types.go:47
const char* const kNoScheduleTaintKey = "alpha.jobset.sigs.k8s.io/no-schedule";   // jobset_types.go:48
const char* const kUnschedulableTaint = "node.kubernetes.io/unschedulable";        // what the node controller sets for spec.unschedulable

bool parse_int64(const std::string& s, int64_t* v) {  // strconv.ParseInt(s, 10, 64)
    if (s.empty()) return false;
    char* end = nullptr;
    errno = 0;
    const long long x = std::strtoll(s.c_str(), &end, 10);
    if (errno != 0 || *end != '\0' || std::isspace((unsigned char)s[0])) return false;
    *v = x;
    return true;
}

const Json& labels_of(const Json& o) { return o.get("metadata").get("labels"); }

}  // namespace

// ------------------------------------------------------------------ dictionaries
bool LabelPred::operator<(const LabelPred& o) const {
    if (key != o.key) return key < o.key;
    if (op != o.op) return op < o.op;
    return values < o.values;
}
bool LabelPred::operator==(const LabelPred& o) const { return key == o.key && op == o.op && values == o.values; }

bool LabelPred::holds(const Json& labels) const {
    if (!has_key(labels, key)) return false;
    const std::string& v = labels.get(key).as_string();
    if (op == "Exists") return true;
    if (op == "In") return std::binary_search(values.begin(), values.end(), v);
    int64_t a = 0, b = 0;
    if (values.size() != 1 || !parse_int64(v, &a) || !parse_int64(values[0], &b)) return false;
    return op == "Gt" ? a > b : a < b;
}

bool TaintKey::operator<(const TaintKey& o) const {
    if (key != o.key) return key < o.key;
    if (value != o.value) return value < o.value;
    return effect < o.effect;
}
bool TaintKey::operator==(const TaintKey& o) const { return key == o.key && value == o.value && effect == o.effect; }

// ToleratesTaint (k8s.io/api/core/v1/toleration.go)
static bool tolerates(const Json& t, const TaintKey& taint) {
    const std::string eff = t.get("effect").as_string(), key = t.get("key").as_string();
    const std::string op = t.get("operator").as_string();
    if (!eff.empty() && eff != taint.effect) return false;
    if (!key.empty() && key != taint.key) return false;
    if (op.empty() || op == "Equal") return t.get("value").as_string() == taint.value;
    return op == "Exists";
}

// ------------------------------------------------------------------ quantities
bool parse_quantity(const std::string& q, const std::string& resource, bool round_up, uint64_t* out) {
    if (q.empty()) return false;
    size_t i = 0;
    if (q[i] == '+') ++i;
    const size_t num_begin = i;
    while (i < q.size() && (std::isdigit((unsigned char)q[i]) || q[i] == '.')) ++i;
    if (i == num_begin) return false;
    long double v = std::strtold(q.substr(num_begin, i - num_begin).c_str(), nullptr);
    const std::string suf = q.substr(i);
    long double mul = 1;
    if (suf.empty()) mul = 1;
    else if (suf == "m") mul = 1e-3L;
    else if (suf == "k") mul = 1e3L;
    else if (suf == "M") mul = 1e6L;
    else if (suf == "G") mul = 1e9L;
    else if (suf == "T") mul = 1e12L;
    else if (suf == "P") mul = 1e15L;
    else if (suf == "E") mul = 1e18L;
    else if (suf == "Ki") mul = 1024.0L;
    else if (suf == "Mi") mul = 1024.0L * 1024;
    else if (suf == "Gi") mul = 1024.0L * 1024 * 1024;
    else if (suf == "Ti") mul = 1024.0L * 1024 * 1024 * 1024;
    else if (suf == "Pi") mul = 1024.0L * 1024 * 1024 * 1024 * 1024;
    else if (suf == "Ei") mul = 1024.0L * 1024 * 1024 * 1024 * 1024 * 1024;
    else if (suf[0] == 'e' || suf[0] == 'E') {
        char* end = nullptr;
        const long e = std::strtol(suf.c_str() + 1, &end, 10);
        if (*end != '\0' || suf.size() < 2) return false;
        mul = std::pow(10.0L, (long double)e);
    } else {
        return false;
    }
    v *= mul;
    long double unit = 1;
    if (resource == "cpu") unit = 1e-3L;                                          // millicores
    else if (resource == "memory" || resource == "ephemeral-storage") unit = 1024.0L * 1024;  // MiB
    long double x = v / unit;
    x = round_up ? std::ceil(x - 1e-9L) : std::floor(x + 1e-9L);
    if (x < 0) x = 0;
    *out = x > 1.8e19L ? ~0ull : (uint64_t)x;
    return true;
}

static uint64_t container_sum(const Json& containers, const std::string& resource) {
    uint64_t s = 0;
    for (const auto& c : containers.elems()) {
        uint64_t v = 0;
        const Json& r = c.get("resources").get("requests");
        if (has_key(r, resource) && parse_quantity(r.get(resource).as_string(), resource, true, &v)) s += v;
    }
    return s;
}

uint64_t pod_request(const Json& podSpec, const std::string& resource) {
    const uint64_t sum = container_sum(podSpec.get("containers"), resource);
    uint64_t init_max = 0;
    for (const auto& c : podSpec.get("initContainers").elems()) {
        Json one = Json::array();
        one.push_back(c);
        init_max = std::max(init_max, container_sum(one, resource));
    }
    return std::max(sum, init_max);
}

// ------------------------------------------------------------------ planner
Planner::Planner(jsp_engine* e, std::vector<std::string> level_keys, std::vector<std::string> resources)
    : eng_(e), level_keys_(std::move(level_keys)), res_(std::move(resources)) {}

int Planner::level_of(const std::string& key) const {
    for (size_t k = 0; k < level_keys_.size(); ++k)
        if (level_keys_[k] == key) return (int)k;
    return -1;
}

bool Planner::row_of(const std::string& node, int32_t* row) const {
    auto it = node_row_.find(node);
    if (it == node_row_.end()) return false;
    *row = it->second;
    return true;
}

int32_t Planner::domain_id(int level, const std::string& value) const {
    if (level < 0 || (size_t)level >= domain_ids_.size()) return -1;
    auto it = domain_ids_[level].find(value);
    return it == domain_ids_[level].end() ? -1 : it->second;
}

void Planner::domain_rows(int level, int32_t d, uint32_t* first, uint32_t* end) const {
    const uint32_t a = first_leaf_[level][d], b = first_leaf_[level][d + 1];
    *first = leaf_start_[a];
    *end = leaf_start_[b];
}

int32_t Planner::row_domain(uint32_t row, int level) const {
    const uint32_t leaf = (uint32_t)(std::upper_bound(leaf_start_.begin(), leaf_start_.end(), row) - leaf_start_.begin()) - 1;
    const auto& fl = first_leaf_[level];
    return (int32_t)(std::upper_bound(fl.begin(), fl.end(), leaf) - fl.begin()) - 1;
}

int Planner::pred_bit(const LabelPred& p) const {
    auto it = std::lower_bound(preds_.begin(), preds_.end(), p);
    return (it != preds_.end() && *it == p) ? (int)(it - preds_.begin()) : -1;
}

Err2 Planner::rebuild(const std::map<std::string, Json>& nodes, const std::map<std::string, Json>& pods) {
    const size_t K = level_keys_.size(), R = res_.size();
    if (K < 1 || K > JSP_MAX_LEVELS) return {"planner: 1.." + std::to_string(JSP_MAX_LEVELS) + " topology keys"};
    if (R < 1 || R > JSP_MAX_RES) return {"planner: 1.." + std::to_string(JSP_MAX_RES) + " resources"};
    if (preds_.size() > 64u * JSP_MAX_LABEL_WORDS)
        return {"planner: " + std::to_string(preds_.size()) + " label predicates exceed the engine's " +
                std::to_string(64 * JSP_MAX_LABEL_WORDS)};
    // nodes carrying every level label, sorted by (level values..., name)
    struct Row {
        std::vector<std::string> key;
        const Json* node;
    };
    std::vector<Row> rows;
    std::vector<std::string> skipped;
    std::set<TaintKey> taint_set;
    for (const auto& kv : nodes) {
        const Json& lab = labels_of(kv.second);
        Row r{{}, &kv.second};
        bool ok = true;
        for (const auto& k : level_keys_) {
            if (!has_key(lab, k)) { ok = false; break; }
            r.key.push_back(lab.get(k).as_string());
        }
        if (!ok) { skipped.push_back(kv.first); continue; }
        r.key.push_back(kv.first);
        rows.push_back(std::move(r));
        for (const auto& t : kv.second.get("spec").get("taints").elems()) {
            const std::string eff = t.get("effect").as_string();
            if (eff == "NoSchedule" || eff == "NoExecute")
                taint_set.insert({t.get("key").as_string(), t.get("value").as_string(), eff});
        }
        if (kv.second.get("spec").get("unschedulable").as_bool()) taint_set.insert({kUnschedulableTaint, "", "NoSchedule"});
    }
    if (taint_set.size() > 32) return {"planner: " + std::to_string(taint_set.size()) + " distinct NoSchedule/NoExecute taints exceed 32"};
    std::sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) { return a.key < b.key; });
    const uint32_t N = (uint32_t)rows.size();
    // domains per level; a level-k value must sit under exactly one level-(k-1) domain
    std::vector<std::vector<std::string>> dv(K);
    std::vector<std::map<std::string, int32_t>> did(K);
    std::vector<std::vector<uint32_t>> dstart(K);  // first row of each domain
    for (uint32_t i = 0; i < N; ++i) {
        for (size_t k = 0; k < K; ++k) {
            bool fresh = i == 0;
            for (size_t j = 0; j <= k && !fresh; ++j) fresh = rows[i].key[j] != rows[i - 1].key[j];
            if (!fresh) continue;
            const std::string& v = rows[i].key[k];
            if (did[k].count(v))
                return {"planner: topology key " + level_keys_[k] + " value " + v + " spans several " +
                        (k ? level_keys_[k - 1] : std::string("")) + " domains (keys must nest)"};
            did[k][v] = (int32_t)dv[k].size();
            dv[k].push_back(v);
            dstart[k].push_back(i);
        }
    }
    const uint32_t L = (uint32_t)dv[K - 1].size();
    std::vector<uint32_t> leaf_start(dstart[K - 1]);
    leaf_start.push_back(N);
    std::vector<std::vector<uint32_t>> fl(K);
    for (size_t k = 0; k < K; ++k) {
        for (uint32_t r0 : dstart[k])  // the leaf that starts at a domain's first row
            fl[k].push_back((uint32_t)(std::lower_bound(dstart[K - 1].begin(), dstart[K - 1].end(), r0) - dstart[K - 1].begin()));
        fl[k].push_back(L);
    }
    // columns
    std::vector<TaintKey> taints(taint_set.begin(), taint_set.end());
    const uint32_t W = std::max<uint32_t>(1, (uint32_t)((preds_.size() + 63) / 64));
    std::vector<uint64_t> lab((size_t)W * N, 0);
    std::vector<uint32_t> tb(N, 0), fr((size_t)R * N, 0);
    std::vector<int32_t> ex(N, -1);
    std::map<std::string, int32_t> node_row;
    std::vector<std::string> row_node(N);
    for (uint32_t i = 0; i < N; ++i) {
        const Json& node = *rows[i].node;
        const std::string name = rows[i].key.back();
        row_node[i] = name;
        node_row[name] = (int32_t)i;
        const Json& nl = labels_of(node);
        for (size_t b = 0; b < preds_.size(); ++b)
            if (preds_[b].holds(nl)) lab[(b >> 6) * N + i] |= 1ull << (b & 63);
        for (const auto& t : node.get("spec").get("taints").elems()) {
            const TaintKey key{t.get("key").as_string(), t.get("value").as_string(), t.get("effect").as_string()};
            auto it = std::lower_bound(taints.begin(), taints.end(), key);
            if (it != taints.end() && *it == key) tb[i] |= 1u << (it - taints.begin());
        }
        if (node.get("spec").get("unschedulable").as_bool()) {
            const TaintKey key{kUnschedulableTaint, "", "NoSchedule"};
            tb[i] |= 1u << (std::lower_bound(taints.begin(), taints.end(), key) - taints.begin());
        }
        const Json& alloc = node.get("status").get("allocatable");
        for (size_t r = 0; r < R; ++r) {
            uint64_t v = 0;
            if (has_key(alloc, res_[r])) parse_quantity(alloc.get(res_[r]).as_string(), res_[r], false, &v);
            fr[r * N + i] = (uint32_t)std::min<uint64_t>(v, 0xFFFFFFFFull);
        }
    }
    // bound, non-terminal pods: their requests come off their node's free
    // resources; an exclusive pod covers its node's domain at its key's level
    std::map<std::string, int32_t> job_ids;  // job-key -> dense id (sorted)
    std::vector<std::pair<std::string, std::pair<int, int32_t>>> covers;  // job-key, (level, domain)
    for (const auto& kv : pods) {
        const Json& pod = kv.second;
        const std::string nn = pod.get("spec").get("nodeName").as_string();
        const std::string phase = pod.get("status").get("phase").as_string();
        if (nn.empty() || phase == "Succeeded" || phase == "Failed") continue;
        auto it = node_row.find(nn);
        if (it == node_row.end()) continue;
        const uint32_t i = (uint32_t)it->second;
        for (size_t r = 0; r < R; ++r) {
            const uint64_t q = pod_request(pod.get("spec"), res_[r]);
            fr[r * N + i] = (uint32_t)(q >= fr[r * N + i] ? 0 : fr[r * N + i] - q);
        }
        const Json& ann = pod.get("metadata").get("annotations");
        if (!has_key(ann, kExclusiveKey) || !has_key(labels_of(pod), kJobKey)) continue;
        const int lvl = level_of(ann.get(kExclusiveKey).as_string());
        if (lvl < 0) continue;  // a key that is not an engine level: not modelled
        const std::string& v = labels_of(*rows[i].node).get(level_keys_[lvl]).as_string();
        covers.push_back({labels_of(pod).get(kJobKey).as_string(), {lvl, did[lvl][v]}});
        job_ids[covers.back().first] = 0;
    }
    int32_t next = 0;
    for (auto& kv : job_ids) kv.second = next++;
    for (const auto& c : covers) {
        const uint32_t a = leaf_start[fl[c.second.first][c.second.second]];
        const uint32_t b = leaf_start[fl[c.second.first][c.second.second + 1]];
        for (uint32_t i = a; i < b; ++i) ex[i] = job_ids[c.first];
    }
    // commit
    taints_ = std::move(taints);
    row_node_ = std::move(row_node);
    node_row_ = std::move(node_row);
    domain_values_ = std::move(dv);
    domain_ids_ = std::move(did);
    first_leaf_ = std::move(fl);
    leaf_start_ = std::move(leaf_start);
    W_ = W;
    labels_ = std::move(lab);
    taint_bits_ = std::move(tb);
    free_ = std::move(fr);
    excl_ = std::move(ex);
    skipped_ = std::move(skipped);
    exclusive_jobs_ = (uint32_t)job_ids.size();
    return {};
}

Err2 Planner::upload_full() {
    const uint32_t K = (uint32_t)level_keys_.size();
    jsp_topology t{};
    t.n_levels = K;
    for (uint32_t k = 0; k < K; ++k) {
        t.n_domains[k] = (uint32_t)domain_values_[k].size();
        t.first_leaf[k] = first_leaf_[k].data();
    }
    if (jsp_topology_upload(eng_, &t) != JSP_OK) return {std::string("placement engine: ") + jsp_last_error()};
    jsp_nodes n{};
    n.n_nodes = (uint32_t)row_node_.size();
    n.leaf_begin = 0;
    n.n_leaves = (uint32_t)leaf_start_.size() - 1;
    n.leaf_start = leaf_start_.data();
    n.n_label_words = W_;
    n.labels = labels_.data();
    n.taints = taint_bits_.data();
    n.n_res = (uint32_t)res_.size();
    n.free_res = free_.data();
    n.excl_owner = excl_.data();
    if (jsp_snapshot_upload(eng_, &n) != JSP_OK) return {std::string("placement engine: ") + jsp_last_error()};
    return {};
}

Err2 Planner::sync(const std::map<std::string, Json>& nodes, const std::map<std::string, Json>& pods, Json* stats) {
    // previous structure and columns, to decide between a patch and a full upload
    const std::vector<std::string> old_rows = row_node_;
    const std::vector<std::vector<uint32_t>> old_fl = first_leaf_;
    const std::vector<uint32_t> old_ls = leaf_start_;
    const std::vector<TaintKey> old_taints = taints_;
    const uint32_t old_W = W_;
    const std::vector<uint64_t> old_lab = labels_;
    const std::vector<uint32_t> old_tb = taint_bits_, old_fr = free_;
    const std::vector<int32_t> old_ex = excl_;
    if (Err2 e = rebuild(nodes, pods); !e.ok()) return e;
    nodes_dirty_ = false;  // the rebuilt host columns reflect every Node event so far
    const uint32_t N = (uint32_t)row_node_.size(), R = (uint32_t)res_.size();
    const bool same = synced_ && !preds_dirty_ && old_rows == row_node_ && old_fl == first_leaf_ &&
                      old_ls == leaf_start_ && old_taints == taints_ && old_W == W_;
    std::string upload = "none";
    uint32_t patched = 0;
    if (eng_ == nullptr) {  // host-only planner (tests of the ingestion itself)
        preds_dirty_ = false;
        synced_ = true;
        upload = "none (no engine)";
    } else if (!same) {
        if (Err2 e = upload_full(); !e.ok()) { synced_ = false; return e; }
        upload = "full";
        preds_dirty_ = false;
        synced_ = true;
    } else {
        std::vector<uint32_t> rows;
        for (uint32_t i = 0; i < N; ++i) {
            bool d = old_tb[i] != taint_bits_[i] || old_ex[i] != excl_[i];
            for (uint32_t w = 0; w < W_ && !d; ++w) d = old_lab[(size_t)w * N + i] != labels_[(size_t)w * N + i];
            for (uint32_t r = 0; r < R && !d; ++r) d = old_fr[(size_t)r * N + i] != free_[(size_t)r * N + i];
            if (d) rows.push_back(i);
        }
        if (!rows.empty()) {
            const uint32_t n = (uint32_t)rows.size();
            std::vector<uint64_t> dl((size_t)W_ * n);
            std::vector<uint32_t> dt(n), df((size_t)R * n);
            std::vector<int32_t> de(n);
            for (uint32_t j = 0; j < n; ++j) {
                const uint32_t i = rows[j];
                for (uint32_t w = 0; w < W_; ++w) dl[(size_t)w * n + j] = labels_[(size_t)w * N + i];
                for (uint32_t r = 0; r < R; ++r) df[(size_t)r * n + j] = free_[(size_t)r * N + i];
                dt[j] = taint_bits_[i];
                de[j] = excl_[i];
            }
            if (jsp_snapshot_patch(eng_, rows.data(), n, dl.data(), dt.data(), df.data(), de.data()) != JSP_OK) {
                // the host columns are already the new ones: without this the
                // next sync would find nothing to patch and the engine would
                // keep the old rows for good; a full upload repairs it
                synced_ = false;
                return {std::string("placement engine: ") + jsp_last_error()};
            }
            upload = "patch";
            patched = n;
        }
    }
    if (stats) {
        Json s = Json::object();
        s["rows"] = (int64_t)N;
        s["leaves"] = (int64_t)(leaf_start_.size() - 1);
        Json dom = Json::array();
        for (const auto& v : domain_values_) dom.push_back((int64_t)v.size());
        s["domains"] = dom;
        s["labelWords"] = (int64_t)W_;
        s["labelPredicates"] = (int64_t)preds_.size();
        s["taintBits"] = (int64_t)taints_.size();
        Json sk = Json::array();
        for (const auto& n : skipped_) sk.push_back(n);
        s["skippedNodes"] = sk;
        s["upload"] = upload;
        s["patchedRows"] = (int64_t)patched;
        s["exclusiveJobs"] = (int64_t)exclusive_jobs_;
        *stats = s;
    }
    return {};
}

Err2 Planner::class_of(const Json& tmpl, int64_t parallelism, const std::string& topology_key, ClassSpec* out) {
    ClassSpec c;
    c.level = level_of(topology_key);
    if (c.level < 0) return {"planner: exclusive-topology key " + topology_key + " is not one of the engine's topology keys"};
    c.pods = (uint32_t)std::max<int64_t>(1, parallelism);
    const Json& spec = tmpl.get("spec");
    for (const auto& kv : spec.get("nodeSelector").items())
        c.req.push_back({kv.first, "In", {kv.second.as_string()}});
    const Json& terms =
        spec.get("affinity").get("nodeAffinity").get("requiredDuringSchedulingIgnoredDuringExecution").get("nodeSelectorTerms");
    if (terms.size() > 1) return {"planner: more than one nodeSelectorTerm (ORed terms) is not supported"};
    for (const auto& term : terms.elems()) {
        if (term.get("matchFields").size() > 0) return {"planner: nodeSelectorTerm matchFields is not supported"};
        for (const auto& e : term.get("matchExpressions").elems()) {
            const std::string key = e.get("key").as_string(), op = e.get("operator").as_string();
            std::vector<std::string> vals;
            for (const auto& v : e.get("values").elems()) vals.push_back(v.as_string());
            std::sort(vals.begin(), vals.end());
            vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
            if (op == "In") c.req.push_back({key, "In", vals});
            else if (op == "NotIn") c.forbid.push_back({key, "In", vals});
            else if (op == "Exists") c.req.push_back({key, "Exists", {}});
            else if (op == "DoesNotExist") c.forbid.push_back({key, "Exists", {}});
            else if ((op == "Gt" || op == "Lt") && vals.size() == 1) c.req.push_back({key, op, vals});
            else return {"planner: node selector operator " + op + " is not supported"};
        }
    }
    c.tolerations = spec.get("tolerations").is_array() ? spec.get("tolerations") : Json::array();
    for (const auto& r : res_) c.res.push_back(pod_request(spec, r));
    // register the predicates (sorted dictionary; a new one changes the columns)
    std::set<LabelPred> all(preds_.begin(), preds_.end());
    const size_t before = all.size();
    for (const auto& p : c.req) all.insert(p);
    for (const auto& p : c.forbid) all.insert(p);
    if (all.size() != before) {
        preds_.assign(all.begin(), all.end());
        preds_dirty_ = true;
    }
    *out = std::move(c);
    return {};
}

Err2 Planner::encode(const std::vector<ClassSpec>& classes, std::vector<jsp_job_class>* out) const {
    std::vector<jsp_job_class>& jc = *out;
    jc.assign(std::max<size_t>(classes.size(), 1), jsp_job_class{});
    for (size_t i = 0; i < classes.size(); ++i) {
        const ClassSpec& c = classes[i];
        jsp_job_class& x = jc[i];
        std::memset(&x, 0, sizeof x);
        for (const auto& p : c.req) {
            const int b = pred_bit(p);
            if (b < 0) return {"planner: unregistered predicate"};
            x.req_labels[b >> 6] |= 1ull << (b & 63);
        }
        for (const auto& p : c.forbid) {
            const int b = pred_bit(p);
            if (b < 0) return {"planner: unregistered predicate"};
            x.forbid_labels[b >> 6] |= 1ull << (b & 63);
        }
        for (size_t t = 0; t < taints_.size(); ++t)
            for (const auto& tol : c.tolerations.elems())
                if (tolerates(tol, taints_[t])) { x.tolerated_taints |= 1u << t; break; }
        x.level = (uint32_t)c.level;
        x.pods = c.pods;
        for (size_t r = 0; r < res_.size(); ++r) x.req_res[r] = (uint32_t)std::min<uint64_t>(c.res[r], 0xFFFFFFFFull);
    }
    return {};
}

Err2 Planner::place(const std::vector<ClassSpec>& classes, const std::vector<uint32_t>& run_class,
                    const std::vector<uint32_t>& run_len, std::vector<int32_t>* assign, jsp_stats* st) {
    if (eng_ == nullptr) return {"planner: no engine bound"};
    if (!synced_ || preds_dirty_) return {"planner: snapshot out of date (sync after registering templates)"};
    std::vector<jsp_job_class> jc;
    if (Err2 e = encode(classes, &jc); !e.ok()) return e;
    if (jsp_classes_upload(eng_, jc.data(), (uint32_t)classes.size()) != JSP_OK)
        return {std::string("placement engine: ") + jsp_last_error()};
    uint64_t J = 0;
    for (uint32_t n : run_len) J += n;
    assign->assign(std::max<uint64_t>(J, 1), -1);
    if (jsp_place(eng_, run_class.data(), run_len.data(), (uint32_t)run_class.size(), assign->data(), nullptr, nullptr,
                  st) != JSP_OK)
        return {std::string("placement engine: ") + jsp_last_error()};
    assign->resize(J);
    return {};
}

Json Planner::columns() const {
    Json c = Json::object();
    Json rows = Json::array();
    for (const auto& n : row_node_) rows.push_back(n);
    c["rows"] = rows;
    const size_t N = row_node_.size();
    Json lab = Json::array(), tb = Json::array(), fr = Json::array(), ex = Json::array();
    for (size_t i = 0; i < N; ++i) {
        Json words = Json::array();
        for (uint32_t w = 0; w < W_; ++w) {
            char buf[24];
            std::snprintf(buf, sizeof buf, "%016llx", (unsigned long long)labels_[(size_t)w * N + i]);
            words.push_back(std::string(buf));
        }
        lab.push_back(words);
        tb.push_back((int64_t)taint_bits_[i]);
        Json f = Json::array();
        for (size_t r = 0; r < res_.size(); ++r) f.push_back((int64_t)free_[r * N + i]);
        fr.push_back(f);
        ex.push_back((int64_t)excl_[i]);
    }
    c["labels"] = lab;
    c["taints"] = tb;
    c["free"] = fr;
    c["excl"] = ex;
    Json ls = Json::array();
    for (uint32_t v : leaf_start_) ls.push_back((int64_t)v);
    c["leafStart"] = ls;
    Json fl = Json::array();
    for (const auto& lv : first_leaf_) {
        Json a = Json::array();
        for (uint32_t v : lv) a.push_back((int64_t)v);
        fl.push_back(a);
    }
    c["firstLeaf"] = fl;
    Json dv = Json::array();
    for (const auto& lv : domain_values_) {
        Json a = Json::array();
        for (const auto& v : lv) a.push_back(v);
        dv.push_back(a);
    }
    c["domainValues"] = dv;
    Json pr = Json::array();
    for (const auto& p : preds_) {
        Json x = Json::object();
        x["key"] = p.key;
        x["op"] = p.op;
        Json vs = Json::array();
        for (const auto& v : p.values) vs.push_back(v);
        x["values"] = vs;
        pr.push_back(x);
    }
    c["predicates"] = pr;
    Json ts = Json::array();
    for (const auto& t : taints_) {
        Json x = Json::object();
        x["key"] = t.key;
        x["value"] = t.value;
        x["effect"] = t.effect;
        ts.push_back(x);
    }
    c["taintKeys"] = ts;
    return c;
}

Json label_nodes(const Planner& pl, int level, const std::vector<std::string>& namespaced_jobs,
                 const std::vector<int32_t>& assign) {
    Json out = Json::array();
    for (size_t j = 0; j < assign.size() && j < namespaced_jobs.size(); ++j) {
        if (assign[j] < 0) continue;
        uint32_t a = 0, b = 0;
        pl.domain_rows(level, assign[j], &a, &b);
        for (uint32_t r = a; r < b; ++r) {
            Json body = Json::object();
            body["metadata"]["labels"][kNamespacedJobKey] = namespaced_jobs[j];
            Json taint = Json::object();
            taint["key"] = kNoScheduleTaintKey;
            taint["value"] = "true";
            taint["effect"] = "NoSchedule";
            body["spec"]["taints"] = Json::array();
            body["spec"]["taints"].push_back(taint);
            Json patch = Json::object();
            patch["node"] = pl.row_node(r);
            patch["body"] = body;
            out.push_back(patch);
        }
    }
    return out;
}

}  // namespace jsk
