// jobset_host.cc — host-side mirror of the reference's exclusive-placement
// path around the engine: the pod webhook (mutation + admission), the leader
// PodReconciler, the child-Job construction / restart bucketing slice of the
// JobSet reconciler, and the placement utilities. Same function names,
// argument meaning and error strings as the Go reference (file:line at each
// function), over Kubernetes objects as JSON (what an AdmissionReview
// carries). The reference's controller-runtime cached client is a small
// in-memory store with the same field indexes and injectable errors (the
// reference's unit tests use controller-runtime's fake client with
// interceptor.Funcs the same way, pkg/controllers/pod_controller_test.go:171-184).
//
// The engine is consulted, behind the unchanged mutation, for the follower's
// topology value (batched A5) and the placement audit (batched A9) when a
// cache is bound to an engine (cache.bindEngine).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../../include/jsk_host.h"
#include "../../../include/jsplace.h"
#include "json.h"
#include "placement.h"
#include "sha1.h"

namespace jsk {

// ---- api/jobset/v1alpha2/jobset_types.go:22-58, pkg/constants/constants.go
const char* const kJobSetNameKey = "jobset.sigs.k8s.io/jobset-name";
const char* const kReplicatedJobReplicas = "jobset.sigs.k8s.io/replicatedjob-replicas";
const char* const kReplicatedJobNameKey = "jobset.sigs.k8s.io/replicatedjob-name";
const char* const kJobIndexKey = "jobset.sigs.k8s.io/job-index";
const char* const kJobGlobalIndexKey = "jobset.sigs.k8s.io/job-global-index";
const char* const kJobKey = "jobset.sigs.k8s.io/job-key";
const char* const kExclusiveKey = "alpha.jobset.sigs.k8s.io/exclusive-topology";
const char* const kNodeSelectorStrategyKey = "alpha.jobset.sigs.k8s.io/node-selector";
const char* const kNamespacedJobKey = "alpha.jobset.sigs.k8s.io/namespaced-job";
const char* const kNoScheduleTaintKey = "alpha.jobset.sigs.k8s.io/no-schedule";
const char* const kCoordinatorKey = "jobset.sigs.k8s.io/coordinator";
const char* const kRestartsKey = "jobset.sigs.k8s.io/restart-attempt";
const char* const kJobCompletionIndexAnnotation = "batch.kubernetes.io/job-completion-index";
const char* const kExclusivePlacementViolationReason = "ExclusivePlacementViolation";
const char* const kExclusivePlacementViolationMessage = "Pod violated JobSet exclusive placement policy";
const char* const kPodNameKey = "podName";      // pkg/controllers/pod_controller.go:43
const char* const kPodJobKey = "podJobKey";     // pkg/controllers/pod_controller.go:48

// ---- Go-like error value
struct Err {
    bool ok = true;
    bool not_found = false;
    std::string msg;
    static Err none() { return Err(); }
    static Err e(std::string m) { Err r; r.ok = false; r.msg = std::move(m); return r; }
    static Err nf(std::string m) { Err r = e(std::move(m)); r.not_found = true; return r; }
};

// fmt %q of a string (strconv.Quote for the ASCII range)
std::string go_quote(const std::string& s) {
    std::string o = "\"";
    for (unsigned char c : s) {
        if (c == '"') o += "\\\"";
        else if (c == '\\') o += "\\\\";
        else if (c == '\n') o += "\\n";
        else if (c == '\t') o += "\\t";
        else if (c == '\r') o += "\\r";
        else if (c < 0x20 || c == 0x7f) {
            char b[8];
            std::snprintf(b, sizeof b, "\\x%02x", c);
            o += b;
        } else o += (char)c;
    }
    return o + "\"";
}

std::string errors_join(const std::vector<std::string>& errs) {  // errors.Join
    std::string o;
    for (size_t i = 0; i < errs.size(); ++i) o += (i ? "\n" : "") + errs[i];
    return o;
}

// ---- object accessors
const Json& meta(const Json& o) { return o.get("metadata"); }
const Json& labels(const Json& o) { return meta(o).get("labels"); }
const Json& annotations(const Json& o) { return meta(o).get("annotations"); }
std::string name_of(const Json& o) { return meta(o).get("name").as_string(); }
std::string ns_of(const Json& o) { return meta(o).get("namespace").as_string(); }
std::string node_name(const Json& pod) { return pod.get("spec").get("nodeName").as_string(); }

// metav1.GetControllerOf: the owner reference with controller == true
const Json* controller_of(const Json& o) {
    for (const auto& r : meta(o).get("ownerReferences").elems())
        if (r.get("controller").as_bool()) return &r;
    return nullptr;
}

Json clone_map(const Json& m) { return m.is_object() ? m : Json::object(); }  // collections.CloneMap

// ============================================================ pkg/util/placement/placement.go
// GenJobName, placement.go:14-16
std::string GenJobName(const std::string& js, const std::string& rjob, int64_t idx) {
    return js + "-" + rjob + "-" + std::to_string(idx);
}
// GenPodName, placement.go:20-22
std::string GenPodName(const std::string& js, const std::string& rjob, const std::string& jobIdx,
                       const std::string& podIdx) {
    return js + "-" + rjob + "-" + jobIdx + "-" + podIdx;
}
// IsLeaderPod, placement.go:26-28
bool IsLeaderPod(const Json& pod) { return str_at(annotations(pod), kJobCompletionIndexAnnotation) == "0"; }

// ============================================================ pkg/controllers/jobset_controller.go
// sha1Hash / jobHashKey, :809-818
std::string sha1Hash(const std::string& s) { return sha1_hex(s); }
std::string jobHashKey(const std::string& ns, const std::string& jobName) { return sha1Hash(ns + "/" + jobName); }
// namespacedJobName, :804-806
std::string namespacedJobName(const std::string& ns, const std::string& job) { return ns + "_" + job; }

// globalJobIndex, :1056-1065
std::string globalJobIndex(const Json& js, const std::string& rjobName, int64_t jobIdx) {
    int64_t total = 0;
    for (const auto& rj : js.get("spec").get("replicatedJobs").elems()) {
        if (rj.get("name").as_string() == rjobName) return std::to_string(total + jobIdx);
        total += rj.get("replicas").as_int();
    }
    return "";
}

// GetSubdomain, :790-798
std::string GetSubdomain(const Json& js) {
    const std::string sd = js.get("spec").get("network").get("subdomain").as_string();
    return sd.empty() ? name_of(js) : sd;
}
bool dnsHostnamesEnabled(const Json& js) { return js.get("spec").get("network").get("enableDNSHostnames").as_bool(); }
bool jobSetSuspended(const Json& js) { return js.get("spec").get("suspend").as_bool(); }

// coordinatorEndpoint, :1034-1036
std::string coordinatorEndpoint(const Json& js) {
    const Json& c = js.get("spec").get("coordinator");
    return name_of(js) + "-" + c.get("replicatedJob").as_string() + "-" + std::to_string(c.get("jobIndex").as_int()) +
           "-" + std::to_string(c.get("podIndex").as_int()) + "." + GetSubdomain(js);
}

// labelAndAnnotateObject, :722-770 (A1: the exclusive-topology block is :751-766)
void labelAndAnnotateObject(Json& objMeta, const Json& js, const Json& rjob, int64_t jobIdx) {
    const std::string jsName = name_of(js), rjName = rjob.get("name").as_string();
    const std::string jobName = GenJobName(jsName, rjName, jobIdx);
    const std::string restarts = std::to_string(js.get("status").get("restarts").as_int());
    const std::string replicas = std::to_string(rjob.get("replicas").as_int());
    const std::string key = jobHashKey(ns_of(js), jobName);
    const std::string gidx = globalJobIndex(js, rjName, jobIdx);
    Json lab = clone_map(objMeta.get("labels"));
    Json ann = clone_map(objMeta.get("annotations"));
    for (Json* m : {&lab, &ann}) {
        (*m)[kJobSetNameKey] = jsName;
        (*m)[kReplicatedJobNameKey] = rjName;
        (*m)[kRestartsKey] = restarts;
        (*m)[kReplicatedJobReplicas] = replicas;
        (*m)[kJobIndexKey] = std::to_string(jobIdx);
        (*m)[kJobKey] = key;
        (*m)[kJobGlobalIndexKey] = gidx;
    }
    if (!js.get("spec").get("coordinator").is_null()) {
        lab[kCoordinatorKey] = coordinatorEndpoint(js);
        ann[kCoordinatorKey] = coordinatorEndpoint(js);
    }
    // JobSet-level exclusive placement
    const Json& jsAnn = annotations(js);
    if (has_key(jsAnn, kExclusiveKey)) {
        ann[kExclusiveKey] = str_at(jsAnn, kExclusiveKey);
        if (has_key(jsAnn, kNodeSelectorStrategyKey)) ann[kNodeSelectorStrategyKey] = str_at(jsAnn, kNodeSelectorStrategyKey);
    }
    // ReplicatedJob-level exclusive placement (overrides)
    const Json& rjAnn = rjob.get("template").get("metadata").get("annotations");
    if (has_key(rjAnn, kExclusiveKey)) {
        ann[kExclusiveKey] = str_at(rjAnn, kExclusiveKey);
        if (has_key(rjAnn, kNodeSelectorStrategyKey)) ann[kNodeSelectorStrategyKey] = str_at(rjAnn, kNodeSelectorStrategyKey);
    }
    objMeta["labels"] = lab;
    objMeta["annotations"] = ann;
}

// addNamespacedJobNodeSelector, :795-800; addTaintToleration, :688-696
void addNamespacedJobNodeSelector(Json& job) {
    Json& ps = job["spec"]["template"]["spec"];
    if (!ps.get("nodeSelector").is_object()) ps["nodeSelector"] = Json::object();
    ps["nodeSelector"][kNamespacedJobKey] = namespacedJobName(ns_of(job), name_of(job));
}
void addTaintToleration(Json& job) {
    Json& ps = job["spec"]["template"]["spec"];
    Json t = Json::object();
    t["key"] = kNoScheduleTaintKey;
    t["operator"] = "Exists";
    t["effect"] = "NoSchedule";
    if (!ps.get("tolerations").is_array()) ps["tolerations"] = Json::array();
    ps["tolerations"].push_back(t);
}

// constructJob, :651-686
Json constructJob(const Json& js, const Json& rjob, int64_t jobIdx) {
    const Json& tmpl = rjob.get("template");
    Json job = Json::object();
    job["metadata"]["labels"] = clone_map(tmpl.get("metadata").get("labels"));
    job["metadata"]["annotations"] = clone_map(tmpl.get("metadata").get("annotations"));
    job["metadata"]["name"] = GenJobName(name_of(js), rjob.get("name").as_string(), jobIdx);
    job["metadata"]["namespace"] = ns_of(js);
    job["spec"] = tmpl.get("spec").is_object() ? tmpl.get("spec") : Json::object();
    labelAndAnnotateObject(job["metadata"], js, rjob, jobIdx);
    labelAndAnnotateObject(job["spec"]["template"]["metadata"], js, rjob, jobIdx);
    if (dnsHostnamesEnabled(js)) job["spec"]["template"]["spec"]["subdomain"] = GetSubdomain(js);
    const Json& ann = job.get("metadata").get("annotations");
    if (has_key(ann, kExclusiveKey) && has_key(ann, kNodeSelectorStrategyKey)) {
        addNamespacedJobNodeSelector(job);
        addTaintToleration(job);
    }
    job["spec"]["suspend"] = jobSetSuspended(js);
    return job;
}

// shouldCreateJob, :698-709
bool shouldCreateJob(const std::string& jobName, const Json& owned) {
    for (const char* b : {"active", "successful", "failed", "delete"})
        for (const auto& j : owned.get(b).elems())
            if (name_of(j) == jobName) return false;
    return true;
}

// constructJobsFromTemplate, :638-649
Json constructJobsFromTemplate(const Json& js, const Json& rjob, const Json& owned) {
    Json jobs = Json::array();
    for (int64_t i = 0; i < rjob.get("replicas").as_int(); ++i) {
        const std::string n = GenJobName(name_of(js), rjob.get("name").as_string(), i);
        if (!shouldCreateJob(n, owned)) continue;
        jobs.push_back(constructJob(js, rjob, i));
    }
    return jobs;
}

// JobFinished, :772-779
std::string jobFinishedType(const Json& job) {
    for (const auto& c : job.get("status").get("conditions").elems()) {
        const std::string t = c.get("type").as_string();
        if ((t == "Complete" || t == "Failed") && c.get("status").as_string() == "True") return t;
    }
    return "";
}

// getChildJobs bucketing, :267-305 (restart attempts older than status.restarts -> delete)
Err getChildJobs(const Json& js, const Json& jobs, Json* out) {
    Json b = Json::object();
    for (const char* k : {"active", "successful", "failed", "delete"}) b[k] = Json::array();
    const int64_t restarts = js.get("status").get("restarts").as_int();
    for (const auto& job : jobs.elems()) {
        const std::string v = str_at(labels(job), kRestartsKey);
        char* end = nullptr;
        const long r = std::strtol(v.c_str(), &end, 10);
        if (v.empty() || *end != '\0') {
            b["delete"].push_back(job);
            *out = b;
            return Err::e("strconv.Atoi: parsing " + go_quote(v) + ": invalid syntax");
        }
        if (r < restarts) {
            b["delete"].push_back(job);
            continue;
        }
        const std::string t = jobFinishedType(job);
        if (t.empty()) b["active"].push_back(job);
        else if (t == "Failed") b["failed"].push_back(job);
        else b["successful"].push_back(job);
    }
    *out = b;
    return Err::none();
}

// failurePolicyRecreateAll, pkg/controllers/failure_policy.go:155-175 (A10 trigger)
void failurePolicyRecreateAll(Json& js, bool shouldCountTowardsMax) {
    Json& st = js["status"];
    st["restarts"] = st.get("restarts").as_int() + 1;
    if (shouldCountTowardsMax) st["restartsCountTowardsMax"] = st.get("restartsCountTowardsMax").as_int() + 1;
}

// ============================================================ pkg/controllers/pod_controller.go
// removePodNameSuffix, :297-306
Err removePodNameSuffix(const std::string& podName, std::string* out) {
    std::vector<std::string> parts;
    size_t st = 0;
    while (true) {
        size_t p = podName.find('-', st);
        parts.push_back(podName.substr(st, p == std::string::npos ? std::string::npos : p - st));
        if (p == std::string::npos) break;
        st = p + 1;
    }
    if (parts.size() < 5) return Err::e("invalid pod name: " + podName);
    std::string r;
    for (size_t i = 0; i + 1 < parts.size(); ++i) r += (i ? "-" : "") + parts[i];
    *out = r;
    return Err::none();
}

// SetupPodIndexes extractors, :75-106 (A11)
std::vector<std::string> podJobKeyIndex(const Json& pod) {
    if (!has_key(annotations(pod), kExclusiveKey)) return {};
    if (!has_key(labels(pod), kJobKey)) return {};
    return {str_at(labels(pod), kJobKey)};
}
std::vector<std::string> podNameIndex(const Json& pod) {
    if (!has_key(annotations(pod), kExclusiveKey)) return {};
    std::string n;
    if (!removePodNameSuffix(name_of(pod), &n).ok) return {};
    return {n};
}

bool usingExclusivePlacement(const Json& pod) { return has_key(annotations(pod), kExclusiveKey); }
bool podScheduled(const Json& pod) { return !node_name(pod).empty(); }
bool podDeleted(const Json& pod) { return !meta(pod).get("deletionTimestamp").is_null(); }

// followerPodTopology, :268-277
Err followerPodTopology(const Json& pod, const std::string& key, std::string* out) {
    const Json& ns = pod.get("spec").get("nodeSelector");
    if (!ns.is_object()) return Err::e("pod " + name_of(pod) + " nodeSelector is nil");
    if (!ns.has(key)) return Err::e("pod " + name_of(pod) + " nodeSelector is missing key: " + key);
    *out = ns.get(key).as_string();
    return Err::none();
}

// updatePodCondition, :309-327 (LastTransitionTime is set by the caller's clock)
bool updatePodCondition(Json& pod, Json cond) {
    Json& conds = pod["status"]["conditions"];
    if (!conds.is_array()) conds = Json::array();
    for (auto& c : conds.elems()) {
        const bool sameType = c.get("type") == cond.get("type");
        if (sameType && c.get("status") != cond.get("status")) {
            c = cond;
            return true;
        }
        if (sameType) return false;
    }
    if (cond.get("status").as_string() == "True") {
        conds.push_back(cond);
        return true;
    }
    return false;
}

// ============================================================ cached client
struct Cache {
    std::mutex mu;
    std::map<std::string, Json> pods;   // ns/name
    std::map<std::string, Json> nodes;  // name
    std::map<std::string, std::string> inject;  // "get/Node", "list/Pod", "update/Pod", "delete/Pod" -> error text
    // engine binding (the snapshot mirrors the node cache)
    jsp_engine* eng = nullptr;
    std::map<std::string, int32_t> node_rows;
    std::vector<std::string> level_keys;
    std::vector<std::vector<std::string>> domain_values;
    std::vector<std::map<std::string, int32_t>> domain_ids;
    // planner: the engine's snapshot built from this cache's objects (placement.h)
    std::unique_ptr<Planner> planner;
    // call counters (tests check which path ran)
    int64_t node_gets = 0, pod_lists = 0, engine_calls = 0;
    std::vector<std::string> deleted, status_updates;
};

Err injected(Cache& c, const std::string& what) {
    auto it = c.inject.find(what);
    if (it == c.inject.end()) return Err::none();
    return Err::e(it->second);
}

Err getNode(Cache& c, const std::string& name, Json* out) {
    ++c.node_gets;
    if (Err e = injected(c, "get/Node"); !e.ok) return e;
    auto it = c.nodes.find(name);
    if (it == c.nodes.end()) return Err::nf("nodes " + go_quote(name) + " not found");
    *out = it->second;
    return Err::none();
}

Err getPod(Cache& c, const std::string& ns, const std::string& name, Json* out) {
    if (Err e = injected(c, "get/Pod"); !e.ok) return e;
    auto it = c.pods.find(ns + "/" + name);
    if (it == c.pods.end()) return Err::nf("pods " + go_quote(name) + " not found");
    *out = it->second;
    return Err::none();
}

// client.List(InNamespace(ns), MatchingFields{field: value})
Err listPods(Cache& c, const std::string& ns, const std::string& field, const std::string& value, Json* out) {
    ++c.pod_lists;
    if (Err e = injected(c, "list/Pod"); !e.ok) return e;
    Json items = Json::array();
    for (const auto& kv : c.pods) {
        if (ns_of(kv.second) != ns) continue;
        const auto idx = field == kPodNameKey ? podNameIndex(kv.second) : podJobKeyIndex(kv.second);
        if (std::find(idx.begin(), idx.end(), value) != idx.end()) items.push_back(kv.second);
    }
    *out = items;
    return Err::none();
}

// Topology value of the node a pod is bound to: pod_mutating_webhook.go:173-194
// and pod_controller.go:242-263 (identical logic). With an engine bound, the
// domain of a node the snapshot holds, at one of its topology levels, comes
// from the resident snapshot (jsp_resolve_leader_domains). Anything else -- a
// key that is not an engine level, a node the snapshot does not hold (absent
// from the cache, or lacking a level label) -- takes the reference's Node Get
// path, so NotFound stays "" + nil and a missing label stays its error.
bool engineTopology(Cache& c, const std::string& node, const std::string& key, int32_t* row, uint32_t* level) {
    if (!c.eng) return false;
    if (c.planner) {
        const int lk = c.planner->level_of(key);
        if (lk < 0 || !c.planner->serving() || !c.planner->row_of(node, row)) return false;
        *level = (uint32_t)lk;
        return true;
    }
    auto lk = std::find(c.level_keys.begin(), c.level_keys.end(), key);
    auto it = c.node_rows.find(node);
    if (lk == c.level_keys.end() || it == c.node_rows.end()) return false;
    *row = it->second;
    *level = (uint32_t)(lk - c.level_keys.begin());
    return true;
}

const std::string& domainValue(Cache& c, uint32_t level, int32_t dom) {
    static const std::string empty;
    const std::vector<std::string>& v = c.planner ? c.planner->domain_values((int)level) : c.domain_values[level];
    return dom >= 0 && (size_t)dom < v.size() ? v[dom] : empty;
}

Err topologyFromPod(Cache& c, const Json& pod, const std::string& key, std::string* out) {
    const std::string node = node_name(pod);
    int32_t row = -1;
    uint32_t level = 0;
    if (engineTopology(c, node, key, &row, &level)) {
        int32_t dom = -1;
        ++c.engine_calls;
        if (jsp_resolve_leader_domains(c.eng, &row, &level, 1, &dom) != JSP_OK)
            return Err::e(std::string("placement engine: ") + jsp_last_error());
        *out = domainValue(c, level, dom);
        return Err::none();
    }
    Json n;
    Err e = getNode(c, node, &n);
    if (!e.ok) {
        *out = "";
        return e.not_found ? Err::none() : e;  // client.IgnoreNotFound
    }
    if (!has_key(labels(n), key)) return Err::e("node does not have topology label: " + key);
    *out = str_at(labels(n), key);
    return Err::none();
}

// ============================================================ pkg/webhooks
// genLeaderPodName, pod_admission_webhook.go:128-144
Err genLeaderPodName(const Json& pod, std::string* out) {
    const Json& l = labels(pod);
    for (const char* k : {kJobSetNameKey, kReplicatedJobNameKey, kJobIndexKey})
        if (!has_key(l, k)) return Err::e(std::string("pod missing label: ") + k);
    *out = GenPodName(str_at(l, kJobSetNameKey), str_at(l, kReplicatedJobNameKey), str_at(l, kJobIndexKey), "0");
    return Err::none();
}

// podsOwnedBySameJob, pod_admission_webhook.go:148-161
Err podsOwnedBySameJob(const Json& leader, const Json& follower) {
    const Json* f = controller_of(follower);
    if (!f) return Err::e("follower pod has no owner reference");
    const Json* l = controller_of(leader);
    if (!l) return Err::e("leader pod " + go_quote(name_of(leader)) + " has no owner reference");
    if (f->get("uid").as_string() != l->get("uid").as_string())
        return Err::e("follower pod owner UID (" + f->get("uid").as_string() + ") != leader pod owner UID (" +
                      l->get("uid").as_string() + ")");
    return Err::none();
}

// leaderPodForFollower, pod_admission_webhook.go:91-124
Err leaderPodForFollower(Cache& c, const Json& pod, Json* leader) {
    std::string ln;
    if (Err e = genLeaderPodName(pod, &ln); !e.ok) return e;
    Json list;
    if (Err e = listPods(c, ns_of(pod), kPodNameKey, ln, &list); !e.ok) return e;
    if (list.size() != 1)
        return Err::e("expected 1 leader pod (" + ln + "), but got " + std::to_string(list.size()) +
                      ". this is an expected, transient error");
    if (Err e = podsOwnedBySameJob(list.at(0), pod); !e.ok) return e;
    *leader = list.at(0);
    return Err::none();
}

// setExclusiveAffinities, pod_mutating_webhook.go:95-135 (A4): appends, never dedupes
void setExclusiveAffinities(Json& pod) {
    const std::string own = str_at(labels(pod), kJobKey);
    const std::string topo = str_at(annotations(pod), kExclusiveKey);
    Json& aff = pod["spec"]["affinity"];
    Json term = Json::object();
    Json req = Json::object();
    req["key"] = kJobKey;
    req["operator"] = "In";
    req["values"] = Json::array();
    req["values"].push_back(own);
    term["labelSelector"]["matchExpressions"] = Json::array();
    term["labelSelector"]["matchExpressions"].push_back(req);
    term["topologyKey"] = topo;
    term["namespaceSelector"] = Json::object();
    Json& pa = aff["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"];
    if (!pa.is_array()) pa = Json::array();
    pa.push_back(term);

    Json anti = Json::object();
    Json e1 = Json::object();
    e1["key"] = kJobKey;
    e1["operator"] = "Exists";
    Json e2 = Json::object();
    e2["key"] = kJobKey;
    e2["operator"] = "NotIn";
    e2["values"] = Json::array();
    e2["values"].push_back(own);
    anti["labelSelector"]["matchExpressions"] = Json::array();
    anti["labelSelector"]["matchExpressions"].push_back(e1);
    anti["labelSelector"]["matchExpressions"].push_back(e2);
    anti["topologyKey"] = topo;
    anti["namespaceSelector"] = Json::object();
    Json& paa = aff["podAntiAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"];
    if (!paa.is_array()) paa = Json::array();
    paa.push_back(anti);
}

// setNodeSelector, pod_mutating_webhook.go:137-171 (A5)
Err setNodeSelector(Cache& c, Json& pod) {
    Json leader;
    if (Err e = leaderPodForFollower(c, pod, &leader); !e.ok) return Err::none();  // validation webhook rejects
    if (node_name(leader).empty()) return Err::none();
    const Json& ann = annotations(pod);
    if (!has_key(ann, kExclusiveKey)) return Err::e(std::string("pod missing annotation: ") + kExclusiveKey);
    const std::string key = str_at(ann, kExclusiveKey);
    std::string value;
    if (Err e = topologyFromPod(c, leader, key, &value); !e.ok) return e;
    Json& ns = pod["spec"]["nodeSelector"];
    if (!ns.is_object()) ns = Json::object();
    ns[key] = value;
    return Err::none();
}

// Default, pod_mutating_webhook.go:64-93
Err Default(Cache& c, Json& pod) {
    const Json& ann = annotations(pod);
    if (!has_key(ann, kExclusiveKey) || has_key(ann, kNodeSelectorStrategyKey)) return Err::none();
    if (str_at(ann, kJobCompletionIndexAnnotation) == "0") {
        setExclusiveAffinities(pod);
        return Err::none();
    }
    return setNodeSelector(c, pod);
}

// Default over a batch of pods -- every pod of a JobSet's (re)created Jobs as
// the Job controller creates them: per pod exactly
// Default's result and error, but the followers whose leader node the engine
// holds at a level key are resolved by ONE jsp_resolve_leader_domains call.
Json DefaultBatch(Cache& c, const Json& pods) {
    struct Pending {
        size_t i;
        int32_t row;
        uint32_t level;
        std::string key;
    };
    std::vector<Pending> pend;
    std::vector<Json> res;
    std::vector<Err> errs;
    for (size_t i = 0; i < pods.size(); ++i) {
        Json pod = pods.at(i);
        Err e = Err::none();
        const Json& ann = annotations(pod);
        if (has_key(ann, kExclusiveKey) && !has_key(ann, kNodeSelectorStrategyKey)) {
            if (str_at(ann, kJobCompletionIndexAnnotation) == "0") {
                setExclusiveAffinities(pod);
            } else {
                // setNodeSelector's order: leader lookup, leader bound, then the topology value
                Json leader;
                if (leaderPodForFollower(c, pod, &leader).ok && !node_name(leader).empty()) {
                    const std::string key = str_at(ann, kExclusiveKey);
                    int32_t row = -1;
                    uint32_t level = 0;
                    if (engineTopology(c, node_name(leader), key, &row, &level)) {
                        pend.push_back({i, row, level, key});
                    } else {
                        std::string value;
                        e = topologyFromPod(c, leader, key, &value);
                        if (e.ok) {
                            Json& ns = pod["spec"]["nodeSelector"];
                            if (!ns.is_object()) ns = Json::object();
                            ns[key] = value;
                        }
                    }
                }
            }
        }
        res.push_back(std::move(pod));
        errs.push_back(e);
    }
    if (!pend.empty()) {
        std::vector<int32_t> rows, doms(pend.size(), -1);
        std::vector<uint32_t> levels;
        for (const auto& p : pend) {
            rows.push_back(p.row);
            levels.push_back(p.level);
        }
        ++c.engine_calls;
        const bool ok = jsp_resolve_leader_domains(c.eng, rows.data(), levels.data(), (uint32_t)rows.size(),
                                                   doms.data()) == JSP_OK;
        const std::string msg = ok ? "" : std::string("placement engine: ") + jsp_last_error();
        for (size_t k = 0; k < pend.size(); ++k) {
            if (!ok) {
                errs[pend[k].i] = Err::e(msg);
                continue;
            }
            Json& ns = res[pend[k].i]["spec"]["nodeSelector"];
            if (!ns.is_object()) ns = Json::object();
            ns[pend[k].key] = domainValue(c, pend[k].level, doms[k]);
        }
    }
    Json out = Json::array();
    for (size_t i = 0; i < res.size(); ++i) {
        Json x = Json::object();
        x["pod"] = res[i];
        x["error"] = errs[i].ok ? Json() : Json(errs[i].msg);
        out.push_back(x);
    }
    return out;
}

// leaderPodScheduled, pod_admission_webhook.go:78-89
Err leaderPodScheduled(Cache& c, const Json& pod, bool* scheduled) {
    Json leader;
    if (Err e = leaderPodForFollower(c, pod, &leader); !e.ok) return e;
    *scheduled = !node_name(leader).empty();
    return Err::none();
}

// ValidateCreate, pod_admission_webhook.go:24-67 (A6)
Err ValidateCreate(Cache& c, const Json& pod) {
    const Json& ann = annotations(pod);
    if (!has_key(ann, kJobSetNameKey)) return Err::none();
    if (has_key(ann, kNodeSelectorStrategyKey)) return Err::none();
    if (!has_key(ann, kExclusiveKey)) return Err::none();
    const std::string key = str_at(ann, kExclusiveKey);
    if (IsLeaderPod(pod)) return Err::none();
    const Json& ns = pod.get("spec").get("nodeSelector");
    if (!ns.is_object()) return Err::e("follower pod node selector not set");
    if (!ns.has(key))
        return Err::e("follower pod node selector for topology domain not found. missing selector: " + key);
    bool scheduled = false;
    if (Err e = leaderPodScheduled(c, pod, &scheduled); !e.ok) return e;
    if (!scheduled)
        return Err::e("leader pod not yet scheduled, not creating follower pod. this is an expected, transient error");
    return Err::none();
}

// ============================================================ PodReconciler
// validatePodPlacements, pod_controller.go:172-194 (A9). With an engine
// holding the leader's node at the key's level, the whole job is checked by
// one jsp_audit_placements call (followers' selector values as domain ids
// against the leader's row); only when it reports a mismatch are the
// followers walked on the host, to return the reference's first error.
Err validatePodPlacements(Cache& c, const Json& leader, const Json& podList, bool* valid) {
    *valid = false;
    const std::string key = str_at(annotations(leader), kExclusiveKey);
    int32_t row = -1;
    uint32_t level = 0;
    if (c.planner && engineTopology(c, node_name(leader), key, &row, &level)) {
        std::vector<int32_t> fdom;
        bool selector_error = false;
        for (const auto& pod : podList.elems()) {
            if (IsLeaderPod(pod)) continue;
            std::string ft;
            if (!followerPodTopology(pod, key, &ft).ok) {
                selector_error = true;
                break;
            }
            const int32_t d = c.planner->domain_id((int)level, ft);
            fdom.push_back(d < 0 ? -2 : d);  // a value no domain has never matches
        }
        if (!selector_error) {
            const uint32_t off[2] = {0, (uint32_t)fdom.size()};
            uint32_t bad = 0;
            ++c.engine_calls;
            if (jsp_audit_placements(c.eng, &row, &level, off, fdom.empty() ? nullptr : fdom.data(), 1, &bad) != JSP_OK)
                return Err::e(std::string("placement engine: ") + jsp_last_error());
            if (bad == 0) {
                *valid = true;
                return Err::none();
            }
        }
        // the reference's walk, for its first error (leader value from the snapshot)
        const std::string lt = domainValue(c, level, c.planner->row_domain((uint32_t)row, (int)level));
        for (const auto& pod : podList.elems()) {
            if (IsLeaderPod(pod)) continue;
            std::string ft;
            if (Err e = followerPodTopology(pod, key, &ft); !e.ok) return e;
            if (ft != lt) return Err::e("follower topology " + go_quote(ft) + " != leader topology " + go_quote(lt));
        }
        *valid = true;
        return Err::none();
    }
    std::string lt;
    if (Err e = topologyFromPod(c, leader, key, &lt); !e.ok) return e;
    for (const auto& pod : podList.elems()) {
        if (IsLeaderPod(pod)) continue;
        std::string ft;
        if (Err e = followerPodTopology(pod, key, &ft); !e.ok) return e;
        if (ft != lt) return Err::e("follower topology " + go_quote(ft) + " != leader topology " + go_quote(lt));
    }
    *valid = true;
    return Err::none();
}

// deleteFollowerPods, pod_controller.go:197-237 (sequential; deterministic order)
Err deleteFollowerPods(Cache& c, const Json& pods, const std::string& now) {
    std::vector<std::string> errs;
    for (auto pod : pods.elems()) {
        if (IsLeaderPod(pod)) continue;
        Json cond = Json::object();
        cond["type"] = "DisruptionTarget";
        cond["status"] = "True";
        cond["reason"] = kExclusivePlacementViolationReason;
        cond["message"] = kExclusivePlacementViolationMessage;
        cond["lastTransitionTime"] = now;
        if (updatePodCondition(pod, cond)) {
            if (Err e = injected(c, "update/Pod"); !e.ok) {
                errs.push_back(e.msg);
                continue;
            }
            c.status_updates.push_back(name_of(pod));
            auto it = c.pods.find(ns_of(pod) + "/" + name_of(pod));
            if (it != c.pods.end()) it->second = pod;
        }
        if (Err e = injected(c, "delete/Pod"); !e.ok) {
            errs.push_back(e.msg);
            continue;
        }
        c.pods.erase(ns_of(pod) + "/" + name_of(pod));  // absent pods are NotFound: ignored
        c.deleted.push_back(name_of(pod));
    }
    return errs.empty() ? Err::none() : Err::e(errors_join(errs));
}

// Reconcile, pod_controller.go:115-157. The reference returns on the
// validation error before its `!valid` branch (:148-155), so a mismatch is an
// error + requeue, never a deletion; kept as is.
Err Reconcile(Cache& c, const std::string& ns, const std::string& name, const std::string& now) {
    Json leader;
    if (Err e = getPod(c, ns, name, &leader); !e.ok) return e.not_found ? Err::none() : e;
    if (!has_key(labels(leader), kJobKey))
        return Err::e("job key label not found on leader pod: " + go_quote(name_of(leader)));
    Json list;
    if (Err e = listPods(c, ns_of(leader), kPodJobKey, str_at(labels(leader), kJobKey), &list); !e.ok) return e;
    bool valid = false;
    if (Err e = validatePodPlacements(c, leader, list, &valid); !e.ok) return e;
    if (!valid) return deleteFollowerPods(c, list, now);
    return Err::none();
}

// ============================================================ engine placement (A10, §8f rows 1 and 4)
// Plan child Jobs through the engine: one requirement class per
// (replicatedJob, exclusive-topology key), runs in the jobs' order (the order
// constructJobsFromTemplate produces them: globalJobIndex), the snapshot
// re-synced from this cache's Node / Pod objects first. Jobs without the
// exclusive annotation, or with the node-selector strategy, are not placed by
// the engine (the reference's webhooks skip them too, pod_mutating_webhook.go:72-76).
Json classesJson(const Planner& pl, const std::vector<ClassSpec>& classes) {
    std::vector<jsp_job_class> jc;
    pl.encode(classes, &jc);
    Json out = Json::array();
    for (size_t i = 0; i < classes.size(); ++i) {
        const jsp_job_class& x = jc[i];
        Json o = Json::object(), req = Json::array(), fb = Json::array(), res = Json::array();
        for (int w = 0; w < JSP_MAX_LABEL_WORDS; ++w) {
            char a[24], b[24];
            std::snprintf(a, sizeof a, "%016llx", (unsigned long long)x.req_labels[w]);
            std::snprintf(b, sizeof b, "%016llx", (unsigned long long)x.forbid_labels[w]);
            req.push_back(std::string(a));
            fb.push_back(std::string(b));
        }
        for (int r = 0; r < JSP_MAX_RES; ++r) res.push_back((int64_t)x.req_res[r]);
        o["reqLabels"] = req;
        o["forbidLabels"] = fb;
        o["toleratedTaints"] = (int64_t)x.tolerated_taints;
        o["level"] = (int64_t)x.level;
        o["pods"] = (int64_t)x.pods;
        o["reqRes"] = res;
        out.push_back(o);
    }
    return out;
}

// The requirement classes of `jobs` and each placed job's class index.
Err jobClasses(Planner& pl, const Json& jobs, std::vector<ClassSpec>* classes, std::vector<uint32_t>* job_class,
               std::vector<std::string>* names, std::vector<std::string>* keys) {
    std::map<std::string, uint32_t> class_of_rj;
    for (const auto& job : jobs.elems()) {
        const Json& ann = annotations(job);
        if (!has_key(ann, kExclusiveKey) || has_key(ann, kNodeSelectorStrategyKey)) continue;
        const std::string key = str_at(ann, kExclusiveKey);
        const std::string ck = str_at(labels(job), kReplicatedJobNameKey) + "\n" + key;
        auto it = class_of_rj.find(ck);
        uint32_t ci = 0;
        if (it == class_of_rj.end()) {
            ClassSpec cs;
            const Json& js = job.get("spec");
            const int64_t par = js.has("parallelism") ? js.get("parallelism").as_int() : 1;
            if (Err2 e = pl.class_of(js.get("template"), par, key, &cs); !e.ok()) return Err::e(e.msg);
            ci = (uint32_t)classes->size();
            classes->push_back(std::move(cs));
            class_of_rj[ck] = ci;
        } else {
            ci = it->second;
        }
        job_class->push_back(ci);
        names->push_back(name_of(job));
        keys->push_back(key);
    }
    if (classes->size() > JSP_MAX_CLASSES) return Err::e("placement planner: more than 64 requirement classes");
    return Err::none();
}

Err planJobs(Cache& c, const Json& jobs, Json* out) {
    if (!c.planner) return Err::e("no placement planner bound to this cache");
    Planner& pl = *c.planner;
    std::vector<ClassSpec> classes;
    std::vector<uint32_t> job_class;
    std::vector<std::string> names, keys;
    if (Err e = jobClasses(pl, jobs, &classes, &job_class, &names, &keys); !e.ok) return e;
    Json stats;
    if (Err2 e = pl.sync(c.nodes, c.pods, &stats); !e.ok()) return Err::e(e.msg);
    std::vector<uint32_t> rc, rl;
    for (uint32_t ci : job_class) {
        if (rc.empty() || rc.back() != ci) {
            rc.push_back(ci);
            rl.push_back(0);
        }
        ++rl.back();
    }
    std::vector<int32_t> assign;
    jsp_stats st{};
    ++c.engine_calls;
    if (Err2 e = pl.place(classes, rc, rl, &assign, &st); !e.ok()) return Err::e(e.msg);
    Json r = Json::object(), js = Json::array(), un = Json::array();
    for (size_t j = 0; j < names.size(); ++j) {
        Json x = Json::object();
        x["name"] = names[j];
        x["topologyKey"] = keys[j];
        x["domainId"] = (int64_t)assign[j];
        if (assign[j] >= 0) {
            x["domain"] = pl.domain_values(pl.level_of(keys[j]))[assign[j]];
        } else {
            x["domain"] = Json();
            un.push_back(names[j]);
        }
        js.push_back(x);
    }
    r["jobs"] = js;
    r["unplaceable"] = un;
    r["placed"] = (int64_t)st.placed;
    r["snapshot"] = stats;
    r["classes"] = classesJson(pl, classes);
    Json jcj = Json::array();
    for (uint32_t ci : job_class) jcj.push_back((int64_t)ci);
    r["jobClass"] = jcj;
    *out = r;
    return Err::none();
}

// The recreate path consulting the engine (A10): the reconcile step after
// failurePolicyRecreateAll bumped status.restarts (failure_policy.go:155-175).
// getChildJobs buckets the old attempt into `delete` (jobset_controller.go:
// 281-290); while any is listed nothing is created (shouldCreateJob, :698-709,
// and the Foreground deletion, :553-576). Once they are gone, every
// replicatedJob's Jobs are constructed (constructJobsFromTemplate, :638-649,
// unchanged) and placed by the engine on the post-delete snapshot. The plan is
// reported beside the Jobs; the Jobs and the pods' mutations are not changed.
Err reconcileRecreate(Cache& c, const Json& js, const Json& jobs, Json* out) {
    Json owned;
    if (Err e = getChildJobs(js, jobs, &owned); !e.ok) return e;
    Json r = Json::object(), del = Json::array(), create = Json::array();
    for (const auto& j : owned.get("delete").elems()) del.push_back(name_of(j));
    if (owned.get("delete").size() == 0)
        for (const auto& rj : js.get("spec").get("replicatedJobs").elems()) {
            const Json made = constructJobsFromTemplate(js, rj, owned);  // outlives the loop below
            for (const auto& j : made.elems()) create.push_back(j);
        }
    r["delete"] = del;
    r["create"] = create;
    r["plan"] = Json();
    if (create.size() > 0 && c.planner) {
        Json plan;
        if (Err e = planJobs(c, create, &plan); !e.ok) r["planError"] = e.msg;
        else r["plan"] = plan;
    }
    *out = r;
    return Err::none();
}

// ============================================================ node-selector strategy
// generate_namespaced_jobs, hack/label_nodes/label_nodes.py:99-112
Json generateNamespacedJobs(const Json& js) {
    const std::string ns = ns_of(js).empty() ? "default" : ns_of(js);
    Json out = Json::array();
    for (const auto& rj : js.get("spec").get("replicatedJobs").elems()) {
        const int64_t n = rj.has("replicas") ? rj.get("replicas").as_int() : 1;
        for (int64_t i = 0; i < n; ++i)
            out.push_back(ns + "_" + name_of(js) + "-" + rj.get("name").as_string() + "-" + std::to_string(i));
    }
    return out;
}

// Deterministic replacement for label_nodes.py (hack/label_nodes/
// label_nodes.py:36-120; its job -> node-pool map iterates a Python set,
// :115-120): the JobSet's jobs (generate_namespaced_jobs order) are placed on
// the exclusive-topology key's domains by the engine's lowest-index rule, and
// every node of a job's domain gets the script's patch body (:65-80).
Err labelNodes(Cache& c, const Json& js, Json* out) {
    if (!c.planner) return Err::e("no placement planner bound to this cache");
    Planner& pl = *c.planner;
    const Json ns_jobs = generateNamespacedJobs(js);
    std::vector<ClassSpec> classes;
    std::vector<uint32_t> rc, rl;
    std::string key;
    for (const auto& rj : js.get("spec").get("replicatedJobs").elems()) {
        std::string k = "cloud.google.com/gke-nodepool";  // label_nodes.py:33 NODE_POOL_KEY
        if (has_key(annotations(js), kExclusiveKey)) k = str_at(annotations(js), kExclusiveKey);
        const Json& rja = rj.get("template").get("metadata").get("annotations");
        if (has_key(rja, kExclusiveKey)) k = str_at(rja, kExclusiveKey);
        if (!key.empty() && k != key) return Err::e("label nodes: replicated jobs use different topology keys");
        key = k;
        const Json& jspec = rj.get("template").get("spec");
        ClassSpec cs;
        const int64_t par = jspec.has("parallelism") ? jspec.get("parallelism").as_int() : 1;
        if (Err2 e = pl.class_of(jspec.get("template"), par, key, &cs); !e.ok()) return Err::e(e.msg);
        rc.push_back((uint32_t)classes.size());
        rl.push_back((uint32_t)(rj.has("replicas") ? rj.get("replicas").as_int() : 1));
        classes.push_back(std::move(cs));
    }
    if (classes.size() > JSP_MAX_CLASSES) return Err::e("label nodes: more than 64 replicated jobs");
    Json stats;
    if (Err2 e = pl.sync(c.nodes, c.pods, &stats); !e.ok()) return Err::e(e.msg);
    std::vector<int32_t> assign;
    jsp_stats st{};
    ++c.engine_calls;
    if (Err2 e = pl.place(classes, rc, rl, &assign, &st); !e.ok()) return Err::e(e.msg);
    std::vector<std::string> names;
    for (const auto& n : ns_jobs.elems()) names.push_back(n.as_string());
    const int level = pl.level_of(key);
    Json mapping = Json::object(), un = Json::array();
    for (size_t j = 0; j < names.size() && j < assign.size(); ++j) {
        if (assign[j] >= 0) mapping[names[j]] = pl.domain_values(level)[assign[j]];
        else un.push_back(names[j]);
    }
    Json r = Json::object();
    r["mapping"] = mapping;
    r["unplaceable"] = un;
    r["patches"] = label_nodes(pl, level, names, assign);
    *out = r;
    return Err::none();
}

// ============================================================ registry of caches
std::mutex g_mu;
std::map<int64_t, std::unique_ptr<Cache>> g_caches;
int64_t g_next = 1;

Cache* cache_of(const Json& req) {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_caches.find(req.get("cache").as_int());
    if (it == g_caches.end()) throw std::runtime_error("unknown cache handle");
    return it->second.get();
}

Json ok(Json v) {
    Json r = Json::object();
    r["result"] = std::move(v);
    return r;
}
Json err_json(const Err& e, Json v = Json()) {
    Json r = Json::object();
    r["result"] = std::move(v);
    if (!e.ok) r["error"] = e.msg;
    return r;
}

Json dispatch(const std::string& m, const Json& q) {
    // ---- stateless
    if (m == "placement.GenJobName") return ok(GenJobName(q.get("jsName").as_string(), q.get("rjobName").as_string(), q.get("jobIndex").as_int()));
    if (m == "placement.GenPodName")
        return ok(GenPodName(q.get("jobSet").as_string(), q.get("replicatedJob").as_string(), q.get("jobIndex").as_string(),
                             q.get("podIndex").as_string()));
    if (m == "placement.IsLeaderPod") return ok(IsLeaderPod(q.get("pod")));
    if (m == "controllers.sha1Hash") return ok(sha1Hash(q.get("s").as_string()));
    if (m == "controllers.jobHashKey") return ok(jobHashKey(q.get("ns").as_string(), q.get("jobName").as_string()));
    if (m == "controllers.namespacedJobName") return ok(namespacedJobName(q.get("ns").as_string(), q.get("jobName").as_string()));
    if (m == "controllers.globalJobIndex")
        return ok(globalJobIndex(q.get("jobSet"), q.get("replicatedJob").as_string(), q.get("jobIdx").as_int()));
    if (m == "controllers.removePodNameSuffix") {
        std::string out;
        Err e = removePodNameSuffix(q.get("podName").as_string(), &out);
        return err_json(e, out);
    }
    if (m == "controllers.labelAndAnnotateObject") {
        Json obj = q.get("obj");
        Json md = obj.get("metadata").is_object() ? obj.get("metadata") : Json::object();
        labelAndAnnotateObject(md, q.get("jobSet"), q.get("replicatedJob"), q.get("jobIdx").as_int());
        obj["metadata"] = md;
        return ok(obj);
    }
    if (m == "controllers.constructJob") return ok(constructJob(q.get("jobSet"), q.get("replicatedJob"), q.get("jobIdx").as_int()));
    if (m == "controllers.constructJobsFromTemplate")
        return ok(constructJobsFromTemplate(q.get("jobSet"), q.get("replicatedJob"), q.get("ownedJobs")));
    if (m == "controllers.shouldCreateJob") return ok(shouldCreateJob(q.get("jobName").as_string(), q.get("ownedJobs")));
    if (m == "controllers.getChildJobs") {
        Json out;
        Err e = getChildJobs(q.get("jobSet"), q.get("jobs"), &out);
        return err_json(e, out);
    }
    if (m == "controllers.failurePolicyRecreateAll") {
        Json js = q.get("jobSet");
        failurePolicyRecreateAll(js, q.get("shouldCountTowardsMax").as_bool());
        return ok(js);
    }
    if (m == "controllers.followerPodTopology") {
        std::string out;
        Err e = followerPodTopology(q.get("pod"), q.get("topologyKey").as_string(), &out);
        return err_json(e, out);
    }
    if (m == "controllers.updatePodCondition") {
        Json pod = q.get("pod");
        const bool changed = updatePodCondition(pod, q.get("condition"));
        Json r = Json::object();
        r["changed"] = changed;
        r["pod"] = pod;
        return ok(r);
    }
    if (m == "controllers.podIndexes") {
        Json r = Json::object();
        r[kPodNameKey] = Json::array();
        r[kPodJobKey] = Json::array();
        for (const auto& v : podNameIndex(q.get("pod"))) r[kPodNameKey].push_back(v);
        for (const auto& v : podJobKeyIndex(q.get("pod"))) r[kPodJobKey].push_back(v);
        return ok(r);
    }
    if (m == "controllers.podPredicate") {  // SetupWithManager event filter, pod_controller.go:66-71
        const Json& p = q.get("pod");
        return ok(IsLeaderPod(p) && podScheduled(p) && usingExclusivePlacement(p) && !podDeleted(p));
    }
    if (m == "webhooks.genLeaderPodName") {
        std::string out;
        Err e = genLeaderPodName(q.get("pod"), &out);
        return err_json(e, out);
    }
    if (m == "webhooks.podsOwnedBySameJob") return err_json(podsOwnedBySameJob(q.get("leaderPod"), q.get("followerPod")));
    if (m == "webhooks.setExclusiveAffinities") {
        Json pod = q.get("pod");
        setExclusiveAffinities(pod);
        return ok(pod);
    }
    if (m == "hack.generateNamespacedJobs") return ok(generateNamespacedJobs(q.get("jobSet")));
    // ---- caches
    if (m == "cache.new") {
        std::lock_guard<std::mutex> g(g_mu);
        const int64_t id = g_next++;
        g_caches[id] = std::make_unique<Cache>();
        return ok(id);
    }
    if (m == "cache.free") {
        std::lock_guard<std::mutex> g(g_mu);
        g_caches.erase(q.get("cache").as_int());
        return ok(true);
    }
    Cache& c = *cache_of(q);
    std::lock_guard<std::mutex> g(c.mu);
    if (m == "cache.add") {  // watch Added / Modified
        const Json& o = q.get("object");
        if (q.get("kind").as_string() == "Node") {
            c.nodes[name_of(o)] = o;
            if (c.planner) c.planner->note_node_event();  // its labels may have moved it to another domain
        } else {
            c.pods[ns_of(o) + "/" + name_of(o)] = o;
        }
        return ok(true);
    }
    if (m == "cache.remove") {  // watch Deleted
        if (q.get("kind").as_string() == "Node") {
            c.nodes.erase(q.get("name").as_string());
            if (c.planner) c.planner->note_node_event();  // a Node Get now answers NotFound -> ""
        } else {
            c.pods.erase(q.get("namespace").as_string() + "/" + q.get("name").as_string());
        }
        return ok(true);
    }
    if (m == "planner.new") {
        std::vector<std::string> lk, res;
        for (const auto& k : q.get("levelKeys").elems()) lk.push_back(k.as_string());
        for (const auto& r : q.get("resources").elems()) res.push_back(r.as_string());
        c.eng = reinterpret_cast<jsp_engine*>((uintptr_t)q.get("engine").as_int());
        c.planner = std::make_unique<Planner>(c.eng, lk, res);
        return ok(true);
    }
    if (m == "planner.sync" || m == "planner.columns") {
        if (!c.planner) return err_json(Err::e("no placement planner bound to this cache"));
        Json stats;
        if (Err2 e = c.planner->sync(c.nodes, c.pods, &stats); !e.ok()) return err_json(Err::e(e.msg));
        return ok(m == "planner.sync" ? stats : c.planner->columns());
    }
    if (m == "planner.encode") {  // classes of `jobs` without placing (tests, oracle inputs)
        if (!c.planner) return err_json(Err::e("no placement planner bound to this cache"));
        std::vector<ClassSpec> classes;
        std::vector<uint32_t> job_class;
        std::vector<std::string> names, keys;
        if (Err e = jobClasses(*c.planner, q.get("jobs"), &classes, &job_class, &names, &keys); !e.ok) return err_json(e);
        Json stats;
        if (Err2 e = c.planner->sync(c.nodes, c.pods, &stats); !e.ok()) return err_json(Err::e(e.msg));
        Json r = Json::object();
        r["classes"] = classesJson(*c.planner, classes);
        Json jcj = Json::array();
        for (uint32_t ci : job_class) jcj.push_back((int64_t)ci);
        r["jobClass"] = jcj;
        return ok(r);
    }
    if (m == "planner.plan") {
        Json out;
        Err e = planJobs(c, q.get("jobs"), &out);
        return err_json(e, out);
    }
    if (m == "controllers.reconcileRecreate") {
        Json out;
        Err e = reconcileRecreate(c, q.get("jobSet"), q.get("jobs"), &out);
        return err_json(e, out);
    }
    if (m == "hack.labelNodes") {
        Json out;
        Err e = labelNodes(c, q.get("jobSet"), &out);
        return err_json(e, out);
    }
    if (m == "webhooks.DefaultBatch") return ok(DefaultBatch(c, q.get("pods")));
    if (m == "cache.inject") {
        if (q.get("error").is_null()) c.inject.erase(q.get("what").as_string());
        else c.inject[q.get("what").as_string()] = q.get("error").as_string();
        return ok(true);
    }
    if (m == "cache.stats") {
        Json r = Json::object();
        r["nodeGets"] = c.node_gets;
        r["podLists"] = c.pod_lists;
        r["engineCalls"] = c.engine_calls;
        r["deleted"] = Json::array();
        for (auto& d : c.deleted) r["deleted"].push_back(d);
        r["statusUpdates"] = Json::array();
        for (auto& d : c.status_updates) r["statusUpdates"].push_back(d);
        r["pods"] = Json::array();
        for (auto& kv : c.pods) r["pods"].push_back(kv.second);
        return ok(r);
    }
    if (m == "cache.bindEngine") {
        c.eng = reinterpret_cast<jsp_engine*>((uintptr_t)q.get("engine").as_int());
        c.node_rows.clear();
        for (const auto& kv : q.get("nodeRows").items()) c.node_rows[kv.first] = (int32_t)kv.second.as_int();
        c.level_keys.clear();
        for (const auto& k : q.get("levelKeys").elems()) c.level_keys.push_back(k.as_string());
        c.domain_values.clear();
        for (const auto& lv : q.get("domainValues").elems()) {
            std::vector<std::string> v;
            for (const auto& x : lv.elems()) v.push_back(x.as_string());
            c.domain_values.push_back(std::move(v));
        }
        return ok(true);
    }
    if (m == "webhooks.Default") {
        Json pod = q.get("pod");
        Err e = Default(c, pod);
        return err_json(e, pod);
    }
    if (m == "webhooks.ValidateCreate") return err_json(ValidateCreate(c, q.get("pod")));
    if (m == "webhooks.leaderPodForFollower") {
        Json leader;
        Err e = leaderPodForFollower(c, q.get("pod"), &leader);
        return err_json(e, leader);
    }
    if (m == "controllers.validatePodPlacements") {
        bool valid = false;
        Err e = validatePodPlacements(c, q.get("leaderPod"), q.get("podList"), &valid);
        return err_json(e, valid);
    }
    if (m == "controllers.deleteFollowerPods")
        return err_json(deleteFollowerPods(c, q.get("pods"), q.get("now").as_string()));
    if (m == "controllers.Reconcile")
        return err_json(Reconcile(c, q.get("namespace").as_string(), q.get("name").as_string(), q.get("now").as_string()));
    throw std::runtime_error("unknown method " + m);
}

}  // namespace jsk

extern "C" int jsk_call(const char* method, const char* request_json, char** response_json) {
    if (!method || !response_json) return JSP_EINVAL;
    std::string out;
    int rc = JSP_OK;
    try {
        const jsk::Json q = jsk::Json::parse(request_json ? request_json : "{}");
        out = jsk::dispatch(method, q).dump();
    } catch (const std::exception& ex) {
        jsk::Json r = jsk::Json::object();
        r["error"] = std::string("jsk_call: ") + ex.what();
        out = r.dump();
        rc = JSP_EINVAL;
    }
    char* p = static_cast<char*>(std::malloc(out.size() + 1));
    if (!p) return JSP_ENOMEM;
    std::memcpy(p, out.c_str(), out.size() + 1);
    *response_json = p;
    return rc;
}

extern "C" void jsk_free(char* p) { std::free(p); }
