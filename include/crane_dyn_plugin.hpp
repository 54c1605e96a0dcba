// crane_dyn_plugin.hpp — C++ mirror of crane-scheduler's Dynamic plugin
// interface, served by the MI355X engine (crane_dyn.h).  Header-only, C++17.
//
// Mirrors (paths into /root/reference):
//   Name = "Dynamic"                                 pkg/plugins/dynamic/plugins.go:20-33
//   DynamicScheduler::Filter                          plugins.go:39-69
//   DynamicScheduler::Score                           plugins.go:73-98
//   DynamicScheduler::ScoreExtensions (nil)           plugins.go:100-102
//   NewDynamicScheduler(args, handle)                 plugins.go:105-120
//   DynamicArgs{PolicyConfigPath} + default           pkg/plugins/apis/config/types.go:10-14,
//                                                     v1beta2/defaults.go:7-12
//   IsDaemonsetPod                                    pkg/utils/utils.go:17-24
// The k8s framework types are reduced to what the plugin touches.  Instead of
// re-parsing annotations per call (stats.go:51-76), the plugin parses a node
// snapshot once per generation (Sync: one bulk, threaded crane_parse_annotations
// call) and answers a pod's Filter/Score calls from one engine evaluation of
// that pod against every node (crane_dyn_eval_compact: int8 first-fail and
// score rows), made once per scheduling cycle and kept in the CycleState.
//
// Threading: the framework calls Filter/Score for one pod from 16 goroutines.
// The first call of a cycle computes the cycle's row under std::call_once; every
// call after that reads the immutable row (and the immutable name -> index map
// of the snapshot generation it was computed against) without taking a lock.
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <cstdlib>
#include <string>
#include <thread>
#include <typeinfo>
#include <unordered_map>
#include <utility>
#include <vector>

#include "crane_dyn.h"

namespace crane {
namespace dynamic {

constexpr const char* Name = "Dynamic";
constexpr const char* NodeHotValue = "node_hot_value";  // stats.go:22
constexpr int64_t MaxNodeScore = 100, MinNodeScore = 0;  // upstream framework

// ------------------------------------------------------------ framework
enum class Code { Success = 0, Error = 1, Unschedulable = 2 };

class Status {
   public:
    Status() = default;
    Status(Code c, std::string m) : code_(c), msg_(std::move(m)) {}
    Code code() const { return code_; }
    const std::string& message() const { return msg_; }
    bool IsSuccess() const { return code_ == Code::Success; }

   private:
    Code code_ = Code::Success;
    std::string msg_;
};
inline Status NewStatus(Code c, const std::string& m) { return Status(c, m); }

struct OwnerReference {
    std::string Kind, Name;
};

struct Pod {
    std::string Namespace, Name, UID;
    std::vector<OwnerReference> OwnerReferences;
};

struct Node {
    std::string Name;
    std::map<std::string, std::string> Annotations;
};

// framework.NodeInfo: Node() may be null.
class NodeInfo {
   public:
    explicit NodeInfo(const Node* n = nullptr) : node_(n) {}
    const Node* node() const { return node_; }

   private:
    const Node* node_;
};

// One scheduling cycle of one pod (framework.CycleState).  time.Now() for the
// whole cycle (the reference calls it per Filter/Score call; declared deviation).
// The Dynamic plugin's per-cycle row lives here (as plugins keep cycle data in
// the framework's CycleState); Clone() (preemption dry runs) shares it.
struct CycleState {
    int64_t now_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::system_clock::now().time_since_epoch())
                         .count();
    CycleState() = default;
    CycleState(const CycleState&) = delete;
    CycleState& operator=(const CycleState&) = delete;
    std::unique_ptr<CycleState> Clone() const {
        std::unique_ptr<CycleState> c(new CycleState());
        c->now_ns = now_ns;
        std::lock_guard<std::mutex> g(clone_mu_);
        if (dyn_done_) {
            c->dyn_row_ = dyn_row_;
            c->dyn_err_ = dyn_err_;
            std::call_once(c->dyn_once_, [] {});
            c->dyn_done_ = true;
        }
        return c;
    }

   private:
    friend class DynamicScheduler;
    mutable std::once_flag dyn_once_;
    mutable std::mutex clone_mu_;
    bool dyn_done_ = false;
    std::shared_ptr<const void> dyn_row_;
    std::string dyn_err_;
};

// The handle's snapshot lister (SnapshotSharedLister().NodeInfos()).
class Snapshot {
   public:
    virtual ~Snapshot() = default;
    virtual std::vector<const Node*> List() const = 0;
    virtual const Node* Get(const std::string& name, std::string* err) const = 0;
    virtual uint64_t Generation() const = 0;  // changes when any node annotation changes
};

struct Handle {
    const Snapshot* snapshot = nullptr;
    int32_t device = 0;
};

// runtime.Object for plugin args
struct Object {
    virtual ~Object() = default;
};

// DynamicArgs (config/types.go:10-14) with the v1beta2 default path.
struct DynamicArgs : Object {
    std::string PolicyConfigPath = "/etc/kubernetes/dynamic-scheduler-policy.yaml";
};

// utils.IsDaemonsetPod (utils.go:17-24)
inline bool IsDaemonsetPod(const Pod& pod) {
    for (const auto& o : pod.OwnerReferences)
        if (o.Kind == "DaemonSet") return true;
    return false;
}

// ---------------------------------------------------------------- plugin
class DynamicScheduler {
   public:
    ~DynamicScheduler() {
        if (eng_) crane_dyn_destroy(eng_);
        if (doc_) crane_policy_free(doc_);
        if (zone_) crane_tz_free(zone_);
    }
    DynamicScheduler(const DynamicScheduler&) = delete;
    DynamicScheduler& operator=(const DynamicScheduler&) = delete;

    std::string name() const { return Name; }
    const void* ScoreExtensions() const { return nullptr; }
    const crane_policy& policy() const { return *crane_policy_view(doc_); }

    // Filter (plugins.go:39-69)
    Status Filter(CycleState& state, const Pod& pod, const NodeInfo& nodeInfo) {
        if (IsDaemonsetPod(pod)) return NewStatus(Code::Success, "");
        const Node* node = nodeInfo.node();
        if (!node) return NewStatus(Code::Error, "node not found");
        const Row* row;
        int64_t idx;
        std::string err;
        if (!row_for(state, pod, node->Name, &row, &idx, &err)) return NewStatus(Code::Error, err);
        const int k = row->first_fail[(size_t)idx];
        if (k >= 0)
            return NewStatus(Code::Unschedulable,
                             "Load[" + std::string(policy().pred_name[k]) + "] of node[" + node->Name + "] is too high");
        return NewStatus(Code::Success, "");
    }

    // Score (plugins.go:73-98)
    std::pair<int64_t, Status> Score(CycleState& state, const Pod& pod, const std::string& nodeName) {
        std::string err;
        const Node* node = handle_.snapshot ? handle_.snapshot->Get(nodeName, &err) : nullptr;
        if (!err.empty() || !handle_.snapshot)
            return {0, NewStatus(Code::Error, "getting node \"" + nodeName + "\" from Snapshot: " + err)};
        if (!node) return {0, NewStatus(Code::Error, "node not found")};
        const Row* row;
        int64_t idx;
        if (!row_for(state, pod, node->Name, &row, &idx, &err)) return {0, NewStatus(Code::Error, err)};
        return {(int64_t)row->score[(size_t)idx], Status()};
    }

    // Re-parse the snapshot's annotations into the engine (once per generation).
    bool Sync(std::string* err) {
        std::lock_guard<std::mutex> g(mu_);
        return sync_locked(err) != nullptr;
    }

    // host threads of the once-per-sync annotation parse (<= 0: all hardware threads)
    void SetParseThreads(int32_t n) { parse_threads_ = n; }

    friend std::pair<std::unique_ptr<DynamicScheduler>, std::string> NewDynamicScheduler(const Object& plArgs,
                                                                                         const Handle& h);

   private:
    // one synced snapshot generation: node name -> engine index (immutable once published)
    struct Synced {
        uint64_t generation;
        std::unordered_map<std::string, int64_t> index;
    };
    // one cycle's answers for every node of `snap` (immutable once published)
    struct Row {
        std::shared_ptr<const Synced> snap;
        std::vector<int8_t> first_fail;
        std::vector<int8_t> score;
    };

    DynamicScheduler() = default;

    std::shared_ptr<const Synced> sync_locked(std::string* err) {
        if (!handle_.snapshot) {
            *err = "no snapshot";
            return nullptr;
        }
        const uint64_t gen = handle_.snapshot->Generation();
        if (synced_ && synced_->generation == gen) return synced_;
        const auto nodes = handle_.snapshot->List();
        const int32_t M = crane_dyn_num_metrics(eng_);
        const size_t N = nodes.size();
        auto snap = std::make_shared<Synced>();
        snap->generation = gen;
        snap->index.reserve(N);
        // rows [metric slot 0..M-1, node_hot_value] x N of annotation strings (NULL = key missing)
        std::vector<const char*> strs((size_t)(M + 1) * N, nullptr);
        std::vector<size_t> lens((size_t)(M + 1) * N, 0);
        std::vector<std::string> keys;
        for (int32_t m = 0; m < M; ++m) keys.emplace_back(crane_dyn_metric_name(eng_, m));
        keys.emplace_back(NodeHotValue);
        for (size_t n = 0; n < N; ++n) {
            snap->index.emplace(nodes[n]->Name, (int64_t)n);
            const auto& a = nodes[n]->Annotations;
            for (int32_t m = 0; m <= M; ++m) {
                auto it = a.find(keys[(size_t)m]);
                if (it == a.end()) continue;
                strs[(size_t)m * N + n] = it->second.data();
                lens[(size_t)m * N + n] = it->second.size();
            }
        }
        std::vector<double> val((size_t)(M + 1) * N);
        std::vector<int64_t> ts((size_t)(M + 1) * N);
        const int prc = zone_ ? crane_parse_annotations_tz((int64_t)strs.size(), strs.data(), lens.data(), zone_,
                                                           val.data(), ts.data(), parse_threads_)
                              : crane_parse_annotations((int64_t)strs.size(), strs.data(), lens.data(), tz_,
                                                        val.data(), ts.data(), parse_threads_);
        if (prc) {
            *err = "annotation parse failed";
            return nullptr;
        }
        const double* hv = val.data() + (size_t)M * N;
        const int64_t* hv_ts = ts.data() + (size_t)M * N;
        if (crane_dyn_upload_nodes(eng_, (int64_t)N, 0, val.data(), ts.data(), hv, hv_ts)) {
            *err = crane_dyn_last_error(eng_);
            return nullptr;
        }
        synced_ = std::move(snap);
        return synced_;
    }

    // The cycle's row (computed by the first caller of the cycle), and the node's index in it.
    bool row_for(CycleState& state, const Pod& pod, const std::string& node_name, const Row** row, int64_t* idx,
                 std::string* err) {
        std::call_once(state.dyn_once_, [&] {
            std::string e;
            std::shared_ptr<Row> r = compute_row(state.now_ns, pod, &e);
            std::lock_guard<std::mutex> g(state.clone_mu_);
            state.dyn_row_ = r;
            state.dyn_err_ = e;
            state.dyn_done_ = true;
        });
        const Row* r = static_cast<const Row*>(state.dyn_row_.get());
        if (!r) {
            *err = state.dyn_err_;
            return false;
        }
        auto ni = r->snap->index.find(node_name);
        if (ni == r->snap->index.end()) {
            *err = "node \"" + node_name + "\" not in the synced snapshot";
            return false;
        }
        *row = r;
        *idx = ni->second;
        return true;
    }

    std::shared_ptr<Row> compute_row(int64_t now_ns, const Pod& pod, std::string* err) {
        std::lock_guard<std::mutex> g(mu_);  // one engine: the sync and the evaluation are serial
        std::shared_ptr<const Synced> snap = sync_locked(err);
        if (!snap) return nullptr;
        auto r = std::make_shared<Row>();
        r->snap = snap;
        const size_t N = snap->index.size();
        r->first_fail.assign(N, -1);
        r->score.assign(N, 0);
        const uint8_t flag = IsDaemonsetPod(pod) ? CRANE_POD_DAEMONSET : 0;
        int64_t chosen, chosen_score;
        if (crane_dyn_eval_compact(eng_, 1, &now_ns, &flag, r->first_fail.data(), r->score.data(), &chosen,
                                   &chosen_score)) {
            *err = crane_dyn_last_error(eng_);
            return nullptr;
        }
        return r;
    }

    Handle handle_;
    crane_policy_doc* doc_ = nullptr;
    crane_dyn* eng_ = nullptr;
    crane_tz* zone_ = nullptr;  // the IANA zone of $TZ, or null: the fixed offset tz_
    int64_t tz_ = 8 * 3600;
    int32_t parse_threads_ = 16;  // the framework's parallelism (upstream default)
    std::mutex mu_;
    std::shared_ptr<const Synced> synced_;
};

// NewDynamicScheduler (plugins.go:105-120): the same error strings.
inline std::pair<std::unique_ptr<DynamicScheduler>, std::string> NewDynamicScheduler(const Object& plArgs,
                                                                                     const Handle& h) {
    const auto* args = dynamic_cast<const DynamicArgs*>(&plArgs);
    if (!args)
        return {nullptr, std::string("want args to be of type DynamicArgs, got ") + typeid(plArgs).name() + "."};
    char err[512] = {0};
    crane_policy_doc* doc = nullptr;
    if (crane_policy_load_file(args->PolicyConfigPath.c_str(), &doc, err, sizeof err))
        return {nullptr, std::string("failed to get scheduler policy from config file: ") + err};
    std::unique_ptr<DynamicScheduler> ds(new DynamicScheduler());
    ds->doc_ = doc;
    ds->handle_ = h;
    // utils.GetLocation: time.LoadLocation($TZ, default Asia/Shanghai) from tzdata; without
    // tzdata files the fixed-offset zones (crane_tz_offset) still load
    const char* tzenv = std::getenv("TZ");
    const std::string zname = tzenv && *tzenv ? tzenv : "Asia/Shanghai";
    if (crane_tz_load(zname.c_str(), nullptr, &ds->zone_) && crane_tz_offset(zname.c_str(), &ds->tz_))
        return {nullptr, "unknown time zone " + zname};
    if (crane_dyn_create(crane_policy_view(doc), h.device, &ds->eng_)) {
        std::string e = ds->eng_ ? crane_dyn_last_error(ds->eng_) : "engine creation failed";
        return {nullptr, "failed to create the Dynamic engine: " + e};
    }
    return {std::move(ds), ""};
}

}  // namespace dynamic
}  // namespace crane
