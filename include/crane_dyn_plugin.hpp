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
// snapshot once (Sync) and answers a pod's Filter/Score calls from one engine
// evaluation of that pod against every node, cached per scheduling cycle.
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
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
struct CycleState {
    int64_t now_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::system_clock::now().time_since_epoch())
                         .count();
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
        return {row->score[(size_t)idx], Status()};
    }

    // Re-parse the snapshot's annotations into the engine (once per generation).
    bool Sync(std::string* err) {
        std::lock_guard<std::mutex> g(mu_);
        return sync_locked(err);
    }

    friend std::pair<std::unique_ptr<DynamicScheduler>, std::string> NewDynamicScheduler(const Object& plArgs,
                                                                                         const Handle& h);

   private:
    struct Row {
        const CycleState* cycle;
        std::vector<int8_t> first_fail;
        std::vector<int64_t> score;
    };

    DynamicScheduler() = default;

    bool sync_locked(std::string* err) {
        if (!handle_.snapshot) {
            *err = "no snapshot";
            return false;
        }
        const uint64_t gen = handle_.snapshot->Generation();
        if (synced_ && gen == generation_) return true;
        const auto nodes = handle_.snapshot->List();
        const int32_t M = crane_dyn_num_metrics(eng_);
        const size_t N = nodes.size();
        std::vector<double> val((size_t)M * N, 0.0), hv(N, 0.0);
        std::vector<int64_t> ts((size_t)M * N, CRANE_TS_INVALID), hv_ts(N, CRANE_TS_INVALID);
        index_.clear();
        for (size_t n = 0; n < N; ++n) {
            index_[nodes[n]->Name] = (int64_t)n;
            const auto& a = nodes[n]->Annotations;
            for (int32_t m = 0; m < M; ++m) {
                auto it = a.find(crane_dyn_metric_name(eng_, m));
                if (it != a.end())
                    crane_parse_annotation(it->second.data(), it->second.size(), tz_, &val[(size_t)m * N + n],
                                           &ts[(size_t)m * N + n]);
            }
            auto it = a.find(NodeHotValue);
            if (it != a.end()) crane_parse_annotation(it->second.data(), it->second.size(), tz_, &hv[n], &hv_ts[n]);
        }
        if (crane_dyn_upload_nodes(eng_, (int64_t)N, 0, val.data(), ts.data(), hv.data(), hv_ts.data())) {
            *err = crane_dyn_last_error(eng_);
            return false;
        }
        generation_ = gen;
        synced_ = true;
        rows_.clear();
        return true;
    }

    bool row_for(CycleState& state, const Pod& pod, const std::string& node_name, const Row** row, int64_t* idx,
                 std::string* err) {
        std::lock_guard<std::mutex> g(mu_);
        if (!sync_locked(err)) return false;
        auto ni = index_.find(node_name);
        if (ni == index_.end()) {
            *err = "node \"" + node_name + "\" not in the synced snapshot";
            return false;
        }
        const std::string key = pod.UID.empty() ? pod.Namespace + "/" + pod.Name : pod.UID;
        auto it = rows_.find(key);
        if (it == rows_.end() || it->second.cycle != &state) {
            Row r;
            r.cycle = &state;
            const size_t N = index_.size();
            r.first_fail.assign(N, -1);
            r.score.assign(N, 0);
            const uint8_t flag = IsDaemonsetPod(pod) ? CRANE_POD_DAEMONSET : 0;
            int64_t chosen, chosen_score;
            if (crane_dyn_eval(eng_, 1, &state.now_ns, &flag, r.first_fail.data(), r.score.data(), &chosen,
                               &chosen_score)) {
                *err = crane_dyn_last_error(eng_);
                return false;
            }
            if (rows_.size() > 4096) rows_.clear();
            it = rows_.insert_or_assign(key, std::move(r)).first;
        }
        *row = &it->second;
        *idx = ni->second;
        return true;
    }

    Handle handle_;
    crane_policy_doc* doc_ = nullptr;
    crane_dyn* eng_ = nullptr;
    int64_t tz_ = 8 * 3600;
    std::mutex mu_;
    bool synced_ = false;
    uint64_t generation_ = 0;
    std::unordered_map<std::string, int64_t> index_;
    std::unordered_map<std::string, Row> rows_;
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
    if (crane_tz_offset(nullptr, &ds->tz_))  // utils.GetLocation: $TZ, default Asia/Shanghai
        return {nullptr, "unsupported time zone in $TZ"};
    if (crane_dyn_create(crane_policy_view(doc), h.device, &ds->eng_)) {
        std::string e = ds->eng_ ? crane_dyn_last_error(ds->eng_) : "engine creation failed";
        return {nullptr, "failed to create the Dynamic engine: " + e};
    }
    return {std::move(ds), ""};
}

}  // namespace dynamic
}  // namespace crane
