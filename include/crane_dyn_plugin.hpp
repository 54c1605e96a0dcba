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
// call).  A node's Filter and Score depend on `now` only through its expiries, so
// the engine returns every node's answers as step functions of time over a horizon
// (crane_dyn_node_steps: int8 first-fail and score per piece, computed by the
// engine's kernels); a pod's per-node calls are then lookups at its `now` — no
// device call per pod, a new table only when a pod's time leaves the horizon or the
// snapshot generation changes.
//
// Threading: the framework calls Filter/Score for one pod from 16 goroutines.
// The first call of a cycle fetches the table under std::call_once; every call
// after that reads the immutable table (and the immutable node -> index maps of
// the snapshot generation it was built from) without taking a lock.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <algorithm>
#include <cstdlib>
#include <cstring>
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
    // the Filter's "Load[%s] of node[%s] is too high", formatted when read: a cycle's tens of
    // thousands of Unschedulable answers are rarely read and need no allocation each
    static Status Overloaded(const char* metric, const std::string* node) {
        Status s(Code::Unschedulable, std::string());
        s.metric_ = metric;
        s.node_ = node;
        return s;
    }
    Code code() const { return code_; }
    std::string message() const {
        if (!metric_) return msg_;
        return "Load[" + std::string(metric_) + "] of node[" + *node_ + "] is too high";
    }
    bool IsSuccess() const { return code_ == Code::Success; }

   private:
    Code code_ = Code::Success;
    std::string msg_;
    const char* metric_ = nullptr;     // (Overloaded: the policy's predicate name, lives with the plugin)
    const std::string* node_ = nullptr;  // (the snapshot's node name, lives with the snapshot)
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
// The Dynamic plugin's answer table of the cycle lives here (as plugins keep cycle
// data in the framework's CycleState); Clone() (preemption dry runs) shares it.
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

// FNV-1a over a node name (names are short; std::hash's murmur costs more per call)
struct NameHash {
    size_t operator()(const std::string& s) const {
        uint64_t h = 1469598103934665603ull;
        for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
        return (size_t)h;
    }
};

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
        const Table* t;
        int64_t idx;
        std::string err;
        if (!table_for(state, node, &t, &idx, &err)) return NewStatus(Code::Error, err);
        const int k = t->first_fail[t->piece(idx, state.now_ns)];
        if (k >= 0) return Status::Overloaded(policy().pred_name[k], &node->Name);  // plugins.go:64
        return Status();
    }

    // Score (plugins.go:73-98).  The node is looked up in the synced generation's index, which
    // is the snapshot's node set; only a name outside it goes to the snapshot's own Get, for
    // the reference's error (plugins.go:74-77).
    std::pair<int64_t, Status> Score(CycleState& state, const Pod& pod, const std::string& nodeName) {
        (void)pod;
        std::string err;
        const Table* t = table_of(state, &err);
        const int64_t idx = t ? t->snap->find_name(nodeName) : -1;
        if (idx < 0) {
            const Node* node = handle_.snapshot ? handle_.snapshot->Get(nodeName, &err) : nullptr;
            if (!err.empty() || !handle_.snapshot)
                return {0, NewStatus(Code::Error, "getting node \"" + nodeName + "\" from Snapshot: " + err)};
            if (!node) return {0, NewStatus(Code::Error, "node not found")};
            if (!t) return {0, NewStatus(Code::Error, err)};
            return {0, NewStatus(Code::Error, "node \"" + nodeName + "\" not in the synced snapshot")};
        }
        return {(int64_t)t->score[t->piece(idx, state.now_ns)], Status()};
    }

    // Re-parse the snapshot's annotations into the engine (once per generation).
    bool Sync(std::string* err) {
        std::lock_guard<std::mutex> g(mu_);
        return sync_locked(err) != nullptr;
    }

    // host threads of the once-per-sync annotation parse (<= 0: all hardware threads)
    void SetParseThreads(int32_t n) { parse_threads_ = n; }
    // time span one answer table covers (a pod later than it gets a new table)
    void SetHorizon(int64_t ns) { horizon_ns_ = ns > 0 ? ns : 1; }
    // answer tables built so far (one per horizon and snapshot generation)
    uint64_t TablesBuilt() const { return tables_built_.load(); }

    friend std::pair<std::unique_ptr<DynamicScheduler>, std::string> NewDynamicScheduler(const Object& plArgs,
                                                                                         const Handle& h);

   private:
    // one synced snapshot generation: node -> engine index (immutable once published).  The
    // framework hands Filter the snapshot's own Node objects and Score their Name strings, so
    // the address of a node's Name field is the key of both (a flat open-addressing table: an
    // address equal to a synced node's &Name is that node's name); a name lookup remains for
    // any other object.
    struct Synced {
        uint64_t generation;
        std::unordered_map<std::string, int64_t, NameHash> index;
        std::vector<const Node*> ptrs;                              // List() order
        std::vector<std::pair<const std::string*, int64_t>> slots;  // power-of-two size, {nullptr, -1} empty
        int shift = 64;
        static uint64_t mix(const std::string* p) { return ((uint64_t)(uintptr_t)p >> 4) * 0x9E3779B97F4A7C15ull; }
        void build(const std::vector<const Node*>& nodes) {
            ptrs = nodes;
            size_t cap = 16;
            while (cap < 2 * nodes.size()) cap <<= 1;
            shift = 64 - __builtin_ctzll(cap);
            slots.assign(cap, {nullptr, -1});
            for (size_t i = 0; i < nodes.size(); ++i) {
                const std::string* k = &nodes[i]->Name;
                size_t h = (size_t)(mix(k) >> shift);
                while (slots[h].first && slots[h].first != k) h = (h + 1) & (cap - 1);
                slots[h] = {k, (int64_t)i};
            }
        }
        int64_t find(const Node* p) const { return find_key(&p->Name); }
        int64_t find_name(const std::string& name) const { return find_key(&name); }
        // the framework walks the nodes in List() order in chunks per goroutine: the node after
        // this thread's last one (or a few further, for the feasible list) first — a pointer
        // compare, no load of the node — then the table, then the name
        int64_t find_key(const std::string* k) const {
            thread_local const Synced* last_snap = nullptr;
            thread_local int64_t last = -1;
            if (last_snap == this) {
                const int64_t n = (int64_t)ptrs.size();
                for (int64_t i = last + 1; i < std::min(n, last + 5); ++i)
                    if (&ptrs[(size_t)i]->Name == k) return last = i;
            }
            const int64_t i = find_slow(k);
            last_snap = this;
            last = i;
            return i;
        }
        int64_t find_slow(const std::string* k) const {
            size_t h = (size_t)(mix(k) >> shift);
            for (;;) {
                const auto& s = slots[h];
                if (s.first == k) return s.second;
                if (!s.first) break;
                h = (h + 1) & (slots.size() - 1);
            }
            auto it = index.find(*k);
            return it == index.end() ? -1 : it->second;
        }
    };
    // every node's answers over [t0, t1) as step functions (immutable once published)
    struct Table {
        std::shared_ptr<const Synced> snap;
        int64_t t0 = 0, t1 = 0;
        size_t S = 0;
        std::vector<uint8_t> n_steps;
        std::vector<int64_t> bp;
        std::vector<int8_t> first_fail, score;
        // index of node i's value at time t (t0 <= t < t1)
        size_t piece(int64_t i, int64_t t) const {
            const size_t nb = n_steps[(size_t)i];
            const int64_t* b = bp.data() + (size_t)i * S;
            size_t j = 0;
            while (j < nb && b[j] <= t) ++j;
            return (size_t)i * (S + 1) + j;
        }
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
        snap->build(nodes);
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
        table_.reset();
        return synced_;
    }

    // The table covering the cycle's time (fetched by the first caller of the cycle).
    const Table* table_of(CycleState& state, std::string* err) {
        std::call_once(state.dyn_once_, [&] {
            std::string e;
            std::shared_ptr<const Table> t = table_at(state.now_ns, &e);
            std::lock_guard<std::mutex> g(state.clone_mu_);
            state.dyn_row_ = t;
            state.dyn_err_ = e;
            state.dyn_done_ = true;
        });
        const Table* t = static_cast<const Table*>(state.dyn_row_.get());
        if (!t) *err = state.dyn_err_;
        return t;
    }

    // ... and the node's index in it.
    bool table_for(CycleState& state, const Node* node, const Table** table, int64_t* idx, std::string* err) {
        const Table* t = table_of(state, err);
        if (!t) return false;
        const int64_t i = t->snap->find(node);
        if (i < 0) {
            *err = "node \"" + node->Name + "\" not in the synced snapshot";
            return false;
        }
        *table = t;
        *idx = i;
        return true;
    }

    std::shared_ptr<const Table> table_at(int64_t now_ns, std::string* err) {
        std::lock_guard<std::mutex> g(mu_);  // one engine: the sync and the table build are serial
        std::shared_ptr<const Synced> snap = sync_locked(err);
        if (!snap) return nullptr;
        if (table_ && table_->snap == snap && table_->t0 <= now_ns && now_ns < table_->t1) return table_;
        auto t = std::make_shared<Table>();
        t->snap = snap;
        t->t0 = now_ns;
        t->t1 = now_ns > INT64_MAX - horizon_ns_ ? INT64_MAX : now_ns + horizon_ns_;
        t->S = (size_t)crane_dyn_step_slots(eng_);
        const size_t N = snap->index.size();
        t->n_steps.resize(N);
        t->bp.resize(N * t->S);
        t->first_fail.resize(N * (t->S + 1));
        t->score.resize(N * (t->S + 1));
        if (crane_dyn_node_steps(eng_, t->t0, t->t1, (int64_t)N, t->n_steps.data(), t->bp.data(),
                                 t->first_fail.data(), t->score.data())) {
            *err = crane_dyn_last_error(eng_);
            return nullptr;
        }
        ++tables_built_;
        table_ = t;
        return table_;
    }

    Handle handle_;
    crane_policy_doc* doc_ = nullptr;
    crane_dyn* eng_ = nullptr;
    crane_tz* zone_ = nullptr;  // the IANA zone of $TZ, or null: the fixed offset tz_
    int64_t tz_ = 8 * 3600;
    int32_t parse_threads_ = 16;  // the framework's parallelism (upstream default)
    int64_t horizon_ns_ = 60LL * 1000000000LL;
    std::atomic<uint64_t> tables_built_{0};
    std::mutex mu_;
    std::shared_ptr<const Synced> synced_;
    std::shared_ptr<const Table> table_;
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
