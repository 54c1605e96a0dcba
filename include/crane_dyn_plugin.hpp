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
// The k8s framework types are reduced to what the plugin touches.  The reference
// re-parses a node's annotations on every call (stats.go:51-76), so it always sees
// the controller's latest patch (node.go:88-96,123-146).  Here the plugin keeps
// every node's parsed annotations in the engine and every node's answers as step
// functions of `now` over a time horizon (crane_dyn_node_steps: int8 first-fail and
// score per piece, computed by the engine's kernels); a pod's per-node calls are
// lookups at its `now`.  At the start of each scheduling cycle the plugin compares
// every NodeInfo of the snapshot with the one it parsed (its Node object, which the
// informer replaces on every update, and its Generation): only the changed nodes
// are re-parsed, scattered into the engine and their table rows rebuilt in one call
// (crane_dyn_update_node_steps).  The whole snapshot is parsed again
// only when the node set changes, and the whole table only when a pod's time leaves
// the horizon.
//
// Threading: the framework calls Filter/Score for one pod from 16 goroutines.
// The first call of a cycle brings the plugin's state up to date — the cycle's other
// first calls, which must wait for it anyway, take chunks of its snapshot scan — and
// every call after that reads it without taking a lock.  The state is patched in place
// at the start of later cycles: the framework runs scheduling cycles one at a time, and
// its binding cycles (which overlap the next scheduling cycle) call neither Filter nor
// Score, so no call reads a row while it is patched.  A CycleState kept past its cycle
// answers from the patched state.
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
    // thousands of Unschedulable answers are rarely read.  The node name is copied (a Status
    // may outlive the Node object, which the informer replaces on update); the metric name
    // points into the plugin's policy, which lives as long as the plugin.
    static Status Overloaded(const char* metric, const std::string& node) {
        Status s(Code::Unschedulable, node);
        s.metric_ = metric;
        return s;
    }
    Code code() const { return code_; }
    std::string message() const {
        if (!metric_) return msg_;
        return "Load[" + std::string(metric_) + "] of node[" + msg_ + "] is too high";
    }
    bool IsSuccess() const { return code_ == Code::Success; }

   private:
    Code code_ = Code::Success;
    std::string msg_;               // (Overloaded: the node's name)
    const char* metric_ = nullptr;  // (Overloaded: the policy's predicate name)
};
inline Status NewStatus(Code c, const std::string& m) { return Status(c, m); }

struct OwnerReference {
    std::string Kind, Name;
};

struct Pod {
    std::string Namespace, Name, UID;
    std::vector<OwnerReference> OwnerReferences;
};

// *v1.Node as the informer cache holds it: immutable once published — an update (such as the
// controller's annotation patch) publishes a new object.
struct Node {
    std::string Name;
    std::map<std::string, std::string> Annotations;
};

// framework.NodeInfo: node() may be null; the object is the snapshot's, stable for the node's
// lifetime, and its Generation changes whenever the NodeInfo does (the framework's
// nextGeneration()).
class NodeInfo {
   public:
    explicit NodeInfo(const Node* n = nullptr, int64_t generation = 0) : Generation(generation), node_(n) {}
    const Node* node() const { return node_; }
    void SetNode(const Node* n) { node_ = n; }
    int64_t Generation;

   private:
    const Node* node_;
};

// One scheduling cycle of one pod (framework.CycleState).  time.Now() for the
// whole cycle (the reference calls it per Filter/Score call; declared deviation).
// The Dynamic plugin's answers of the cycle are referenced from here (as plugins keep
// cycle data in the framework's CycleState); Clone() (preemption dry runs) shares them.
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
            c->dyn_done_ = true;
            c->dyn_phase_.store(3, std::memory_order_relaxed);
            c->dyn_ready_.store(true, std::memory_order_release);
        }
        return c;
    }

   private:
    friend class DynamicScheduler;
    mutable std::mutex clone_mu_;
    // the plugin's per-cycle sync: 0 not started, 1 the first caller brings the plugin up to
    // date, 2 its scan of the snapshot is open to the cycle's other callers (dyn_job_), 4 its
    // parse of the changed nodes' annotations is (dyn_parse_), 3 done
    std::atomic<int> dyn_phase_{0};
    std::atomic<bool> dyn_ready_{false};  // the cycle's answers are set (the lock-free fast path)
    std::shared_ptr<void> dyn_job_;       // the open scan (set before phase 2, kept until the state dies)
    std::shared_ptr<void> dyn_parse_;     // the open parse (set before phase 4, likewise)
    bool dyn_done_ = false;
    std::shared_ptr<const void> dyn_row_;
    std::string dyn_err_;
};

// The handle's snapshot lister (SnapshotSharedLister().NodeInfos()), fixed for the length of
// a scheduling cycle (the framework updates it before the cycle's first Filter).
class Snapshot {
   public:
    virtual ~Snapshot() = default;
    virtual const std::vector<const NodeInfo*>& List() const = 0;
    virtual const NodeInfo* Get(const std::string& name, std::string* err) const = 0;
};

struct Handle {
    const Snapshot* snapshot = nullptr;
    int32_t device = 0;
    // more than one: the plugin's nodes are sharded over these devices (crane_dyn_group_*: each
    // device holds a contiguous range of the synced rows; the same answers as one engine)
    std::vector<int32_t> devices;
};

// The engine the plugin keeps its nodes in: one engine, or a group of node shards over several
// devices (the same calls routed by node row, crane_dyn_group_*)
class Backend {
   public:
    ~Backend() {
        if (eng_) crane_dyn_destroy(eng_);
        if (grp_) crane_dyn_group_destroy(grp_);
    }
    int create(const crane_policy* pol, const Handle& h) {
        if (h.devices.size() > 1) {
            int rc = crane_dyn_group_create(pol, (int32_t)h.devices.size(), h.devices.data(), 1, &grp_);
            if (!rc) rc = crane_dyn_group_set_option(grp_, "collective", 0);  // (answer tables only: no batches)
            return rc;
        }
        return crane_dyn_create(pol, h.devices.size() == 1 ? h.devices[0] : h.device, &eng_);
    }
    const char* error() const {
        return grp_ ? crane_dyn_group_last_error(grp_) : eng_ ? crane_dyn_last_error(eng_) : "engine creation failed";
    }
    crane_dyn* first() const { return grp_ ? crane_dyn_group_engine(grp_, 0, 0) : eng_; }
    int32_t num_metrics() const { return crane_dyn_num_metrics(first()); }
    const char* metric_name(int32_t m) const { return crane_dyn_metric_name(first(), m); }
    int32_t step_slots() const { return crane_dyn_step_slots(first()); }
    int set_option(const char* name, int64_t v) {
        return grp_ ? crane_dyn_group_set_option(grp_, name, v) : crane_dyn_set_option(eng_, name, v);
    }
    int upload_nodes(int64_t n, const double* val, const int64_t* ts, const double* hv, const int64_t* hv_ts) {
        return grp_ ? crane_dyn_group_upload_nodes(grp_, n, val, ts, hv, hv_ts)
                    : crane_dyn_upload_nodes(eng_, n, 0, val, ts, hv, hv_ts);
    }
    int node_steps(int64_t t0, int64_t t1, int64_t n, uint8_t* ns, int64_t* bp, int8_t* ff, int8_t* sc) {
        return grp_ ? crane_dyn_group_node_steps(grp_, t0, t1, n, ns, bp, ff, sc)
                    : crane_dyn_node_steps(eng_, t0, t1, n, ns, bp, ff, sc);
    }
    int update_nodes(int64_t k, const int64_t* idx, const double* val, const int64_t* ts, const double* hv,
                     const int64_t* hv_ts) {
        return grp_ ? crane_dyn_group_update_nodes(grp_, k, idx, val, ts, hv, hv_ts)
                    : crane_dyn_update_nodes(eng_, k, idx, val, ts, hv, hv_ts);
    }
    int update_node_steps(int64_t k, const int64_t* idx, const double* val, const int64_t* ts, const double* hv,
                          const int64_t* hv_ts, int64_t t0, int64_t t1, uint8_t* ns, int64_t* bp, int8_t* ff,
                          int8_t* sc) {
        return grp_ ? crane_dyn_group_update_node_steps(grp_, k, idx, val, ts, hv, hv_ts, t0, t1, ns, bp, ff, sc)
                    : crane_dyn_update_node_steps(eng_, k, idx, val, ts, hv, hv_ts, t0, t1, ns, bp, ff, sc);
    }
    int resize_nodes(int64_t n) { return grp_ ? crane_dyn_group_resize_nodes(grp_, n) : crane_dyn_resize_nodes(eng_, n); }
    int32_t shards() const { return grp_ ? crane_dyn_group_size(grp_) : 1; }

   private:
    crane_dyn* eng_ = nullptr;
    crane_dyn_group* grp_ = nullptr;
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

// Open-addressing map from an object address to a node index (power-of-two size, linear
// probing, no deletion: a lookup is validated by the caller against the node's current
// object, so an entry left behind by a replaced object is harmless).
class AddrIndex {
   public:
    void reset(size_t n) {
        size_t cap = 16;
        while (cap < 2 * n + 16) cap <<= 1;
        shift_ = 64 - __builtin_ctzll(cap);
        slots_.assign(cap, {nullptr, -1});
        used_ = 0;
        base_ = n;
    }
    // (keeps the table at most half full itself: a caller may put more entries than it sized the
    // table for — nodes joining in one cycle — and a full table would make put / get spin)
    void put(const void* k, int64_t i) {
        if (slots_.empty()) reset(0);
        if (2 * (used_ + 1) > slots_.size()) rehash(2 * slots_.size());
        size_t h = hash(k);
        while (slots_[h].first && slots_[h].first != k) h = (h + 1) & (slots_.size() - 1);
        if (!slots_[h].first) ++used_;
        slots_[h] = {k, i};
    }
    int64_t get(const void* k) const {
        if (slots_.empty()) return -1;
        size_t h = hash(k);
        for (;;) {
            const auto& s = slots_[h];
            if (s.first == k) return s.second;
            if (!s.first) return -1;
            h = (h + 1) & (slots_.size() - 1);
        }
    }
    // stale entries (replaced or departed objects) past the node count the table was built for:
    // time to rebuild it from the live rows
    bool crowded() const { return used_ > 2 * base_ + 64; }

    size_t capacity() const { return slots_.size(); }

   private:
    void rehash(size_t cap) {
        std::vector<std::pair<const void*, int64_t>> old;
        old.swap(slots_);
        shift_ = 64 - __builtin_ctzll(cap);
        slots_.assign(cap, {nullptr, -1});
        used_ = 0;
        for (const auto& s : old)
            if (s.first) {
                size_t h = hash(s.first);
                while (slots_[h].first) h = (h + 1) & (cap - 1);
                slots_[h] = s;
                ++used_;
            }
    }
    size_t hash(const void* k) const { return (size_t)((((uint64_t)(uintptr_t)k >> 4) * 0x9E3779B97F4A7C15ull) >> shift_); }
    std::vector<std::pair<const void*, int64_t>> slots_;
    int shift_ = 64;
    size_t used_ = 0, base_ = 0;
};

// ---------------------------------------------------------------- plugin
class DynamicScheduler {
   public:
    ~DynamicScheduler() {
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
        std::string err;
        const View* v = view_of(state, &err);
        if (!v) return NewStatus(Code::Error, err);
        const int64_t i = v->find_info(&nodeInfo, node);
        if (i < 0) return NewStatus(Code::Error, "node \"" + node->Name + "\" not in the synced snapshot");
        const int k = v->first_fail[v->piece(i, state.now_ns)];
        if (k >= 0) return Status::Overloaded(policy().pred_name[k], node->Name);  // plugins.go:64
        return Status();
    }

    // Score (plugins.go:73-98).  The node is looked up in the synced node set, which is the
    // snapshot's; only a name outside it goes to the snapshot's own Get, for the reference's
    // error (plugins.go:74-77).
    std::pair<int64_t, Status> Score(CycleState& state, const Pod& pod, const std::string& nodeName) {
        (void)pod;
        std::string err;
        const View* v = view_of(state, &err);
        const int64_t i = v ? v->find_name(nodeName) : -1;
        if (i < 0) {
            const NodeInfo* ni = handle_.snapshot ? handle_.snapshot->Get(nodeName, &err) : nullptr;
            if (!err.empty() || !handle_.snapshot)
                return {0, NewStatus(Code::Error, "getting node \"" + nodeName + "\" from Snapshot: " + err)};
            if (!ni || !ni->node()) return {0, NewStatus(Code::Error, "node not found")};
            if (!v) return {0, NewStatus(Code::Error, err)};
            return {0, NewStatus(Code::Error, "node \"" + nodeName + "\" not in the synced snapshot")};
        }
        return {(int64_t)v->score[v->piece(i, state.now_ns)], Status()};
    }

    // Bring the plugin's state up to date with the snapshot now (the first Filter / Score of a
    // cycle does this itself).  Only between scheduling cycles: it patches the state the
    // cycle's lock-free Filter / Score calls read.
    bool Sync(std::string* err) {
        std::lock_guard<std::mutex> g(mu_);
        return sync_locked(std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::system_clock::now().time_since_epoch())
                               .count(),
                           err) != nullptr;
    }

    // host threads of the full-snapshot annotation parse (<= 0: all hardware threads)
    void SetParseThreads(int32_t n) { parse_threads_ = n; }
    // an engine option (crane_dyn_set_option: alternative kernel forms, tests and A/B tools)
    bool SetEngineOption(const char* name, int64_t value) { return eng_.set_option(name, value) == 0; }
    // node shards the plugin's engine spans (Handle::devices)
    int32_t Shards() const { return eng_.shards(); }
    // time span one answer table covers from the pod that builds it (a later pod gets a new
    // table); by default (and ns <= 0) the whole time axis, which never needs a new table
    void SetHorizon(int64_t ns) { horizon_ns_ = ns > 0 ? ns : kAllTime; }
    // work done so far: full tables built (the first sync, a finite horizon passed), full snapshot
    // parses, cycles that found changed or joining nodes and the rows re-parsed over them, nodes
    // that joined / left, times the shard grew (sync_ns: wall time of the cycles' syncs, scan +
    // update, as their leaders saw it)
    struct Counters {
        uint64_t tables_built = 0, full_syncs = 0, incremental_syncs = 0, nodes_updated = 0, sync_ns = 0,
                 nodes_joined = 0, nodes_left = 0, grows = 0;
        // the incremental syncs' parts: snapshot scan, joins / departures, the changed nodes'
        // parse, the engine call
        uint64_t scan_ns = 0, membership_ns = 0, parse_ns = 0, engine_ns = 0;
    };
    Counters counters() const {
        std::lock_guard<std::mutex> g(mu_);
        return cnt_;
    }
    uint64_t TablesBuilt() const { return counters().tables_built; }

    friend std::pair<std::unique_ptr<DynamicScheduler>, std::string> NewDynamicScheduler(const Object& plArgs,
                                                                                         const Handle& h);

   private:
    // The synced node set and every node's answers.  Rows are the engine's node indices: a node
    // keeps its row while it stays in the snapshot; a node that leaves frees its row (never read
    // again) and a joining node takes a free row, or the shard grows (crane_dyn_resize_nodes) —
    // the reference looks a node up per call (plugins.go:45-50,74-84), so a node set change costs
    // it nothing, and here it costs the joining nodes' rows.  The answers cover [t0, t1): by
    // default the whole time axis (every expiry of a node fits its row), so no pod time ever
    // needs a new table.
    struct View {
        std::vector<const NodeInfo*> infos;  // row -> the snapshot's NodeInfo (null: a free row)
        std::vector<const Node*> nodes;      // row -> the Node object the row was parsed from
        std::vector<std::string> names;      // ... its name (a departed node's objects may be freed)
        std::vector<int64_t> gens;           // ... and its NodeInfo's Generation
        std::vector<uint32_t> seen;          // row -> the last snapshot scan that found its NodeInfo
        std::vector<int64_t> free_rows;      // (popped from the back: lowest row first)
        size_t live = 0;
        std::unordered_map<std::string, int64_t, NameHash> by_name;
        AddrIndex info_idx;  // NodeInfo address -> row (a stale entry is rejected against infos)
        AddrIndex name_idx;  // address of a node's Name -> row (entries added as Nodes are replaced)
        int64_t t0 = 0, t1 = 0;
        size_t S = 0;
        std::vector<uint8_t> n_steps;
        std::vector<int64_t> bp;
        std::vector<int8_t> first_fail, score;

        size_t rows() const { return infos.size(); }
        void grow(size_t n) {
            infos.resize(n, nullptr);
            nodes.resize(n, nullptr);
            names.resize(n);
            gens.resize(n, 0);
            seen.resize(n, 0);
            n_steps.resize(n, 0);
            bp.resize(n * S, 0);
            first_fail.resize(n * (S + 1), 0);
            score.resize(n * (S + 1), 0);
        }
        void index_infos() {
            info_idx.reset(rows());
            for (size_t i = 0; i < rows(); ++i)
                if (infos[i]) info_idx.put(infos[i], (int64_t)i);
        }
        void index_names() {
            name_idx.reset(rows());
            for (size_t i = 0; i < rows(); ++i)
                if (infos[i] && nodes[i]) name_idx.put(&nodes[i]->Name, (int64_t)i);
        }
        // index of node i's value at time t (t0 <= t < t1)
        size_t piece(int64_t i, int64_t t) const {
            const size_t nb = n_steps[(size_t)i];
            const int64_t* b = bp.data() + (size_t)i * S;
            size_t j = 0;
            while (j < nb && b[j] <= t) ++j;
            return (size_t)i * (S + 1) + j;
        }
        // The framework walks the nodes in List() order in chunks per goroutine: the row after
        // this thread's last one (or a few further, for the feasible list) first — a pointer
        // compare; rows follow List() order until nodes join or leave —, then the address index,
        // then the name.
        int64_t find_info(const NodeInfo* ni, const Node* node) const {
            thread_local const View* lv = nullptr;
            thread_local int64_t last = -1;
            const int64_t n = (int64_t)rows();
            if (lv == this)
                for (int64_t i = last + 1; i < std::min(n, last + 5); ++i)
                    if (infos[(size_t)i] == ni) return last = i;
            int64_t i = info_idx.get(ni);
            if (i >= 0 && infos[(size_t)i] != ni) i = -1;  // a departed NodeInfo's entry
            if (i < 0) {  // a NodeInfo object that is not the snapshot's: by name
                auto it = by_name.find(node->Name);
                i = it == by_name.end() ? -1 : it->second;
            }
            lv = this;
            last = i;
            return i;
        }
        int64_t find_name(const std::string& name) const {
            thread_local const View* lv = nullptr;
            thread_local int64_t last = -1;
            const int64_t n = (int64_t)rows();
            auto mine = [&](int64_t i) { return infos[(size_t)i] && nodes[(size_t)i] && &nodes[(size_t)i]->Name == &name; };
            if (lv == this)
                for (int64_t i = last + 1; i < std::min(n, last + 5); ++i)
                    if (mine(i)) return last = i;
            int64_t i = name_idx.get(&name);
            if (i >= 0 && !mine(i)) i = -1;  // a replaced or departed Node's
            if (i < 0) {
                auto it = by_name.find(name);
                i = it == by_name.end() ? -1 : it->second;
            }
            lv = this;
            last = i;
            return i;
        }
    };

    DynamicScheduler() = default;

    const std::vector<std::string>& keys() {  // rows: metric slots 0..M-1, node_hot_value
        if (keys_.empty()) {
            const int32_t M = eng_.num_metrics();
            for (int32_t m = 0; m < M; ++m) keys_.emplace_back(eng_.metric_name(m));
            keys_.emplace_back(NodeHotValue);
        }
        return keys_;
    }

    // The changed nodes parsed in chunks of nodes by the cycle's callers — the annotation lookups
    // and the parses (a cycle at the controller's rate at one pod per second re-parses ~1,400
    // nodes, ~10k strings: 1-2 ms on one thread while the other callers wait).
    struct ParseJob {
        const Node* const* nodes;
        const std::string* keys;
        size_t R = 0, n = 0, nchunks = 0;
        double* val;
        int64_t* ts;
        const crane_tz* zone;
        int64_t tz;
        std::atomic<size_t> next{0}, done{0};
        void work() {
            for (;;) {
                const size_t c = next.fetch_add(1, std::memory_order_relaxed);
                if (c >= nchunks) return;
                const size_t hi = std::min(n, (c + 1) * kParseChunk);
                for (size_t i = c * kParseChunk; i < hi; ++i)
                    for (size_t m = 0; m < R; ++m) {
                        double* v = val + m * n + i;
                        int64_t* t = ts + m * n + i;
                        const Node* nd = nodes[i];
                        auto it = nd ? nd->Annotations.find(keys[m]) : decltype(nd->Annotations.end()){};
                        if (!nd || it == nd->Annotations.end()) {
                            *v = 0;  // key not found (stats.go:52-55)
                            *t = CRANE_TS_INVALID;
                        } else if (zone) {
                            crane_parse_annotation_tz(it->second.data(), it->second.size(), zone, v, t);
                        } else {
                            crane_parse_annotation(it->second.data(), it->second.size(), tz, v, t);
                        }
                    }
                done.fetch_add(1, std::memory_order_acq_rel);
            }
        }
    };
    static constexpr size_t kParseChunk = 64;  // nodes

    // parse rows [key][n] of the nodes' annotation strings (NULL = key missing); with the cycle's
    // state, a parse of more than a few chunks is shared with the cycle's other callers
    bool parse(const std::vector<const Node*>& nodes, int32_t threads, std::vector<double>* val,
               std::vector<int64_t>* ts, std::string* err, CycleState* state = nullptr) {
        const std::vector<std::string>& ks = keys();
        const size_t R = ks.size(), n = nodes.size();
        val->resize(R * n);
        ts->resize(R * n);
        if (state && n >= 4 * kParseChunk) {
            auto job = std::make_shared<ParseJob>();
            job->nodes = nodes.data();
            job->keys = ks.data();
            job->R = R;
            job->n = n;
            job->nchunks = (n + kParseChunk - 1) / kParseChunk;
            job->val = val->data();
            job->ts = ts->data();
            job->zone = zone_;
            job->tz = tz_;
            state->dyn_parse_ = job;
            state->dyn_phase_.store(4, std::memory_order_release);
            job->work();
            while (job->done.load(std::memory_order_acquire) < job->nchunks) relax();
            return true;
        }
        strs_.assign(R * n, nullptr);
        lens_.assign(R * n, 0);
        for (size_t i = 0; i < n; ++i) {
            if (!nodes[i]) continue;
            const auto& a = nodes[i]->Annotations;
            for (size_t m = 0; m < R; ++m) {
                auto it = a.find(ks[m]);
                if (it == a.end()) continue;
                strs_[m * n + i] = it->second.data();
                lens_[m * n + i] = it->second.size();
            }
        }
        const int rc = zone_ ? crane_parse_annotations_tz((int64_t)(R * n), strs_.data(), lens_.data(), zone_,
                                                         val->data(), ts->data(), threads)
                             : crane_parse_annotations((int64_t)(R * n), strs_.data(), lens_.data(), tz_, val->data(),
                                                       ts->data(), threads);
        if (rc) *err = "annotation parse failed";
        return rc == 0;
    }

    // every row's answers over the table's span into v: the whole time axis by default, else
    // [now, now + horizon).  (The span is recorded only once the rows hold it: on a failure the
    // caller drops the View, so no later cycle answers from rows of another span.)
    bool build_table(View* v, int64_t now, std::string* err) {
        const size_t N = v->rows();
        int64_t t0 = INT64_MIN, t1 = INT64_MAX;
        if (horizon_ns_ != kAllTime) {
            t0 = now;
            t1 = now > INT64_MAX - horizon_ns_ ? INT64_MAX : now + horizon_ns_;
        }
        if (eng_.node_steps(t0, t1, (int64_t)N, v->n_steps.data(), v->bp.data(), v->first_fail.data(),
                            v->score.data())) {
            *err = eng_.error();
            return false;
        }
        v->t0 = t0;
        v->t1 = t1;
        ++cnt_.tables_built;
        return true;
    }

    // the first sync (or a change of most of the node set): parse the whole snapshot, upload it,
    // index it, build the table
    std::shared_ptr<View> full_sync(const std::vector<const NodeInfo*>& L, int64_t now, std::string* err) {
        auto v = std::make_shared<View>();
        const size_t N = L.size();
        v->S = (size_t)eng_.step_slots();
        v->grow(N);
        v->by_name.reserve(N);
        for (size_t i = 0; i < N; ++i) {
            v->infos[i] = L[i];
            v->nodes[i] = L[i]->node();
            v->gens[i] = L[i]->Generation;
            if (v->nodes[i]) {
                v->names[i] = v->nodes[i]->Name;
                v->by_name.emplace(v->names[i], (int64_t)i);
            }
        }
        v->live = N;
        v->index_infos();
        v->index_names();
        std::vector<double> val;
        std::vector<int64_t> ts;
        if (!parse(v->nodes, parse_threads_, &val, &ts, err)) return nullptr;
        const size_t M = (size_t)eng_.num_metrics();
        if (eng_.upload_nodes((int64_t)N, val.data(), ts.data(), val.data() + M * N, ts.data() + M * N)) {
            *err = eng_.error();
            return nullptr;
        }
        ++cnt_.full_syncs;
        if (!build_table(v.get(), now, err)) return nullptr;
        // warm the incremental path (its staging buffers, its kernel) with row 0's own columns,
        // which rewrites row 0 unchanged: the first cycle that finds changed nodes then costs
        // what the later ones do
        if (N > 0) {
            std::vector<double> cv(M + 1);
            std::vector<int64_t> ct(M + 1);
            for (size_t m = 0; m <= M; ++m) {
                cv[m] = val[m * N];
                ct[m] = ts[m * N];
            }
            const int64_t r0 = 0;
            if (eng_.update_node_steps(1, &r0, cv.data(), ct.data(), cv.data() + M, ct.data() + M, v->t0, v->t1,
                                       v->n_steps.data(), v->bp.data(), v->first_fail.data(), v->score.data())) {
                *err = eng_.error();
                return nullptr;
            }
        }
        return v;
    }

    // Nodes that left give their rows back; joining nodes take free rows (the shard grows by an
    // eighth when none is left) and join the changed rows, whose columns update() writes.
    bool membership(View* v, const std::vector<const NodeInfo*>& L, std::string* err) {
        for (int64_t r : removed_) {
            // (by the kept name: the snapshot may have freed the departed node's objects)
            auto it = v->by_name.find(v->names[(size_t)r]);
            if (it != v->by_name.end() && it->second == r) v->by_name.erase(it);
            v->infos[(size_t)r] = nullptr;
            v->nodes[(size_t)r] = nullptr;
            v->names[(size_t)r].clear();
            v->free_rows.push_back(r);
            --v->live;
        }
        std::sort(v->free_rows.begin(), v->free_rows.end(), std::greater<int64_t>());
        if (added_.size() > v->free_rows.size()) {
            const size_t rows = v->rows(), need = added_.size() - v->free_rows.size();
            const size_t cap = rows + std::max(need, rows / 8 + 64);
            if (eng_.resize_nodes((int64_t)cap)) {
                *err = eng_.error();
                return false;
            }
            v->grow(cap);
            std::vector<int64_t> fresh;
            for (size_t r = cap; r-- > rows;) fresh.push_back((int64_t)r);
            v->free_rows.insert(v->free_rows.begin(), fresh.begin(), fresh.end());  // (after the old ones)
            ++cnt_.grows;
        }
        for (int64_t j : added_) {
            const int64_t r = v->free_rows.back();
            v->free_rows.pop_back();
            const NodeInfo* ni = L[(size_t)j];
            v->infos[(size_t)r] = ni;
            v->nodes[(size_t)r] = nullptr;  // (parsed by update(), which records the Node)
            v->gens[(size_t)r] = ni->Generation;
            v->seen[(size_t)r] = epoch_;
            v->info_idx.put(ni, r);
            if (ni->node()) {
                v->names[(size_t)r] = ni->node()->Name;
                v->by_name[v->names[(size_t)r]] = r;
            }
            ++v->live;
            changed_.push_back(r);
        }
        if (v->info_idx.crowded()) v->index_infos();  // entries of departed NodeInfos pile up
        cnt_.nodes_joined += added_.size();
        cnt_.nodes_left += removed_.size();
        return true;
    }

    // the changed rows: re-parse, scatter into the engine, rebuild their table rows.  The View
    // records the new Node objects only once the engine holds them (a failed call makes the
    // caller drop the View: the next cycle resyncs in full).
    bool update(View* v, int64_t now, std::string* err, CycleState* state) {
        const size_t k = changed_.size();
        cnodes_.resize(k);
        for (size_t j = 0; j < k; ++j) cnodes_[j] = v->infos[(size_t)changed_[j]]->node();
        std::vector<double> val;
        std::vector<int64_t> ts;
        const auto tp = std::chrono::steady_clock::now();
        if (!parse(cnodes_, 1, &val, &ts, err, state)) return false;
        const auto te = std::chrono::steady_clock::now();
        cnt_.parse_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(te - tp).count();
        struct EngineTime {  // (the engine call and the rows' copy, however update() returns)
            Counters& c;
            std::chrono::steady_clock::time_point t;
            ~EngineTime() {
                c.engine_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                   std::chrono::steady_clock::now() - t)
                                   .count();
            }
        } et{cnt_, te};
        const size_t M = (size_t)eng_.num_metrics();
        auto record = [&] {
            for (size_t j = 0; j < k; ++j) {
                const size_t i = (size_t)changed_[j];
                v->nodes[i] = cnodes_[j];
                v->gens[i] = v->infos[i]->Generation;
                if (cnodes_[j]) v->name_idx.put(&cnodes_[j]->Name, (int64_t)i);
            }
            if (v->name_idx.crowded()) v->index_names();  // entries of replaced Nodes pile up
            ++cnt_.incremental_syncs;
            cnt_.nodes_updated += k;
        };
        if (now < v->t0 || now >= v->t1) {  // the caller rebuilds the whole table: the columns only
            if (eng_.update_nodes((int64_t)k, changed_.data(), val.data(), ts.data(), val.data() + M * k,
                                  ts.data() + M * k)) {
                *err = eng_.error();
                return false;
            }
            record();
            return true;
        }
        // the columns, the records and the changed nodes' rows in one launch (one round trip)
        const size_t S = v->S;
        rns_.resize(k);
        rbp_.resize(k * S);
        rff_.resize(k * (S + 1));
        rsc_.resize(k * (S + 1));
        if (eng_.update_node_steps((int64_t)k, changed_.data(), val.data(), ts.data(), val.data() + M * k,
                                   ts.data() + M * k, v->t0, v->t1, rns_.data(), rbp_.data(), rff_.data(),
                                   rsc_.data())) {
            *err = eng_.error();
            return false;
        }
        for (size_t j = 0; j < k; ++j) {
            const size_t i = (size_t)changed_[j];
            v->n_steps[i] = rns_[j];
            std::memcpy(&v->bp[i * S], &rbp_[j * S], 8 * S);
            std::memcpy(&v->first_fail[i * (S + 1)], &rff_[j * (S + 1)], S + 1);
            std::memcpy(&v->score[i * (S + 1)], &rsc_[j * (S + 1)], S + 1);
        }
        record();
        return true;
    }

    // The snapshot scan: every NodeInfo looked up in the synced rows and compared with the one
    // its row was parsed from, in chunks any of the cycle's callers may take.  A NodeInfo with no
    // row is a joining node; the rows no NodeInfo claimed are the nodes that left.
    struct ScanJob {
        const NodeInfo* const* L;
        const View* v;
        uint32_t* seen;
        uint32_t epoch = 0;
        size_t n = 0, chunk = 0, nchunks = 0;
        std::atomic<size_t> next{0}, done{0};
        std::vector<std::vector<int64_t>> changed;  // per chunk: rows
        std::vector<std::vector<int64_t>> added;    // per chunk: List() positions
        void work() {
            for (;;) {
                const size_t c = next.fetch_add(1, std::memory_order_relaxed);
                if (c >= nchunks) return;
                const size_t hi = std::min(n, (c + 1) * chunk);
                std::vector<int64_t>& ch = changed[c];
                std::vector<int64_t>& ad = added[c];
                const NodeInfo* const* vi = v->infos.data();
                const Node* const* vn = v->nodes.data();
                const int64_t* vg = v->gens.data();
                const int64_t rows = (int64_t)v->rows();
                for (size_t i = c * chunk; i < hi; ++i) {
                    const NodeInfo* x = L[i];
                    // rows follow List() order until the set changes: the same position first
                    int64_t r = (int64_t)i < rows && vi[i] == x ? (int64_t)i : v->info_idx.get(x);
                    if (r < 0 || vi[r] != x) {
                        ad.push_back((int64_t)i);
                        continue;
                    }
                    seen[r] = epoch;
                    if (x->node() != vn[r] || x->Generation != vg[r]) ch.push_back(r);
                }
                done.fetch_add(1, std::memory_order_acq_rel);
            }
        }
    };
    static constexpr size_t kScanChunk = 4096;

    // The state for a cycle at `now`: compare the snapshot's NodeInfos with the synced rows (with
    // the cycle's other callers when `state` is given), then apply the joins, departures and
    // changes.
    std::shared_ptr<View> sync_locked(int64_t now, std::string* err, CycleState* state = nullptr) {
        if (!handle_.snapshot) {
            *err = "no snapshot";
            return nullptr;
        }
        const std::vector<const NodeInfo*>& L = handle_.snapshot->List();
        std::shared_ptr<View> v = view_;
        if (!v) {
            view_ = full_sync(L, now, err);
            return view_;
        }
        changed_.clear();
        added_.clear();
        removed_.clear();
        ++epoch_;
        const auto ts0 = std::chrono::steady_clock::now();
        {
            auto job = std::make_shared<ScanJob>();
            job->L = L.data();
            job->v = v.get();
            job->seen = v->seen.data();
            job->epoch = epoch_;
            job->n = L.size();
            job->chunk = kScanChunk;
            job->nchunks = (job->n + kScanChunk - 1) / kScanChunk;
            // every chunk's lists hold a whole chunk already (kept across cycles): the cycle's
            // other callers never allocate (a first allocation on a thread maps a malloc arena)
            job->changed = std::move(scan_changed_);
            job->added = std::move(scan_added_);
            if (job->changed.size() < job->nchunks) job->changed.resize(job->nchunks);
            if (job->added.size() < job->nchunks) job->added.resize(job->nchunks);
            for (size_t c = 0; c < job->nchunks; ++c) {
                job->changed[c].clear();
                job->added[c].clear();
                job->changed[c].reserve(kScanChunk);
                job->added[c].reserve(kScanChunk);
            }
            if (state && job->nchunks > 1) {
                state->dyn_job_ = job;
                state->dyn_phase_.store(2, std::memory_order_release);
            }
            job->work();
            while (job->done.load(std::memory_order_acquire) < job->nchunks) relax();
            for (size_t c = 0; c < job->nchunks; ++c) {
                changed_.insert(changed_.end(), job->changed[c].begin(), job->changed[c].end());
                added_.insert(added_.end(), job->added[c].begin(), job->added[c].end());
            }
            scan_changed_ = std::move(job->changed);  // (every chunk is done: no caller touches them)
            scan_added_ = std::move(job->added);
        }
        // the live rows no NodeInfo of this snapshot claimed: the nodes that left
        if (L.size() - added_.size() != v->live)
            for (size_t r = 0; r < v->rows(); ++r)
                if (v->infos[r] && v->seen[r] != epoch_) removed_.push_back((int64_t)r);
        const auto ts1 = std::chrono::steady_clock::now();
        cnt_.scan_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(ts1 - ts0).count();
        if (4 * (added_.size() + removed_.size()) > L.size() + 256) {  // most of the set: resync whole
            view_.reset();
            view_ = full_sync(L, now, err);
            return view_;
        }
        // a failed engine call drops the View: the next cycle starts from a full sync instead of
        // answering from rows the engine no longer matches
        if ((!added_.empty() || !removed_.empty()) && !membership(v.get(), L, err)) {
            view_.reset();
            return nullptr;
        }
        cnt_.membership_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                  std::chrono::steady_clock::now() - ts1)
                                  .count();
        if (!changed_.empty() && !update(v.get(), now, err, state)) {
            view_.reset();
            return nullptr;
        }
        if ((now < v->t0 || now >= v->t1) && !build_table(v.get(), now, err)) {
            view_.reset();
            return nullptr;
        }
        return v;
    }

    // The state of the cycle.  Its first caller brings the plugin up to date; the cycle's other
    // callers (the framework's 16 goroutines, all waiting for the same answers) take chunks of
    // the snapshot scan and of the changed nodes' parse meanwhile, then wait for the leader's
    // engine update.
    const View* view_of(CycleState& state, std::string* err) {
        if (!state.dyn_ready_.load(std::memory_order_acquire)) {
            int ph = 0;
            if (state.dyn_phase_.compare_exchange_strong(ph, 1, std::memory_order_acq_rel)) {
                std::string e;
                std::shared_ptr<const View> v;
                {
                    std::lock_guard<std::mutex> g(mu_);  // one engine: syncs are serial
                    const auto t0 = std::chrono::steady_clock::now();
                    v = sync_locked(state.now_ns, &e, &state);
                    cnt_.sync_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                        std::chrono::steady_clock::now() - t0)
                                        .count();
                }
                std::lock_guard<std::mutex> g(state.clone_mu_);
                state.dyn_row_ = v;
                state.dyn_err_ = e;
                state.dyn_done_ = true;
                state.dyn_phase_.store(3, std::memory_order_relaxed);
                state.dyn_ready_.store(true, std::memory_order_release);
            } else {
                bool scanned = false, parsed = false;
                for (uint32_t k = 0; !state.dyn_ready_.load(std::memory_order_acquire); ++k) {
                    const int ph = state.dyn_phase_.load(std::memory_order_acquire);
                    if (ph == 2 && !scanned) {
                        static_cast<ScanJob*>(state.dyn_job_.get())->work();
                        scanned = true;
                        k = 0;
                    } else if (ph == 4 && !parsed) {
                        static_cast<ParseJob*>(state.dyn_parse_.get())->work();
                        parsed = true;
                        k = 0;
                    }
                    if (k < 4096) relax();
                    else std::this_thread::yield();
                }
            }
        }
        const View* v = static_cast<const View*>(state.dyn_row_.get());
        if (!v) *err = state.dyn_err_;
        return v;
    }

    static void relax() { __builtin_ia32_pause(); }

    Handle handle_;
    crane_policy_doc* doc_ = nullptr;
    Backend eng_;
    crane_tz* zone_ = nullptr;  // the IANA zone of $TZ, or null: the fixed offset tz_
    int64_t tz_ = 8 * 3600;
    int32_t parse_threads_ = 16;  // the framework's parallelism (upstream default)
    static constexpr int64_t kAllTime = INT64_MAX;
    int64_t horizon_ns_ = kAllTime;  // the table's span: the whole time axis unless SetHorizon
    uint32_t epoch_ = 0;             // snapshot scans so far
    mutable std::mutex mu_;
    Counters cnt_;
    std::shared_ptr<View> view_;
    // scratch of the syncs (under mu_)
    std::vector<std::string> keys_;
    std::vector<int64_t> changed_, added_, removed_;
    std::vector<std::vector<int64_t>> scan_changed_, scan_added_;  // ScanJob's per-chunk lists, reused
    std::vector<const Node*> cnodes_;
    std::vector<const char*> strs_;
    std::vector<size_t> lens_;
    std::vector<uint8_t> rns_;
    std::vector<int64_t> rbp_;
    std::vector<int8_t> rff_, rsc_;
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
    if (ds->eng_.create(crane_policy_view(doc), h))
        return {nullptr, std::string("failed to create the Dynamic engine: ") + ds->eng_.error()};
    return {std::move(ds), ""};
}

}  // namespace dynamic
}  // namespace crane
