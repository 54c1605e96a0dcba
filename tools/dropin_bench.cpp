// dropin_bench.cpp — per-pod scheduling-cycle latency of the drop-in plugin
// mirror (include/crane_dyn_plugin.hpp) the way the upstream framework drives
// it: Filter on every node and Score on every feasible node from a pool of 16
// threads (kube-scheduler's default parallelism), then selectHost — while the
// controller keeps patching node annotations.
//
//   dropin_bench <policy file> <snapshot tsv> <pods tsv> [--threads N] [--cpu]
//                [--churn X] [--churn-log path] [--seed S]
//     snapshot tsv:  N<TAB>name   starts a node;  A<TAB>key<TAB>value  adds an annotation
//     pods tsv:      P<TAB>uid<TAB>now_ns<TAB>daemonset(0/1)
// Prints one JSON object: the per-pod cycle times with their parts (the Filter fan-out —
// whose first calls bring the plugin up to date: "first_call" is that sync's wall time as
// the plugin measured it —, the Score fan-out, selectHost), the plugin's sync counters, and
// the chosen node of every pod (highest
// score, lowest index on ties: the engine's declared tie-break, in place of upstream's
// random reservoir choice).
//
// Churn (--churn X, X > 0): the controller's patch stream at X times its rate.  Every node
// is re-synced for every syncPolicy metric at that metric's period / X (node.go:148-177,
// each (node, metric) with its own phase); a sync patches the metric's annotation and then
// node_hot_value (node.go:88-96,113-146), each stamped with the patch time in the local zone
// (utils.GetLocalTime, Asia/Shanghai).  Pod p's cycle runs at its now_ns; the patches due in
// (now_{p-1}, now_p] are published before it, as the informer would: each one a new Node
// object and a new NodeInfo Generation.  --churn-log writes them (pod, node, key, value) so
// the caller can recompute every pod's answer on the churned annotations.  At X = 1 and
// 100k nodes with the shipped policy that is ~2,700 patches per simulated second.
//
// Node set changes (--node-events E, E > 0): every E-th cycle one node joins the cluster (a new
// Node with every syncPolicy metric and node_hot_value, stamped at the cycle's time) and, in
// between, one node leaves (a random live node; its NodeInfo and Node are freed).  Nodes are
// identified by creation index (the snapshot's nodes 0..N-1, then the joining ones); the churn
// log records joins ("J pod id name") and departures ("L pod id") and the chosen node of every
// pod is a creation index.  The slowest cycles are reported with their parts (slowest).
//
// "--cpu" (the dropin_cpu build, -DDROPIN_CPU, linked with the CPU oracle — bench.py's CPU
// baseline only): the same harness driving a CPU plugin whose Filter and Score re-parse
// the node's annotations on every call, as the reference's getResourceUsage does
// (stats.go:51-76), through the oracle's string mode (oracle/crane_oracle.c).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <memory>
#include <numeric>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "crane_dyn_plugin.hpp"
#ifdef DROPIN_CPU
#include "../oracle/crane_oracle.h"
#endif

using namespace crane::dynamic;
using Clock = std::chrono::steady_clock;

// The scheduler's snapshot as the informer keeps it: stable NodeInfo objects, each pointing
// at the node's current (immutable) Node object; an update publishes a new Node object.
struct BenchSnap : Snapshot {
    std::vector<std::unique_ptr<Node>> objs;
    std::vector<std::unique_ptr<NodeInfo>> infos;
    std::vector<const NodeInfo*> list;
    std::vector<int64_t> ids;          // list position -> creation index
    std::vector<int64_t> pos_of;       // creation index -> list position (-1: left)
    std::unordered_map<std::string, size_t, NameHash> by_name;  // name -> list position
    int64_t gen = 0;
    const std::vector<const NodeInfo*>& List() const override { return list; }
    const NodeInfo* Get(const std::string& name, std::string* err) const override {
        auto it = by_name.find(name);
        if (it == by_name.end()) {
            *err = "nodeinfo not found for node name \"" + name + "\"";
            return nullptr;
        }
        return infos[it->second].get();
    }
    const Node& node(size_t i) const { return *objs[i]; }
    void add(const std::string& name) {
        by_name[name] = objs.size();
        pos_of.push_back((int64_t)objs.size());
        ids.push_back((int64_t)pos_of.size() - 1);
        objs.emplace_back(new Node{name, {}});
        infos.emplace_back(new NodeInfo(objs.back().get(), ++gen));
        list.push_back(infos.back().get());
    }
    // a joining node, published whole (its annotations set before any reader sees it)
    void join(const std::string& name, std::map<std::string, std::string> ann) {
        add(name);
        objs.back()->Annotations = std::move(ann);
    }
    // node at list position i leaves: dropped from the list, its objects freed
    void leave(size_t i) {
        by_name.erase(objs[i]->Name);
        pos_of[(size_t)ids[i]] = -1;
        list.erase(list.begin() + (long)i);
        infos.erase(infos.begin() + (long)i);
        objs.erase(objs.begin() + (long)i);
        ids.erase(ids.begin() + (long)i);
        for (size_t j = i; j < ids.size(); ++j) {
            pos_of[(size_t)ids[j]] = (int64_t)j;
            by_name[objs[j]->Name] = j;
        }
    }
    void patch(size_t i, const std::string& key, const std::string& value) {
        std::unique_ptr<Node> n(new Node(*objs[i]));
        n->Annotations[key] = value;
        infos[i]->SetNode(n.get());
        infos[i]->Generation = ++gen;
        objs[i] = std::move(n);
    }
};

// "YYYY-MM-DDTHH:MM:SSZ" of Unix second t in a fixed-offset zone (utils.TimeFormat, utils.go:11;
// Asia/Shanghai has had no transition since 1991)
static std::string local_stamp(int64_t t, int64_t off) {
    int64_t s = t + off, days = s / 86400, sod = s % 86400;
    if (sod < 0) {
        sod += 86400;
        --days;
    }
    // civil_from_days (Howard Hinnant)
    days += 719468;
    const int64_t era = (days >= 0 ? days : days - 146096) / 146097;
    const int64_t doe = days - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    const int64_t d = doy - (153 * mp + 2) / 5 + 1;
    const int64_t m = mp < 10 ? mp + 3 : mp - 9;
    if (m <= 2) ++y;
    char buf[32];
    std::snprintf(buf, sizeof buf, "%04lld-%02lld-%02lldT%02lld:%02lld:%02lldZ", (long long)y, (long long)m,
                  (long long)d, (long long)(sod / 3600), (long long)(sod / 60 % 60), (long long)(sod % 60));
    return buf;
}

static uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// The controller's patch stream (node.go:148-177): (node, syncPolicy entry) pairs due in time
// order, each at its own phase within the entry's period.
class Churn {
   public:
    struct Patch {
        size_t node;
        std::string key, value;
    };
    Churn(const crane_policy& pol, size_t n_nodes, int64_t t_start_ns, double scale, uint64_t seed) : seed_(seed) {
        for (int32_t m = 0; m < pol.n_sync; ++m) {
            if (pol.sync_period_ns[m] <= 0) continue;
            names_.emplace_back(pol.sync_name[m]);
            period_.push_back(std::max<int64_t>(1, (int64_t)((double)pol.sync_period_ns[m] / scale)));
        }
        std::vector<Ev> evs;
        evs.reserve(n_nodes * names_.size());
        for (size_t n = 0; n < n_nodes; ++n)
            for (size_t m = 0; m < names_.size(); ++m) {
                const int64_t ph = (int64_t)(mix64(seed_ ^ (n * 64 + m)) % (uint64_t)period_[m]);
                evs.push_back({t_start_ns + ph, (uint32_t)n, (uint32_t)m});
            }
        q_ = std::priority_queue<Ev, std::vector<Ev>, std::greater<Ev>>(std::greater<Ev>(), std::move(evs));
    }
    // the patches due in (.., t_ns], in time order: metric m's value, then node_hot_value
    void due(int64_t t_ns, std::vector<Patch>* out) {
        while (!q_.empty() && q_.top().t <= t_ns) {
            Ev e = q_.top();
            q_.pop();
            const uint64_t r = mix64(seed_ * 31 + (uint64_t)e.t * 1315423911ull + e.n * 7 + e.m);
            const std::string st = local_stamp(e.t / 1000000000LL, 8 * 3600);
            char v[64];
            std::snprintf(v, sizeof v, "%.5f,%s", (double)(r % 120001) / 1e5, st.c_str());  // prometheus.go:124
            out->push_back({e.n, names_[e.m], v});
            std::snprintf(v, sizeof v, "%d,%s", (int)((r >> 20) % 13), st.c_str());  // strconv.Itoa, node.go:120
            out->push_back({e.n, NodeHotValue, v});
            e.t += period_[e.m];
            q_.push(e);
        }
    }

   private:
    struct Ev {
        int64_t t;
        uint32_t n, m;
        bool operator>(const Ev& o) const { return t != o.t ? t > o.t : (n != o.n ? n > o.n : m > o.m); }
    };
    uint64_t seed_;
    std::vector<std::string> names_;
    std::vector<int64_t> period_;
    std::priority_queue<Ev, std::vector<Ev>, std::greater<Ev>> q_;
};

// framework.Parallelizer().Until(ctx, n, f) on a fixed pool: the caller and n - 1 workers
// take chunks of 64 pieces.  Between fan-outs a worker spins on the epoch for a while
// (~0.1 ms) before it sleeps, and the caller spins on the count of busy workers: the
// framework's goroutines start in about a microsecond, a condition-variable wake of
// sixteen threads per fan-out cost ~0.13 ms of the cycle (the harness's no-op fan-outs).
class Pool {
   public:
    explicit Pool(int n) {
        for (int i = 1; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_.store(true, std::memory_order_relaxed);
            epoch_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void until(int64_t n, const std::function<void(int64_t)>& f) {
        f_ = &f;
        n_ = n;
        next_.store(0, std::memory_order_relaxed);
        busy_.store((int)th_.size(), std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(mu_);  // (a worker between its check and its wait sees it)
            epoch_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        work();
        for (int k = 0; busy_.load(std::memory_order_acquire) != 0; ++k) {
            if (k < kSpin) {
                relax();
                continue;
            }
            std::unique_lock<std::mutex> lk(mu_);
            done_.wait(lk, [&] { return busy_.load(std::memory_order_acquire) == 0; });
        }
    }

   private:
    static constexpr int kSpin = 4096;
    static void relax() { __builtin_ia32_pause(); }
    void work() {
        const std::function<void(int64_t)>& f = *f_;
        const int64_t n = n_;
        for (;;) {  // chunks of 64 pieces, like the framework's chunked work queue
            const int64_t i0 = next_.fetch_add(64, std::memory_order_relaxed);
            if (i0 >= n) break;
            for (int64_t i = i0; i < std::min(n, i0 + 64); ++i) f(i);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            uint64_t e = epoch_.load(std::memory_order_acquire);
            for (int k = 0; e == seen && k < kSpin; ++k) {
                relax();
                e = epoch_.load(std::memory_order_acquire);
            }
            if (e == seen) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return (e = epoch_.load(std::memory_order_acquire)) != seen; });
            }
            seen = e;
            if (stop_.load(std::memory_order_relaxed)) return;
            work();
            if (busy_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> g(mu_);
                done_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int64_t)>* f_ = nullptr;
    int64_t n_ = 0;
    std::atomic<int64_t> next_{0};
    std::atomic<int> busy_{0};
    std::atomic<uint64_t> epoch_{0};
    std::atomic<bool> stop_{false};
};

#ifdef DROPIN_CPU
// Filter / Score re-parsing the node's annotations on every call (stats.go:51-76): one
// (pod, node) evaluation of the oracle's string mode per call, on the node's current object.
class CpuPlugin {
   public:
    CpuPlugin(const crane_policy& p, const BenchSnap& snap, int64_t tz) : tz_(tz), snap_(&snap) {
        pol_ = or_policy{p.n_sync, p.sync_name, p.sync_period_ns, p.n_pred, p.pred_name, p.pred_limit,
                         p.n_prio, p.prio_name, p.prio_weight, p.n_hot, p.hot_tr_ns, p.hot_count};
        for (size_t i = 0; i < snap.infos.size(); ++i) idx_[snap.infos[i].get()] = (int64_t)i;
    }
    Status Filter(CycleState& st, const Pod& pod, const NodeInfo& ni) {
        if (IsDaemonsetPod(pod)) return NewStatus(Code::Success, "");
        const Node* n = ni.node();
        if (!n) return NewStatus(Code::Error, "node not found");
        int8_t ff = -1;
        eval(*n, st.now_ns, 0, &ff, nullptr);
        if (ff >= 0)
            return NewStatus(Code::Unschedulable,
                             "Load[" + std::string(pol_.pred_name[ff]) + "] of node[" + n->Name + "] is too high");
        return NewStatus(Code::Success, "");
    }
    std::pair<int64_t, Status> Score(CycleState& st, const Pod&, const std::string& name) {
        std::string err;
        const NodeInfo* ni = snap_->Get(name, &err);
        if (!ni) return {0, NewStatus(Code::Error, "getting node \"" + name + "\" from Snapshot: " + err)};
        int64_t s = 0;
        eval(*ni->node(), st.now_ns, 1, nullptr, &s);  // (flag 1: the Filter part is skipped)
        return {s, Status()};
    }

   private:
    void eval(const Node& n, int64_t now, uint8_t ds, int8_t* ff, int64_t* score) {
        thread_local std::vector<const char*> keys, vals;
        keys.clear();
        vals.clear();
        for (const auto& kv : n.Annotations) {
            keys.push_back(kv.first.c_str());
            vals.push_back(kv.second.c_str());
        }
        const int64_t off[2] = {0, (int64_t)keys.size()};
        or_eval_strings(&pol_, 1, off, keys.data(), vals.data(), 1, &now, &ds, tz_, 1, ff, score, nullptr);
    }
    or_policy pol_;
    int64_t tz_;
    const BenchSnap* snap_;
    std::unordered_map<const NodeInfo*, int64_t> idx_;
};
#endif

static std::vector<std::string> split_tab(const std::string& s) {
    std::vector<std::string> out;
    size_t a = 0;
    for (;;) {
        size_t b = s.find('\t', a);
        out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) break;
        a = b + 1;
    }
    return out;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: dropin_bench <policy> <snapshot.tsv> <pods.tsv> [--threads N] [--cpu] "
                             "[--churn X] [--churn-log path] [--seed S] [--engine-opt name=value]\n");
        return 2;
    }
    int threads = 16;
    int node_events = 0;
    bool cpu = false;
    bool lead_main = false;  // the caller's thread makes each cycle's first Filter call (probe)
    double churn_scale = 0.0;
    std::string churn_log;
    uint64_t seed = 1;
    std::vector<std::string> engine_opts;  // name=value
    for (int a = 4; a < argc; ++a) {
        const std::string k = argv[a];
        auto next = [&]() -> std::string { return a + 1 < argc ? argv[++a] : ""; };
        if (k == "--threads") threads = std::atoi(next().c_str());
        else if (k == "--cpu") cpu = true;
        else if (k == "--lead-main") lead_main = true;
        else if (k == "--churn") churn_scale = std::atof(next().c_str());
        else if (k == "--churn-log") churn_log = next();
        else if (k == "--seed") seed = std::strtoull(next().c_str(), nullptr, 10);
        else if (k == "--node-events") node_events = std::atoi(next().c_str());
        else if (k == "--engine-opt") engine_opts.push_back(next());
        else {
            std::fprintf(stderr, "unknown argument %s\n", k.c_str());
            return 2;
        }
    }
    BenchSnap snap;
    {
        std::ifstream f(argv[2]);
        std::string line;
        std::vector<std::pair<std::string, std::string>> pend;
        auto flush = [&] {
            if (snap.objs.empty()) return;
            Node& n = *snap.objs.back();  // (not yet published to any reader)
            for (auto& kv : pend) n.Annotations[kv.first] = kv.second;
            pend.clear();
        };
        while (std::getline(f, line)) {
            auto t = split_tab(line);
            if (t[0] == "N") {
                flush();
                snap.add(t[1]);
            } else if (t[0] == "A" && t.size() >= 3) {
                pend.emplace_back(t[1], t[2]);
            }
        }
        flush();
    }
    struct PodIn {
        Pod pod;
        int64_t now;
    };
    std::vector<PodIn> pods;
    {
        std::ifstream f(argv[3]);
        std::string line;
        while (std::getline(f, line)) {
            auto t = split_tab(line);
            if (t[0] != "P") continue;
            PodIn p;
            p.pod.UID = p.pod.Name = t[1];
            p.pod.Namespace = "default";
            if (t[3] == "1") p.pod.OwnerReferences.push_back({"DaemonSet", "ds"});
            p.now = std::stoll(t[2]);
            pods.push_back(std::move(p));
        }
    }
    Handle h;
    h.snapshot = &snap;
    DynamicArgs a;
    a.PolicyConfigPath = argv[1];
#ifndef DROPIN_CPU
    if (cpu) {
        std::fprintf(stderr, "the cpu mode is the dropin_cpu build\n");
        return 2;
    }
#endif
    auto r = NewDynamicScheduler(a, h);
    if (!r.first) {
        std::fprintf(stderr, "NewDynamicScheduler: %s\n", r.second.c_str());
        return 1;
    }
    DynamicScheduler& ds = *r.first;
    ds.SetParseThreads(threads);
#ifndef DROPIN_CPU
    for (const std::string& o : engine_opts) {
        const size_t eq = o.find('=');
        if (eq == std::string::npos || !ds.SetEngineOption(o.substr(0, eq).c_str(), std::atoll(o.c_str() + eq + 1))) {
            std::fprintf(stderr, "bad --engine-opt %s\n", o.c_str());
            return 2;
        }
    }
#endif
    std::string err;
    double sync_ms = 0.0;
    if (!cpu) {  // the first full sync (parse + upload of the whole snapshot + table), before the pods
        CycleState st;
        st.now_ns = pods.empty() ? 0 : pods[0].now;
        Pod none;
        const auto s0 = Clock::now();
        if (!snap.list.empty() && ds.Filter(st, none, *snap.list[0]).code() == Code::Error) {
            std::fprintf(stderr, "first sync failed\n");
            return 1;
        }
        sync_ms = std::chrono::duration<double, std::milli>(Clock::now() - s0).count();
    }
#ifdef DROPIN_CPU
    CpuPlugin cp(ds.policy(), snap, 8 * 3600);
#endif
    std::unique_ptr<Churn> churn;
    if (churn_scale > 0 && !pods.empty())
        churn.reset(new Churn(ds.policy(), snap.objs.size(), pods[0].now, churn_scale, seed));
    FILE* clog = churn_log.empty() ? nullptr : std::fopen(churn_log.c_str(), "w");
    Pool pool(threads);
    const int64_t N0 = (int64_t)snap.objs.size();
    std::vector<uint8_t> feas((size_t)N0);
    std::vector<int64_t> fidx((size_t)N0), fscore((size_t)N0);
    int64_t n_joins = 0, n_leaves = 0;
    std::vector<double> cyc_ms, first_ms, filt_ms, score_ms, sel_ms, pool_ms, cyc_changed_ms;
    std::vector<int64_t> chosen;
    std::vector<Churn::Patch> due;
    int64_t n_patches = 0, changed_cycles = 0;
    struct Slow {
        double cyc, first, filt, score;
        size_t pod;
        int64_t patches;
        double scan, memb, parse, eng;  // the cycle's sync parts (plugin counters)
        long long upd;
    };
    std::vector<char> changed_flag;  // per cycle: the engine was updated
    std::vector<Slow> slow;
    std::atomic<int> errors{0};
    for (size_t pi = 0; pi < pods.size(); ++pi) {
        auto& p = pods[pi];
        {  // the harness's own cost: the two fan-outs over no-op calls
            const int64_t Nn = (int64_t)snap.list.size();
            const auto q0 = Clock::now();
            pool.until(Nn, [&](int64_t i) { feas[(size_t)i] = (uint8_t)(i & 1); });
            pool.until(Nn * 7 / 10, [&](int64_t j) { fscore[(size_t)j] = j; });
            pool_ms.push_back(std::chrono::duration<double, std::milli>(Clock::now() - q0).count());
        }
        due.clear();
        const int64_t patches0 = n_patches;
        if (churn && pi > 0) churn->due(p.now, &due);  // published between the cycles (informer)
        if (cpu && node_events > 0) {
            std::fprintf(stderr, "--node-events needs the engine plugin\n");
            return 2;
        }
        for (const auto& x : due) {
            const int64_t at = snap.pos_of[x.node];
            if (at < 0) continue;  // (a node that left)
            snap.patch((size_t)at, x.key, x.value);
            ++n_patches;
            if (clog) std::fprintf(clog, "%zu\t%zu\t%s\t%s\n", pi, x.node, x.key.c_str(), x.value.c_str());
        }
        if (node_events > 0 && pi > 0 && pi % (size_t)node_events == 0) {  // a node joins
            std::map<std::string, std::string> ann;
            const std::string st = local_stamp(p.now / 1000000000LL, 8 * 3600);
            uint64_t r = mix64(seed * 977 + pi);
            char v[64];
            for (int32_t m = 0; m < ds.policy().n_sync; ++m) {
                r = mix64(r);
                std::snprintf(v, sizeof v, "%.5f,%s", (double)(r % 120001) / 1e5, st.c_str());
                ann[ds.policy().sync_name[m]] = v;
            }
            std::snprintf(v, sizeof v, "%d,%s", (int)((r >> 20) % 13), st.c_str());
            ann[NodeHotValue] = v;
            const std::string name = "joined-" + std::to_string(pi);
            snap.join(name, ann);
            ++n_joins;
            if (clog) {
                std::fprintf(clog, "J\t%zu\t%lld\t%s\n", pi, (long long)snap.ids.back(), name.c_str());
                for (const auto& kv : ann)
                    std::fprintf(clog, "%zu\t%lld\t%s\t%s\n", pi, (long long)snap.ids.back(), kv.first.c_str(),
                                 kv.second.c_str());
            }
        } else if (node_events > 0 && pi > 0 && pi % (size_t)node_events == (size_t)node_events / 2) {  // one leaves
            const size_t i = (size_t)(mix64(seed * 131 + pi) % snap.list.size());
            if (clog) std::fprintf(clog, "L\t%zu\t%lld\n", pi, (long long)snap.ids[i]);
            snap.leave(i);
            ++n_leaves;
        }
        const int64_t N = (int64_t)snap.list.size();
        if ((int64_t)feas.size() < N) {
            feas.resize((size_t)N);
            fidx.resize((size_t)N);
            fscore.resize((size_t)N);
        }
        const auto c0 = cpu ? decltype(ds.counters()){} : ds.counters();
        const uint64_t sync0 = c0.sync_ns;
        const auto t0 = Clock::now();
        CycleState st;
        st.now_ns = p.now;
        // (the cycle's first Filter calls bring the plugin up to date: the first one leads the
        // sync, the pool's other threads take chunks of its snapshot scan)
        if (lead_main && !cpu && N > 0) (void)ds.Filter(st, p.pod, *snap.list[0]);
        pool.until(N, [&](int64_t i) {  // findNodesThatPassFilters
            Status s;
#ifdef DROPIN_CPU
            if (cpu) s = cp.Filter(st, p.pod, *snap.list[(size_t)i]);
            else
#endif
                s = ds.Filter(st, p.pod, *snap.list[(size_t)i]);
            feas[(size_t)i] = s.IsSuccess();
            if (s.code() == Code::Error) errors++;
        });
        const auto t1 = Clock::now();
        int64_t F = 0;  // the feasible list in node order (branch-free: ~30 % of the nodes fail at random)
        for (int64_t i = 0; i < N; ++i) {
            fidx[(size_t)F] = i;
            F += feas[(size_t)i];
        }
        pool.until(F, [&](int64_t j) {  // prioritizeNodes -> RunScorePlugins
            std::pair<int64_t, Status> sr;
            const std::string& name = snap.node((size_t)fidx[(size_t)j]).Name;
#ifdef DROPIN_CPU
            if (cpu) sr = cp.Score(st, p.pod, name);
            else
#endif
                sr = ds.Score(st, p.pod, name);
            fscore[(size_t)j] = sr.first * 3;  // plugin weight (scheduler-config.yaml:16)
            if (!sr.second.IsSuccess()) errors++;
        });
        const auto t2 = Clock::now();
        int64_t best = -1, bs = -1;  // selectHost over the feasible list (index order)
        for (int64_t j = 0; j < F; ++j)
            if (fscore[(size_t)j] > bs) {
                bs = fscore[(size_t)j];
                best = fidx[(size_t)j];
            }
        const auto t3 = Clock::now();
        auto ms = [](Clock::time_point x, Clock::time_point y) {
            return std::chrono::duration<double, std::milli>(y - x).count();
        };
        cyc_ms.push_back(ms(t0, t3));
        changed_flag.push_back(cpu ? !due.empty() : ds.counters().nodes_updated != c0.nodes_updated);
        if (!due.empty()) {
            cyc_changed_ms.push_back(ms(t0, t3));
            ++changed_cycles;
        }
        first_ms.push_back(cpu ? 0.0 : (double)(ds.counters().sync_ns - sync0) / 1e6);
        filt_ms.push_back(ms(t0, t1));
        score_ms.push_back(ms(t1, t2));
        sel_ms.push_back(ms(t2, t3));
        chosen.push_back(best < 0 ? -1 : snap.ids[(size_t)best]);
        const auto c1 = cpu ? decltype(ds.counters()){} : ds.counters();
        slow.push_back({ms(t0, t3), first_ms.back(), ms(t0, t1), ms(t1, t2), pi, n_patches - patches0,
                        (double)(c1.scan_ns - c0.scan_ns) / 1e6, (double)(c1.membership_ns - c0.membership_ns) / 1e6,
                        (double)(c1.parse_ns - c0.parse_ns) / 1e6, (double)(c1.engine_ns - c0.engine_ns) / 1e6,
                        (long long)(c1.nodes_updated - c0.nodes_updated)});
    }
    std::sort(slow.begin(), slow.end(), [](const Slow& a, const Slow& b) { return a.cyc > b.cyc; });
    if (clog) std::fclose(clog);
    auto med = [](std::vector<double> v) {
        if (v.empty()) return 0.0;
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    std::vector<double> sorted = cyc_ms;
    std::sort(sorted.begin(), sorted.end());
    auto pct = [&](double q) { return sorted.empty() ? 0.0 : sorted[(size_t)(q * (double)(sorted.size() - 1))]; };
    // the slowest cycle past the first one that changed the engine (that one pays the GPU's
    // first work after the initial sync's idle gap: DESIGN 4.9)
    double max_after_first = 0.0;
    {
        bool seen_change = false;
        for (size_t i = 0; i < cyc_ms.size(); ++i) {
            if (seen_change) max_after_first = std::max(max_after_first, cyc_ms[i]);
            if (changed_flag[i]) seen_change = true;
        }
    }
    const auto c = ds.counters();
    double sim_s = pods.size() > 1 ? (double)(pods.back().now - pods.front().now) / 1e9 : 0.0;
    std::printf("{\"nodes\": %lld, \"pods\": %zu, \"threads\": %d, \"mode\": \"%s\", \"sync_ms\": %.3f, "
                "\"cycle_ms_median\": %.4f, \"cycle_ms_p90\": %.4f, \"cycle_ms_min\": %.4f, \"cycle_ms_max\": %.4f, "
                "\"cycle_ms_max_after_first_change\": %.4f, "
                "\"cycle_ms_mean\": %.4f, \"changed_cycle_ms_median\": %.4f, "
                "\"first_call_ms_median\": %.4f, \"filter_fanout_ms_median\": %.4f, \"score_fanout_ms_median\": %.4f, "
                "\"select_ms_median\": %.4f, \"pool_noop_ms_median\": %.4f, \"churn_scale\": %.3f, "
                "\"patches\": %lld, \"simulated_s\": %.4f, \"cycles_with_patches\": %lld, \"tables_built\": %llu, "
                "\"full_syncs\": %llu, \"incremental_syncs\": %llu, \"nodes_updated\": %llu, \"errors\": %d, "
                "\"nodes_joined\": %lld, \"nodes_left\": %lld, \"plugin_joined\": %llu, \"plugin_left\": %llu, "
                "\"shard_grows\": %llu, \"nodes_end\": %zu, \"slowest\": [",
                (long long)N0, pods.size(), threads, cpu ? "cpu" : "engine", sync_ms, pct(0.5), pct(0.9), pct(0.0),
                pct(1.0), max_after_first, cyc_ms.empty() ? 0.0 : std::accumulate(cyc_ms.begin(), cyc_ms.end(), 0.0) / (double)cyc_ms.size(),
                med(cyc_changed_ms), med(first_ms), med(filt_ms), med(score_ms), med(sel_ms), med(pool_ms), churn_scale,
                (long long)n_patches, sim_s, (long long)changed_cycles, (unsigned long long)c.tables_built,
                (unsigned long long)c.full_syncs, (unsigned long long)c.incremental_syncs,
                (unsigned long long)c.nodes_updated, errors.load(), (long long)n_joins, (long long)n_leaves,
                (unsigned long long)c.nodes_joined, (unsigned long long)c.nodes_left, (unsigned long long)c.grows,
                snap.list.size());
    for (size_t i = 0; i < std::min<size_t>(5, slow.size()); ++i)
        std::printf("%s{\"pod\": %zu, \"cycle_ms\": %.4f, \"first_call_ms\": %.4f, \"filter_ms\": %.4f, "
                    "\"score_ms\": %.4f, \"patches\": %lld, \"scan_ms\": %.4f, \"membership_ms\": %.4f, "
                    "\"parse_ms\": %.4f, \"engine_ms\": %.4f, \"nodes_updated\": %lld}",
                    i ? ", " : "", slow[i].pod, slow[i].cyc, slow[i].first, slow[i].filt, slow[i].score,
                    (long long)slow[i].patches, slow[i].scan, slow[i].memb, slow[i].parse, slow[i].eng, slow[i].upd);
    std::printf("], \"chosen\": [");
    for (size_t i = 0; i < chosen.size(); ++i) std::printf("%s%lld", i ? ", " : "", (long long)chosen[i]);
    std::printf("]}\n");
    return 0;
}
