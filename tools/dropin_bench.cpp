// dropin_bench.cpp — per-pod scheduling-cycle latency of the drop-in plugin
// mirror (include/crane_dyn_plugin.hpp) the way the upstream framework drives
// it: Filter on every node and Score on every feasible node from a pool of 16
// threads (kube-scheduler's default parallelism), then selectHost.
//
//   dropin_bench <policy file> <snapshot tsv> <pods tsv> [threads] [cpu]
//     snapshot tsv:  N<TAB>name   starts a node;  A<TAB>key<TAB>value  adds an annotation
//     pods tsv:      P<TAB>uid<TAB>now_ns<TAB>daemonset(0/1)
// Prints one JSON object: sync time (bulk parse + upload of the snapshot), the
// per-pod cycle times with their parts (Filter fan-out, Score fan-out, selectHost),
// and the chosen node of every pod (highest score, lowest index on ties: the
// engine's declared tie-break, in place of upstream's random reservoir choice).
//
// "cpu" (the dropin_cpu build, -DDROPIN_CPU, linked with the CPU oracle — bench.py's CPU
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

struct BenchSnap : Snapshot {
    std::vector<Node> nodes;
    std::unordered_map<std::string, size_t, NameHash> by_name;
    std::vector<const Node*> List() const override {
        std::vector<const Node*> v;
        v.reserve(nodes.size());
        for (const auto& n : nodes) v.push_back(&n);
        return v;
    }
    const Node* Get(const std::string& name, std::string* err) const override {
        auto it = by_name.find(name);
        if (it == by_name.end()) {
            *err = "nodeinfo not found for node name \"" + name + "\"";
            return nullptr;
        }
        return &nodes[it->second];
    }
    uint64_t Generation() const override { return 1; }
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
// (pod, node) evaluation of the oracle's string mode per call.
class CpuPlugin {
   public:
    CpuPlugin(const crane_policy& p, const std::vector<Node>& nodes, int64_t tz) : tz_(tz) {
        pol_ = or_policy{p.n_sync, p.sync_name, p.sync_period_ns, p.n_pred, p.pred_name, p.pred_limit,
                         p.n_prio, p.prio_name, p.prio_weight, p.n_hot, p.hot_tr_ns, p.hot_count};
        for (const auto& n : nodes) {
            off_.push_back((int64_t)keys_.size());
            for (const auto& kv : n.Annotations) {
                keys_.push_back(kv.first.c_str());
                vals_.push_back(kv.second.c_str());
            }
        }
        off_.push_back((int64_t)keys_.size());
        for (size_t i = 0; i < nodes.size(); ++i) idx_[&nodes[i]] = (int64_t)i;
        names_ = &nodes;
    }
    Status Filter(CycleState& st, const Pod& pod, const NodeInfo& ni) {
        if (IsDaemonsetPod(pod)) return NewStatus(Code::Success, "");
        const Node* n = ni.node();
        if (!n) return NewStatus(Code::Error, "node not found");
        int8_t ff = -1;
        eval(idx_.at(n), st.now_ns, 0, &ff, nullptr);
        if (ff >= 0)
            return NewStatus(Code::Unschedulable,
                             "Load[" + std::string(pol_.pred_name[ff]) + "] of node[" + n->Name + "] is too high");
        return NewStatus(Code::Success, "");
    }
    std::pair<int64_t, Status> Score(CycleState& st, const Pod&, const std::string& name, const Snapshot& snap) {
        std::string err;
        const Node* n = snap.Get(name, &err);
        if (!n) return {0, NewStatus(Code::Error, "getting node \"" + name + "\" from Snapshot: " + err)};
        int64_t s = 0;
        eval(idx_.at(n), st.now_ns, 1, nullptr, &s);  // (flag 1: the Filter part is skipped)
        return {s, Status()};
    }

   private:
    void eval(int64_t i, int64_t now, uint8_t ds, int8_t* ff, int64_t* score) {
        const int64_t off[2] = {0, off_[(size_t)i + 1] - off_[(size_t)i]};
        or_eval_strings(&pol_, 1, off, keys_.data() + off_[(size_t)i], vals_.data() + off_[(size_t)i], 1, &now, &ds,
                        tz_, 1, ff, score, nullptr);
    }
    or_policy pol_;
    int64_t tz_;
    std::vector<int64_t> off_;
    std::vector<const char*> keys_, vals_;
    std::unordered_map<const Node*, int64_t> idx_;
    const std::vector<Node>* names_;
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
        std::fprintf(stderr, "usage: dropin_bench <policy> <snapshot.tsv> <pods.tsv> [threads]\n");
        return 2;
    }
    const int threads = argc > 4 ? std::atoi(argv[4]) : 16;
    BenchSnap snap;
    {
        std::ifstream f(argv[2]);
        std::string line;
        while (std::getline(f, line)) {
            auto t = split_tab(line);
            if (t[0] == "N") {
                snap.by_name[t[1]] = snap.nodes.size();
                snap.nodes.push_back(Node{t[1], {}});
            } else if (t[0] == "A" && t.size() >= 3) {
                snap.nodes.back().Annotations[t[1]] = t[2];
            }
        }
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
    const bool cpu = argc > 5 && std::string(argv[5]) == "cpu";
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
    std::string err;
    double sync_ms = 0.0;
    if (!cpu) {
        const auto s0 = Clock::now();
        if (!ds.Sync(&err)) {
            std::fprintf(stderr, "Sync: %s\n", err.c_str());
            return 1;
        }
        sync_ms = std::chrono::duration<double, std::milli>(Clock::now() - s0).count();
    }
#ifdef DROPIN_CPU
    CpuPlugin cp(ds.policy(), snap.nodes, 8 * 3600);
#endif
    Pool pool(threads);
    const int64_t N = (int64_t)snap.nodes.size();
    std::vector<uint8_t> feas((size_t)N);
    std::vector<int64_t> fidx((size_t)N), fscore((size_t)N);
    std::vector<double> cyc_ms, filt_ms, score_ms, sel_ms, pool_ms;
    std::vector<int64_t> chosen;
    std::atomic<int> errors{0};
    for (auto& p : pods) {
        {  // the harness's own cost: the two fan-outs over no-op calls
            const auto q0 = Clock::now();
            pool.until(N, [&](int64_t i) { feas[(size_t)i] = (uint8_t)(i & 1); });
            pool.until(N * 7 / 10, [&](int64_t j) { fscore[(size_t)j] = j; });
            pool_ms.push_back(std::chrono::duration<double, std::milli>(Clock::now() - q0).count());
        }
        const auto t0 = Clock::now();
        CycleState st;
        st.now_ns = p.now;
        pool.until(N, [&](int64_t i) {  // findNodesThatPassFilters
            Status s;
#ifdef DROPIN_CPU
            if (cpu) s = cp.Filter(st, p.pod, NodeInfo(&snap.nodes[(size_t)i]));
            else
#endif
                s = ds.Filter(st, p.pod, NodeInfo(&snap.nodes[(size_t)i]));
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
#ifdef DROPIN_CPU
            if (cpu) sr = cp.Score(st, p.pod, snap.nodes[(size_t)fidx[(size_t)j]].Name, snap);
            else
#endif
                sr = ds.Score(st, p.pod, snap.nodes[(size_t)fidx[(size_t)j]].Name);
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
        filt_ms.push_back(ms(t0, t1));
        score_ms.push_back(ms(t1, t2));
        sel_ms.push_back(ms(t2, t3));
        chosen.push_back(best);
    }
    auto med = [](std::vector<double> v) {
        if (v.empty()) return 0.0;
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    std::vector<double> sorted = cyc_ms;
    std::sort(sorted.begin(), sorted.end());
    auto pct = [&](double q) { return sorted.empty() ? 0.0 : sorted[(size_t)(q * (double)(sorted.size() - 1))]; };
    std::printf("{\"nodes\": %lld, \"pods\": %zu, \"threads\": %d, \"mode\": \"%s\", \"sync_ms\": %.3f, "
                "\"cycle_ms_median\": %.4f, \"cycle_ms_p90\": %.4f, \"cycle_ms_min\": %.4f, \"cycle_ms_max\": %.4f, "
                "\"filter_fanout_ms_median\": %.4f, \"score_fanout_ms_median\": %.4f, \"select_ms_median\": %.4f, "
                "\"pool_noop_ms_median\": %.4f, \"tables_built\": %llu, \"errors\": %d, \"chosen\": [",
                (long long)N, pods.size(), threads, cpu ? "cpu" : "engine", sync_ms, pct(0.5), pct(0.9), pct(0.0),
                pct(1.0), med(filt_ms), med(score_ms), med(sel_ms), med(pool_ms), (unsigned long long)ds.TablesBuilt(),
                errors.load());
    for (size_t i = 0; i < chosen.size(); ++i) std::printf("%s%lld", i ? ", " : "", (long long)chosen[i]);
    std::printf("]}\n");
    return 0;
}
