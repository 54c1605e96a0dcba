// dropin_bench.cpp — per-pod scheduling-cycle latency of the drop-in plugin
// mirror (include/crane_dyn_plugin.hpp) the way the upstream framework drives
// it: Filter on every node and Score on every feasible node from a pool of 16
// threads (kube-scheduler's default parallelism), then selectHost.
//
//   dropin_bench <policy file> <snapshot tsv> <pods tsv> [threads]
//     snapshot tsv:  N<TAB>name   starts a node;  A<TAB>key<TAB>value  adds an annotation
//     pods tsv:      P<TAB>uid<TAB>now_ns<TAB>daemonset(0/1)
// Prints one JSON object: sync time (bulk parse + upload of the snapshot), the
// per-pod cycle times and the chosen node of every pod (highest score, lowest
// index on ties: the engine's declared tie-break, in place of upstream's
// random reservoir choice).
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

using namespace crane::dynamic;
using Clock = std::chrono::steady_clock;

struct BenchSnap : Snapshot {
    std::vector<Node> nodes;
    std::unordered_map<std::string, size_t> by_name;
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

// framework.Parallelizer().Until(ctx, n, f) on a fixed pool of workers
class Pool {
   public:
    explicit Pool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
            ++epoch_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void until(int64_t n, const std::function<void(int64_t)>& f) {
        {
            std::lock_guard<std::mutex> g(mu_);
            f_ = &f;
            n_ = n;
            next_ = 0;
            busy_ = (int)th_.size();
            ++epoch_;
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return busy_ == 0; });
    }

   private:
    void loop(int) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int64_t)>* f;
            int64_t n;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return epoch_ != seen; });
                seen = epoch_;
                if (stop_) return;
                f = f_;
                n = n_;
            }
            for (;;) {  // chunks of 64 pieces, like the framework's chunked work queue
                const int64_t i0 = next_.fetch_add(64);
                if (i0 >= n) break;
                for (int64_t i = i0; i < std::min(n, i0 + 64); ++i) (*f)(i);
            }
            std::lock_guard<std::mutex> g(mu_);
            if (--busy_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int64_t)>* f_ = nullptr;
    int64_t n_ = 0;
    std::atomic<int64_t> next_{0};
    int busy_ = 0;
    uint64_t epoch_ = 0;
    bool stop_ = false;
};

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
    auto r = NewDynamicScheduler(a, h);
    if (!r.first) {
        std::fprintf(stderr, "NewDynamicScheduler: %s\n", r.second.c_str());
        return 1;
    }
    DynamicScheduler& ds = *r.first;
    ds.SetParseThreads(threads);
    std::string err;
    const auto s0 = Clock::now();
    if (!ds.Sync(&err)) {
        std::fprintf(stderr, "Sync: %s\n", err.c_str());
        return 1;
    }
    const double sync_ms = std::chrono::duration<double, std::milli>(Clock::now() - s0).count();
    Pool pool(threads);
    const int64_t N = (int64_t)snap.nodes.size();
    std::vector<uint8_t> feas((size_t)N);
    std::vector<int64_t> fidx((size_t)N), fscore((size_t)N);
    std::vector<double> cyc_ms;
    std::vector<int64_t> chosen;
    std::atomic<int> errors{0};
    for (auto& p : pods) {
        const auto t0 = Clock::now();
        CycleState st;
        st.now_ns = p.now;
        pool.until(N, [&](int64_t i) {  // findNodesThatPassFilters
            Status s = ds.Filter(st, p.pod, NodeInfo(&snap.nodes[(size_t)i]));
            feas[(size_t)i] = s.IsSuccess();
            if (s.code() == Code::Error) errors++;
        });
        int64_t F = 0;
        for (int64_t i = 0; i < N; ++i)
            if (feas[(size_t)i]) fidx[(size_t)F++] = i;
        pool.until(F, [&](int64_t j) {  // prioritizeNodes -> RunScorePlugins
            auto sr = ds.Score(st, p.pod, snap.nodes[(size_t)fidx[(size_t)j]].Name);
            fscore[(size_t)j] = sr.first * 3;  // plugin weight (scheduler-config.yaml:16)
            if (!sr.second.IsSuccess()) errors++;
        });
        int64_t best = -1, bs = -1;  // selectHost over the feasible list (index order)
        for (int64_t j = 0; j < F; ++j)
            if (fscore[(size_t)j] > bs) {
                bs = fscore[(size_t)j];
                best = fidx[(size_t)j];
            }
        cyc_ms.push_back(std::chrono::duration<double, std::milli>(Clock::now() - t0).count());
        chosen.push_back(best);
    }
    std::vector<double> sorted = cyc_ms;
    std::sort(sorted.begin(), sorted.end());
    auto pct = [&](double q) { return sorted.empty() ? 0.0 : sorted[(size_t)(q * (double)(sorted.size() - 1))]; };
    std::printf("{\"nodes\": %lld, \"pods\": %zu, \"threads\": %d, \"sync_ms\": %.3f, \"cycle_ms_median\": %.4f, "
                "\"cycle_ms_p90\": %.4f, \"cycle_ms_min\": %.4f, \"errors\": %d, \"chosen\": [",
                (long long)N, pods.size(), threads, sync_ms, pct(0.5), pct(0.9), pct(0.0), errors.load());
    for (size_t i = 0; i < chosen.size(); ++i) std::printf("%s%lld", i ? ", " : "", (long long)chosen[i]);
    std::printf("]}\n");
    return 0;
}
