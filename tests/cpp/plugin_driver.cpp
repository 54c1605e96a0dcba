// Drives crane::dynamic::DynamicScheduler (include/crane_dyn_plugin.hpp) from a
// tab-separated script on stdin, printing every Filter/Score result.  Used by
// tests/test_plugin_cpp.py.
//   policy <path>            NewDynamicScheduler(DynamicArgs{path})
//   badargs                  NewDynamicScheduler(<not DynamicArgs>)
//   node <name>              start a node
//   anno <key> <value>       annotation of the current node
//   pod <uid> <now_ns> <ds>  run Filter + Score of this pod on every node
//   nilnode <uid> <now_ns>   Filter with NodeInfo(nullptr)
//   missing <uid> <now_ns> <name>  Score of a node absent from the snapshot
//   mt <uid> <now_ns> <ds>   as pod, but Filter/Score called from 16 threads at once, half
//                            of them on a Clone() of the cycle state (preemption dry runs)
#include <iostream>
#include <thread>
#include <sstream>
#include <string>
#include <vector>

#include "crane_dyn_plugin.hpp"

using namespace crane::dynamic;

struct Snap : Snapshot {
    std::vector<Node> nodes;
    // (linear Get: small test snapshots)
    uint64_t gen = 1;
    std::vector<const Node*> List() const override {
        std::vector<const Node*> v;
        for (const auto& n : nodes) v.push_back(&n);
        return v;
    }
    const Node* Get(const std::string& name, std::string* err) const override {
        for (const auto& n : nodes)
            if (n.Name == name) return &n;
        *err = "nodeinfo not found for node name \"" + name + "\"";
        return nullptr;
    }
    uint64_t Generation() const override { return gen; }
};

struct Other : Object {};

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

int main() {
    Snap snap;
    Handle h;
    h.snapshot = &snap;
    std::unique_ptr<DynamicScheduler> ds;
    std::string line;
    while (std::getline(std::cin, line)) {
        auto f = split_tab(line);
        if (f.empty() || f[0].empty()) continue;
        if (f[0] == "policy") {
            DynamicArgs a;
            a.PolicyConfigPath = f[1];
            auto r = NewDynamicScheduler(a, h);
            if (!r.first) {
                std::cout << "NEWERR\t" << r.second << "\n";
                return 0;
            }
            ds = std::move(r.first);
            std::cout << "NEW\t" << ds->name() << "\t" << (ds->ScoreExtensions() == nullptr) << "\n";
        } else if (f[0] == "badargs") {
            auto r = NewDynamicScheduler(Other(), h);
            std::cout << "NEWERR\t" << r.second << "\n";
        } else if (f[0] == "node") {
            snap.nodes.push_back(Node{f[1], {}});
            snap.gen++;
        } else if (f[0] == "anno") {
            snap.nodes.back().Annotations[f[1]] = f.size() > 2 ? f[2] : "";
            snap.gen++;
        } else if (f[0] == "mt") {
            Pod pod;
            pod.UID = pod.Name = f[1];
            if (f[3] == "1") pod.OwnerReferences.push_back({"DaemonSet", "ds"});
            CycleState st;
            st.now_ns = std::stoll(f[2]);
            const size_t N = snap.nodes.size();
            std::vector<Status> fs(N);
            std::vector<std::pair<int64_t, Status>> ss(N);
            std::vector<std::thread> th;
            // threads 8..15 work on a clone taken before the first call (it evaluates the pod
            // itself); a second clone is taken after the cycle's row exists (it shares it)
            std::unique_ptr<CycleState> clone = st.Clone();
            for (int t = 0; t < 16; ++t)
                th.emplace_back([&, t] {
                    CycleState* s = t < 8 ? &st : clone.get();
                    for (size_t i = t; i < N; i += 16) {
                        fs[i] = ds->Filter(*s, pod, NodeInfo(&snap.nodes[i]));
                        ss[i] = ds->Score(*s, pod, snap.nodes[i].Name);
                    }
                });
            for (auto& x : th) x.join();
            for (size_t i = 0; i < N; ++i) {
                std::cout << "F\t" << pod.UID << "\t" << snap.nodes[i].Name << "\t" << (int)fs[i].code() << "\t"
                          << fs[i].message() << "\n";
                std::cout << "S\t" << pod.UID << "\t" << snap.nodes[i].Name << "\t" << ss[i].first << "\t"
                          << (int)ss[i].second.code() << "\t" << ss[i].second.message() << "\n";
            }
            // a clone of the evaluated cycle answers like its parent
            std::unique_ptr<CycleState> late = st.Clone();
            for (size_t i = 0; i < N; ++i)
                if (ds->Filter(*late, pod, NodeInfo(&snap.nodes[i])).code() != fs[i].code() ||
                    ds->Score(*late, pod, snap.nodes[i].Name).first != ss[i].first)
                    std::cout << "CLONE_MISMATCH\t" << i << "\n";
        } else if (f[0] == "pod" || f[0] == "nilnode" || f[0] == "missing") {
            Pod pod;
            pod.UID = f[1];
            pod.Name = f[1];
            CycleState st;
            st.now_ns = std::stoll(f[2]);
            if (f[0] == "nilnode") {
                Status s = ds->Filter(st, pod, NodeInfo(nullptr));
                std::cout << "F\t" << pod.UID << "\t-\t" << (int)s.code() << "\t" << s.message() << "\n";
                continue;
            }
            if (f[0] == "missing") {
                auto r = ds->Score(st, pod, f[3]);
                std::cout << "S\t" << pod.UID << "\t" << f[3] << "\t" << r.first << "\t" << (int)r.second.code()
                          << "\t" << r.second.message() << "\n";
                continue;
            }
            if (f[3] == "1") pod.OwnerReferences.push_back({"DaemonSet", "ds"});
            for (const auto& n : snap.nodes) {
                Status s = ds->Filter(st, pod, NodeInfo(&n));
                std::cout << "F\t" << pod.UID << "\t" << n.Name << "\t" << (int)s.code() << "\t" << s.message() << "\n";
                auto r = ds->Score(st, pod, n.Name);
                std::cout << "S\t" << pod.UID << "\t" << n.Name << "\t" << r.first << "\t" << (int)r.second.code()
                          << "\t" << r.second.message() << "\n";
            }
        }
    }
    return 0;
}
