// Drives crane::dynamic::DynamicScheduler (include/crane_dyn_plugin.hpp) from a
// tab-separated script on stdin, printing every Filter/Score result.  Used by
// tests/test_plugin_cpp.py.
//   policy <path>            NewDynamicScheduler(DynamicArgs{path})
//   badargs                  NewDynamicScheduler(<not DynamicArgs>)
//   node <name>              start a node
//   anno <key> <value>       annotation of the current node
//   patch <i> <key> <value>  the controller's patch of node i's annotation (the informer publishes a
//                            new Node object and bumps the NodeInfo's Generation; the old object
//                            is freed, so its address may be reused)
//   unset <i> <key>          the same with the annotation removed
//   pod <uid> <now_ns> <ds>  run Filter + Score of this pod on every node
//   nilnode <uid> <now_ns>   Filter with NodeInfo(nullptr)
//   missing <uid> <now_ns> <name>  Score of a node absent from the snapshot
//   mt <uid> <now_ns> <ds>   as pod, but Filter/Score called from 16 threads at once, half
//                            of them on a Clone() of the cycle state (preemption dry runs)
//   counters                 the plugin's sync counters
#include <iostream>
#include <memory>
#include <thread>
#include <sstream>
#include <string>
#include <vector>

#include "crane_dyn_plugin.hpp"

using namespace crane::dynamic;

struct Snap : Snapshot {
    std::vector<std::unique_ptr<Node>> objs;       // the current Node object of each node
    std::vector<std::unique_ptr<NodeInfo>> infos;  // stable NodeInfo objects
    std::vector<const NodeInfo*> list;
    int64_t gen = 0;
    const std::vector<const NodeInfo*>& List() const override { return list; }
    // (linear Get: small test snapshots)
    const NodeInfo* Get(const std::string& name, std::string* err) const override {
        for (const auto& ni : infos)
            if (ni->node()->Name == name) return ni.get();
        *err = "nodeinfo not found for node name \"" + name + "\"";
        return nullptr;
    }
    void add(const std::string& name) {
        objs.emplace_back(new Node{name, {}});
        infos.emplace_back(new NodeInfo(objs.back().get(), ++gen));
        list.push_back(infos.back().get());
    }
    // an update: a new Node object replaces the old one (which is freed)
    void replace(size_t i, const std::string& key, const std::string* value) {
        std::unique_ptr<Node> n(new Node(*objs[i]));
        if (value) n->Annotations[key] = *value;
        else n->Annotations.erase(key);
        infos[i]->SetNode(n.get());
        infos[i]->Generation = ++gen;
        objs[i] = std::move(n);
    }
    const Node& node(size_t i) const { return *objs[i]; }
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
            snap.add(f[1]);
        } else if (f[0] == "anno") {
            const std::string v = f.size() > 2 ? f[2] : "";
            snap.replace(snap.objs.size() - 1, f[1], &v);
        } else if (f[0] == "patch") {
            const std::string v = f.size() > 3 ? f[3] : "";
            snap.replace((size_t)std::stoll(f[1]), f[2], &v);
        } else if (f[0] == "unset") {
            snap.replace((size_t)std::stoll(f[1]), f[2], nullptr);
        } else if (f[0] == "counters") {
            const auto c = ds->counters();
            std::cout << "C\t" << c.tables_built << "\t" << c.full_syncs << "\t" << c.incremental_syncs << "\t"
                      << c.nodes_updated << "\n";
        } else if (f[0] == "mt") {
            Pod pod;
            pod.UID = pod.Name = f[1];
            if (f[3] == "1") pod.OwnerReferences.push_back({"DaemonSet", "ds"});
            CycleState st;
            st.now_ns = std::stoll(f[2]);
            const size_t N = snap.list.size();
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
                        fs[i] = ds->Filter(*s, pod, *snap.list[i]);
                        ss[i] = ds->Score(*s, pod, snap.node(i).Name);
                    }
                });
            for (auto& x : th) x.join();
            for (size_t i = 0; i < N; ++i) {
                std::cout << "F\t" << pod.UID << "\t" << snap.node(i).Name << "\t" << (int)fs[i].code() << "\t"
                          << fs[i].message() << "\n";
                std::cout << "S\t" << pod.UID << "\t" << snap.node(i).Name << "\t" << ss[i].first << "\t"
                          << (int)ss[i].second.code() << "\t" << ss[i].second.message() << "\n";
            }
            // a clone of the evaluated cycle answers like its parent
            std::unique_ptr<CycleState> late = st.Clone();
            for (size_t i = 0; i < N; ++i)
                if (ds->Filter(*late, pod, *snap.list[i]).code() != fs[i].code() ||
                    ds->Score(*late, pod, snap.node(i).Name).first != ss[i].first)
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
            for (size_t i = 0; i < snap.list.size(); ++i) {
                const Node& n = snap.node(i);
                // odd nodes through a NodeInfo that is not the snapshot's (found by name)
                const NodeInfo tmp(&n);
                Status s = ds->Filter(st, pod, i % 2 ? tmp : *snap.list[i]);
                std::cout << "F\t" << pod.UID << "\t" << n.Name << "\t" << (int)s.code() << "\t" << s.message() << "\n";
                auto r = ds->Score(st, pod, n.Name);
                std::cout << "S\t" << pod.UID << "\t" << n.Name << "\t" << r.first << "\t" << (int)r.second.code()
                          << "\t" << r.second.message() << "\n";
            }
        }
    }
    return 0;
}
