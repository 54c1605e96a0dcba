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
//   remove <i>               node i leaves the cluster: dropped from the snapshot, its NodeInfo and
//                            Node freed (their addresses may be reused by a later node)
//   pod <uid> <now_ns> <ds>  run Filter + Score of this pod on every node
//   nilnode <uid> <now_ns>   Filter with NodeInfo(nullptr)
//   missing <uid> <now_ns> <name>  Score of a node absent from the snapshot
//   mt <uid> <now_ns> <ds>   as pod, but Filter/Score called from 16 threads at once, half
//                            of them on a Clone() of the cycle state (preemption dry runs)
//   counters                 the plugin's sync counters
//   horizon <ns>             SetHorizon (a finite table span; default: the whole time axis)
//   devices <list>           Handle::devices for the next `policy` (comma-separated: the plugin's nodes
//                            sharded over them through the group, crane_dyn_group_*)
// The node-shard group through the C ABI (crane_dyn_group_*), over the same snapshot and policy:
//   group <devices> <depth> <collective> <threads>   crane_dyn_group_create over the comma-separated
//                            device list, options set, the snapshot's annotations parsed (the plugin's
//                            keys, $TZ) and uploaded whole (each device keeps its shard)
//   gbind <node> <ts_s>      a binding of global node <node> (collected; gbinds uploads them)
//   gbinds                   crane_dyn_group_upload_bindings of the collected log
//   gpod <now_ns> <ds>       a pod of the next batch
//   gsched <now_ns>          crane_dyn_group_schedule of the collected pods at <now_ns> (hot values
//                            from the bindings stamped now): "G <pod> <node> <score>" per pod
//   gshard <i>               "GS <i> <device> <lo> <hi>"
#include <iostream>
#include <memory>
#include <thread>
#include <sstream>
#include <string>
#include <vector>

#include "crane_dyn_plugin.hpp"

#include <cstdlib>

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
    crane_dyn_group* grp = nullptr;
    std::vector<int32_t> gbn;
    std::vector<int64_t> gbt, gnow;
    std::vector<uint8_t> gds;
    auto gcheck = [&](int rc, const char* what) {
        if (rc) std::cout << "GERR\t" << what << "\t" << crane_dyn_group_last_error(grp) << "\n";
        return rc == 0;
    };
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
        } else if (f[0] == "devices") {
            h.devices.clear();
            for (size_t a = 0, b; a <= f[1].size(); a = b + 1) {
                b = f[1].find(',', a);
                if (b == std::string::npos) b = f[1].size();
                h.devices.push_back((int32_t)std::stoi(f[1].substr(a, b - a)));
            }
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
        } else if (f[0] == "remove") {
            const size_t i = (size_t)std::stoll(f[1]);
            snap.list.erase(snap.list.begin() + (long)i);
            snap.infos.erase(snap.infos.begin() + (long)i);
            snap.objs.erase(snap.objs.begin() + (long)i);
        } else if (f[0] == "group") {
            std::vector<int32_t> devs;
            for (size_t a = 0, b; a <= f[1].size(); a = b + 1) {
                b = f[1].find(',', a);
                if (b == std::string::npos) b = f[1].size();
                devs.push_back((int32_t)std::stoi(f[1].substr(a, b - a)));
            }
            if (grp) crane_dyn_group_destroy(grp);
            grp = nullptr;
            if (!gcheck(crane_dyn_group_create(&ds->policy(), (int32_t)devs.size(), devs.data(), std::stoi(f[2]), &grp),
                        "create") ||
                !gcheck(crane_dyn_group_set_option(grp, "collective", std::stoll(f[3])), "collective") ||
                !gcheck(crane_dyn_group_set_option(grp, "threads", std::stoll(f[4])), "threads"))
                continue;
            // the snapshot's annotation strings, rows [metric slots..., node_hot_value][node]
            crane_dyn* e0 = crane_dyn_group_engine(grp, 0, 0);
            std::vector<std::string> keys;
            for (int32_t m = 0; m < crane_dyn_num_metrics(e0); ++m) keys.emplace_back(crane_dyn_metric_name(e0, m));
            keys.emplace_back(NodeHotValue);
            const size_t R = keys.size(), N = snap.objs.size();
            std::vector<const char*> strs(R * N, nullptr);
            std::vector<size_t> lens(R * N, 0);
            for (size_t i = 0; i < N; ++i)
                for (size_t m = 0; m < R; ++m) {
                    auto it = snap.node(i).Annotations.find(keys[m]);
                    if (it == snap.node(i).Annotations.end()) continue;
                    strs[m * N + i] = it->second.data();
                    lens[m * N + i] = it->second.size();
                }
            std::vector<double> val(R * N);
            std::vector<int64_t> ts(R * N);
            // (the plugin's zone: tzdata when present, else the fixed-offset table, as NewDynamicScheduler)
            crane_tz* zone = nullptr;
            const char* tzenv = std::getenv("TZ");
            const char* zname = tzenv && *tzenv ? tzenv : "Asia/Shanghai";
            int64_t off = 0;
            if (crane_tz_load(zname, nullptr, &zone) == 0) {
                crane_parse_annotations_tz((int64_t)(R * N), strs.data(), lens.data(), zone, val.data(), ts.data(), 4);
                crane_tz_free(zone);
            } else if (crane_tz_offset(zname, &off) == 0) {
                crane_parse_annotations((int64_t)(R * N), strs.data(), lens.data(), off, val.data(), ts.data(), 4);
            } else {
                std::cout << "GERR\tzone\n";
                continue;
            }
            const size_t M = R - 1;
            if (gcheck(crane_dyn_group_upload_nodes(grp, (int64_t)N, val.data(), ts.data(), val.data() + M * N,
                                                    ts.data() + M * N),
                       "upload_nodes"))
                std::cout << "GROUP\t" << crane_dyn_group_size(grp) << "\n";
        } else if (f[0] == "gbind") {
            gbn.push_back((int32_t)std::stoll(f[1]));
            gbt.push_back(std::stoll(f[2]));
        } else if (f[0] == "gbinds") {
            gcheck(crane_dyn_group_upload_bindings(grp, (int64_t)gbn.size(), gbn.data(), gbt.data()), "upload_bindings");
        } else if (f[0] == "gpod") {
            gnow.push_back(std::stoll(f[1]));
            gds.push_back((uint8_t)std::stoi(f[2]));
        } else if (f[0] == "gshard") {
            int32_t d = -1;
            int64_t lo = -1, hi = -1;
            crane_dyn_group_shard(grp, std::stoi(f[1]), &d, &lo, &hi);
            std::cout << "GS\t" << f[1] << "\t" << d << "\t" << lo << "\t" << hi << "\n";
        } else if (f[0] == "gsched") {
            const int64_t now = std::stoll(f[1]);
            std::vector<int64_t> ch(gnow.size()), sc(gnow.size());
            if (gcheck(crane_dyn_group_schedule(grp, now, now, (int64_t)gnow.size(), gnow.data(), gds.data(), ch.data(),
                                                sc.data()),
                       "schedule"))
                for (size_t p = 0; p < gnow.size(); ++p) std::cout << "G\t" << p << "\t" << ch[p] << "\t" << sc[p] << "\n";
            gnow.clear();
            gds.clear();
        } else if (f[0] == "horizon") {
            ds->SetHorizon(std::stoll(f[1]));
        } else if (f[0] == "counters") {
            const auto c = ds->counters();
            std::cout << "C\t" << c.tables_built << "\t" << c.full_syncs << "\t" << c.incremental_syncs << "\t"
                      << c.nodes_updated << "\t" << c.nodes_joined << "\t" << c.nodes_left << "\t" << c.grows << "\t"
                      << ds->Shards() << "\n";
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
    if (grp) crane_dyn_group_destroy(grp);
    return 0;
}
