// Latency of crane_dyn_update_node_steps (the drop-in's per-cycle engine call) after the engine
// sat idle for a given gap, at 100k nodes: does the first update after the initial sync pay for
// the time since the last GPU work?  Prints one line per gap: the update's wall time (three
// updates per gap, each after the gap).  Usage: update_gap_probe <policy.yaml>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#include "crane_dyn.h"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    // a host thread started before the engine exists (a framework goroutine's thread), used at
    // the end: its first update
    std::mutex pm;
    std::condition_variable pcv;
    int ptask = 0;  // 1: run the update, 2: done
    std::function<double(int64_t)> pupdate;
    double pfirst = 0, psecond = 0;
    std::thread pre([&] {
        std::unique_lock<std::mutex> l(pm);
        pcv.wait(l, [&] { return ptask == 1; });
        pfirst = pupdate(40);
        psecond = pupdate(41);
        ptask = 2;
        pcv.notify_all();
    });
    crane_policy_doc* doc = nullptr;
    char err[512];
    if (crane_policy_load_file(argv[1], &doc, err, sizeof err)) {
        std::fprintf(stderr, "policy: %s\n", err);
        return 1;
    }
    crane_dyn* h = nullptr;
    if (crane_dyn_create(crane_policy_view(doc), 0, &h)) {
        std::fprintf(stderr, "create: %s\n", crane_dyn_last_error(h));
        return 1;
    }
    const int64_t N = 100000, M = crane_dyn_num_metrics(h);
    const int64_t now = 1700000000LL * 1000000000LL;
    std::vector<double> val((size_t)(M * N));
    std::vector<int64_t> ts((size_t)(M * N));
    std::vector<double> hv((size_t)N);
    std::vector<int64_t> hvt((size_t)N, now - 60LL * 1000000000LL);
    for (int64_t m = 0; m < M; ++m)
        for (int64_t i = 0; i < N; ++i) {
            val[(size_t)(m * N + i)] = (double)((i * 7919 + m * 131) % 1000) / 1000.0;
            ts[(size_t)(m * N + i)] = now - (int64_t)((i * 104729 + m) % 600) * 1000000000LL;
        }
    for (int64_t i = 0; i < N; ++i) hv[(size_t)i] = (double)(i % 5);
    if (crane_dyn_upload_nodes(h, N, 0, val.data(), ts.data(), hv.data(), hvt.data())) {
        std::fprintf(stderr, "upload: %s\n", crane_dyn_last_error(h));
        return 1;
    }
    const int64_t S = crane_dyn_step_slots(h);
    std::vector<uint8_t> ns((size_t)N);
    std::vector<int64_t> bp((size_t)(N * S));
    std::vector<int8_t> ff((size_t)(N * (S + 1))), sc((size_t)(N * (S + 1)));
    if (crane_dyn_node_steps(h, INT64_MIN, INT64_MAX, N, ns.data(), bp.data(), ff.data(), sc.data())) {
        std::fprintf(stderr, "node_steps: %s\n", crane_dyn_last_error(h));
        return 1;
    }
    using Clock = std::chrono::steady_clock;
    std::vector<double> cv((size_t)(M + 1));
    std::vector<int64_t> ct((size_t)(M + 1));
    auto update = [&](int64_t row) {
        for (int64_t m = 0; m < M; ++m) {
            cv[(size_t)m] = val[(size_t)(m * N + row)];
            ct[(size_t)m] = ts[(size_t)(m * N + row)];
        }
        cv[(size_t)M] = hv[(size_t)row];
        ct[(size_t)M] = hvt[(size_t)row];
        const auto t0 = Clock::now();
        if (crane_dyn_update_node_steps(h, 1, &row, cv.data(), ct.data(), cv.data() + M, ct.data() + M, INT64_MIN,
                                        INT64_MAX, &ns[(size_t)row], &bp[(size_t)(row * S)],
                                        &ff[(size_t)(row * (S + 1))], &sc[(size_t)(row * (S + 1))])) {
            std::fprintf(stderr, "update: %s\n", crane_dyn_last_error(h));
            return -1.0;
        }
        return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    };
    std::printf("first update after the table build: %.3f ms\n", update(0));
    for (int gap_us : {0, 100, 1000, 3000, 10000, 30000, 100000, 300000, 1000000}) {
        std::printf("gap %7d us:", gap_us);
        for (int r = 0; r < 3; ++r) {
            std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
            std::printf(" %.3f", update(1 + r));
        }
        std::printf(" ms\n");
        std::fflush(stdout);
    }
    // the same after a gap during which 16 threads read the answer tables (a drop-in cycle's
    // Filter / Score fan-out), then with them spinning through the update
    std::vector<std::thread> th;
    std::atomic<bool> stop{false};
    std::atomic<int64_t> sink{0};
    for (int gap_us : {1000, 10000, 100000}) {
        std::printf("busy gap %7d us:", gap_us);
        for (int r = 0; r < 3; ++r) {
            stop = false;
            for (int t = 0; t < 16; ++t)
                th.emplace_back([&, t] {
                    int64_t acc = 0;
                    size_t i = (size_t)t * 4096;
                    while (!stop.load(std::memory_order_relaxed)) {
                        acc += sc[i % sc.size()] + bp[i % bp.size()];
                        i += 64;
                    }
                    sink += acc;
                });
            std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
            const double ms = update(10 + r);
            stop = true;
            for (auto& x : th) x.join();
            th.clear();
            std::printf(" %.3f", ms);
        }
        std::printf(" ms\n");
        std::fflush(stdout);
    }
    // the update from host threads that have not called HIP before (a drop-in cycle's leader is
    // whichever framework thread calls Filter first), and again from each
    for (int t = 0; t < 3; ++t) {
        double first = 0, second = 0;
        std::thread x([&] {
            first = update(20 + t);
            second = update(30 + t);
        });
        x.join();
        std::printf("new thread %d: first %.3f ms, second %.3f ms\n", t, first, second);
        std::fflush(stdout);
    }
    pupdate = update;
    {
        std::unique_lock<std::mutex> l(pm);
        ptask = 1;
        pcv.notify_all();
        pcv.wait(l, [&] { return ptask == 2; });
    }
    pre.join();
    std::printf("thread started before the engine: first %.3f ms, second %.3f ms\n", pfirst, psecond);
    crane_dyn_destroy(h);
    crane_policy_free(doc);
    return 0;
}
