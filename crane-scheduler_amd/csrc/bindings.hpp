// bindings.hpp — BindingRecords (pkg/controller/annotator/binding.go:50-123)
// kept on the host next to the device binding log.
//
// The reference keeps the recent bindings in a container/heap min-heap over
// Binding.Timestamp: AddBinding pops the minimum when the heap holds `size`
// entries (binding.go:69-78) and BindingsGC pops every entry with Timestamp <=
// now - gcTimeRange, pushing the first younger one back (binding.go:100-123).
// Which of several equal-timestamp entries leaves the heap depends on the
// heap's swap sequence, so the heap is restated operation for operation
// (go1.17 src/container/heap/heap.go: Push = append + up, Pop = swap(0, n-1) +
// down + remove last).  Each heap entry owns a slot of the device log (node,
// timestamp); a pop frees its slot (node = -1: counts for no node), a push takes
// the most recently freed slot.  The slots a call changed are re-uploaded as
// contiguous runs, so a controller sync moves only its new bindings to HBM.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <utility>
#include <vector>

namespace crane {

class BindingHeap {
   public:
    void reset(int64_t size, int64_t gc_time_range_ns) {
        h_.clear();
        free_.clear();
        dirty_.clear();
        size_ = size;
        gc_tr_ns_ = gc_time_range_ns;
        next_ = 0;
        node_ = nullptr;
        ts_ = nullptr;
    }
    void bind(int32_t* node, int64_t* ts) {  // slot mirror, `size` entries
        node_ = node;
        ts_ = ts;
    }
    int64_t len() const { return (int64_t)h_.size(); }

    // AddBinding (binding.go:69-78)
    void add(int32_t node, int64_t ts) {
        if ((int64_t)h_.size() == size_) release(pop());
        int32_t slot;
        if (!free_.empty()) {
            slot = free_.back();
            free_.pop_back();
        } else {
            slot = (int32_t)next_++;
        }
        node_[slot] = node;
        ts_[slot] = ts;
        dirty_.push_back(slot);
        push(E{ts, slot});
    }

    // BindingsGC (binding.go:100-123) at time.Now().UTC().Unix() = now_unix
    void gc(int64_t now_unix) {
        if (gc_tr_ns_ == 0) return;
        const int64_t timeline = now_unix - seconds_trunc(gc_tr_ns_);
        while (!h_.empty()) {
            const E b = pop();
            if (b.ts > timeline) {
                push(b);
                return;
            }
            release(b);
        }
    }

    // slots changed since the last call, as sorted [lo, hi) runs
    void take_dirty_runs(std::vector<std::pair<int64_t, int64_t>>* runs) {
        runs->clear();
        if (dirty_.empty()) return;
        std::sort(dirty_.begin(), dirty_.end());
        dirty_.erase(std::unique(dirty_.begin(), dirty_.end()), dirty_.end());
        for (int32_t s : dirty_) {
            if (!runs->empty() && runs->back().second == s) runs->back().second = s + 1;
            else runs->emplace_back(s, s + 1);
        }
        if (runs->size() > 64) {  // scattered: one copy of the covering range
            const int64_t lo = runs->front().first, hi = runs->back().second;
            runs->assign(1, {lo, hi});
        }
        dirty_.clear();
    }

   private:
    struct E {
        int64_t ts;
        int32_t slot;
    };
    // int64(d.Seconds()) for a Duration (binding.go:85, 110)
    static int64_t seconds_trunc(int64_t d) {
        const double s = (double)(d / 1000000000LL) + (double)(d % 1000000000LL) / 1e9;
        if (!(s >= -9223372036854775808.0 && s < 9223372036854775808.0)) return INT64_MIN;
        return (int64_t)s;
    }
    bool less(size_t i, size_t j) const { return h_[i].ts < h_[j].ts; }  // BindingHeap.Less
    void up(size_t j) {
        for (;;) {
            const size_t i = j == 0 ? 0 : (j - 1) / 2;  // Go: (j-1)/2 truncates to 0 at j = 0
            if (i == j || !less(j, i)) break;
            std::swap(h_[i], h_[j]);
            j = i;
        }
    }
    void down(size_t i, size_t n) {
        for (;;) {
            const size_t j1 = 2 * i + 1;
            if (j1 >= n) break;
            size_t j = j1;
            if (j1 + 1 < n && less(j1 + 1, j1)) j = j1 + 1;
            if (!less(j, i)) break;
            std::swap(h_[i], h_[j]);
            i = j;
        }
    }
    void push(const E& e) {  // heap.Push
        h_.push_back(e);
        up(h_.size() - 1);
    }
    E pop() {  // heap.Pop
        const size_t n = h_.size() - 1;
        std::swap(h_[0], h_[n]);
        down(0, n);
        const E e = h_.back();
        h_.pop_back();
        return e;
    }
    void release(const E& e) {
        node_[e.slot] = -1;
        dirty_.push_back(e.slot);
        free_.push_back(e.slot);
    }

    std::vector<E> h_;
    std::vector<int32_t> free_, dirty_;
    int64_t size_ = 0, gc_tr_ns_ = 0, next_ = 0;
    int32_t* node_ = nullptr;
    int64_t* ts_ = nullptr;
};

}  // namespace crane
