// Sanitizer fuzz of the host-side parsers (tests/test_sanitize.py builds this with
// -fsanitize=address,undefined and runs it).  Test infrastructure: the oracle is
// linked here only as the checker.
//
//  1. annotation values "<float>,<timestamp>" (stats.go:51-76): random grammar
//     pieces + byte mutations; crane_parse_annotation (csrc/annotations.cpp) must
//     agree with the oracle's strconv.ParseFloat / time.ParseInLocation
//     restatement (or_parse_annotation) on usability, timestamp and value bits;
//  2. policy documents (policyfile.go:11-33): mutations of the default policy
//     through crane_policy_load_bytes (csrc/policy.cpp) — no crash, no leak, and a
//     loaded policy views consistently;
//  3. scheduler events (event.go:127-137): mutations of "Successfully assigned
//     ns/pod to node" through crane_translate_event (csrc/events.cpp) — no
//     crash, parts inside the message.
//
//  4. TZif files (tz.cpp, LoadLocationFromTZData): byte mutations and truncations
//     of real zone files through crane_tz_load_bytes, lookups and wall-clock
//     conversions with every zone that loads.
//
//   fuzz_parse <iterations> <seed> <policy.yaml> [tzif files...]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <string>

#include "crane_dyn.h"

extern "C" void or_parse_annotation(const char* s, int64_t n, int64_t tz_offset_s, uint8_t* ok, double* val,
                                    int64_t* ts_ns);

static std::mt19937_64 rng;
static uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }
static std::string pick(std::initializer_list<const char*> xs) {
    const uint64_t i = rnd(xs.size());
    return *(xs.begin() + i);
}

static std::string digits(int n) {
    std::string s;
    for (int i = 0; i < n; ++i) s += (char)('0' + rnd(10));
    return s;
}

static std::string rand_float() {
    switch (rnd(8)) {
        case 0: return pick({"inf", "+Inf", "-infinity", "NaN", "nan", "-0", "0", "1e308", "1e309", "4.9e-324",
                             "2e-324", "0x1p-2", "0x1.8p1", "1_000", "0x_1p0", ".5", "5.", "+.e1", "1e", "e1", ""});
        case 1: return digits(1 + (int)rnd(25));
        case 2: return digits(1 + (int)rnd(5)) + "." + digits((int)rnd(20));
        case 3: return digits(1 + (int)rnd(3)) + "e" + pick({"", "+", "-"}) + digits(1 + (int)rnd(4));
        case 4: return "0x" + digits(1 + (int)rnd(6)) + "p" + pick({"", "-", "+"}) + digits(1 + (int)rnd(3));
        case 5: return pick({"-", "+", " ", ""}) + "0." + digits((int)rnd(30));
        case 6: {
            char b[64];
            std::snprintf(b, sizeof b, "%.17g", std::ldexp((double)rng() / 18446744073709551616.0, (int)rnd(80) - 40));
            return b;
        }
        default: return std::to_string((int64_t)rng() >> rnd(64));
    }
}

static std::string rand_time() {
    auto f2 = [](int lo, int hi) {
        char b[8];
        std::snprintf(b, sizeof b, "%02d", lo + (int)rnd((uint64_t)(hi - lo + 1)));
        return std::string(b);
    };
    std::string y = rnd(4) ? std::to_string(1990 + rnd(120)) : digits(4);
    std::string s = y + "-" + f2(0, 13) + "-" + f2(0, 33) + "T" + f2(0, 25) + ":" + f2(0, 61) + ":" + f2(0, 61);
    if (rnd(8) == 0) s += "." + digits(1 + (int)rnd(10));
    if (rnd(10) == 0) s = s.substr(0, 11) + std::to_string(rnd(10)) + s.substr(13);  // one-digit hour
    return s + (rnd(12) ? "Z" : pick({"", "z", "+08:00", "ZZ"}));
}

static void mutate(std::string& s, int k) {
    for (int i = 0; i < k; ++i) {
        const uint64_t op = rnd(4), at = rnd(s.size() + 1);
        const char c = (char)(rnd(3) ? "0123456789,.:-TZe+x_ \t\n"[rnd(24)] : (char)rnd(256));
        if (op == 0) s.insert(s.begin() + (long)at, c);
        else if (op == 1 && !s.empty() && at < s.size()) s.erase(at, 1);
        else if (op == 2 && at < s.size()) s[at] = c;
        else if (op == 3 && !s.empty()) s = s.substr(0, at);
    }
}

static long n_usable = 0, n_policy_ok = 0, n_event_ok = 0;

static int fuzz_annotations(long iters) {
    for (long it = 0; it < iters; ++it) {
        std::string s = rand_float() + "," + rand_time();
        if (rnd(3) == 0) mutate(s, 1 + (int)rnd(3));
        const int64_t tz = (int64_t)rnd(3) * 3600 * (rnd(2) ? 8 : -5);
        double v = 0;
        int64_t ts = 0;
        // a heap copy with no terminator past n: ASan sees any over-read
        char* buf = (char*)std::malloc(s.size() ? s.size() : 1);
        std::memcpy(buf, s.data(), s.size());
        crane_parse_annotation(buf, s.size(), tz, &v, &ts);
        uint8_t ok = 0;
        double ov = 0;
        int64_t ots = 0;
        or_parse_annotation(buf, (int64_t)s.size(), tz, &ok, &ov, &ots);
        std::free(buf);
        const bool usable = ts != CRANE_TS_INVALID;
        n_usable += usable;
        bool same = usable == (ok != 0);
        if (same && usable) {
            uint64_t a, b;
            std::memcpy(&a, &v, 8);
            std::memcpy(&b, &ov, 8);
            same = ts == ots && (a == b || (std::isnan(v) && std::isnan(ov)));
        }
        if (!same) {
            std::fprintf(stderr, "annotation mismatch: \"%s\" tz %lld: engine (%d, %.17g, %lld) oracle (%d, %.17g, %lld)\n",
                         s.c_str(), (long long)tz, (int)usable, v, (long long)ts, (int)ok, ov, (long long)ots);
            return 1;
        }
    }
    return 0;
}

static int fuzz_policy(long iters, const std::string& base) {
    char err[256];
    for (long it = 0; it < iters; ++it) {
        std::string s = base;
        if (rnd(4) == 0) {  // line-level edits: drop / duplicate a line
            std::istringstream in(s);
            std::string line, out;
            const uint64_t target = rnd(48);
            uint64_t i = 0;
            while (std::getline(in, line)) {
                if (i++ == target) {
                    if (rnd(2)) continue;
                    out += line + "\n";
                }
                out += line + "\n";
            }
            s = out;
        }
        mutate(s, 1 + (int)rnd(6));
        crane_policy_doc* doc = nullptr;
        char* buf = (char*)std::malloc(s.size() ? s.size() : 1);
        std::memcpy(buf, s.data(), s.size());
        const int rc = crane_policy_load_bytes(buf, s.size(), &doc, err, sizeof err);
        std::free(buf);
        if (rc == 0) {
            ++n_policy_ok;
            const crane_policy* p = crane_policy_view(doc);
            if (!p || p->n_sync < 0 || p->n_pred < 0 || p->n_prio < 0 || p->n_hot < 0) {
                std::fprintf(stderr, "policy view inconsistent\n");
                return 1;
            }
            for (int32_t i = 0; i < p->n_sync; ++i) (void)std::strlen(p->sync_name[i]);
            for (int32_t i = 0; i < p->n_pred; ++i) (void)std::strlen(p->pred_name[i]);
            for (int32_t i = 0; i < p->n_prio; ++i) (void)std::strlen(p->prio_name[i]);
            crane_policy_free(doc);
        } else if (doc) {
            std::fprintf(stderr, "policy error left a document\n");
            return 1;
        }
    }
    return 0;
}

static int fuzz_events(long iters) {
    for (long it = 0; it < iters; ++it) {
        std::string s = "Successfully assigned " + pick({"default", "kube-system", "", "a/b"}) + "/" +
                        pick({"pod-1", "p", "", "x y"}) + " to " + pick({"node-7", "n", "", "node with space"});
        if (rnd(2)) mutate(s, 1 + (int)rnd(4));
        char* buf = (char*)std::malloc(s.size() ? s.size() : 1);
        std::memcpy(buf, s.data(), s.size());
        const char *node = nullptr, *ns = nullptr, *pod = nullptr;
        size_t nl = 0, nsl = 0, pl = 0;
        int64_t ts = 0;
        const int rc = crane_translate_event(buf, s.size(), (int32_t)rnd(3), (int64_t)(rng() >> 2),
                                             (int64_t)(rng() >> 2), &node, &nl, &ns, &nsl, &pod, &pl, &ts);
        if (rc == 0) {
            ++n_event_ok;
            auto inside = [&](const char* p, size_t n) { return !n || (p >= buf && p + n <= buf + s.size()); };
            if (!inside(node, nl) || !inside(ns, nsl) || !inside(pod, pl)) {
                std::fprintf(stderr, "event parts outside the message: \"%s\"\n", s.c_str());
                std::free(buf);
                return 1;
            }
        }
        std::free(buf);
    }
    return 0;
}

static long n_tz_ok = 0;

static int fuzz_tzif(long iters, const std::string& base) {
    for (long it = 0; it < iters; ++it) {
        std::string s = base;
        const int k = (int)rnd(4);
        for (int i = 0; i < k; ++i) {  // byte flips and truncations (headers, counts, footer)
            if (s.empty()) break;
            const uint64_t at = rnd(s.size());
            if (rnd(4) == 0) s = s.substr(0, at);
            else s[at] = (char)rnd(256);
        }
        uint8_t* buf = (uint8_t*)std::malloc(s.size() ? s.size() : 1);
        std::memcpy(buf, s.data(), s.size());
        crane_tz* tz = nullptr;
        const int rc = crane_tz_load_bytes(buf, s.size(), &tz);
        std::free(buf);
        if (rc == 0) {
            ++n_tz_ok;
            for (int j = 0; j < 8; ++j) {
                const int64_t t = (int64_t)(rng() % 8000000000ull) - 2000000000;
                int32_t off;
                int64_t st, en;
                // (no containment check: like Go's, a period from the footer rule after the DST
                // end runs to the year start + 365 days, a day short in leap years)
                crane_tz_lookup(tz, t, &off, &st, &en);
                (void)crane_tz_date(tz, t);
            }
            double v;
            int64_t ts;
            const std::string a = "0.5," + rand_time();
            crane_parse_annotation_tz(a.data(), a.size(), tz, &v, &ts);
            crane_tz_free(tz);
        } else if (tz) {
            std::fprintf(stderr, "tz error left a zone\n");
            return 1;
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const long iters = std::atol(argv[1]);
    rng.seed(std::strtoull(argv[2], nullptr, 10));
    std::ifstream f(argv[3]);
    std::stringstream ss;
    ss << f.rdbuf();
    int rc = fuzz_annotations(iters);
    if (!rc) rc = fuzz_policy(iters / 10, ss.str());
    if (!rc) rc = fuzz_events(iters / 4);
    for (int i = 4; i < argc && !rc; ++i) {
        std::ifstream zf(argv[i], std::ios::binary);
        std::stringstream zs;
        zs << zf.rdbuf();
        rc = fuzz_tzif(iters / 100, zs.str());
    }
    if (!rc)
        std::printf("ok %ld usable %ld policies %ld events %ld zones %ld\n", iters, n_usable, n_policy_ok, n_event_ok,
                    n_tz_ok);
    return rc;
}
