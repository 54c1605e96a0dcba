// annotations.cpp — host parser for Dynamic-plugin node annotations.
//
// Value format written by the controller: "<float>,<local time>" —
// strconv.FormatFloat(v,'f',5,64) / strconv.Itoa for the value
// (pkg/controller/prometheus/prometheus.go:124, pkg/controller/annotator/node.go:120)
// and utils.GetLocalTime() = time.Now().In($TZ).Format("2006-01-02T15:04:05Z")
// (pkg/utils/utils.go:11,26-45) for the stamp, joined in node.go:142.
//
// The plugin re-reads it with strings.Split(v, ",") (exactly 2 parts),
// time.ParseInLocation(TimeFormat, parts[1], GetLocation()) and
// strconv.ParseFloat(parts[0], 64) (pkg/plugins/dynamic/stats.go:51-76).  This
// file restates those Go stdlib (go1.17) semantics so that parsing once per
// sync gives exactly the value/timestamp the reference would see per call.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/crane_dyn.h"

namespace {

inline int lower(int c) { return c | 0x20; }
inline bool digit(char c) { return c >= '0' && c <= '9'; }

int prefix_fold(const char* s, size_t n, const char* w) {
    size_t i = 0;
    while (i < n && w[i] && lower((unsigned char)s[i]) == w[i]) ++i;
    return (int)i;
}

// strconv.underscoreOK
bool underscores_ok(const char* s, size_t n) {
    char saw = '^';
    size_t i = 0;
    if (n >= 1 && (s[0] == '+' || s[0] == '-')) { ++s; --n; }
    bool hex = false;
    if (n >= 2 && s[0] == '0' && (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
        i = 2;
        saw = '0';
        hex = lower(s[1]) == 'x';
    }
    for (; i < n; ++i) {
        const char c = s[i];
        if (digit(c) || (hex && lower(c) >= 'a' && lower(c) <= 'f')) { saw = '0'; continue; }
        if (c == '_') {
            if (saw != '0') return false;
            saw = '_';
            continue;
        }
        if (saw == '_') return false;
        saw = '!';
    }
    return saw != '_';
}

}  // namespace

// strconv.ParseFloat(s, 64): true + value on success; false on ErrSyntax or
// ErrRange (the plugin treats both as an error, stats.go:66-69).
bool crane_go_parse_float(const char* s, size_t n, double* out) {
    *out = 0;
    if (n == 0) return false;
    // Fast path for the controller's own formats ([-]d+[.d*], FormatFloat 'f' /
    // Itoa): with the decimal mantissa <= 2^53 and at most 22 fraction digits,
    // mantissa / 10^k is one correctly rounded IEEE division of two exact
    // doubles, i.e. the same double strtod (and Go) return.  Anything else falls
    // through to the full grammar below.
    {
        static const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                       1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        size_t i = (s[0] == '-' || s[0] == '+') ? 1 : 0;
        const size_t d0 = i;
        uint64_t mant = 0;
        int nd = 0, frac = -1;
        for (; i < n; ++i) {
            const char c = s[i];
            if (digit(c)) {
                if (++nd > 19) break;
                mant = mant * 10 + (uint64_t)(c - '0');
                if (frac >= 0) ++frac;
            } else if (c == '.' && frac < 0 && i > d0) {
                frac = 0;
            } else {
                break;
            }
        }
        if (i == n && nd > 0 && mant <= (1ull << 53) && frac <= 22) {
            const double v = frac > 0 ? (double)mant / p10[frac] : (double)mant;
            *out = s[0] == '-' ? -v : v;
            return true;
        }
    }
    // special(): [+-]inf|infinity (case-folded), unsigned nan
    {
        size_t off = 0;
        double sign = 1;
        if (s[0] == '+' || s[0] == '-') { sign = s[0] == '-' ? -1 : 1; off = 1; }
        if (off < n && lower((unsigned char)s[off]) == 'i') {
            int k = prefix_fold(s + off, n - off, "infinity");
            if (k > 3 && k < 8) k = 3;
            if (k == 3 || k == 8) {
                if (off + (size_t)k != n) return false;
                *out = sign * INFINITY;
                return true;
            }
        } else if (off == 0 && lower((unsigned char)s[0]) == 'n') {
            if (prefix_fold(s, n, "nan") == 3) {
                if (n != 3) return false;
                *out = NAN;
                return true;
            }
        }
    }
    // readFloat() grammar
    size_t i = 0;
    bool unders = false, dot = false, digits = false;
    if (s[i] == '+' || s[i] == '-') ++i;
    bool hex = false;
    if (i + 2 < n && s[i] == '0' && lower(s[i + 1]) == 'x') { hex = true; i += 2; }
    for (; i < n; ++i) {
        const char c = s[i];
        if (c == '_') { unders = true; continue; }
        if (c == '.') {
            if (dot) break;
            dot = true;
            continue;
        }
        if (digit(c) || (hex && lower(c) >= 'a' && lower(c) <= 'f')) { digits = true; continue; }
        break;
    }
    if (!digits) return false;
    const char expc = hex ? 'p' : 'e';
    if (i < n && lower(s[i]) == expc) {
        ++i;
        if (i >= n) return false;
        if (s[i] == '+' || s[i] == '-') ++i;
        if (i >= n || !digit(s[i])) return false;
        for (; i < n && (digit(s[i]) || s[i] == '_'); ++i)
            if (s[i] == '_') unders = true;
    } else if (hex) {
        return false;  // a hex mantissa needs a 'p' exponent
    }
    if (unders && !underscores_ok(s, i)) return false;
    if (i != n) return false;  // trailing bytes
    char small[64];
    std::string big;
    char* buf = small;
    if (n >= sizeof small) {
        big.resize(n + 1);
        buf = &big[0];
    }
    size_t m = 0;
    for (size_t j = 0; j < n; ++j)
        if (s[j] != '_') buf[m++] = s[j];
    buf[m] = 0;
    char* end = nullptr;
    const double v = std::strtod(buf, &end);  // correctly rounded, like Go
    if (end != buf + m) return false;
    if (std::isinf(v)) return false;  // ErrRange on overflow; underflow is not an error in Go
    *out = v;
    return true;
}

namespace {

bool getnum(const char* s, size_t n, size_t* p, bool fixed, int* out) {
    const size_t i = *p;
    if (i >= n || !digit(s[i])) return false;
    if (i + 1 >= n || !digit(s[i + 1])) {
        if (fixed) return false;
        *out = s[i] - '0';
        *p = i + 1;
        return true;
    }
    *out = (s[i] - '0') * 10 + (s[i + 1] - '0');
    *p = i + 2;
    return true;
}

bool lit(const char* s, size_t n, size_t* p, char c) {
    if (*p >= n || s[*p] != c) return false;
    ++*p;
    return true;
}

int month_days(int m, int64_t y) {
    static const int d[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
    return (m == 2 && leap) ? 29 : d[m - 1];
}

// days since 1970-01-01 in the proleptic Gregorian calendar (Go's time.Date)
int64_t civil_days(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

}  // namespace

// time.ParseInLocation("2006-01-02T15:04:05Z", s, loc): the wall clock as
// seconds since the epoch taken as UTC (`local`) and the fraction.  Layout chunks
// (go1.17 time/format.go): stdLongYear '-' stdZeroMonth '-' stdZeroDay 'T'
// stdHour ':' stdZeroMinute ':' stdZeroSecond [.frac] 'Z' (a literal).
static bool parse_local(const char* s, size_t n, int64_t* local, int64_t* nsec_out) {
    // Fast path for the exact 20-byte stamp the controller writes: fixed
    // digit/separator positions, same range checks, and a per-thread memo of
    // the last date (a snapshot's stamps share a handful of days), so the
    // calendar arithmetic runs once per distinct date.  Anything else (a
    // fraction, one-digit hour, bad byte) takes the general path below.
    if (n == 20) {
        auto d2 = [&](int i) { return (s[i] - '0') * 10 + (s[i + 1] - '0'); };
        bool ok = s[4] == '-' && s[7] == '-' && s[10] == 'T' && s[13] == ':' && s[16] == ':' && s[19] == 'Z';
        for (int i : {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18}) ok = ok && digit(s[i]);
        if (ok) {
            const int year = d2(0) * 100 + d2(2), mon = d2(5), day = d2(8), hour = d2(11), min = d2(14),
                      sec = d2(17);
            if (mon < 1 || mon > 12 || day < 1 || day > 31 || hour > 23 || min > 59 || sec > 59) return false;
            thread_local int memo_key = -1;
            thread_local int64_t memo_days = 0;
            const int key = (year * 16 + mon) * 32 + day;  // one key per (year, mon, day): day <= 31
            if (key != memo_key) {
                if (day > month_days(mon, year)) return false;
                memo_days = civil_days(year, mon, day);
                memo_key = key;
            }
            *local = memo_days * 86400 + hour * 3600 + min * 60 + sec;
            *nsec_out = 0;
            return true;
        }
    }
    if (n < 4 || !digit(s[0])) return false;
    int year = 0;
    for (int k = 0; k < 4; ++k) {
        if (!digit(s[k])) return false;
        year = year * 10 + (s[k] - '0');
    }
    size_t p = 4;
    int mon, day, hour, min, sec;
    if (!lit(s, n, &p, '-') || !getnum(s, n, &p, true, &mon) || mon < 1 || mon > 12) return false;
    if (!lit(s, n, &p, '-') || !getnum(s, n, &p, true, &day)) return false;
    if (!lit(s, n, &p, 'T') || !getnum(s, n, &p, false, &hour) || hour > 23) return false;
    if (!lit(s, n, &p, ':') || !getnum(s, n, &p, true, &min) || min > 59) return false;
    if (!lit(s, n, &p, ':') || !getnum(s, n, &p, true, &sec) || sec > 59) return false;
    int64_t nsec = 0;
    if (n - p >= 2 && s[p] == '.' && digit(s[p + 1])) {  // fraction not in the layout: accepted
        size_t q = p + 2;
        while (q < n && digit(s[q])) ++q;
        const size_t nb = q - p, lim = nb > 10 ? 10 : nb;
        int64_t v = 0;
        for (size_t k = p + 1; k < p + lim; ++k) v = v * 10 + (s[k] - '0');
        for (size_t k = lim; k < 10; ++k) v *= 10;
        nsec = v;
        p = q;
    }
    if (!lit(s, n, &p, 'Z') || p != n) return false;
    if (day < 1 || day > month_days(mon, year)) return false;
    *local = civil_days(year, mon, day) * 86400 + hour * 3600 + min * 60 + sec;
    *nsec_out = nsec;
    return true;
}

// int64 ns spans 1678..2262; saturate so "long ago" stays stale and "far future"
// stays fresh, as with Go's wider Time
static int64_t to_ns(int64_t unix_s, int64_t nsec) {
    const __int128 t = (__int128)unix_s * 1000000000 + nsec;
    const __int128 lo = (__int128)INT64_MIN / 2, hi = (__int128)INT64_MAX / 2;
    return (int64_t)(t < lo ? lo : (t > hi ? hi : t));
}

// loc a fixed offset
bool crane_go_parse_time(const char* s, size_t n, int64_t tz_offset_s, int64_t* out_ns) {
    int64_t local, nsec;
    if (!parse_local(s, n, &local, &nsec)) return false;
    *out_ns = to_ns(local - tz_offset_s, nsec);
    return true;
}

// loc an IANA zone (tz.cpp: time.Date's offset choice)
bool crane_go_parse_time_tz(const char* s, size_t n, const crane_tz* tz, int64_t* out_ns) {
    int64_t local, nsec;
    if (!parse_local(s, n, &local, &nsec)) return false;
    *out_ns = to_ns(crane_tz_date(tz, local), nsec);
    return true;
}

extern "C" {

// utils.GetLocation (utils.go:35-45): $TZ, default Asia/Shanghai.  No tzdata
// is read: supported zones are those with a fixed offset for every
// timestamp a live controller can write (Asia/Shanghai = UTC+8 since 1991).
int crane_tz_offset(const char* tz_name, int64_t* offset_s) {
    std::string z = tz_name && *tz_name ? tz_name : "";
    if (z.empty()) {
        const char* env = std::getenv("TZ");
        z = env && *env ? env : "Asia/Shanghai";
    }
    static const struct { const char* name; int64_t off; } zones[] = {
        {"UTC", 0}, {"Etc/UTC", 0}, {"GMT", 0}, {"Etc/GMT", 0}, {"Universal", 0}, {"Zulu", 0},
        {"Asia/Shanghai", 8 * 3600}, {"Asia/Chongqing", 8 * 3600}, {"Asia/Harbin", 8 * 3600}, {"PRC", 8 * 3600},
        {"Asia/Singapore", 8 * 3600}, {"Asia/Taipei", 8 * 3600}, {"Asia/Tokyo", 9 * 3600}, {"Asia/Seoul", 9 * 3600},
        {"Asia/Kolkata", 19800},
    };
    for (const auto& e : zones)
        if (z == e.name) {
            *offset_s = e.off;
            return CRANE_OK;
        }
    if (z.rfind("Etc/GMT", 0) == 0 && z.size() > 7) {  // POSIX-inverted sign: Etc/GMT-8 = UTC+8
        char* end = nullptr;
        const long h = std::strtol(z.c_str() + 7, &end, 10);
        if (end && *end == 0 && h >= -14 && h <= 12) {
            *offset_s = -h * 3600;
            return CRANE_OK;
        }
    }
    return CRANE_E_INVALID;
}

}  // extern "C"

template <class ParseTime>
static void parse_annotation(const char* s, size_t n, double* value, int64_t* ts_ns, ParseTime&& parse_time) {
    *value = 0;
    *ts_ns = CRANE_TS_INVALID;
    size_t comma = (size_t)-1, ncomma = 0;
    for (size_t i = 0; i < n; ++i)
        if (s[i] == ',') {
            if (!ncomma) comma = i;
            ++ncomma;
        }
    if (ncomma != 1) return;  // strings.Split must give exactly two parts
    const char* t = s + comma + 1;
    const size_t tn = n - comma - 1;
    int64_t ts;
    if (tn < 5 || !parse_time(t, tn, &ts)) return;  // stats.go:31-40
    double v;
    if (!crane_go_parse_float(s, comma, &v)) return;
    *value = v;
    *ts_ns = ts;
}

template <class One>
static int parse_bulk(int64_t n, const char* const* strs, const size_t* lens, double* value, int64_t* ts_ns,
                      int32_t n_threads, One&& one) {
    if (n < 0 || (n > 0 && (!strs || !lens || !value || !ts_ns))) return CRANE_E_INVALID;
    int64_t nt = n_threads > 0 ? n_threads : (int64_t)std::thread::hardware_concurrency();
    if (nt < 1) nt = 1;
    // >= 32k strings per thread: a thread parses ~1e7 strings/s, so spawning one costs
    // more than it saves below that (measured: 170 threads on a 700k-string snapshot
    // 4.6 ms, 16 threads 1.7 ms)
    nt = std::min<int64_t>(nt, std::max<int64_t>(1, n / 32768));
    auto work = [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            if (!strs[i]) {
                value[i] = 0;
                ts_ns[i] = CRANE_TS_INVALID;  // key not found (stats.go:52-55)
            } else {
                one(strs[i], lens[i], &value[i], &ts_ns[i]);
            }
        }
    };
    if (nt == 1) {
        work(0, n);
        return CRANE_OK;
    }
    std::vector<std::thread> th;
    for (int64_t t = 0; t < nt; ++t) th.emplace_back(work, n * t / nt, n * (t + 1) / nt);
    for (auto& x : th) x.join();
    return CRANE_OK;
}

extern "C" {

void crane_parse_annotation(const char* s, size_t n, int64_t tz_offset_s, double* value, int64_t* ts_ns) {
    parse_annotation(s, n, value, ts_ns,
                     [&](const char* t, size_t tn, int64_t* o) { return crane_go_parse_time(t, tn, tz_offset_s, o); });
}

void crane_parse_annotation_tz(const char* s, size_t n, const crane_tz* tz, double* value, int64_t* ts_ns) {
    parse_annotation(s, n, value, ts_ns,
                     [&](const char* t, size_t tn, int64_t* o) { return crane_go_parse_time_tz(t, tn, tz, o); });
}

int crane_parse_annotations(int64_t n, const char* const* strs, const size_t* lens, int64_t tz_offset_s,
                            double* value, int64_t* ts_ns, int32_t n_threads) {
    return parse_bulk(n, strs, lens, value, ts_ns, n_threads, [&](const char* s, size_t l, double* v, int64_t* t) {
        crane_parse_annotation(s, l, tz_offset_s, v, t);
    });
}

int crane_parse_annotations_tz(int64_t n, const char* const* strs, const size_t* lens, const crane_tz* tz,
                               double* value, int64_t* ts_ns, int32_t n_threads) {
    if (!tz) return CRANE_E_INVALID;
    return parse_bulk(n, strs, lens, value, ts_ns, n_threads, [&](const char* s, size_t l, double* v, int64_t* t) {
        crane_parse_annotation_tz(s, l, tz, v, t);
    });
}

}  // extern "C"
