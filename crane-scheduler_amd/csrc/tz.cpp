// tz.cpp — IANA time zones for the annotation timestamps, with Go's semantics.
//
// The reference parses every annotation stamp with time.ParseInLocation in
// utils.GetLocation() = time.LoadLocation($TZ, default Asia/Shanghai)
// (pkg/utils/utils.go:35-45, stats.go:36-40).  go1.17 (go.mod:3) reads the
// zone from a TZif file ($ZONEINFO, then /usr/share/zoneinfo, ...; the
// reference image installs tzdata, Dockerfile:30) and turns a wall-clock time
// into an instant with time.Date: look the zone up at the wall time taken as
// UTC, and again at the corrected instant if that falls outside the zone
// period found (so a skipped or repeated wall time gets one of its two
// offsets, as Go's own algorithm picks).  Restated here from the published
// go1.17 sources (time/zoneinfo_read.go LoadLocationFromTZData,
// time/zoneinfo.go lookup, lookupFirstZone, tzset*, tzruleTime, time/time.go
// Date); the checker is oracle/tz.py, an independent Python restatement.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/crane_dyn.h"

namespace {

constexpr int64_t kAlpha = INT64_MIN, kOmega = INT64_MAX;  // Go's alpha / omega
constexpr int64_t kSecPerDay = 86400;

struct Zone {
    int32_t offset;
    bool isdst;
};
struct Rule {  // tzset rule
    int kind = 0;  // 0 Julian (J n), 1 day of year (n), 2 month-week-day (M m.w.d)
    int day = 0, week = 0, mon = 0;
    int time = 2 * 3600;
};

bool is_leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }

int64_t days_from_civil(int64_t y, int m, int d) {  // days since 1970-01-01 (proleptic Gregorian)
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

// year and day of year (0-based) of the UTC instant sec (Go's absDate, yday from 0)
void year_yday(int64_t sec, int64_t* year, int64_t* yday) {
    int64_t days = sec / kSecPerDay;
    if (sec % kSecPerDay < 0) --days;  // floor
    // civil from days (inverse of days_from_civil)
    int64_t z = days + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    const int64_t m = mp + (mp < 10 ? 3 : -9);
    y += m <= 2;
    *year = y;
    *yday = days - days_from_civil(y, 1, 1);
}

// tzsetNum / tzsetOffset / tzsetName / tzsetRule (time/zoneinfo.go)
bool tz_num(const std::string& s, size_t& p, int mn, int mx, int* out) {
    if (p >= s.size()) return false;
    int num = 0;
    size_t i = p;
    for (; i < s.size(); ++i) {
        const char r = s[i];
        if (r < '0' || r > '9') {
            if (i == p || num < mn) return false;
            *out = num;
            p = i;
            return true;
        }
        num = num * 10 + (r - '0');
        if (num > mx) return false;
    }
    if (num < mn) return false;
    *out = num;
    p = i;
    return true;
}

bool tz_offset(const std::string& s, size_t& p, int* out) {
    if (p >= s.size()) return false;
    bool neg = false;
    if (s[p] == '+') ++p;
    else if (s[p] == '-') {
        ++p;
        neg = true;
    }
    int hours;
    if (!tz_num(s, p, 0, 24 * 7, &hours)) return false;
    int off = hours * 3600;
    if (p < s.size() && s[p] == ':') {
        ++p;
        int mins;
        if (!tz_num(s, p, 0, 59, &mins)) return false;
        off += mins * 60;
        if (p < s.size() && s[p] == ':') {
            ++p;
            int secs;
            if (!tz_num(s, p, 0, 59, &secs)) return false;
            off += secs;
        }
    }
    *out = neg ? -off : off;
    return true;
}

bool tz_name(const std::string& s, size_t& p) {
    if (p >= s.size()) return false;
    if (s[p] != '<') {
        for (size_t i = p; i < s.size(); ++i) {
            const char r = s[i];
            if ((r >= '0' && r <= '9') || r == ',' || r == '-' || r == '+') {
                if (i - p < 3) return false;
                p = i;
                return true;
            }
        }
        if (s.size() - p < 3) return false;
        p = s.size();
        return true;
    }
    for (size_t i = p; i < s.size(); ++i)
        if (s[i] == '>') {
            p = i + 1;
            return true;
        }
    return false;
}

bool tz_rule(const std::string& s, size_t& p, Rule* r) {
    if (p >= s.size()) return false;
    if (s[p] == 'J') {
        ++p;
        if (!tz_num(s, p, 1, 365, &r->day)) return false;
        r->kind = 0;
    } else if (s[p] == 'M') {
        ++p;
        if (!tz_num(s, p, 1, 12, &r->mon) || p >= s.size() || s[p] != '.') return false;
        ++p;
        if (!tz_num(s, p, 1, 5, &r->week) || p >= s.size() || s[p] != '.') return false;
        ++p;
        if (!tz_num(s, p, 0, 6, &r->day)) return false;
        r->kind = 2;
    } else {
        if (!tz_num(s, p, 0, 365, &r->day)) return false;
        r->kind = 1;
    }
    if (p >= s.size() || s[p] != '/') {
        r->time = 2 * 3600;
        return true;
    }
    ++p;
    return tz_offset(s, p, &r->time);
}

int tz_rule_time(int64_t year, const Rule& r, int off) {  // tzruleTime: seconds into the year, UTC
    static const int before[13] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334, 365};
    int s = 0;
    if (r.kind == 0) {
        s = (r.day - 1) * 86400;
        if (is_leap(year) && r.day >= 60) s += 86400;
    } else if (r.kind == 1) {
        s = r.day * 86400;
    } else {
        const int m1 = (r.mon + 9) % 12 + 1;  // Zeller's congruence
        int64_t yy0 = year;
        if (r.mon <= 2) --yy0;
        const int64_t yy1 = yy0 / 100, yy2 = yy0 % 100;
        int dow = (int)(((26 * m1 - 2) / 10 + 1 + yy2 + yy2 / 4 + yy1 / 4 - 2 * yy1) % 7);
        if (dow < 0) dow += 7;
        int d = r.day - dow;
        if (d < 0) d += 7;
        const int dim = before[r.mon] - before[r.mon - 1] + ((r.mon == 2 && is_leap(year)) ? 1 : 0);
        for (int i = 1; i < r.week; ++i) {
            if (d + 7 >= dim) break;
            d += 7;
        }
        d += before[r.mon - 1];
        if (is_leap(year) && r.mon > 2) ++d;
        s = d * 86400;
    }
    return s + r.time - off;
}

// tzset(s, initEnd, sec): offset, start, end of the zone period holding sec
bool tz_set(const std::string& s, int64_t init_end, int64_t sec, int32_t* offset, int64_t* start, int64_t* end) {
    size_t p = 0;
    int std_off, dst_off;
    if (!tz_name(s, p) || !tz_offset(s, p, &std_off)) return false;
    std_off = -std_off;  // POSIX offsets are added to local time to get UTC
    if (p >= s.size() || s[p] == ',') {  // no daylight saving time
        *offset = std_off;
        *start = init_end;
        *end = kOmega;
        return true;
    }
    if (!tz_name(s, p)) return false;
    if (p >= s.size() || s[p] == ',') {
        dst_off = std_off + 3600;
    } else {
        if (!tz_offset(s, p, &dst_off)) return false;
        dst_off = -dst_off;
    }
    std::string rules = p >= s.size() ? std::string(",M3.2.0,M11.1.0") : s.substr(p);  // tzcode's default
    if (rules[0] != ',' && rules[0] != ';') return false;
    size_t q = 1;
    Rule sr, er;
    if (!tz_rule(rules, q, &sr) || q >= rules.size() || rules[q] != ',') return false;
    ++q;
    if (!tz_rule(rules, q, &er) || q != rules.size()) return false;
    int64_t year, yday;
    year_yday(sec, &year, &yday);
    const int64_t ysec = yday * kSecPerDay + sec % kSecPerDay;  // (Go's % truncates)
    const int64_t abs = days_from_civil(year, 1, 1) * kSecPerDay;
    int64_t ss = tz_rule_time(year, sr, std_off), es = tz_rule_time(year, er, dst_off);
    int32_t so = std_off, doff = dst_off;
    if (es < ss) {  // southern hemisphere: the labels flip
        std::swap(ss, es);
        std::swap(so, doff);
    }
    if (ysec < ss) {
        *offset = so;
        *start = abs;
        *end = ss + abs;
    } else if (ysec >= es) {
        *offset = so;
        *start = es + abs;
        *end = abs + 365 * kSecPerDay;
    } else {
        *offset = doff;
        *start = ss + abs;
        *end = es + abs;
    }
    return true;
}

uint32_t be32(const uint8_t* b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; }
uint64_t be64(const uint8_t* b) { return (uint64_t)be32(b) << 32 | be32(b + 4); }

}  // namespace

struct crane_tz {
    std::vector<Zone> zone;
    std::vector<int64_t> tx_when;
    std::vector<uint8_t> tx_index;
    std::string extend;
    int first_zone = 0;

    // time/zoneinfo.go lookup: the zone in effect at the UTC instant sec, and its period
    void lookup(int64_t sec, int32_t* offset, int64_t* start, int64_t* end) const {
        if (zone.empty()) {
            *offset = 0;
            *start = kAlpha;
            *end = kOmega;
            return;
        }
        if (tx_when.empty() || sec < tx_when[0]) {
            *offset = zone[first_zone].offset;
            *start = kAlpha;
            *end = tx_when.empty() ? kOmega : tx_when[0];
            return;
        }
        int64_t e = kOmega;
        size_t lo = 0, hi = tx_when.size();
        while (hi - lo > 1) {
            const size_t m = lo + (hi - lo) / 2;
            if (sec < tx_when[m]) {
                e = tx_when[m];
                hi = m;
            } else {
                lo = m;
            }
        }
        *offset = zone[tx_index[lo]].offset;
        *start = tx_when[lo];
        *end = e;
        if (lo == tx_when.size() - 1 && !extend.empty()) {
            int32_t eo;
            int64_t es, ee;
            if (tz_set(extend, e, sec, &eo, &es, &ee)) {
                *offset = eo;
                *start = es;
                *end = ee;
            }
        }
    }

    // time.Date: the instant of the wall clock `local` (seconds, as if UTC) in this zone;
    // go1.17 re-looks the zone up at start-1 (utc < start) or at end (utc >= end)
    int64_t date(int64_t local) const {
        int32_t off;
        int64_t start, end;
        lookup(local, &off, &start, &end);
        if (off != 0) {
            const int64_t utc = local - off;
            int64_t s2, e2;
            if (utc < start)
                lookup(start - 1, &off, &s2, &e2);
            else if (utc >= end)
                lookup(end, &off, &s2, &e2);
            local -= off;
        }
        return local;
    }
};

// LoadLocationFromTZData (time/zoneinfo_read.go, go1.17)
static bool tz_parse(const uint8_t* d, size_t n, crane_tz* z) {
    if (n < 44 || std::memcmp(d, "TZif", 4) != 0) return false;
    // go1.17 reads versions 1 ('\0'), '2' and '3' only
    const int version = d[4] == 0 ? 1 : ((d[4] == '2' || d[4] == '3') ? 2 : 0);
    if (version == 0) return false;
    auto counts = [&](const uint8_t* h, uint32_t* c) {  // isutcnt isstdcnt leapcnt timecnt typecnt charcnt
        for (int i = 0; i < 6; ++i) c[i] = be32(h + 20 + 4 * i);
    };
    uint32_t c[6];
    counts(d, c);
    size_t p = 44;
    int tsize = 4;
    if (version >= 2) {  // skip the 32-bit data block: the 64-bit one follows its own header
        const size_t skip = (size_t)c[3] * 4 + c[3] + (size_t)c[4] * 6 + c[5] + (size_t)c[2] * 8 + c[1] + c[0];
        if (p + skip + 44 > n || std::memcmp(d + p + skip, "TZif", 4) != 0) return false;
        counts(d + p + skip, c);
        p += skip + 44;
        tsize = 8;
    }
    const uint32_t isut = c[0], isstd = c[1], leap = c[2], ntx = c[3], ntyp = c[4], nchar = c[5];
    const size_t need = (size_t)ntx * tsize + ntx + (size_t)ntyp * 6 + nchar + (size_t)leap * (tsize + 4) + isstd + isut;
    if (p + need > n || ntyp == 0 || ntyp > 256) return false;
    const uint8_t* txt = d + p;
    const uint8_t* txi = txt + (size_t)ntx * tsize;
    const uint8_t* typ = txi + ntx;
    z->zone.resize(ntyp);
    for (uint32_t i = 0; i < ntyp; ++i) {
        z->zone[i].offset = (int32_t)be32(typ + 6 * i);
        z->zone[i].isdst = typ[6 * i + 4] != 0;
    }
    z->tx_when.resize(ntx);
    z->tx_index.resize(ntx);
    for (uint32_t i = 0; i < ntx; ++i) {
        z->tx_when[i] = tsize == 8 ? (int64_t)be64(txt + 8 * i) : (int64_t)(int32_t)be32(txt + 4 * i);
        z->tx_index[i] = txi[i];
        if (txi[i] >= ntyp) return false;
    }
    if (ntx == 0) {  // a fixed zone: one fake transition covering all time
        z->tx_when.push_back(kAlpha);
        z->tx_index.push_back(0);
    }
    p += need;
    if (version >= 2 && p < n && d[p] == '\n') {  // the footer: a POSIX TZ string for later times
        const size_t e = std::string((const char*)d + p + 1, n - p - 1).find('\n');
        if (e != std::string::npos) z->extend.assign((const char*)d + p + 1, e);
    }
    // lookupFirstZone
    bool used0 = false;
    for (uint8_t i : z->tx_index) used0 = used0 || i == 0;
    z->first_zone = 0;
    if (used0) {
        int fz = -1;
        if (!z->tx_index.empty() && z->zone[z->tx_index[0]].isdst)
            for (int zi = (int)z->tx_index[0] - 1; zi >= 0 && fz < 0; --zi)
                if (!z->zone[zi].isdst) fz = zi;
        for (int zi = 0; zi < (int)ntyp && fz < 0; ++zi)
            if (!z->zone[zi].isdst) fz = zi;
        z->first_zone = fz < 0 ? 0 : fz;
    }
    return true;
}

extern "C" {

int crane_tz_load_bytes(const uint8_t* data, size_t n, crane_tz** out) {
    if (!out || (!data && n)) return CRANE_E_INVALID;
    *out = nullptr;
    auto* z = new crane_tz();
    if (!tz_parse(data, n, z)) {
        delete z;
        return CRANE_E_INVALID;
    }
    *out = z;
    return CRANE_OK;
}

// time.LoadLocation: "" / "UTC" = UTC; names with ".." or a leading '/' are
// invalid; $ZONEINFO (or zoneinfo_dir when given), then the platform
// directories Go searches on Linux.
int crane_tz_load(const char* name, const char* zoneinfo_dir, crane_tz** out) {
    if (!out) return CRANE_E_INVALID;
    *out = nullptr;
    std::string z = name ? name : "";
    if (z.empty() || z == "UTC") {
        *out = new crane_tz();  // no zones: UTC
        return CRANE_OK;
    }
    if (z.find("..") != std::string::npos || z[0] == '/' || z[0] == '\\') return CRANE_E_INVALID;
    std::vector<std::string> dirs;
    if (zoneinfo_dir && *zoneinfo_dir) dirs.push_back(zoneinfo_dir);
    else {
        const char* env = std::getenv("ZONEINFO");
        if (env && *env) dirs.push_back(env);
        dirs.insert(dirs.end(), {"/usr/share/zoneinfo", "/usr/share/lib/zoneinfo", "/usr/lib/locale/TZ"});
    }
    for (const auto& d : dirs) {
        const std::string path = d + "/" + z;
        FILE* f = std::fopen(path.c_str(), "rb");
        if (!f) continue;
        std::vector<uint8_t> buf;
        uint8_t tmp[4096];
        size_t k;
        while ((k = std::fread(tmp, 1, sizeof tmp, f)) > 0 && buf.size() < (1u << 20)) buf.insert(buf.end(), tmp, tmp + k);
        std::fclose(f);
        return crane_tz_load_bytes(buf.data(), buf.size(), out);
    }
    return CRANE_E_INVALID;
}

void crane_tz_free(crane_tz* tz) { delete tz; }

int crane_tz_lookup(const crane_tz* tz, int64_t unix_s, int32_t* offset_s, int64_t* start_s, int64_t* end_s) {
    if (!tz || !offset_s || !start_s || !end_s) return CRANE_E_INVALID;
    tz->lookup(unix_s, offset_s, start_s, end_s);
    return CRANE_OK;
}

int64_t crane_tz_date(const crane_tz* tz, int64_t local_s) { return tz ? tz->date(local_s) : local_s; }

}  // extern "C"
